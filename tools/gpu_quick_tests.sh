#!/bin/bash
# a subset of the GPU suite: bash tools/gpu_quick_tests.sh <pytest -k expression>
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -k "$1" -x -v --timeout 300 --timeout-method thread > gpurun_out/quick.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/quick.log | head -40
tail -3 gpurun_out/quick.log
exit $rc
