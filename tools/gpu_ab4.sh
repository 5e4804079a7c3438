#!/bin/bash
# parity subset on the walk hulls, then variant timings and stats
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_narrow_parity.py tests/test_gpu_parity.py tests/test_multi_art.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sub.log
[ $rc -eq 0 ] || exit $rc
bash tools/sweep.sh && bash tools/stats2.sh
