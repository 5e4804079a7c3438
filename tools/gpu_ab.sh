#!/bin/bash
# full GPU suite, then kernel timings of every variants/*.so, the NO_WALK
# ablation and the stats build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/sweep.sh && bash tools/kt.sh nowalk MPG_DEBUG_NO_WALK=1 > /tmp/kt2.out 2>&1 && grep -E "==|narrow|cull" /tmp/kt2.out && bash tools/stats2.sh
