#!/bin/bash
# full GPU test suite, then the cfg3 bench under rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/kt.sh head > /tmp/kt.out 2>&1 && grep -E "==|narrow|cull" /tmp/kt.out && grep -h '^{' gpurun_out/kt/head.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['value']/1e6), 'Mcfg/s', r['ms_per_step'], {k: round(v['ms_per_step'],3) for k,v in r['stages'].items()})"
