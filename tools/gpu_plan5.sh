#!/bin/bash
# cfg5 planner check on the GPU: device-vs-oracle path test, then cfg5 bench lines
# (default, and each --spec-nodes value given as an argument)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_planner.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/plan_tests.log 2>&1 || { tail -30 gpurun_out/plan_tests.log; exit 1; }
tail -2 gpurun_out/plan_tests.log
timeout -k 10 300 python bench.py --cfg 5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { tail gpurun_out/bench_cfg5.err; exit 1; }
cat gpurun_out/bench_cfg5.json
for k in "$@"; do
  timeout -k 10 300 python bench.py --cfg 5 --cpu-plans 0 --spec-nodes $k > gpurun_out/bench_cfg5_s$k.json 2> gpurun_out/bench_cfg5_s$k.err || { tail gpurun_out/bench_cfg5_s$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_cfg5_s$k.json'));print($k,{k:d[k] for k in ['value','mean_batches','mean_check_ms','mean_spec_nodes','mean_spec_wait_nodes','mean_spec_ms','mean_states_checked']})"
done
