#!/bin/bash
# latency path: parity tests, then the cfg5 bench (one-state round trip, plans/s)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_planner.py -m gpu -k "latency or oracle_path" -x -q --timeout 240 --timeout-method thread > gpurun_out/lat_tests.log 2>&1 || { tail -30 gpurun_out/lat_tests.log; exit 1; }
tail -2 gpurun_out/lat_tests.log
timeout -k 10 300 python bench.py --cfg 5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { tail gpurun_out/bench_cfg5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_cfg5.json'));print({k:d[k] for k in ['value','mean_batches','mean_check_ms','mean_spec_nodes','mean_spec_wait_nodes','mean_spec_ms','mean_states_checked','one_state_round_trip_us_median']}, d['cpu_baseline']['value'], d['roofline']['kernel_ms'])"
for k in "$@"; do
  timeout -k 10 300 python bench.py --cfg 5 --cpu-plans 0 --spec-nodes $k > gpurun_out/bench_cfg5_s$k.json 2> gpurun_out/bench_cfg5_s$k.err || { tail gpurun_out/bench_cfg5_s$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_cfg5_s$k.json'));print($k,{k:d[k] for k in ['value','mean_batches','mean_check_ms','mean_spec_nodes','mean_spec_wait_nodes','mean_spec_ms','mean_states_checked']})"
done
