# cfg5 planner: GPU parity tests of the planner, then the far / near bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_planner.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?
tail -2 gpurun_out/pt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --cfg 5 --steps 16 --warmup 2 > gpurun_out/bench_cfg5.json 2>gpurun_out/bench_cfg5.err || exit 1
timeout -k 10 300 python bench.py --cfg 5 --goal near --steps 64 --warmup 2 > gpurun_out/bench_cfg5_near.json 2>gpurun_out/bench_cfg5n.err || exit 1
for f in bench_cfg5 bench_cfg5_near; do
  python3 -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f', d['value'], d['mean_batches'], d['roofline']['kernel_ms'], d['cpu_baseline']['value'], d['cpu_baseline']['gpu_matches_cpu_on_sample'])"
done
