# quick GPU iteration: full GPU tests, latency micro-bench, headline bench line, cfg5 / cfg6 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/latency.py > gpurun_out/latency.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_cfg3.json 2>gpurun_out/bench_cfg3.err || exit 1
timeout -k 10 300 python bench.py --cfg 6 --cpu-sample 8192 > gpurun_out/bench_cfg6.json 2>gpurun_out/bench_cfg6.err || exit 1
timeout -k 10 400 python bench.py --cfg 5 --steps 16 --warmup 2 > gpurun_out/bench_cfg5.json 2>gpurun_out/bench_cfg5.err || exit 1
timeout -k 10 300 python bench.py --cfg 5 --goal near --steps 64 --warmup 2 > gpurun_out/bench_cfg5_near.json 2>gpurun_out/bench_cfg5n.err || exit 1
for f in cfg3 cfg6 cfg5 cfg5_near; do python3 -c "import json;d=json.load(open('gpurun_out/bench_$f.json'));print('$f', d['value'], d['unit'], d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('gpu_matches_cpu_on_sample'))"; done
