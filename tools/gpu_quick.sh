# quick GPU iteration: full GPU tests, latency micro-bench, cfg5 planner bench, cfg3 bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/latency.py > gpurun_out/latency.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/latency.log
timeout -k 10 400 python -u tools/bench_plan.py --seeds 16 --cpu-seeds 4 --out gpurun_out/bench_plan.json > gpurun_out/bench_plan.log 2>&1 || exit 1
grep -v "sampled a new\|invalid start\|amdgpu.ids" gpurun_out/bench_plan.log | cut -c1-400
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_q.json 2>gpurun_out/bench_q.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_q.json'));print(d['value'], d['stages'])"
