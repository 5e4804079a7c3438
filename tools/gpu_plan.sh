set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_planner.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_plan.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_plan.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_plan.py --seeds 16 --cpu-seeds 4 --out gpurun_out/bench_plan.json > gpurun_out/bench_plan.log 2>&1; rc=$?
grep -v "sampled a new\|invalid start" gpurun_out/bench_plan.log | tail -5
exit $rc
