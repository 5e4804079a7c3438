set -o pipefail
TAG=${1:-cur}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/prof_${TAG}.log 2>&1; echo "prof rc=$?"
cat gpurun_out/prof_${TAG}/trace_kernel_stats.csv | cut -c1-200
