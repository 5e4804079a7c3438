#!/bin/bash
# Round evidence in one GPU call: full GPU suite, smoke, bench lines for
# cfg3 (default), cfg2, cfg4, cfg5, then the rocprofv3 kernel-trace and PMC
# passes of the cfg3 bench (tools/profile.sh).
# usage: bash tools/gpu_round2.sh <tag>
set -o pipefail
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
for c in 2 4 5; do
  timeout -k 10 300 python bench.py --cfg $c > gpurun_out/bench_${TAG}_cfg$c.json 2> gpurun_out/bench_${TAG}_cfg$c.err || { tail gpurun_out/bench_${TAG}_cfg$c.err; exit 1; }
  head -c 400 gpurun_out/bench_${TAG}_cfg$c.json; echo
done
NCFG=524288 bash tools/profile.sh $TAG
# the bench line again with the PMC record of this very build (valu_roofline, traffic)
cp gpurun_out/prof_$TAG/pmc_summary.json profiles/pmc_cfg3.json
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}_final.json 2> gpurun_out/bench_${TAG}_final.err || { tail gpurun_out/bench_${TAG}_final.err; exit 1; }
cat gpurun_out/bench_${TAG}_final.json
