#!/bin/bash
# Round evidence in one GPU call: full GPU suite, smoke, then rocprofv3
# kernel-trace + PMC passes of the cfg3, cfg2 and cfg4 benches (tools/profile.sh,
# each config's PMC record keyed to this build), then the bench lines for
# cfg3 (default), cfg2, cfg4 and cfg5 with those records.
# usage: bash tools/gpu_round3.sh <tag>
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
NCFG=524288 bash tools/profile.sh $TAG || exit 1
cp gpurun_out/prof_$TAG/pmc_summary.json profiles/pmc_cfg3.json
NCFG=65536 bash tools/profile.sh ${TAG}_cfg2 --cfg 2 || exit 1
cp gpurun_out/prof_${TAG}_cfg2/pmc_summary.json profiles/pmc_cfg2.json
NCFG=1048576 bash tools/profile.sh ${TAG}_cfg4 --cfg 4 || exit 1
cp gpurun_out/prof_${TAG}_cfg4/pmc_summary.json profiles/pmc_cfg4.json
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}_final.json 2> gpurun_out/bench_${TAG}_final.err || { tail gpurun_out/bench_${TAG}_final.err; exit 1; }
cat gpurun_out/bench_${TAG}_final.json
for c in 2 4 5; do
  timeout -k 10 300 python bench.py --cfg $c > gpurun_out/bench_${TAG}_cfg$c.json 2> gpurun_out/bench_${TAG}_cfg$c.err || { tail gpurun_out/bench_${TAG}_cfg$c.err; exit 1; }
  head -c 300 gpurun_out/bench_${TAG}_cfg$c.json; echo
done
