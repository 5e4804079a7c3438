#!/bin/bash
# One GPU call for a round's evidence.
#   bash tools/gpu_round.sh <tag> [tests] [prof] [bench]
#   tests : full GPU suite + smoke
#   prof  : rocprofv3 kernel-trace/stats + PMC passes for cfg3, cfg2, cfg4
#           (tools/profile.sh; each config's PMC record keyed to this build)
#   bench : bench lines for cfg3 (default), cfg2, cfg4, cfg5
#   extra : bench.py --host and --capi-multi 1 --gather
# Every step has its own time limit; the first failure ends the call.
set -o pipefail
TAG=${1:-r04}; shift
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
    echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
    tail -1 gpurun_out/smoke.log ;;
  prof)
    NCFG=1048576 bash tools/profile.sh $TAG || exit 1
    cp gpurun_out/prof_$TAG/pmc_summary.json profiles/pmc_cfg3.json
    NCFG=65536 bash tools/profile.sh ${TAG}_cfg2 --cfg 2 || exit 1
    cp gpurun_out/prof_${TAG}_cfg2/pmc_summary.json profiles/pmc_cfg2.json
    NCFG=1048576 bash tools/profile.sh ${TAG}_cfg4 --cfg 4 || exit 1
    cp gpurun_out/prof_${TAG}_cfg4/pmc_summary.json profiles/pmc_cfg4.json ;;
  bench)
    timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}_final.json 2> gpurun_out/bench_${TAG}_final.err || { tail gpurun_out/bench_${TAG}_final.err; exit 1; }
    head -c 400 gpurun_out/bench_${TAG}_final.json; echo
    for c in 2 4 5; do
      timeout -k 10 300 python bench.py --cfg $c > gpurun_out/bench_${TAG}_cfg$c.json 2> gpurun_out/bench_${TAG}_cfg$c.err || { tail gpurun_out/bench_${TAG}_cfg$c.err; exit 1; }
      head -c 300 gpurun_out/bench_${TAG}_cfg$c.json; echo
    done ;;
  extra)  # round 6: host-buffer line, the in-process multi-GPU C route (one GPU here)
    timeout -k 10 300 python bench.py --host > gpurun_out/bench_${TAG}_host.json 2> gpurun_out/bench_${TAG}_host.err || { tail gpurun_out/bench_${TAG}_host.err; exit 1; }
    head -c 400 gpurun_out/bench_${TAG}_host.json; echo
    timeout -k 10 300 python bench.py --capi-multi 1 --gather > gpurun_out/bench_${TAG}_capi1.json 2> gpurun_out/bench_${TAG}_capi1.err || { tail gpurun_out/bench_${TAG}_capi1.err; exit 1; }
    head -c 400 gpurun_out/bench_${TAG}_capi1.json; echo ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
