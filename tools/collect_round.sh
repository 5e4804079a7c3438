#!/bin/bash
# Copy one tools/gpu_round.sh run's outputs from gpurun_out/ into
# profiles/<tag>/ (tracked): bench lines, rocprofv3 kernel stats and PMC
# counters per config, pytest / smoke summaries; the PMC summaries also to
# profiles/pmc_cfg{2,3,4}.json, which bench.py reads for its lib_hash.
# usage: bash tools/collect_round.sh <tag>
set -e
TAG=$1
D=profiles/$TAG
mkdir -p $D
[ -f gpurun_out/bench_${TAG}_final.json ] && cp gpurun_out/bench_${TAG}_final.json $D/bench.json
for c in 2 4 5; do [ -f gpurun_out/bench_${TAG}_cfg$c.json ] && cp gpurun_out/bench_${TAG}_cfg$c.json $D/bench_cfg$c.json; done
if [ -d gpurun_out/prof_$TAG ]; then
  cp gpurun_out/prof_$TAG/trace/trace_kernel_stats.csv $D/kernel_stats.csv
  for p in gpurun_out/prof_$TAG/pmc_*/; do cp $p/pmc_counter_collection.csv $D/$(basename $p).csv; done
  cp gpurun_out/prof_$TAG/pmc_summary.json $D/pmc_summary.json
  cp gpurun_out/prof_$TAG/pmc_summary.json profiles/pmc_cfg3.json
fi
for c in 2 4; do
  if [ -f gpurun_out/prof_${TAG}_cfg$c/pmc_summary.json ]; then
    cp gpurun_out/prof_${TAG}_cfg$c/pmc_summary.json $D/pmc_summary_cfg$c.json
    cp gpurun_out/prof_${TAG}_cfg$c/pmc_summary.json profiles/pmc_cfg$c.json
    cp gpurun_out/prof_${TAG}_cfg$c/trace/trace_kernel_stats.csv $D/kernel_stats_cfg$c.csv
  fi
done
[ -f gpurun_out/pytest_gpu.log ] && tail -3 gpurun_out/pytest_gpu.log > $D/pytest_gpu.txt
[ -f gpurun_out/smoke.log ] && cp gpurun_out/smoke.log $D/smoke.txt
ls $D
