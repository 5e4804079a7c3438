#!/bin/bash
# Copy one tools/gpu_round2.sh run's outputs from gpurun_out/ into
# profiles/<tag>/ (tracked) and its PMC summary into profiles/pmc_cfg3.json.
# usage: bash tools/collect_round.sh <tag>
set -e
TAG=$1
D=profiles/$TAG
mkdir -p $D
cp gpurun_out/bench_${TAG}_final.json $D/bench.json
for c in 2 4 5; do cp gpurun_out/bench_${TAG}_cfg$c.json $D/bench_cfg$c.json; done
cp gpurun_out/prof_$TAG/trace/trace_kernel_stats.csv $D/kernel_stats.csv
for p in gpurun_out/prof_$TAG/pmc_*/; do
  n=$(basename $p)
  cp $p/pmc_counter_collection.csv $D/$n.csv
done
cp gpurun_out/prof_$TAG/pmc_summary.json $D/pmc_summary.json
cp gpurun_out/prof_$TAG/pmc_summary.json profiles/pmc_cfg3.json
for c in 2 4; do  # tools/gpu_round3.sh: per-config PMC records
  if [ -f gpurun_out/prof_${TAG}_cfg$c/pmc_summary.json ]; then
    cp gpurun_out/prof_${TAG}_cfg$c/pmc_summary.json $D/pmc_summary_cfg$c.json
    cp gpurun_out/prof_${TAG}_cfg$c/pmc_summary.json profiles/pmc_cfg$c.json
    cp gpurun_out/prof_${TAG}_cfg$c/trace/trace_kernel_stats.csv $D/kernel_stats_cfg$c.csv
  fi
done
tail -3 gpurun_out/pytest_gpu.log > $D/pytest_gpu.txt
cp gpurun_out/smoke.log $D/smoke.txt
ls $D
