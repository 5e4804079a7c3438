#!/bin/bash
# Copy one gpurun profile run (tools/gpu_round.sh <tag>) into profiles/<dest>:
# bench line, rocprofv3 kernel stats, PMC counter CSVs and their summary.
# usage: bash tools/collect_profile.sh <tag> <dest>
set -e
TAG=$1; DEST=profiles/$2
SRC=gpurun_out/prof_$TAG
mkdir -p $DEST
cp gpurun_out/bench_$TAG.json $DEST/bench.json
cp $SRC/trace/trace_kernel_stats.csv $DEST/kernel_stats.csv
cp $SRC/pmc_summary.json $DEST/pmc_summary.json
for d in $SRC/pmc_*/; do
  n=$(basename $d)
  cp $d/pmc_counter_collection.csv $DEST/$n.csv
done
cp $DEST/pmc_summary.json profiles/pmc_cfg3.json  # keyed by lib_hash: bench.py uses it only for this build
