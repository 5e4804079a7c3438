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
python3 - "$DEST" <<'PY'
import json, sys
d = sys.argv[1]
s = json.load(open(f"{d}/pmc_summary.json"))
out = {"configs_per_launch": s["configs_per_launch"],
       "source": f"{d} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py cfg3)",
       "correction": "bytes = 2*FETCH_SIZE(KiB)*1024 + WRITE_SIZE(KiB)*1024 (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE counts half of wide reads)",
       "hbm_bytes_per_launch": {k: s["hbm_bytes_per_launch"][k] for k in ("cull", "narrow") if k in s["hbm_bytes_per_launch"]}}
json.dump(out, open("profiles/pmc_cfg3.json", "w"), indent=1)
PY
