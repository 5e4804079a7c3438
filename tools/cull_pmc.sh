#!/bin/bash
# PMC counters of cull_kernel alone (MPG_OVERLAP_MIN=0, one stream) under the
# MPG_DIAG build's MPG_DEBUG_CULL modes (tools/cull_iso.sh lists them); one
# counter group per rocprofv3 pass.  usage: bash tools/cull_pmc.sh <out> [bench args]
set -o pipefail
OUT=${1:-gpurun_out/cull_pmc}; shift
mkdir -p $OUT
export TMPDIR=/tmp MPG_OVERLAP_MIN=0
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_base.so
[ -f mplib_amd/lib/var_diag.so ] && cp mplib_amd/lib/var_diag.so mplib_amd/lib/libmpgpu.so
for m in ${MODES:-13 0}; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU"; do
    name=$(echo $grp | cut -d' ' -f1-2 | tr ' ' '_')
    MPG_DEBUG_CULL=$m timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex cull_kernel -d $OUT/m${m}_$name -o pmc \
      --output-format csv -- python3 bench.py --cpu-sample 0 --steps 4 --warmup 1 "$@" > $OUT/m${m}_$name.log 2>&1 || { echo "mode $m $grp failed"; tail -5 $OUT/m${m}_$name.log; cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so; exit 1; }
  done
  python3 - $OUT $m <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"{sys.argv[1]}/m{sys.argv[2]}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 0
disp = {}
for f in glob.glob(f"{sys.argv[1]}/m{sys.argv[2]}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        disp.setdefault(f, set()).add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
nd = max(len(v) for v in disp.values()) if disp else 1
w = acc.get("SQ_WAVES", 1.0) or 1.0
print(f"mode {sys.argv[2]} dispatches {nd}: " + ", ".join(f"{k}={v / nd:.4g}" for k, v in sorted(acc.items())))
print(f"  per wave: " + ", ".join(f"{k}={v / w:.1f}" for k, v in sorted(acc.items()) if k != "SQ_WAVES"))
PY
done
cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
