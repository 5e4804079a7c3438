#!/bin/bash
# Where the cull kernel's time goes, one stream (MPG_OVERLAP_MIN=0: no
# second stream sharing the CUs, so the rocprof kernel time is the kernel's
# own): the MPG_DIAG build (tools/build_variant.sh diag -DMPG_DIAG) under
# MPG_DEBUG_CULL modes
#   0 full, 1 FK + records, 2 no SAT (sphere survivors kept), 8 bounding
#   tests + SAT, 9 all but sincos, 11 bounding tests only (no queue / SAT),
#   12 full without the static-partner bounding tests, 13 FK without the
#   rq stores, 14 launch + output zeroing only
# usage: bash tools/cull_iso.sh <out dir> [bench args]
set -o pipefail
OUT=${1:-gpurun_out/cull_iso}; shift
mkdir -p $OUT
export TMPDIR=/tmp MPG_OVERLAP_MIN=0
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_base.so
cp mplib_amd/lib/var_diag.so mplib_amd/lib/libmpgpu.so
for m in ${MODES:-0 1 2 8 9 11 12}; do
  MPG_DEBUG_CULL=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/m$m -o t --output-format csv -- \
    python3 bench.py --cpu-sample 0 --steps 10 --warmup 2 "$@" > $OUT/m$m.log 2>&1 || { tail $OUT/m$m.log; cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so; exit 1; }
  python3 - $OUT/m$m $m <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "cull_kernel" in r["Name"]:
        print("mode", sys.argv[2], "cull avg us", round(float(r["AverageNs"]) / 1e3, 1), "calls", r["Calls"])
PY
done
cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
