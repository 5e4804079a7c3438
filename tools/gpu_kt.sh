#!/bin/bash
# Per-kernel durations of library variants, each kernel alone on the GPU
# (MPG_OVERLAP_MIN=0: one stream, no two-half overlap), from rocprofv3
# --kernel-trace --stats, plus the overlapped bench line of each variant.
# usage: CFG=3 bash tools/gpu_kt.sh name1 name2 ...  ("base" = in-tree build)
set -o pipefail
CFG=${CFG:-3}
export TMPDIR=/tmp
mkdir -p gpurun_out/kt
cp mplib_amd/lib/libmpgpu.so gpurun_out/kt/libmpgpu_base.so
rc=0
for v in "$@"; do
  if [ "$v" = base ]; then src=gpurun_out/kt/libmpgpu_base.so; else src=variants/libmpgpu_$v.so; fi
  cp $src mplib_amd/lib/libmpgpu.so
  timeout -k 10 200 python3 bench.py --cfg $CFG --cpu-sample 0 > gpurun_out/kt/$v.json 2> gpurun_out/kt/$v.err || { echo "$v bench failed"; tail -5 gpurun_out/kt/$v.err; rc=1; break; }
  MPG_OVERLAP_MIN=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/$v -o t --output-format csv -- python3 bench.py --cfg $CFG --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/kt/$v.log 2>&1 || { echo "$v trace failed"; rc=1; break; }
  python3 - "$v" <<'PY'
import csv, glob, json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/kt/{v}.json"))
print("%-10s %.4e configs/s %.4f ms/step (overlapped)" % (v, d["value"], d["ms_per_step"]))
f = glob.glob(f"gpurun_out/kt/{v}/**/*kernel_stats.csv", recursive=True)[0]
tot = 0.0
for r in csv.DictReader(open(f)):
    n, avg = int(r["Calls"]), float(r["AverageNs"]) / 1e3
    tot += float(r["TotalDurationNs"]) / 1e3
    print("   %-40s %4d x %8.1f us" % (r["Name"][:40], n, avg))
print("   alone sum per step: %.1f us" % (tot / 6))
PY
done
cp gpurun_out/kt/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
exit $rc
