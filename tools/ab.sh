#!/bin/bash
# A/B the library builds mplib_amd/lib/var_<name>.so (built here with
# tools/build_variant.sh) on one box: each is copied over lib/libmpgpu.so in
# turn and benched (cfg given by CFG, default 3); the in-tree build is "base".
# usage: CFG=3 bash tools/ab.sh name1 name2 ...   -> gpurun_out/ab_<name>.json
set -o pipefail
CFG=${CFG:-3}
mkdir -p gpurun_out
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_base.so
for v in base "$@"; do
  if [ "$v" = base ]; then cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so; else cp mplib_amd/lib/var_$v.so mplib_amd/lib/libmpgpu.so; fi
  timeout -k 10 300 python bench.py --cfg $CFG --cpu-sample 0 $BENCH_ARGS > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail gpurun_out/ab_$v.err; cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));s=d.get('stages',{});print('$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms', {k: round(x['ms_per_step']*1e3,1) for k,x in s.items()})"
done
cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
