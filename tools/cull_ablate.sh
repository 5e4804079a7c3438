#!/bin/bash
# Where the cull kernel's time goes: the MPG_DIAG build (var_diag.so, built
# with tools/build_variant.sh diag -DMPG_DIAG) under MPG_DEBUG_CULL modes
#   0 full, 1 FK + records only, 2 no SAT (sphere survivors kept), 8 bounding tests + SAT only (no survivor
#   words / tile counts / sincos), 9 everything but the sincos pass
# one cfg3 bench each (stage times from HIP events).
set -o pipefail
mkdir -p gpurun_out
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_base.so
cp mplib_amd/lib/var_diag.so mplib_amd/lib/libmpgpu.so
for m in 0 1 2 8 9; do
  MPG_DEBUG_CULL=$m timeout -k 10 300 python bench.py --cfg ${CFG:-3} --cpu-sample 0 --steps 10 > gpurun_out/abl_$m.json 2> gpurun_out/abl_$m.err || { tail gpurun_out/abl_$m.err; cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/abl_$m.json'));s=d['stages'];print('mode $m cull us/launch', round(s['cull']['ms_per_step']*1e3/2,1))"
done
cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
