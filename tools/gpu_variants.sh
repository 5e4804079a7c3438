#!/bin/bash
# A/B of library variants on one GPU box: each variants/libmpgpu_<name>.so is
# swapped in for mplib_amd/lib/libmpgpu.so and the bench runs (cfg given by
# CFG, default 3); the MPG_STATS variant prints its narrow-phase counters.
# usage: bash tools/gpu_variants.sh name1 name2 ...   (name "base" = in-tree build)
set -o pipefail
CFG=${CFG:-3}
mkdir -p gpurun_out/var
cp mplib_amd/lib/libmpgpu.so gpurun_out/var/libmpgpu_base.so
rc=0
for v in "$@"; do
  if [ "$v" = base ]; then src=gpurun_out/var/libmpgpu_base.so; else src=variants/libmpgpu_$v.so; fi
  cp $src mplib_amd/lib/libmpgpu.so
  env ${VENV:-A=1} MPG_STATS=1 timeout -k 10 200 python3 bench.py --cfg $CFG --cpu-sample 0 > gpurun_out/var/$v.json 2> gpurun_out/var/$v.err || { echo "$v failed"; tail -5 gpurun_out/var/$v.err; rc=1; break; }
  python3 -c "
import json
d = json.load(open('gpurun_out/var/$v.json'))
print('%-12s %.4e configs/s %.4f ms' % ('$v', d['value'], d['ms_per_step']), {k: round(x['ms_per_step'], 4) for k, x in d.get('stages', {}).items()})
"
  grep "mpg stats" gpurun_out/var/$v.err | head -2
done
cp gpurun_out/var/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
exit $rc
