#!/bin/bash
# narrow_kernel per-wave timeline (var_trace.so from tools/build_trace_variant.sh):
# the last launch's wave starts / ends, slowest waves, lifetimes.
# usage: bash tools/gpu_wave_trace.sh "<cfg> <per-gpu>" ...
set -o pipefail
mkdir -p gpurun_out
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_base.so
cp mplib_amd/lib/var_${VAR:-trace}.so mplib_amd/lib/libmpgpu.so
rc=0
for cn in "$@"; do
  set -- $cn
  echo "== ${VAR:-trace} cfg$1 n=$2"
  MPG_STATS=1 timeout -k 10 200 python3 bench.py --cfg $1 --per-gpu $2 --cpu-sample 0 --steps 5 --warmup 1 > gpurun_out/trace.json 2> gpurun_out/trace.err || { rc=1; break; }
  grep -h "mpg trace" gpurun_out/trace.err || true
  python3 -c "import json;d=json.load(open('gpurun_out/trace.json'));print({k: round(v['ms_per_step']*1e3,1) for k,v in d['stages'].items()})"
done
cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
exit $rc
