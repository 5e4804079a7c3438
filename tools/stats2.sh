#!/bin/bash
# narrow-phase stats of the MPG_STATS build under two settings (walk / no walk)
set -o pipefail
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_orig.so
cp variants_stats/libmpgpu_stats.so mplib_amd/lib/libmpgpu.so
for e in A=1 MPG_DEBUG_NO_WALK=1; do
  echo "== $e"
  env $e MPG_STATS=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 2>&1 >/dev/null | grep "mpg stats" | head -2
done
cp /tmp/libmpgpu_orig.so mplib_amd/lib/libmpgpu.so
