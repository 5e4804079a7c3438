#!/bin/bash
# latency-path split with the MPG_DIAG library (var_diag.so): full (0), no
# narrow test (3), the bare launch (10)
set -o pipefail
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_base.so
cp mplib_amd/lib/var_diag.so mplib_amd/lib/libmpgpu.so
for m in 0 3 10; do
  MPG_DEBUG_CULL=$m timeout -k 10 120 python tools/lat_ab.py diag_mode$m || { cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so; exit 1; }
done
cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
