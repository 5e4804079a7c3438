#!/bin/bash
# Build mplib_amd/lib/var_trace.so: the product kernels plus tools/wave_trace.patch
# (narrow_kernel per-wave timeline and latency probe, -DMPG_WAVE_TRACE), for
# tools/gpu_wave_trace.sh.  The product source stays untouched, so the product
# library and its lib_hash do not change.
set -e
cd "$(dirname "$0")/../mplib_amd"
tmp=csrc/mpg_kernels_trace.hip
trap 'rm -f $tmp' EXIT
patch -s -o $tmp csrc/mpg_kernels.hip < ../tools/wave_trace.patch
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result \
  -Wno-unused-value -DMPG_WAVE_TRACE -shared -o lib/var_trace.so $tmp
