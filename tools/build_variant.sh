#!/bin/bash
# Build mplib_amd/lib/var_<name>.so with extra hipcc flags (A/B experiments,
# tools/ab.sh).  usage: bash tools/build_variant.sh <name> "-DFOO=1 ..."
set -e
cd mplib_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result \
  -Wno-unused-value $2 -shared -o lib/var_$1.so csrc/mpg_kernels.hip
