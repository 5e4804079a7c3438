#!/bin/bash
# Build mplib_amd/lib/var_<name>.so from the kernel sources of a git commit
# (A/B against an earlier state on one box, tools/ab.sh).  The C ABI must be
# the in-tree one's (the Python host module is not rebuilt).
# usage: bash tools/build_commit.sh <commit> <name>
set -e
C=$1; NAME=$2
T=$(mktemp -d)
mkdir -p $T/mplib_amd/csrc $T/include
for f in $(git ls-tree --name-only $C mplib_amd/csrc/ | grep -E '\.(hip|h)$'); do git show $C:$f > $T/$f; done
git show $C:include/mpgpu.h > $T/include/mpgpu.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result \
  -Wno-unused-value -shared -o mplib_amd/lib/var_$NAME.so $T/mplib_amd/csrc/mpg_kernels.hip
rm -rf $T
