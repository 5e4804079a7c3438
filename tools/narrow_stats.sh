#!/bin/bash
# MPG_STATS counters of the narrow stage (tools/build_variant.sh stats
# -DMPG_STATS): support / update ticks, steps, lanes per step.
# usage: bash tools/narrow_stats.sh <out file> [bench args]
set -o pipefail
OUT=${1:-gpurun_out/narrow_stats.txt}; shift
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_base.so
cp mplib_amd/lib/var_stats.so mplib_amd/lib/libmpgpu.so
MPG_STATS=1 timeout -k 10 200 python3 bench.py --cpu-sample 0 --steps 5 --warmup 1 "$@" > $OUT 2>&1; rc=$?
cp /tmp/libmpgpu_base.so mplib_amd/lib/libmpgpu.so
exit $rc
