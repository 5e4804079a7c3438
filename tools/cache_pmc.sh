#!/bin/bash
# Cache-level PMC of the narrow / cull kernels (cfg3): instruction and scalar
# caches (SQC), vector L1 (TCP), L2 (TCC); one rocprofv3 pass per block.
# usage: bash tools/cache_pmc.sh <tag> [bench args]  -> gpurun_out/cache_<tag>/
set -o pipefail
TAG=${1:-x}; shift
OUT=gpurun_out/cache_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 $*"
KRE="cull_kernel|narrow_kernel"
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $grp | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d $OUT/pmc_$name -o pmc --output-format csv -- $BENCH > $OUT/pmc_$name.log 2>&1 || { echo "pass $grp failed rc=$?"; tail -5 $OUT/pmc_$name.log; exit 1; }
  echo "pass $grp ok"
done
