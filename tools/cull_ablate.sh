#!/bin/bash
# Cull-kernel phase ablation (cfg3, overlap off): the MPG_DIAG build in
# variants/diag.so under MPG_DEBUG_CULL = 0 (full), 1 (FK + records only),
# 2 (no SAT stage), 8 (no tail: survivor words, tile counts, sincos),
# 9 (no sincos).  Timing only: modes != 0 change results.
set -o pipefail
export TMPDIR=/tmp MPG_OVERLAP_MIN=0
OUT=gpurun_out/${1:-abl}; mkdir -p $OUT
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_orig.so
cp variants/${DIAG:-diag}.so mplib_amd/lib/libmpgpu.so
for m in ${MODES:-0 1 2 8 9}; do
  MPG_DEBUG_CULL=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/m$m -o t --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 > $OUT/m$m.log 2>&1 || { cp /tmp/libmpgpu_orig.so mplib_amd/lib/libmpgpu.so; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/m$m/t_kernel_stats.csv')):
    if 'cull' in r['Name']: print('mode $m cull %.1f us' % (float(r['AverageNs']) / 1e3))
"
done
cp /tmp/libmpgpu_orig.so mplib_amd/lib/libmpgpu.so
