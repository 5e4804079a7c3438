# Phase-timing ablation of the collide pipeline (diagnostic env switches, read
# only by a library built with `make -C mplib_amd EXTRA=-DMPG_DIAG`, in
# mpg_kernels.hip): MPG_DEBUG_CULL=1 records only, 2 no SAT, 3 no MPR, 8 cull
# without its tail (survivor words, tile counts, sincos), 9 cull without sincos;
# MPG_STATS=1 prints narrow-phase candidate/support counts.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ablate
MPG_STATS=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/ablate/stats.log 2>&1 || exit 1
grep "mpg stats" gpurun_out/ablate/stats.log
for mode in ${MODES:-0 3}; do
  MPG_DEBUG_CULL=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ablate/m$mode -o t --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/ablate/m$mode.log 2>&1 || exit 1
  echo "mode $mode"; python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/ablate/m$mode/t_kernel_stats.csv')): print('  %-40s %10.1f us' % (r['Name'][:40], float(r['AverageNs'])/1e3))"
done
