set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ablate
for mode in 0 1 2; do
  MPG_DEBUG_CULL=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ablate/m$mode -o t --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/ablate/m$mode.log 2>&1 || exit 1
  echo "mode $mode"; cut -d, -f1,4 gpurun_out/ablate/m$mode/t_kernel_stats.csv | cut -c1-60,150-
done
