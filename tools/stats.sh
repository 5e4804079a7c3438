# narrow-phase section timing (s_memtime stamps) with the MPG_STATS build
set -o pipefail
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_orig.so
cp variants/libmpgpu_stats.so mplib_amd/lib/libmpgpu.so
MPG_STATS=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 > gpurun_out/stats.log 2>&1; rc=$?
cp /tmp/libmpgpu_orig.so mplib_amd/lib/libmpgpu.so
grep "mpg stats" gpurun_out/stats.log; exit $rc
