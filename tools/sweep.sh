# time prebuilt library variants (variants/libmpgpu_*.so) with the same bench
# (extra VAR=VALUE arguments are exported, e.g. MPG_DEBUG_CULL=1)
set -o pipefail
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_orig.so
for f in variants/libmpgpu_*.so; do
  cp $f mplib_amd/lib/libmpgpu.so
  bash tools/kt.sh $(basename $f .so) "$@" > /tmp/kt.out 2>&1 || { cat /tmp/kt.out; cp /tmp/libmpgpu_orig.so mplib_amd/lib/libmpgpu.so; exit 1; }
  grep -E "==|narrow|cull" /tmp/kt.out
done
cp /tmp/libmpgpu_orig.so mplib_amd/lib/libmpgpu.so
