# Host-buffer pipeline settings A/B on one box (round 6):
#   bash tools/host_ab.sh "TAG ENV=VAL ..." ...
set -o pipefail
mkdir -p gpurun_out/hp
for spec in "$@"; do
  set -- $spec
  tag=$1; shift
  ( for kv in "$@"; do export "$kv"; done
    MPG_STATS=1 timeout -k 10 200 python3 bench.py --host --steps 20 --warmup 3 --cpu-sample 0 \
      > gpurun_out/hp/$tag.json 2> gpurun_out/hp/$tag.stats ) || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/hp/$tag.json'));print('%-12s %.3e cfg/s  %.3f ms/step' % ('$tag', d['value'], d['ms_per_step']))"
  grep "host pipeline" gpurun_out/hp/$tag.stats
done
