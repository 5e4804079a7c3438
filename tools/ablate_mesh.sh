set -o pipefail
for m in 0 5 6; do
  MPG_DEBUG_CULL=$m timeout -k 10 200 python bench.py --cfg 7 --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/abl_$m.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/abl_$m.json'));print('mode $m', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms')"
done
