# A/B of the overlapped parts on the headline bench
set -o pipefail
mkdir -p gpurun_out
for parts in 2 4 3 6 2 4; do
  MPG_OVERLAP_PARTS=$parts timeout -k 10 300 python bench.py --cpu-sample 0 --steps 30 > gpurun_out/ab_$parts.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$parts.json'));print('$parts', round(d['value']/1e9,4), 'e9', round(d['step_ms_events'],4))"
done
