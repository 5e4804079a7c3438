# headline bench, 3 repetitions (quick A/B against the previous commit's numbers)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-sample 0 --steps 30 > gpurun_out/ab_$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print(round(d['value']/1e9,4), 'e9', round(d['step_ms_events'],4), {k:round(v['ms_per_step'],4) for k,v in d['stages'].items()})"
done
