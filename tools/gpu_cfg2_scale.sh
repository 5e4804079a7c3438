#!/bin/bash
# cfg2 stage times against the batch size: is the narrow phase at 2^16 a
# fixed latency (slowest wave) or throughput?  usage: bash tools/gpu_cfg2_scale.sh
set -o pipefail
mkdir -p gpurun_out
for n in 1024 4096 16384 65536 262144; do
  timeout -k 10 200 python bench.py --cfg 2 --per-gpu $n --cpu-sample 0 --steps 20 --warmup 3 > gpurun_out/s.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/s.json'));s=d['stages'];print('cfg2 n=$n', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,1), 'us', {k: (round(v['ms_per_step']*1e3,1), int(v['units_per_launch'])) for k,v in s.items()})"
done
