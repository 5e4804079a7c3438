#!/bin/bash
# narrow-phase minimum task size (MPG_TASK_MIN builds in variants/tmN): cfg2 and cfg3 bench lines
set -o pipefail
for v in product tm16 tm32 tm64; do
  if [ $v = product ]; then LP=""; else LP=$PWD/variants/$v; fi
  for c in 2 3; do
    LD_LIBRARY_PATH=$LP timeout -k 10 200 python bench.py --cfg $c --cpu-sample 0 > gpurun_out/tm.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/tm.json'));s=d['stages'];print('$v cfg$c', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,1), 'us', {k: round(v['ms_per_step']*1e3,1) for k,v in s.items()})"
  done
done
