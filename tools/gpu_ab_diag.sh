#!/bin/bash
# same-box A/B: product library vs the MPG_DIAG build (variants/diag), cfg2 and cfg3 stage times
set -o pipefail
for rep in 1 2; do
for v in product diag; do
  if [ $v = product ]; then LP=""; else LP=$PWD/variants/diag; fi
  for c in 2 3; do
    LD_LIBRARY_PATH=$LP timeout -k 10 200 python bench.py --cfg $c --cpu-sample 0 > gpurun_out/ab.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));s=d['stages'];print('$v cfg$c', round(d['value']/1e6,1), 'M/s', {k: round(v['ms_per_step']*1e3,1) for k,v in s.items()}, d['lib_hash'])"
  done
done
done
