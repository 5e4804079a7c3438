#!/bin/bash
# cfg2 / cfg3 narrow time with the walk-hull support off (MPG_DIAG library, linear support): how much of
# the narrow phase the neighbour-walk climbs cost
set -o pipefail
for nw in 0 1; do
  for c in 2 3; do
    MPG_DEBUG_NO_WALK=$nw LD_LIBRARY_PATH=$PWD/variants/diag timeout -k 10 200 python bench.py --cfg $c --cpu-sample 0 > gpurun_out/nw.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/nw.json'));s=d['stages'];print('nowalk=$nw cfg$c', round(d['value']/1e6,1), 'M/s', {k: round(v['ms_per_step']*1e3,1) for k,v in s.items()})"
  done
done
