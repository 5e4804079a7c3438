#!/bin/bash
# cfg2 bench under overlap settings (MPG_OVERLAP_MIN / MPG_OVERLAP_PARTS)
set -o pipefail
for v in "1048576 2" "65536 2" "65536 4" "32768 2"; do
  set -- $v
  MPG_OVERLAP_MIN=$1 MPG_OVERLAP_PARTS=$2 timeout -k 10 200 python bench.py --cfg 2 --cpu-sample 0 > gpurun_out/c2.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/c2.json'));print('$1 $2', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,1), 'us')"
done
