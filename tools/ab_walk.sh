#!/bin/bash
# ablation of the float-libccd / FCL-walk semantics costs (results differ from
# the oracle under the MPG_DEBUG_* knobs; timing only)
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 120 env "$@" python bench.py --cpu-sample 0 --steps 10 2>/dev/null | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$*', round(r['value']/1e6), 'Mcfg/s', round(r['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in r['stages'].items()}, int(r['stages']['narrow']['units_per_launch']))"; }
run A=1 && run MPG_DEBUG_NO_WALK=1 && run MPG_DEBUG_MARGIN=1e-4 && run MPG_DEBUG_NO_WALK=1 MPG_DEBUG_MARGIN=1e-4
