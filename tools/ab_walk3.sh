#!/bin/bash
set -o pipefail
run() { timeout -k 10 120 env "$@" python bench.py --cpu-sample 0 --steps 10 2>/dev/null | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$*', round(r['value']/1e6), 'Mcfg/s', round(r['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in r['stages'].items()})"; }
run MPG_WALK_SUBK=1 && run MPG_WALK_SUBK=2 && run MPG_WALK_SUBK=4 && run MPG_WALK_SUBK=8 && run MPG_DEBUG_NO_WALK=1
