#!/bin/bash
# One iteration on the GPU box: the GPU suite (or a -k subset), the cfg3 and
# cfg2 bench lines, rocprofv3 kernel stats of both, and the MPG_STATS build in
# variants/ (if present) for the narrow-phase counters.
# usage: bash tools/gpu_iter.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-it}; K=${2:-}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KA[@]}" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/$TAG/bench3.json 2> gpurun_out/$TAG/bench3.err || { tail gpurun_out/$TAG/bench3.err; exit 1; }
timeout -k 10 300 python bench.py --cfg 2 --cpu-sample 0 > gpurun_out/$TAG/bench2.json 2> gpurun_out/$TAG/bench2.err || { tail gpurun_out/$TAG/bench2.err; exit 1; }
python3 -c "
import json
for c in (3, 2):
    d = json.load(open('gpurun_out/$TAG/bench%d.json' % c))
    print('cfg%d' % c, '%.3e configs/s' % d['value'], '%.4f ms/step' % d['ms_per_step'], {k: round(v['ms_per_step'], 4) for k, v in d.get('stages', {}).items()})
"
for c in 3 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/kt$c -o t --output-format csv -- python3 bench.py --cfg $c --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/$TAG/kt$c.log 2>&1 || exit 1
  echo "== kernels cfg$c"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/$TAG/kt$c/t_kernel_stats.csv')):
    print('  %-44s %6d calls %10.1f us' % (r['Name'][:44], int(r['Calls']), float(r['AverageNs']) / 1e3))
"
done
