# kernel timings of one bench config under rocprofv3: bash tools/kt.sh TAG [ENV=VAL ...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/kt
env "$@" true
for kv in "$@"; do export "$kv"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/$tag -o t --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 ${BENCH_ARGS} > gpurun_out/kt/$tag.log 2>&1 || exit 1
echo "== $tag $*"; python3 -c "
import csv
tot=0
for r in csv.DictReader(open('gpurun_out/kt/$tag/t_kernel_stats.csv')):
    a=float(r['AverageNs'])/1e3; tot+=a*int(r['Calls'])
    print('  %-40s %10.1f us' % (r['Name'][:40], a))
"
