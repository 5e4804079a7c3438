# Host-buffer pipeline diagnosis (round 6): MPG_STATS host phase sums and a
# rocprofv3 kernel + memory-copy timeline of bench.py --host.
#   bash tools/host_prof.sh TAG [ENV=VAL ...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
for kv in "$@"; do export "$kv"; done
mkdir -p gpurun_out/hp
MPG_STATS=1 timeout -k 10 200 python3 bench.py --host --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/hp/$tag.json 2> gpurun_out/hp/$tag.stats || exit 1
grep "host pipeline" gpurun_out/hp/$tag.stats
python3 -c "import json;d=json.load(open('gpurun_out/hp/$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace -d gpurun_out/hp/${tag}_trace -o t --output-format csv -- python3 bench.py --host --steps 4 --warmup 1 --cpu-sample 0 > gpurun_out/hp/${tag}_trace.log 2>&1 || exit 1
