#!/bin/bash
# Step time and kernel times of the in-tree library and every
# variants/libmpgpu_*.so on cfg3 and cfg2: the bench line (ms per step), then
# rocprofv3 kernel stats with the two-stream overlap off (MPG_OVERLAP_MIN=0,
# so each kernel runs alone), then the MPG_STATS counters of variants/stats.so
# (if present).  usage: bash tools/gpu_sweep.sh <tag> [cfgs]
set -o pipefail
TAG=${1:-sw}; CFGS=${2:-"3 2"}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
cp mplib_amd/lib/libmpgpu.so /tmp/libmpgpu_orig.so
restore() { cp /tmp/libmpgpu_orig.so mplib_amd/lib/libmpgpu.so; }
# ENVS="A=1;B=0 C=1": extra runs of the in-tree library under those settings
IFS=';' read -ra EXTRA <<< "${ENVS:-}"
RUNS=(/tmp/libmpgpu_orig.so)
for e in "${EXTRA[@]}"; do RUNS+=("env:$e"); done
for f in variants/libmpgpu_*.so; do RUNS+=("$f"); done
for f in "${RUNS[@]}"; do
  if [[ $f == env:* ]]; then
    v=$(echo "${f#env:}" | tr ' =' '_-'); cp /tmp/libmpgpu_orig.so mplib_amd/lib/libmpgpu.so
    for kv in ${f#env:}; do export "$kv"; done
  else
    [ -f "$f" ] || continue
    v=$(basename $f .so); cp $f mplib_amd/lib/libmpgpu.so
  fi
  for c in $CFGS; do
    timeout -k 10 200 python3 bench.py --cfg $c --cpu-sample 0 > gpurun_out/$TAG/$v-$c.json 2> gpurun_out/$TAG/$v-$c.err || { restore; tail gpurun_out/$TAG/$v-$c.err; exit 1; }
    MPG_OVERLAP_MIN=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/$v-$c -o t --output-format csv -- python3 bench.py --cfg $c --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/$TAG/$v-$c.log 2>&1 || { restore; exit 1; }
    python3 -c "
import csv, json, re
d = json.load(open('gpurun_out/$TAG/$v-$c.json'))
r = {}
for row in csv.DictReader(open('gpurun_out/$TAG/$v-$c/t_kernel_stats.csv')):
    m = re.search(r'(\w+_kernel|\w+Buffer\w*)', row['Name'])
    r[(m.group(1) if m else row['Name'])[:18]] = float(row['AverageNs']) / 1e3
print('%-16s cfg$c %.4f ms %.3e/s |' % ('$v', d['ms_per_step'], d['value']), ' '.join('%s=%.1f' % (k.replace('_kernel', ''), v) for k, v in sorted(r.items(), key=lambda kv: -kv[1])[:6]))
"
  done
  if [[ $f == env:* ]]; then for kv in ${f#env:}; do unset "${kv%%=*}"; done; fi
done
restore
if [ -f variants/stats.so ]; then
  cp variants/stats.so mplib_amd/lib/libmpgpu.so
  for c in $CFGS; do
    MPG_OVERLAP_MIN=0 MPG_STATS=1 timeout -k 10 200 python3 bench.py --cfg $c --steps 2 --warmup 0 --cpu-sample 0 > gpurun_out/$TAG/stats$c.log 2>&1; rc=$?
    echo "== stats cfg$c"; grep "mpg stats" gpurun_out/$TAG/stats$c.log
    [ $rc -eq 0 ] || { restore; exit $rc; }
  done
  restore
fi
