#!/bin/bash
# kernel durations of the latency path (n = 1 and 12 states) under rocprofv3
set -o pipefail
mkdir -p gpurun_out/latprof
export TMPDIR=/tmp
for n in 1 12; do
  LAT_N=$n timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/latprof/n$n -o lat --output-format csv -- python3 tools/lat_ab.py prof_n$n > gpurun_out/latprof/n$n.log 2>&1 || { tail gpurun_out/latprof/n$n.log; exit 1; }
  tail -1 gpurun_out/latprof/n$n.log
  python3 - <<PY
import csv, glob
for f in glob.glob('gpurun_out/latprof/n$n/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('n=$n', r['Name'][:70], r['Calls'], 'avg us', round(float(r['AverageNs'])/1e3, 2), 'min', round(float(r['MinNs'])/1e3, 2))
PY
done
