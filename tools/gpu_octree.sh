# Point-cloud workload: GPU parity tests of the octree walk, cfg6 bench line, rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "cloud" -x -q --timeout 240 --timeout-method thread > gpurun_out/oct.log 2>&1; rc=$?
tail -2 gpurun_out/oct.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --cfg 6 --steps 10 --warmup 2 ${CPU:-} > gpurun_out/bench_cfg6.json 2> gpurun_out/bench_cfg6.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_cfg6.json'));print(d['value'], d['ms_per_step'], d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('gpu_matches_cpu_on_sample'))"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg6 -o trace --output-format csv -- python3 bench.py --cfg 6 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_cfg6.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_cfg6/trace_kernel_stats.csv')):
    print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e6, 4), 'ms')
"
