set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcq; mkdir -p $OUT
BENCH="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0"
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  name=$(echo $grp | cut -c1-20 | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-narrow_kernel}" -d $OUT/$name -o pmc --output-format csv -- $BENCH > $OUT/$name.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv,glob,collections
v=collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmcq/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)): v[r['Counter_Name']].append(float(r['Counter_Value']))
for k,x in sorted(v.items()): print(k, sum(x)/len(x))
PY
