#!/bin/bash
# PMC counters of the collide kernels, the two-stream overlap off so each
# kernel runs alone (one pass per counter group; --pmc never combined with
# trace domains).  usage: bash tools/pmc_quick.sh <tag> [cfg]
set -o pipefail
TAG=${1:-pq}; CFG=${2:-3}
export TMPDIR=/tmp MPG_OVERLAP_MIN=0
OUT=gpurun_out/$TAG; mkdir -p $OUT
KRE="cull_kernel|narrow_kernel|cand_pose_kernel|pose_pass_kernel|scatter_kernel|closed_form"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d $OUT/p$i -o pmc --output-format csv -- python3 bench.py --cfg $CFG --steps 3 --warmup 1 --cpu-sample 0 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<PY
import csv, glob, re
from collections import defaultdict
v = defaultdict(lambda: defaultdict(list))
for f in glob.glob("$OUT/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"]); k = m.group(1) if m else r["Kernel_Name"][:20]
        v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in v.items():
    a = {n: sum(x) / len(x) for n, x in c.items()}
    wc = a.get("SQ_WAVE_CYCLES", 1)
    print(k, {n: "%.3g" % x for n, x in sorted(a.items())})
    print("   wait_any %.2f wait_inst %.2f active %.2f | lane_act %.2f | valu/wave %.0f salu/wave %.0f f64/wave %.0f" % (
        a.get("SQ_WAIT_ANY", 0) / wc, a.get("SQ_WAIT_INST_ANY", 0) / wc, a.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        a.get("SQ_THREAD_CYCLES_VALU", 0) / max(1, 64 * a.get("SQ_ACTIVE_INST_VALU", 1)),
        a.get("SQ_INSTS_VALU", 0) / max(1, a.get("SQ_WAVES", 1)), a.get("SQ_INSTS_SALU", 0) / max(1, a.get("SQ_WAVES", 1)),
        sum(a.get(x, 0) for x in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")) / max(1, a.get("SQ_WAVES", 1))))
PY
