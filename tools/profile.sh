#!/bin/bash
# rocprofv3 evidence for the round: one kernel-trace/stats pass, then PMC passes
# one counter group each (FETCH_SIZE and WRITE_SIZE never share a pass; --pmc
# never combined with trace domains), as MI355X_MICROARCH.md prescribes.
# usage: bash tools/profile.sh <tag> [bench args...]   -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 $*"
KRE="cull_kernel|narrow_kernel|scatter_kernel|pair_scan|chunk_scan|closed_form"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- $BENCH > $OUT/trace.log 2>&1 || exit 1
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  name=$(echo $grp | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d $OUT/pmc_$name -o pmc --output-format csv -- $BENCH > $OUT/pmc_$name.log 2>&1 || { echo "pass $grp failed rc=$?"; exit 1; }
done
python3 tools/pmc_summary.py $OUT ${NCFG:-1048576} $OUT/pmc_summary.json
