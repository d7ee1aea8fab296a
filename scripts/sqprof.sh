#!/bin/bash
# SQ instruction / stall counters per kernel (one rocprofv3 --pmc pass per
# group, each under its own kill timer; never with sys/runtime traces).
# usage: bash scripts/sqprof.sh <tag> [workload]   -> gpurun_out/sq_<tag>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-x}; WL=${2:-c2}
OUT=gpurun_out/sq_${TAG}
mkdir -p $OUT
i=0
[ -n "$SQ_GROUPS" ] || SQ_GROUPS="1 2 3"
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU" \
         "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  [[ " $SQ_GROUPS " == *" $i "* ]] || continue
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $OUT/g$i -o run -- \
    python3 scripts/profile_run.py --workload $WL --steps 2 > $OUT/g$i.log 2>&1 || { echo "group $i failed"; tail -5 $OUT/g$i.log; exit 1; }
done
python3 scripts/sq_summary.py $OUT
