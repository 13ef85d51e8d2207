#!/bin/bash
# GPU-box script: rocprofv3 PMC passes for one kernel (KRE) -> gpurun_out/pmc_$TAG_*/
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
W=${WORDS:-2000000}; T=${TAG:-x}; WL=${WORKLOAD:-c3}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-k_expand_fast}" -d $R/gpurun_out/pmc_${T}_$i -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --words $W --workload $WL > $R/gpurun_out/pmc_${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmc_${T}_$i.log; exit 21; }
done <<GROUPS
${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH
SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD
WRITE_SIZE GRBM_GUI_ACTIVE
FETCH_SIZE}
GROUPS
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_${T}_
