#!/bin/bash
# GPU-box script: rocprofv3 PMC passes over tools/mb_rounds (one counter group per pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
T=${TAG:-mb}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_${T}_$i -o run --output-format csv -- $R/tools/mb_rounds > $R/gpurun_out/pmc_${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmc_${T}_$i.log; exit 21; }
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR
GROUPS
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_${T}_
