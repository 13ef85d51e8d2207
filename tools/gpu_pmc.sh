#!/bin/bash
# GPU-box script: rocprofv3 PMC passes on the expansion kernel (outputs under gpurun_out/pmc*)
# usage: WORDS=2000000 TAG=r1 bash tools/gpu_pmc.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
W=${WORDS:-2000000}; T=${TAG:-x}; WL=${WORKLOAD:-c3}
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --words $W --workload $WL"
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc_list_$T.txt 2>&1 || true
i=0
for grp in "${PMC_GROUPS[@]:-}"; do :; done
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-k_expand_fast}" -d $R/gpurun_out/pmc_${T}_$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_${T}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmc_${T}_$i.log; exit 21; }
done <<GROUPS
${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH
WRITE_SIZE
FETCH_SIZE
GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL}
GROUPS
echo pmc done
