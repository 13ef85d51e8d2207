#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export A5X_LIB_PATH=$R/hashcat_a5_table_generator_amd/_build_abl/liba5x.so
for ab in 0 8; do
 i=0
 while read -r grp; do
  i=$((i+1))
  A5X_ABLATE=$ab timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex k_expand_fast -d $R/gpurun_out/pmcg${ab}_$i -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --words 2000000 > $R/gpurun_out/pmcg${ab}_$i.log 2>&1 || { echo "pmc failed"; tail -3 $R/gpurun_out/pmcg${ab}_$i.log; exit 21; }
 done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_MISC
GROUPS
 echo "== ablate $ab"; python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcg${ab}_ | grep -v "^k_\|^__" 
done
