#!/bin/bash
# instruction mix of k_expand_fast: full vs no rounds (FX_ABL=8) vs no big entries (FX_ABL=16)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=$GRAFT_REPO_ROOT/hashcat_a5_table_generator_amd
G="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH"
for v in full abl8 abl16; do
  if [ $v = full ]; then unset A5X_LIB_PATH; else export A5X_LIB_PATH=$P/_build_$v/liba5x.so; fi
  TAG=$v PMC="$G
$G2" bash tools/gpu_pmc2.sh > gpurun_out/pmcsum_$v.txt 2>&1 || { cat gpurun_out/pmcsum_$v.txt | tail; exit 21; }
  echo "== $v"; grep -A40 "^k_expand_fast$" gpurun_out/pmcsum_$v.txt | grep -E "per wave|WAVE_CYCLES|SQ_WAVES "
done
