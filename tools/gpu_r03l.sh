#!/bin/bash
# k_expand_fast instruction mix, wait states and LDS bank conflicts on HEAD (C3, 2M words)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_BRANCH"
G3="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
TAG=r02wmix PMC="$G1
$G2
$G3" bash tools/gpu_pmc2.sh > gpurun_out/pmcsum_r02wmix.txt 2>&1 || { tail gpurun_out/pmcsum_r02wmix.txt; exit 21; }
cat gpurun_out/pmcsum_r02wmix.txt
