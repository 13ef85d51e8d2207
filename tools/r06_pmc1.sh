#!/bin/bash
# round 6: memory-pipeline / LDS-queue counters of k_expand_fast (C3 2M words), nt vs plain vs no stores
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
L=hashcat_a5_table_generator_amd/_build
PMC="SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD GRBM_GUI_ACTIVE
TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TCP_TA_DATA_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCP_WRITE_TAGCONFLICT_STALL_CYCLES TCP_TCC_WRITE_REQ_LATENCY GRBM_GUI_ACTIVE
TCC_EA0_WRREQ_STALL TCC_TAG_STALL TCC_TOO_MANY_EA_WRREQS_STALL TCC_BUSY GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS_STORE
SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for v in cur st1 abl4; do
  lib=""; [ $v != cur ] && lib=$PWD/${L}_$v/liba5x.so
  A5X_LIB_PATH=$lib PMC="$PMC" TAG=r06e_$v bash tools/gpu.sh pmc > gpurun_out/r06e_pmc_$v.txt 2>&1 || { tail -20 gpurun_out/r06e_pmc_$v.txt; exit 5; }
  echo "== $v"; cat gpurun_out/r06e_pmc_$v.txt
done
