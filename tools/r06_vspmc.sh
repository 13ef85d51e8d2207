#!/bin/bash
# round 6: counters of k_keyspace_vsub (C5 -s keyspace, 10M words) for the product and the VS_ABL=1
# build (no build pass): where the build pass's 7.8 ms go
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
mkdir -p gpurun_out
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES"
for v in cur vsabl1; do
  lib=""
  [ $v != cur ] && lib=$R/hashcat_a5_table_generator_amd/_build_$v/liba5x.so
  i=0
  for G in "$G1" "$G2"; do
    i=$((i + 1))
    ( cd /tmp && export TMPDIR=/tmp && KSMODE=2 A5X_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $G \
        --kernel-include-regex k_keyspace_vsub -d $R/gpurun_out/vspmc_${v}_$i -o run --output-format csv -- \
        python3 $R/tools/ks_time.py c5 10000000 > $R/gpurun_out/vspmc_${v}_$i.log 2>&1 ) \
      || { echo "vspmc $v $i failed"; tail -3 gpurun_out/vspmc_${v}_$i.log; exit 15; }
  done
  echo "== $v"
  python3 tools/pmc_summary.py mix gpurun_out/vspmc_${v}_
done
