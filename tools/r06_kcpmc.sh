#!/bin/bash
# round 6: counters of k_keyspace_cplx (C3, 10M words)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
mkdir -p gpurun_out
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
G2="SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for v in c3:0; do
  wl=${v%%:*}; m=${v#*:}
  i=0
  for G in "$G1" "$G2"; do
    i=$((i + 1))
    ( cd /tmp && export TMPDIR=/tmp && KSMODE=$m timeout -s KILL 120 rocprofv3 --pmc $G \
        --kernel-include-regex k_keyspace_cplx -d $R/gpurun_out/kcpmc_${wl}_$i -o run --output-format csv -- \
        python3 $R/tools/ks_time.py $wl 10000000 > $R/gpurun_out/kcpmc_${wl}_$i.log 2>&1 ) \
      || { echo "kspmc $wl $i failed"; tail -3 gpurun_out/kcpmc_${wl}_$i.log; exit 15; }
  done
  echo "== $wl mode $m"
  python3 tools/pmc_summary.py mix gpurun_out/kcpmc_${wl}_
done
