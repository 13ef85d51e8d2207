#!/bin/bash
# round 6 A/B 5: whole-line flushes (FX_LALIGN) vs current; batched flush; write-latency counters
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
L=hashcat_a5_table_generator_amd/_build
echo "== parity lalign $(date +%T)"
A5X_LIB_PATH=$PWD/${L}_lalign/liba5x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/r06f_parity_lalign.log 2>&1 || { tail -20 gpurun_out/r06f_parity_lalign.log; exit 3; }
tail -1 gpurun_out/r06f_parity_lalign.log
VARIANTS="cur:X=0 lalign:LIB=${L}_lalign/liba5x.so cur2:X=0 lalign2:LIB=${L}_lalign/liba5x.so cur3:X=0 lalign3:LIB=${L}_lalign/liba5x.so" \
  TAG=r06f BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh ab || exit 4
PMC="TCP_TCC_WRITE_REQ_LATENCY TCP_TCC_WRITE_REQ TCP_PENDING_STALL_CYCLES TD_TC_STALL TD_TD_BUSY GRBM_GUI_ACTIVE"
for v in cur lalign; do
  lib=""; [ $v != cur ] && lib=$PWD/${L}_$v/liba5x.so
  A5X_LIB_PATH=$lib PMC="$PMC" TAG=r06f_$v bash tools/gpu.sh pmc > gpurun_out/r06f_pmc_$v.txt 2>&1 || { tail -20 gpurun_out/r06f_pmc_$v.txt; exit 5; }
  echo "== $v"; grep -E "TCP|TD_|GRBM" gpurun_out/r06f_pmc_$v.txt
done
