#!/bin/bash
# round 6 A/B 8: flush stores as scalar base + 32-bit lane offset (FX_SADDR: 4 B of address per lane)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
L=hashcat_a5_table_generator_amd/_build
A5X_LIB_PATH=$PWD/${L}_saddr/liba5x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/r06l_parity_saddr.log 2>&1 || { tail -20 gpurun_out/r06l_parity_saddr.log; exit 3; }
tail -1 gpurun_out/r06l_parity_saddr.log
VARIANTS="cur:X=0 saddr:LIB=${L}_saddr/liba5x.so cur2:X=0 saddr2:LIB=${L}_saddr/liba5x.so cur3:X=0 saddr3:LIB=${L}_saddr/liba5x.so" \
  TAG=r06l BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh ab
