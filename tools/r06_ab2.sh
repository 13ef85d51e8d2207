#!/bin/bash
# round 6 A/B 2: output store policy (nt / plain / sc1) x 128-B grid in k_expand_fast; store ceilings
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
B=hashcat_a5_table_generator_amd
L=$B/_build
echo "== parity st2grid $(date +%T)"
A5X_LIB_PATH=$PWD/${L}_st2grid/liba5x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/r06b_parity_st2grid.log 2>&1 || { tail -20 gpurun_out/r06b_parity_st2grid.log; exit 3; }
tail -1 gpurun_out/r06b_parity_st2grid.log
echo "== mb_ustore $(date +%T)"
timeout -k 10 200 tools/mb_ustore 1800000000 1 > gpurun_out/r06b_mb_ustore.txt 2>&1 || { cat gpurun_out/r06b_mb_ustore.txt; exit 4; }
cat gpurun_out/r06b_mb_ustore.txt
echo "== ab $(date +%T)"
VARIANTS="cur:X=0 st1:LIB=${L}_st1/liba5x.so st1grid:LIB=${L}_st1grid/liba5x.so st2:LIB=${L}_st2/liba5x.so st2grid:LIB=${L}_st2grid/liba5x.so cur2:X=0 st1b:LIB=${L}_st1/liba5x.so st1gridb:LIB=${L}_st1grid/liba5x.so st2b:LIB=${L}_st2/liba5x.so st2gridb:LIB=${L}_st2grid/liba5x.so" \
  TAG=r06b BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh ab
