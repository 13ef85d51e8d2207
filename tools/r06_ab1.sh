#!/bin/bash
# round 6 first A/B: 128-B store grid, XOR-swizzled ring, ablations; store-pattern ceilings
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
B=hashcat_a5_table_generator_amd
echo "== parity swzgrid $(date +%T)"
A5X_LIB_PATH=$PWD/$B/_build_swzgrid/liba5x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/r06a_parity_swzgrid.log 2>&1 || { tail -20 gpurun_out/r06a_parity_swzgrid.log; exit 3; }
tail -1 gpurun_out/r06a_parity_swzgrid.log
echo "== mb_ustore $(date +%T)"
timeout -k 10 200 tools/mb_ustore 1800000000 1 > gpurun_out/r06a_mb_ustore.txt 2>&1 || { cat gpurun_out/r06a_mb_ustore.txt; exit 4; }
cat gpurun_out/r06a_mb_ustore.txt
echo "== ab $(date +%T)"
L=$B/_build
VARIANTS="cur:X=0 grid:LIB=${L}_grid/liba5x.so swz:LIB=${L}_swz/liba5x.so swzgrid:LIB=${L}_swzgrid/liba5x.so abl64:LIB=${L}_abl64/liba5x.so abl4:LIB=${L}_abl4/liba5x.so abl68:LIB=${L}_abl68/liba5x.so cur2:X=0 grid2:LIB=${L}_grid/liba5x.so swz2:LIB=${L}_swz/liba5x.so swzgrid2:LIB=${L}_swzgrid/liba5x.so" \
  TAG=r06a BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh ab
