#!/bin/bash
# round 6 A/B 9: store cache-policy bits -- the round-flush pattern alone (mb_ustore modes 8-18) and
# k_expand_fast with sc0 nt / sc1 nt / sc0 sc1 nt stores (FX_ST=3, FX_STPOL)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
L=hashcat_a5_table_generator_amd/_build
timeout -k 10 200 tools/mb_ustore 1800000000 2 > gpurun_out/r06m_mb_ustore_policy.txt 2>&1 || { cat gpurun_out/r06m_mb_ustore_policy.txt; exit 4; }
cat gpurun_out/r06m_mb_ustore_policy.txt
A5X_LIB_PATH=$PWD/${L}_p01n/liba5x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/r06m_parity.log 2>&1 || { tail -20 gpurun_out/r06m_parity.log; exit 3; }
tail -1 gpurun_out/r06m_parity.log
VARIANTS="cur:X=0 p0n:LIB=${L}_p0n/liba5x.so p1n:LIB=${L}_p1n/liba5x.so p01n:LIB=${L}_p01n/liba5x.so cur2:X=0 p0n2:LIB=${L}_p0n/liba5x.so p1n2:LIB=${L}_p1n/liba5x.so p01n2:LIB=${L}_p01n/liba5x.so" \
  TAG=r06m BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh ab
