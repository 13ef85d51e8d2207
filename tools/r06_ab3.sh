#!/bin/bash
# round 6 A/B 3: does waiting for the stores (vmcnt) cost more with plain stores?  stamps nt vs plain
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
B=hashcat_a5_table_generator_amd
L=$B/_build
echo "== stamps nt $(date +%T)"
A5X_LIB_PATH=$PWD/${L}_diag/liba5x.so timeout -k 10 120 python tools/stamps.py c3 2000000 > gpurun_out/r06c_stamps_nt.txt 2>&1 || { tail -5 gpurun_out/r06c_stamps_nt.txt; exit 3; }
cat gpurun_out/r06c_stamps_nt.txt
echo "== stamps plain $(date +%T)"
A5X_LIB_PATH=$PWD/${L}_diagst1/liba5x.so timeout -k 10 120 python tools/stamps.py c3 2000000 > gpurun_out/r06c_stamps_plain.txt 2>&1 || { tail -5 gpurun_out/r06c_stamps_plain.txt; exit 3; }
cat gpurun_out/r06c_stamps_plain.txt
echo "== ab $(date +%T)"
VARIANTS="cur:X=0 drain:LIB=${L}_drain/liba5x.so drainst1:LIB=${L}_drainst1/liba5x.so st1:LIB=${L}_st1/liba5x.so cur2:X=0 drain2:LIB=${L}_drain/liba5x.so drainst12:LIB=${L}_drainst1/liba5x.so st12:LIB=${L}_st1/liba5x.so" \
  TAG=r06c BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh ab
