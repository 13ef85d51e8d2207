#!/bin/bash
# round 6 A/B 4: batched flush reads (one LDS round trip per flush)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
B=hashcat_a5_table_generator_amd
L=$B/_build
echo "== parity batch $(date +%T)"
A5X_LIB_PATH=$PWD/${L}_batch/liba5x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/r06d_parity_batch.log 2>&1 || { tail -20 gpurun_out/r06d_parity_batch.log; exit 3; }
tail -1 gpurun_out/r06d_parity_batch.log
VARIANTS="cur:X=0 batch:LIB=${L}_batch/liba5x.so cur2:X=0 batch2:LIB=${L}_batch/liba5x.so cur3:X=0 batch3:LIB=${L}_batch/liba5x.so" \
  TAG=r06d BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh ab
