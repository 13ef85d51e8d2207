#!/bin/bash
# fused NTLM parity + L2 prefetch of the next window's records (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_configs.py -q -m gpu -x --timeout 300 --timeout-method thread -k "fused or lookup or digest" > gpurun_out/ta.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ta.log
grep -E "Error|assert|FAILED" gpurun_out/ta.log | head -8
[ $rc -eq 0 ] || exit 10
VARIANTS="base:X=0 pf16:LIB=$P/_build_l2pf16/liba5x.so pf32:LIB=$P/_build_l2pf32/liba5x.so pf64:LIB=$P/_build_l2pf64/liba5x.so base2:X=0 pf32b:LIB=$P/_build_l2pf32/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
