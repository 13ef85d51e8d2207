#!/bin/bash
# parity of the fast kernel (+ fused digest) then A/B of FX_AB (fx8_put) vs fx7_put
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digest.py tests/test_gpu_configs.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
grep -E "Error|assert|FAILED" gpurun_out/tv.log | head -6
[ $rc -eq 0 ] || exit 10
VARIANTS="fx7:LIB=$P/_build_fx7/liba5x.so cur:X=0 fx7b:LIB=$P/_build_fx7/liba5x.so cur2:X=0" STEPS=5 bash tools/gpu_ab.sh
