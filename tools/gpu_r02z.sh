#!/bin/bash
# wave-pair windows: parity, then A/B vs one wave per window
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_long.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
grep -E "Error|assert|FAILED" gpurun_out/tv.log | head -8
[ $rc -eq 0 ] || exit 10
VARIANTS="pair:X=0 pair16k:A5X_CHUNK=16384 nopair:LIB=$P/_build_nopair/liba5x.so pair2:X=0 pair16kb:A5X_CHUNK=16384 nopair2:LIB=$P/_build_nopair/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
