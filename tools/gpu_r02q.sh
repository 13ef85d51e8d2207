#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -m gpu -x -k "golden or oracle or c3 or c4_shape_one" --timeout 300 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
grep -E "Error|assert|FAILED" gpurun_out/tv.log | head -6
[ $rc -eq 0 ] || exit 10
VARIANTS="prev:LIB=$P/_build_prev/liba5x.so cur:X=0 prev2:LIB=$P/_build_prev/liba5x.so cur2:X=0" STEPS=3 bash tools/gpu_ab.sh
