#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
[ $rc -eq 0 ] || exit 10
A5X_LIB_PATH=$GRAFT_REPO_ROOT/$P/_build_flb/liba5x.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tv2.log 2>&1; rc=$?; echo "flb pytest rc=$rc"; tail -2 gpurun_out/tv2.log
[ $rc -eq 0 ] || exit 10
VARIANTS="prev:LIB=$P/_build_prev/liba5x.so cur:X=0 flb:LIB=$P/_build_flb/liba5x.so a4:LIB=$P/_build_a4/liba5x.so prev2:LIB=$P/_build_prev/liba5x.so cur2:X=0 flb2:LIB=$P/_build_flb/liba5x.so" STEPS=3 bash tools/gpu_ab.sh
