#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
A5X_LIB_PATH=$GRAFT_REPO_ROOT/$P/_build_pf1/liba5x.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pf1 pytest rc=$rc"; tail -2 gpurun_out/tv.log
[ $rc -eq 0 ] || exit 10
VARIANTS="cur:X=0 pf1:LIB=$P/_build_pf1/liba5x.so pf2:LIB=$P/_build_pf2/liba5x.so cur2:X=0 pf1b:LIB=$P/_build_pf1/liba5x.so pf2b:LIB=$P/_build_pf2/liba5x.so" STEPS=3 bash tools/gpu_ab.sh
