#!/bin/bash
# parity of a variant build (VLIB) + A/B bench vs the default build
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
A5X_LIB_PATH=$GRAFT_REPO_ROOT/$P/_build_${VAR:-or}/liba5x.so timeout -k 10 400 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "variant pytest rc=$rc"; tail -2 gpurun_out/tv.log
grep -E "Error|assert" gpurun_out/tv.log | head -5
[ $rc -eq 0 ] || exit 10
VARIANTS="cur:X=0 ${VAR:-or}:LIB=$P/_build_${VAR:-or}/liba5x.so cur2:X=0 ${VAR:-or}2:LIB=$P/_build_${VAR:-or}/liba5x.so" STEPS=3 bash tools/gpu_ab.sh
