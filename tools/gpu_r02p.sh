#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
[ $rc -eq 0 ] || exit 10
VARIANTS="nodw3:LIB=$P/_build_nodw3/liba5x.so cur:X=0 nodw3b:LIB=$P/_build_nodw3/liba5x.so cur2:X=0 nodw3c:LIB=$P/_build_nodw3/liba5x.so cur3:X=0" STEPS=3 bash tools/gpu_ab.sh
