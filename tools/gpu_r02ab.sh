#!/bin/bash
# round prefetch (FX_RPF): parity, then A/B vs the previous product build
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_digest.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
grep -E "Error|assert|FAILED" gpurun_out/tv.log | head -8
[ $rc -eq 0 ] || exit 10
VARIANTS="cur:X=0 base:LIB=$P/_build_base/liba5x.so nopfm:LIB=$P/_build_nopfm/liba5x.so rpfh2:LIB=$P/_build_rpfh2/liba5x.so cur2:X=0 base2:LIB=$P/_build_base/liba5x.so nopfm2:LIB=$P/_build_nopfm/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
