#!/bin/bash
# parity of the fast kernel, A/B of metadata prefetch (FX_PFM) and fx8_put (FX_AB), ablations, stamps
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digest.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
[ $rc -eq 0 ] || exit 10
VARIANTS="cur:X=0 pfm0:LIB=$P/_build_pfm0/liba5x.so fx7:LIB=$P/_build_fx7/liba5x.so cur2:X=0 pfm0b:LIB=$P/_build_pfm0/liba5x.so fx7b:LIB=$P/_build_fx7/liba5x.so abl4:LIB=$P/_build_abl4/liba5x.so abl8:LIB=$P/_build_abl8/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
timeout -k 10 120 python tools/stamps.py c3 2000000 > gpurun_out/stamps.txt 2>&1 || { tail -5 gpurun_out/stamps.txt; exit 12; }
cat gpurun_out/stamps.txt
