#!/bin/bash
# cplx striping parity + keyspace ablations (timing only)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
[ $rc -eq 0 ] || exit 10
VARIANTS="cur:X=0 ks1:LIB=$P/_build_ks1/liba5x.so ks3:LIB=$P/_build_ks3/liba5x.so cur2:X=0" STEPS=5 bash tools/gpu_ab.sh || exit 11
TAG=r02x STEPS=5 bash tools/gpu_prof.sh | grep keyspace
