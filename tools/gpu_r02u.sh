#!/bin/bash
# parity (fast/slow/cplx paths) + bench + kernel stats after: side-stream slow kernel, LDS-staged cplx keyspace
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_digest.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log
grep -E "Error|assert|FAILED" gpurun_out/tv.log | head -6
[ $rc -eq 0 ] || exit 10
VARIANTS="cur:X=0 cur2:X=0" STEPS=5 bash tools/gpu_ab.sh || exit 11
TAG=r02u STEPS=5 bash tools/gpu_prof.sh || exit 12
