#!/bin/bash
# GPU-box script: fused digest parity tests, then the whole GPU suite (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_digest.py -v -x --timeout 120 --timeout-method thread > gpurun_out/td.log 2>&1; rc=$?
echo "digest rc=$rc"; tail -3 gpurun_out/td.log; grep -E "Error|assert" gpurun_out/td.log | head -8
[ $rc -eq 0 ] || exit 10
[ -n "$ONLY" ] && exit 0
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tq.log 2>&1 || { tail -5 gpurun_out/tq.log; exit 11; }
tail -1 gpurun_out/tq.log
