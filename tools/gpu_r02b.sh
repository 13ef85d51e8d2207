#!/bin/bash
# GPU-box script: parity tests, then an A/B of workgroup sizes on C3
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tq.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tq.log
grep -E "Error|assert" gpurun_out/tq.log | head -5
[ $rc -eq 0 ] || exit 10
VARIANTS="w4:A5X_WAVES=4 w2:A5X_WAVES=2 w1:A5X_WAVES=1" STEPS=5 bash tools/gpu_ab.sh
