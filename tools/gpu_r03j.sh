#!/bin/bash
# fused NTLM multi-block test
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_digest.py -v -m gpu -x --timeout 200 --timeout-method thread -k "multi_block" > gpurun_out/tn.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tn.log
grep -E "Error|assert|FAILED" gpurun_out/tn.log | head -8
exit $rc
