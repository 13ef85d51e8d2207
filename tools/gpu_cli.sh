#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_cli.py -v -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/cli.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/cli.log
grep -E "Error|assert" gpurun_out/cli.log | head -8
exit $rc
