#!/bin/bash
# pass G (long lines) parity + the per-word path regressions
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_long.py -v -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/tl.log 2>&1; rc=$?; echo "long rc=$rc"; tail -12 gpurun_out/tl.log
[ $rc -eq 0 ] || exit 10
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/tv.log
exit $rc
