#!/bin/bash
# mode pass G (long -r/-s lines) + full GPU parity suite
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_long.py -v -m gpu -x --timeout 200 --timeout-method thread -k mode > gpurun_out/tg.log 2>&1; rc=$?; echo "long-mode pytest rc=$rc"; tail -4 gpurun_out/tg.log
grep -E "Error|assert|FAILED" gpurun_out/tg.log | head -8
[ $rc -eq 0 ] || exit 10
timeout -k 10 500 python -u -m pytest tests/ -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/tq.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tq.log
grep -E "Error|assert|FAILED" gpurun_out/tq.log | head -8
[ $rc -eq 0 ] || exit 11
