#!/bin/bash
# C4 shape tests + c3 / c4 bench lines on the partitioned global list
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/c4t.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/c4t.log
[ $rc -eq 0 ] || exit 10
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err || { echo "bench c3 failed"; tail -5 gpurun_out/b_c3.err; exit 11; }
cat gpurun_out/b_c3.json
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload c4 --words 12500000 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err || { echo "bench c4 failed"; tail -5 gpurun_out/b_c4.err; exit 12; }
cat gpurun_out/b_c4.json
