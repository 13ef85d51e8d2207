#!/bin/bash
# C5 shape tests + digest profiles (kernel stats + VALU counters) + --digest bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -v -m gpu -x -k c5 --timeout 300 --timeout-method thread > gpurun_out/c5t.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/c5t.log
[ $rc -eq 0 ] || exit 10
timeout -k 10 900 bash tools/gpu_digest_prof.sh > gpurun_out/dprof.txt 2>&1 || { echo "digest prof failed"; tail -20 gpurun_out/dprof.txt; exit 11; }
tail -4 gpurun_out/dprof.txt
for A in md5 ntlm; do
  timeout -k 10 300 python bench.py --digest $A --workload c5 --words 2000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bd_$A.json 2> gpurun_out/bd_$A.err || { echo "bench $A failed"; tail -5 gpurun_out/bd_$A.err; exit 12; }
  cat gpurun_out/bd_$A.json
done
