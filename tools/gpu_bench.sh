#!/bin/bash
# GPU-box script: parity, bench JSON (with CPU baseline), digest verify, rocprofv3
# kernel-trace/stats, PMC traffic (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
T=${TAG:-r01}
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tq.log 2>&1 || { tail -5 gpurun_out/tq.log; exit 10; }
tail -1 gpurun_out/tq.log
SECONDS=0; timeout -k 10 400 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail -5 gpurun_out/bench_$T.err; exit 11; }
echo "bench wall ${SECONDS} s"; tail -3 gpurun_out/bench_$T.err
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --words 2000000 --verify --no-cpu-baseline > gpurun_out/bench_verify.json 2> gpurun_out/bench_verify.err || { tail -3 gpurun_out/bench_verify.err; exit 12; }
grep verify gpurun_out/bench_verify.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$T.log 2>&1 || { tail -5 $R/gpurun_out/prof_$T.log; exit 13; }
cd $R && TAG=$T WL=c3 bash tools/gpu_pmc_traffic.sh || exit 14
echo done
