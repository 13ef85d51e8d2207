#!/bin/bash
# GPU-box script: bench JSON + verify + rocprofv3 kernel-trace/stats (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 11
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --words 1000000 --verify --no-cpu-baseline > gpurun_out/bench_verify.json 2> gpurun_out/bench_verify.err || exit 12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof1.log 2>&1 || exit 13
echo done
