#!/bin/bash
# round 6 final measurements, part 2b: the C5 -r / -s / -s -r lines, their kernel stats, the stdout path
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
T=${TAG:-r06w}
for m in 1 2 3; do
  TAG=$T NAME=_c5_mode$m BENCH_ARGS="--mode $m --workload c5 --steps 3 --warmup 1 --no-cpu-baseline" bash tools/gpu.sh bench || exit 11
done
for m in 1 2; do
  TAG=${T}_m$m BENCH_ARGS="--mode $m --workload c5 --steady-batches 0" STEPS=2 bash tools/gpu.sh prof || exit 13
done
TAG=$T NAME=_stdout BENCH_ARGS="--stdout --no-cpu-baseline" bash tools/gpu.sh bench
