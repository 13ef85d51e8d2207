#!/bin/bash
# round 6 final measurements, part 1: the C3 headline line (+ CPU baseline, steady state), its rocprof
# kernel stats and PMC traffic, then C4 and C2a (tools/gpu.sh steps; TAG names the outputs)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
T=${TAG:-r06w}
TAG=$T NAME=_c3 BENCH_ARGS="" bash tools/gpu.sh bench &&
TAG=$T BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh prof &&
TAG=$T WL=c3 bash tools/gpu.sh traffic &&
TAG=$T NAME=_c4 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --workload c4 --words 12500000 --steady-batches 0" bash tools/gpu.sh bench &&
TAG=$T WL=c4 WORDS=12500000 bash tools/gpu.sh traffic &&
TAG=$T NAME=_c2a BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --workload c2a --words 1000000 --steady-batches 0" bash tools/gpu.sh bench
