#!/bin/bash
# round 6 final measurements, part 2b: the fused-digest lines again now that their sha-matched VALU profiles are
# committed (the roofline fractions come from them), then the C5 -r / -s / -s -r lines, kernel stats, stdout path
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
T=${TAG:-r06fin}
TAG=$T NAME=_digest_md5 BENCH_ARGS="--digest md5 --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1" bash tools/gpu.sh bench &&
TAG=$T NAME=_digest_ntlm BENCH_ARGS="--digest ntlm --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1" bash tools/gpu.sh bench &&
TAG=$T NAME=_digest_md5_m3 BENCH_ARGS="--digest md5 --mode 3 --min 1 --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1 --no-cpu-baseline" bash tools/gpu.sh bench &&
TAG=$T bash tools/r06_final3.sh
