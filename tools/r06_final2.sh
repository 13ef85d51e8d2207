#!/bin/bash
# round 6 final measurements, part 2a: fused digests (C5, 1M targets) -- kernel stats + VALU counters,
# the bench lines, the op breakdown (FX_DABL variant builds), and the -s -r -m 1 MD5 line with its counters
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
T=${TAG:-r06w}
TAG=$T ALGOS="md5 ntlm" bash tools/gpu.sh digestprof &&
TAG=$T NAME=_digest_md5 BENCH_ARGS="--digest md5 --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1" bash tools/gpu.sh bench &&
TAG=$T NAME=_digest_ntlm BENCH_ARGS="--digest ntlm --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1" bash tools/gpu.sh bench &&
TAG=$T bash tools/gpu.sh dabl &&
TAG=$T ALGOS=md5 KRE="k_expand_fast_md5|k_mode_digest" KNAME="k_expand_fast_md5+k_mode_digest_*" DARGS="--mode 3 --min 1" bash tools/gpu.sh digestprof &&
TAG=$T NAME=_digest_md5_m3 BENCH_ARGS="--digest md5 --mode 3 --min 1 --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1 --no-cpu-baseline" bash tools/gpu.sh bench
