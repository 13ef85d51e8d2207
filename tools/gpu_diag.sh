#!/bin/bash
# GPU-box script: kernel-stats profile + per-phase stamps of k_expand_fast
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py ${WL:-c3} ${SW:-2000000} > gpurun_out/stamps.txt 2>&1 || { tail -5 gpurun_out/stamps.txt; exit 12; }
cat gpurun_out/stamps.txt
TAG=${TAG:-x} WORDS=${WORDS:-10000000} WORKLOAD=${WL:-c3} timeout -k 10 400 bash tools/gpu_prof.sh
