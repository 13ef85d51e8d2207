#!/bin/bash
# PMC instruction mix of the keyspace kernels + HBM traffic of the current k_expand_fast
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=ks KRE="k_keyspace" WORDS=2000000 bash tools/gpu_pmc2.sh > gpurun_out/pmc2_ks.txt 2>&1 || { tail -5 gpurun_out/pmc2_ks.txt; exit 11; }
cat gpurun_out/pmc2_ks.txt
TAG=r02w WL=c3 bash tools/gpu_pmc_traffic.sh || exit 12
