#!/bin/bash
# lane run length K = 2 / 3 / 4 (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="base:X=0 k3:LIB=$P/_build_k3/liba5x.so k2:LIB=$P/_build_k2/liba5x.so base2:X=0 k3b:LIB=$P/_build_k3/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
