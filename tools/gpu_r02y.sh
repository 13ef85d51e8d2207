#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="cur:X=0 ks4:LIB=$P/_build_ks4/liba5x.so ks1:LIB=$P/_build_ks1/liba5x.so cur2:X=0 ks4b:LIB=$P/_build_ks4/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
