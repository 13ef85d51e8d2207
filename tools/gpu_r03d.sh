#!/bin/bash
# occupancy: 5 waves/SIMD with 128-entry windows (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="base:X=0 o5a:LIB=$P/_build_o5a/liba5x.so o5b:LIB=$P/_build_o5b/liba5x.so o5c:LIB=$P/_build_o5c/liba5x.so o4s:LIB=$P/_build_o4s/liba5x.so base2:X=0 o5b2:LIB=$P/_build_o5b/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
