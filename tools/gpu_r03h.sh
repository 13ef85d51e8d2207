#!/bin/bash
# VALU-boundness probe: +32 / +96 independent VALU ops per round
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="base:X=0 padv32:LIB=$P/_build_padv32/liba5x.so padv96:LIB=$P/_build_padv96/liba5x.so base2:X=0 padv32b:LIB=$P/_build_padv32/liba5x.so padv96b:LIB=$P/_build_padv96/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
