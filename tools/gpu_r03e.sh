#!/bin/bash
# L2 prefetch of the next window's records (inline-asm loads, no early waits): A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="base:X=0 pf16:LIB=$P/_build_pf16/liba5x.so pf32:LIB=$P/_build_pf32/liba5x.so base2:X=0 pf16b:LIB=$P/_build_pf16/liba5x.so pf32b:LIB=$P/_build_pf32/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
