#!/bin/bash
# bigger rounds: 6 KiB ring + 128-entry windows with 5 / 6 candidates per lane run (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="base:X=0 r6k6:LIB=$P/_build_r6k6/liba5x.so r6k5:LIB=$P/_build_r6k5/liba5x.so r6k6h0:LIB=$P/_build_r6k6h0/liba5x.so base2:X=0 r6k6b:LIB=$P/_build_r6k6/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
