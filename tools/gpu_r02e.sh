#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="cur:A5X_WAVES=1 np4:A5X_WAVES=1,LIB=$P/_build_np4/liba5x.so np3:A5X_WAVES=1,LIB=$P/_build_np3/liba5x.so r4:A5X_WAVES=1,LIB=$P/_build_r4/liba5x.so np4w4:A5X_WAVES=4,LIB=$P/_build_np4/liba5x.so cur2:A5X_WAVES=1" STEPS=3 bash tools/gpu_ab.sh
