#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="cur:A5X_WAVES=1 v1:A5X_WAVES=1,LIB=$P/_build_v1/liba5x.so v2:A5X_WAVES=1,LIB=$P/_build_v2/liba5x.so v3:A5X_WAVES=1,LIB=$P/_build_v3/liba5x.so ch16k:A5X_WAVES=1,A5X_CHUNK=16384 ch4k:A5X_WAVES=1,A5X_CHUNK=4096 v1ch16k:A5X_WAVES=1,A5X_CHUNK=16384,LIB=$P/_build_v1/liba5x.so" STEPS=3 bash tools/gpu_ab.sh
