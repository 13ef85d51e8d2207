#!/bin/bash
# keyspace occupancy: KS_ULOG 8 (<= 32 KB LDS per 256-word tile block: 5 blocks per CU) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="base:X=0 ulog8:LIB=$P/_build_ulog8/liba5x.so base2:X=0 ulog8b:LIB=$P/_build_ulog8/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
WL=c4 WORDS=4000000 VARIANTS="c4base:X=0 c4ulog8:LIB=$P/_build_ulog8/liba5x.so" STEPS=3 bash tools/gpu_ab.sh || exit 12
