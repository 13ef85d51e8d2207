#!/bin/bash
# timing ablations: expand ms of compile-time FX_ABL variant builds (_build_a<mask>)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
V="cur:X=0"
for ab in ${ABL:-64 128 4 8 24}; do V="$V a$ab:LIB=$P/_build_a$ab/liba5x.so"; done
VARIANTS="$V cur2:X=0" STEPS=3 bash tools/gpu_ab.sh
