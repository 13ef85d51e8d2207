#!/bin/bash
# does waiting for the stores cost much?  (vmcnt(0) after every flush) + HOLDNB=1
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
VARIANTS="cur:X=0 fw:LIB=$P/_build_fw/liba5x.so hold1:LIB=$P/_build_hold1/liba5x.so cur2:X=0 fw2:LIB=$P/_build_fw/liba5x.so hold1b:LIB=$P/_build_hold1/liba5x.so" STEPS=5 bash tools/gpu_ab.sh || exit 11
