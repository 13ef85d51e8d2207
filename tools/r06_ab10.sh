#!/bin/bash
# round 6 A/B 10: would store-free compute waves keep their speed at lower occupancy?  (emulating a
# design with dedicated store waves: no stores (FX_ABL=4) at 16 / 12 / 8 waves per CU via LDS padding)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
L=hashcat_a5_table_generator_amd/_build
VARIANTS="cur:X=0 abl4:LIB=${L}_abl4/liba5x.so o12:LIB=${L}_o12/liba5x.so o8:LIB=${L}_o8/liba5x.so o12s:LIB=${L}_o12s/liba5x.so cur2:X=0 abl42:LIB=${L}_abl4/liba5x.so o122:LIB=${L}_o12/liba5x.so o82:LIB=${L}_o8/liba5x.so o12s2:LIB=${L}_o12s/liba5x.so" \
  TAG=r06n BENCH_ARGS="--steady-batches 0" bash tools/gpu.sh ab
