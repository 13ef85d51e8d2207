#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
A5X_LIB_PATH=$R/$P/_build_t16/liba5x.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tv.log 2>&1; rc=$?; echo "t16 pytest rc=$rc"; tail -2 gpurun_out/tv.log
[ $rc -eq 0 ] || exit 10
VARIANTS="cur:X=0 t16:LIB=$P/_build_t16/liba5x.so cur2:X=0 t16b:LIB=$P/_build_t16/liba5x.so" STEPS=3 bash tools/gpu_ab.sh || exit 11
cd /tmp && export TMPDIR=/tmp
export A5X_LIB_PATH=$R/$P/_build_abl/liba5x.so
for ab in 8 24 56; do
  A5X_ABLATE=$ab timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex k_expand_fast -d $R/gpurun_out/pmci${ab}_1 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --words 2000000 > $R/gpurun_out/pmci${ab}_1.log 2>&1 || { echo "pmc failed"; tail -3 $R/gpurun_out/pmci${ab}_1.log; exit 21; }
  echo "== ablate $ab"; python3 $R/tools/pmc_summary.py $R/gpurun_out/pmci${ab}_ | grep "per wave"
done
