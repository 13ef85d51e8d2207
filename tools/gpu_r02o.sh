#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_modes.py -v -m gpu -x -k "long_candidates or 32_bit or negative_min" --timeout 300 --timeout-method thread > gpurun_out/adv.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/adv.log
grep -E "Error|assert|FAILED" gpurun_out/adv.log | head -8
[ $rc -eq 0 ] || exit 10
VARIANTS="cur:X=0 ch16k:A5X_CHUNK=16384 ch32k:A5X_CHUNK=32768 ch4k:A5X_CHUNK=4096 cur2:X=0" STEPS=3 bash tools/gpu_ab.sh || exit 11
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-include-regex k_keyspace_thread -d $R/gpurun_out/pks_1 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --words 2000000 > $R/gpurun_out/pks_1.log 2>&1 || { echo "pmc failed"; tail -3 $R/gpurun_out/pks_1.log; exit 21; }
python3 $R/tools/pmc_summary.py $R/gpurun_out/pks_ | grep -v "^__"
