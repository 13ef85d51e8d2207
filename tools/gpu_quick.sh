#!/bin/bash
# GPU-box script: parity tests + one bench line (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tq.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tq.log
grep -E "Error|assert" gpurun_out/tq.log | head -5
[ $rc -eq 0 ] || exit 10
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --words ${WORDS:-10000000} ${BENCH_ARGS} > gpurun_out/bq.json 2> gpurun_out/bq.err || { echo "bench failed"; tail -5 gpurun_out/bq.err; exit 11; }
python -c "import json;d=json.load(open('gpurun_out/bq.json'));r=d['roofline'];print('value %.3e cand/s  expand %.2f ms  %.0f GB/s  frac %.3f  ks %.2f ms  step %.2f ms'%(d['value'],r['ms_per_launch'],r['achieved'],r['frac'],r['ms_keyspace_scan_plan'],d['ms_per_step']))"
