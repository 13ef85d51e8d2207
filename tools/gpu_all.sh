#!/bin/bash
# GPU-box script: parity tests, bench line, per-phase stamps, kernel stats (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/tq.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tq.log
grep -E "Error|assert" gpurun_out/tq.log | head -5
[ $rc -eq 0 ] || exit 10
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --words ${WORDS:-10000000} --workload ${WL:-c3} > gpurun_out/bq.json 2> gpurun_out/bq.err || { echo "bench failed"; tail -5 gpurun_out/bq.err; exit 11; }
python -c "import json;d=json.load(open('gpurun_out/bq.json'));r=d['roofline'];print('value %.3e cand/s  expand %.2f ms  %.0f GB/s  frac %.3f  ks %.2f ms  step %.2f ms'%(d['value'],r['ms_per_launch'],r['achieved'],r['frac'],r['ms_keyspace_scan_plan'],d['ms_per_step']))"
[ -n "$NOSTAMPS" ] || { timeout -k 10 120 python tools/stamps.py ${WL:-c3} ${SW:-2000000} > gpurun_out/stamps.txt 2>&1 || { tail -5 gpurun_out/stamps.txt; exit 12; }; cat gpurun_out/stamps.txt; }
[ -n "$NOPROF" ] || TAG=${TAG:-x} WORDS=${WORDS:-10000000} WORKLOAD=${WL:-c3} timeout -k 10 400 bash tools/gpu_prof.sh | grep -v "^W20"
