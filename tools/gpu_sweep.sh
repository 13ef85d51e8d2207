#!/bin/bash
# GPU-box script: env sweep of the bench (A5X_CHUNK / A5X_WAVES ...); prints one line per setting
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for cfg in ${SWEEP:-"A5X_CHUNK=1024"}; do
  env $cfg timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --words ${WORDS:-10000000} --workload ${WORKLOAD:-c3} > gpurun_out/sw.json 2> gpurun_out/sw.err || { echo "$cfg failed"; tail -3 gpurun_out/sw.err; exit 11; }
  python -c "import json,sys;d=json.load(open('gpurun_out/sw.json'));r=d['roofline'];print('%-22s value %.3e cand/s  expand %.2f ms  %.0f GB/s  frac %.3f ks %.2f ms'%(sys.argv[1],d['value'],r['ms_per_launch'],r['achieved'],r['frac'],r['ms_keyspace_scan_plan']))" "$cfg"
done
