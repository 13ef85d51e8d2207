#!/bin/bash
# GPU-box script: bench sweep over A5X_CHUNK values (expand ms / GB/s per setting)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for ch in ${CHUNKS:-4096 16384 65536}; do
  A5X_CHUNK=$ch timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --words ${WORDS:-10000000} --workload ${WL:-c3} > gpurun_out/sw_$ch.json 2> gpurun_out/sw_$ch.err || { echo "bench failed"; tail -5 gpurun_out/sw_$ch.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/sw_$ch.json'));r=d['roofline'];print('chunk $ch: expand %.2f ms  %.0f GB/s  ks %.2f ms'%(r['ms_per_launch'],r['achieved'],r['ms_keyspace_scan_plan']))"
done
