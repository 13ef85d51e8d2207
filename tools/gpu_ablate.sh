#!/bin/bash
# GPU-box script: expansion time under phase ablations (timing only; output invalid when A5X_ABLATE != 0)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for ab in ${ABL:-0 2 4 6}; do
  A5X_ABLATE=$ab A5X_CHUNK=${CH:-8192} timeout -k 10 60 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --words ${WORDS:-10000000} --workload ${WL:-c3} > gpurun_out/ab_$ab.json 2> gpurun_out/ab_$ab.err || { echo "bench failed"; tail -5 gpurun_out/ab_$ab.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$ab.json'));r=d['roofline'];print('ablate $ab: expand %.2f ms  %.0f GB/s'%(r['ms_per_launch'],r['achieved']))"
done
