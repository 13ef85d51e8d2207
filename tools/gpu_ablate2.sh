#!/bin/bash
# GPU-box script: expansion time of both FAST kernels under ablations (timing only)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for wg in ${WGS:-1 0}; do
  for ab in ${ABL:-0 6 8}; do
    A5X_FASTWG=$wg A5X_ABLATE=$ab timeout -k 10 60 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --words ${WORDS:-10000000} --workload ${WL:-c3} > gpurun_out/ab2_${wg}_$ab.json 2> gpurun_out/ab2_${wg}_$ab.err || { echo "bench failed"; tail -5 gpurun_out/ab2_${wg}_$ab.err; exit 11; }
    python -c "import json;d=json.load(open('gpurun_out/ab2_${wg}_$ab.json'));r=d['roofline'];print('fastwg $wg ablate $ab: expand %.2f ms  %.0f GB/s'%(r['ms_per_launch'],r['achieved']))"
  done
done
