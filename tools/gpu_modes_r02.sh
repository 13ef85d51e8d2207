#!/bin/bash
# -r / -s / -s -r bench lines + rocprofv3 kernel stats on the C5 shape (greek-hebrew x Greek words)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
W=${WORDS:-2000000}
for spec in "1 0" "2 0" "3 0" "3 1"; do
  set -- $spec; M=$1; MN=$2
  timeout -k 10 300 python bench.py --workload c5 --mode $M --min $MN --words $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bm_${M}_${MN}.json 2> gpurun_out/bm_${M}_${MN}.err || { echo "bench mode $M failed"; tail -5 gpurun_out/bm_${M}_${MN}.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/bm_${M}_${MN}.json'));r=d['roofline'];print('mode $M min $MN: %.3e cand/s  expand %.2f ms  %.0f GB/s  frac %.3f  ks %.2f ms step %.2f ms  cands %d'%(d['value'],r['ms_per_launch'],r['achieved'],r['frac'],r['ms_keyspace_scan_plan'],d['ms_per_step'],d['config']['candidates_per_gpu_step']))"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mprof_${M}_${MN} -o run --output-format csv -- python3 $R/bench.py --workload c5 --mode $M --min $MN --words $W --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/mprof_${M}_${MN}.log 2>&1) || { echo "prof mode $M failed"; tail -5 gpurun_out/mprof_${M}_${MN}.log; exit 12; }
  python3 - <<PY
import csv
for r in csv.DictReader(open("gpurun_out/mprof_${M}_${MN}/run_kernel_stats.csv")):
    if float(r["Percentage"]) > 1: print("   %-40s calls %4s avg %10.1f us  %5.1f%%"%(r["Name"][:40], r["Calls"], float(r["AverageNs"])/1e3, float(r["Percentage"])))
PY
done
