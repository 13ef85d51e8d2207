#!/bin/bash
# GPU-box script: bench lines of the -r / -s / -s -r engines on C3 words (+ digest verify) and a
# rocprofv3 kernel-stats pass (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
T=${TAG:-m}
for m in 1 2 3; do
  timeout -k 10 300 python bench.py --mode $m --steps 5 --warmup 1 --words ${WORDS:-10000000} ${BARGS} > gpurun_out/bench_${T}_mode$m.json 2> gpurun_out/bench_${T}_mode$m.err || { tail -5 gpurun_out/bench_${T}_mode$m.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_mode$m.json'));r=d['roofline'];c=d['cpu_baseline'];print('mode $m value %.3e cand/s  expand %.2f ms  %.0f GB/s  ks %.2f ms  step %.2f ms cpu %s'%(d['value'],r['ms_per_launch'],r['achieved'],r['ms_keyspace_scan_plan'],d['ms_per_step'],c and '%.3e'%c['value']))"
done
timeout -k 10 300 python bench.py --mode 2 --steps 2 --warmup 1 --words 2000000 --verify --no-cpu-baseline > gpurun_out/bench_${T}_verify2.json 2> gpurun_out/bench_${T}_verify2.err || { tail -3 gpurun_out/bench_${T}_verify2.err; exit 12; }
grep verify gpurun_out/bench_${T}_verify2.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_mode2 -o run --output-format csv -- python3 $R/bench.py --mode 2 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_${T}_mode2.log 2>&1 || { tail -5 $R/gpurun_out/prof_${T}_mode2.log; exit 13; }
echo done
