#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_modes.py tests/test_gpu_configs.py -v -m gpu -x -k "modes or substitute_all or ranges or golden or multi_value" --timeout 300 --timeout-method thread > gpurun_out/md.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/md.log
grep -E "Error|assert" gpurun_out/md.log | head -8
[ $rc -eq 0 ] || exit 10
for spec in "2 0" "3 1"; do
  set -- $spec
  timeout -k 10 300 python bench.py --workload c5 --mode $1 --min $2 --words 2000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bm_$1_$2.json 2> gpurun_out/bm_$1_$2.err || { echo "bench failed"; tail -5 gpurun_out/bm_$1_$2.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/bm_$1_$2.json'));r=d['roofline'];print('mode $1 min $2: %.3e cand/s  expand %.2f ms  %.0f GB/s  ks %.2f ms step %.2f ms'%(d['value'],r['ms_per_launch'],r['achieved'],r['ms_keyspace_scan_plan'],d['ms_per_step']))"
done
