#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_modes.py tests/test_gpu_configs.py tests/test_gpu_digest.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/md.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/md.log
grep -E "Error|assert|FAILED" gpurun_out/md.log | head -8
[ $rc -eq 0 ] || exit 10
for spec in "2 0" "3 1"; do
  set -- $spec
  timeout -k 10 300 python bench.py --workload c5 --mode $1 --min $2 --words 2000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bm_$1_$2.json 2> gpurun_out/bm_$1_$2.err || { echo "bench failed"; tail -5 gpurun_out/bm_$1_$2.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/bm_$1_$2.json'));r=d['roofline'];print('mode $1 min $2: %.3e cand/s  expand %.2f ms  %.0f GB/s  ks %.2f ms step %.2f ms'%(d['value'],r['ms_per_launch'],r['achieved'],r['ms_keyspace_scan_plan'],d['ms_per_step']))"
done
for A in md5 ntlm; do
  timeout -k 10 300 python bench.py --digest $A --workload c5 --words 2000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bd_$A.json 2> gpurun_out/bd_$A.err || { echo "bench $A failed"; tail -5 gpurun_out/bd_$A.err; exit 12; }
  python -c "import json;d=json.load(open('gpurun_out/bd_$A.json'));r=d['roofline'];print('$A: %.3e cand/s step %.2f ms  fused %s  stage %.0f Mcand/s'%(d['value'],d['ms_per_step'],r['fused'],r['digest_cand_per_s']/1e6))"
done
ALGOS=md5 KRE=k_expand_fast_md5 timeout -k 10 600 bash tools/gpu_digest_prof.sh > gpurun_out/dprof_f.txt 2>&1 || { echo "prof failed"; tail -5 gpurun_out/dprof_f.txt; exit 13; }
tail -2 gpurun_out/dprof_f.txt
