#!/bin/bash
# branch-free NTLM unit decoder: digest parity + C5 NTLM bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_configs.py -q -m gpu -x --timeout 300 --timeout-method thread -k "fused or lookup or digest or c5" > gpurun_out/ta.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ta.log
grep -E "Error|assert|FAILED" gpurun_out/ta.log | head -8
[ $rc -eq 0 ] || exit 10
timeout -k 10 300 python bench.py --digest ntlm --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bd_ntlm.json 2> gpurun_out/bd_ntlm.err || { tail -5 gpurun_out/bd_ntlm.err; exit 11; }
python -c "import json;d=json.load(open('gpurun_out/bd_ntlm.json'));r=d['roofline'];print('ntlm value %.3e cand/s step %.1f ms (%.3e cand/s)'%(d['value'],d['ms_per_step'],r['digest_cand_per_s']))"
