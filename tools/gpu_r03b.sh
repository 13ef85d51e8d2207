#!/bin/bash
# fused NTLM: C5 bench lines (md5 + ntlm, fused) and kernel stats + VALU counters of k_expand_fast_ntlm
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for alg in md5 ntlm; do
  timeout -k 10 300 python bench.py --digest $alg --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1 > gpurun_out/bd_$alg.json 2> gpurun_out/bd_$alg.err || { tail -5 gpurun_out/bd_$alg.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/bd_$alg.json'));r=d['roofline'];c=d['cpu_baseline'];print('$alg value %.3e cand/s step %.1f ms digest %.1f ms (%.3e cand/s) cpu %s'%(d['value'],d['ms_per_step'],r['ms_digest_per_step'],r['digest_cand_per_s'],c and '%.3e'%c['value']))"
done
ALGOS=ntlm KRE=k_expand_fast_ntlm bash tools/gpu_digest_prof.sh
