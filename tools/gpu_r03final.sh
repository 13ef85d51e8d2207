#!/bin/bash
# Round-2 closing evidence on HEAD: full GPU parity suite, C3 bench line (with CPU
# baseline) + rocprof kernel stats + PMC traffic, C4 / C5-digest (md5, ntlm fused) /
# C5 -s bench lines, fused-digest VALU counters.  Outputs under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r02w}
timeout -k 10 500 python -u -m pytest tests/ -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/tq_$T.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tq_$T.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/tq_$T.log | head -8; exit 10; }
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}_c3.json 2> gpurun_out/bench_${T}_c3.err || { tail -5 gpurun_out/bench_${T}_c3.err; exit 11; }
python -c "import json;d=json.load(open('gpurun_out/bench_${T}_c3.json'));r=d['roofline'];print('c3 value %.3e frac %.3f expand %.2f ms step %.2f ms cpu %.3e'%(d['value'],r['frac'],r['ms_per_launch'],d['ms_per_step'],d['cpu_baseline']['value']))"
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$T.log 2>&1) || { tail -5 gpurun_out/prof_$T.log; exit 13; }
TAG=$T WL=c3 bash tools/gpu_pmc_traffic.sh || exit 14
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload c4 --words 12500000 > gpurun_out/bench_${T}_c4.json 2> gpurun_out/bench_${T}_c4.err || { tail -5 gpurun_out/bench_${T}_c4.err; exit 15; }
ALGOS="md5" KRE=k_expand_fast_md5 bash tools/gpu_digest_prof.sh || exit 16
ALGOS="ntlm" KRE=k_expand_fast_ntlm bash tools/gpu_digest_prof.sh || exit 17
for alg in md5 ntlm; do
  timeout -k 10 300 python bench.py --digest $alg --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1 > gpurun_out/bench_${T}_digest_$alg.json 2> gpurun_out/bench_${T}_digest_$alg.err || { tail -5 gpurun_out/bench_${T}_digest_$alg.err; exit 18; }
done
for m in 1 2 3; do
  timeout -k 10 300 python bench.py --mode $m --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${T}_c5_mode$m.json 2> gpurun_out/bench_${T}_c5_mode$m.err || { tail -5 gpurun_out/bench_${T}_c5_mode$m.err; exit 19; }
done
echo done
