#!/bin/bash
# GPU-box script: fused digest bench lines (C5 shape), rocprofv3 kernel stats and one PMC
# pass (VALU instruction counts) of k_digest_stream (outputs under gpurun_out/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
T=${TAG:-d}; W=${WORDS:-1000000}
for alg in md5 ntlm; do
  timeout -k 10 400 python bench.py --digest $alg --workload c5 --words $W --steps 3 --warmup 1 ${BARGS} > gpurun_out/bench_${T}_$alg.json 2> gpurun_out/bench_${T}_$alg.err || { tail -5 gpurun_out/bench_${T}_$alg.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${T}_$alg.json'));r=d['roofline'];c=d['cpu_baseline'];print('$alg value %.3e cand/s step %.1f ms digest %.1f ms (%.3e cand/s) expand %.1f ms cpu %s'%(d['value'],d['ms_per_step'],r['ms_digest_per_step'],r['digest_cand_per_s'],r['ms_expand_per_step'],c and '%.3e'%c['value']))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T} -o run --output-format csv -- python3 $R/bench.py --digest md5 --workload c5 --words $W --steps 2 --warmup 0 --no-cpu-baseline > $R/gpurun_out/prof_${T}.log 2>&1 || { tail -5 $R/gpurun_out/prof_${T}.log; exit 13; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-include-regex k_digest_stream -d $R/gpurun_out/pmcd_${T}_1 -o run --output-format csv -- python3 $R/bench.py --digest md5 --workload c5 --words 200000 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmcd_${T}_1.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/pmcd_${T}_1.log; exit 21; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD --kernel-include-regex k_digest_stream -d $R/gpurun_out/pmcd_${T}_2 -o run --output-format csv -- python3 $R/bench.py --digest md5 --workload c5 --words 200000 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmcd_${T}_2.log 2>&1 || { echo "pmc2 failed"; tail -5 $R/gpurun_out/pmcd_${T}_2.log; exit 22; }
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcd_${T}_ && grep -h "candidates" gpurun_out/pmcd_${T}_1.log | head -2
echo done
