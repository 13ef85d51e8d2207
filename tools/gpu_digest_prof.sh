#!/bin/bash
# GPU-box script: fused-digest (C5) evidence per algorithm: rocprofv3 kernel stats +
# VALU counters of k_digest_stream -> gpurun_out/pmc_digest_<algo>_c5.json (read by
# bench.py --digest when its kernel_src_sha matches the sources).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
W=${WORDS:-2000000}
for A in ${ALGOS:-md5 ntlm}; do
  ARGS="--digest $A --workload c5 --words $W --no-cpu-baseline --targets 1000000"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dprof_$A -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 2 --warmup 1 > $R/gpurun_out/dprof_$A.log 2>&1 || { echo "trace $A failed"; tail -5 $R/gpurun_out/dprof_$A.log; exit 21; }
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex ${KRE:-k_digest_stream} -d $R/gpurun_out/dpmc1_$A -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 1 --warmup 0 > $R/gpurun_out/dpmc1_$A.log 2>&1 || { echo "pmc1 $A failed"; tail -5 $R/gpurun_out/dpmc1_$A.log; exit 22; }
  timeout -s KILL 200 rocprofv3 --pmc VALUBusy VALUUtilization --kernel-include-regex ${KRE:-k_digest_stream} -d $R/gpurun_out/dpmc2_$A -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 1 --warmup 0 > $R/gpurun_out/dpmc2_$A.log 2>&1 || echo "derived VALUBusy pass $A failed (raw counters only)"
  cd $R && python3 tools/digest_prof_summary.py $A $W ${KRE:-k_digest_stream} && cd /tmp
done
