#!/bin/bash
# instruction-cache behaviour of the expansion and keyspace kernels (one SQC pair per pass)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
PMC="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES
SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_WAVES SQ_INSTS_VALU" TAG=ic KRE="k_expand_fast|k_keyspace" WORDS=2000000 bash tools/gpu_pmc2.sh > gpurun_out/pmc_ic.txt 2>&1; rc=$?
cat gpurun_out/pmc_ic.txt | grep -v "^\s*$"
exit $rc
