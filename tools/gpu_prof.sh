#!/bin/bash
# GPU-box script: rocprofv3 kernel-trace + stats of a short bench run (gpurun_out/prof_$TAG)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
T=${TAG:-x}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --words ${WORDS:-10000000} --workload ${WORKLOAD:-c3} > $R/gpurun_out/prof_$T.log 2>&1 || { tail -20 $R/gpurun_out/prof_$T.log; exit 13; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$R/gpurun_out/prof_$T/run_kernel_stats.csv")))
for r in rows: print("%-28s calls %4s avg %10.1f us  total %8.2f ms  %5s%%"%(r["Name"][:28], r["Calls"], float(r["AverageNs"])/1e3, float(r["TotalDurationNs"])/1e6, r["Percentage"]))
PY
tail -2 $R/gpurun_out/prof_$T.log
