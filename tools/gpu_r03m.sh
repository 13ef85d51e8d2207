#!/bin/bash
# -s on C5 words: kernel breakdown
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_s5 -o run --output-format csv -- python3 $R/bench.py --mode 2 --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_s5.log 2>&1) || { tail -5 gpurun_out/prof_s5.log; exit 13; }
python3 - <<PY
import csv
rows=list(csv.DictReader(open("gpurun_out/prof_s5/run_kernel_stats.csv")))
for r in rows[:10]: print("%-28s calls %4s avg %10.1f us  total %8.2f ms"%(r["Name"][:28], r["Calls"], float(r["AverageNs"])/1e3, float(r["TotalDurationNs"])/1e6))
PY
tail -3 gpurun_out/prof_s5.log
