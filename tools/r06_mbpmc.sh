#!/bin/bash
# round 6: write-request latency per store pattern (tools/mb_ustore, C3 layout) under rocprofv3 --pmc
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
R=$PWD
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_WRITE_REQ TCP_TCC_WRITE_REQ_LATENCY TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE \
   -d $R/gpurun_out/mbpmc -o run --output-format csv -- $R/tools/mb_ustore 1800000000 1 > $R/gpurun_out/r06g_mbpmc.log 2>&1 ) || { tail -5 gpurun_out/r06g_mbpmc.log; exit 3; }
python3 - <<'PY'
import csv, collections, glob
f = glob.glob("gpurun_out/mbpmc/**/run_counter_collection.csv", recursive=True) or glob.glob("gpurun_out/mbpmc/run_counter_collection.csv")
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"].split("(")[0].strip()
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, d in agg.items():
    req = d.get("TCP_TCC_WRITE_REQ", 0) or 1
    print("%-40s disp %d  req/disp %.3e  lat/req %.0f  pending %.3e  grbm %.3e" % (k, len(n[k]), req / len(n[k]), d.get("TCP_TCC_WRITE_REQ_LATENCY", 0) / req,
          d.get("TCP_PENDING_STALL_CYCLES", 0) / len(n[k]), d.get("GRBM_GUI_ACTIVE", 0) / len(n[k])))
PY
grep -E "round|aligned" gpurun_out/r06g_mbpmc.log | head -30
