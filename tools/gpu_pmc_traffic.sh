#!/bin/bash
# GPU-box script: HBM traffic of the expansion kernel from rocprofv3 PMC passes (one
# counter group per pass, MI355X_MICROARCH.md HBM section): WRITE_SIZE and FETCH_SIZE
# are KiB; gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads,
# so it is doubled.  Writes profiles/pmc_${TAG}_${WL}.json (read by bench.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
W=${WORDS:-10000000}; T=${TAG:-x}; WL=${WL:-c3}
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --words $W --workload $WL"
for grp in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_expand_fast" -d $R/gpurun_out/pmct_${T}_$grp -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmct_${T}_$grp.log 2>&1 || { echo "pmc $grp failed"; tail -5 $R/gpurun_out/pmct_${T}_$grp.log; exit 21; }
done
cd $R && python3 - <<PY
import csv, glob, json, sys
sys.path.insert(0, ".")
from bench import kernel_src_sha
vals = {}
for grp in ("WRITE_SIZE", "FETCH_SIZE"):
    rows = list(csv.DictReader(open(glob.glob("gpurun_out/pmct_${T}_%s/run_counter_collection.csv" % grp)[0])))
    v = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == grp]
    vals[grp] = sum(v) / len(v)   # per dispatch (KiB)
write_b = vals["WRITE_SIZE"] * 1024
fetch_b = vals["FETCH_SIZE"] * 1024 * 2
out = {"workload": "${WL}", "words": ${W}, "kernel": "k_expand_fast", "kernel_src_sha": kernel_src_sha(),
       "write_size_kib": vals["WRITE_SIZE"], "fetch_size_kib": vals["FETCH_SIZE"],
       "bytes_per_launch": write_b + fetch_b, "write_bytes": write_b, "fetch_bytes_corrected": fetch_b,
       "note": "rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE in separate passes; KiB; FETCH_SIZE x2 (gfx950)"}
json.dump(out, open("gpurun_out/pmc_${T}_${WL}.json", "w"), indent=1)
print(json.dumps(out))
PY
