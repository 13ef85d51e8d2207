"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_<tag>_<i>/run_counter_collection.csv) per kernel."""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
pat = f"{tag}*/run_counter_collection.csv" if "/" in tag else f"gpurun_out/pmc_{tag}_*/run_counter_collection.csv"
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(pat)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
kern = sorted({k for k, _ in agg})
for k in kern:
    print(k)
    d = {c: v / max(1, len(disp[(k, c)])) for (kk, c), v in agg.items() if kk == k}
    for c in sorted(d):
        print(f"   {c:28s} {d[c]:.4g}  (per dispatch)")
    if "SQ_WAVES" in d:
        w = d["SQ_WAVES"]
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM",
                  "SQ_INSTS_BRANCH"):
            if c in d:
                print(f"   {c:28s} per wave {d[c] / w:10.1f}")
    if "SQ_WAVE_CYCLES" in d:
        wc = d["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if c in d:
                print(f"   {c:28s} / WAVE_CYCLES {d[c] / wc:.3f}")
