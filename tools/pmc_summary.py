"""Summarise rocprofv3 --pmc passes (tools/gpu.sh steps ``pmc`` and ``traffic``).

    python tools/pmc_summary.py mix <prefix>                 # per-kernel counters per dispatch
    python tools/pmc_summary.py traffic <tag> <wl> <words> [kernel]
        -> gpurun_out/pmc_<tag>_<wl>.json (read by bench.py when kernel_src_sha matches)

HBM traffic per launch follows MI355X_MICROARCH.md's rocprofv3 section: WRITE_SIZE and
FETCH_SIZE in separate passes, in KiB; gfx950 FETCH_SIZE counts half the bytes of
16-B-per-lane streaming reads, so it is doubled.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mix(prefix):
    pat = f"{prefix}*/run_counter_collection.csv"
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in sorted(glob.glob(pat)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    for k in sorted({k for k, _ in agg}):
        print(k)
        d = {c: v / max(1, len(disp[(k, c)])) for (kk, c), v in agg.items() if kk == k}
        for c in sorted(d):
            print(f"   {c:28s} {d[c]:.4g}  (per dispatch)")
        if "SQ_WAVES" in d:
            w = d["SQ_WAVES"]
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD",
                      "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
                if c in d:
                    print(f"   {c:28s} per wave {d[c] / w:10.1f}")
        if "SQ_WAVE_CYCLES" in d:
            wc = d["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in d:
                    print(f"   {c:28s} / WAVE_CYCLES {d[c] / wc:.3f}")
        if "SQ_LDS_BANK_CONFLICT" in d and "SQ_LDS_IDX_ACTIVE" in d and d["SQ_LDS_IDX_ACTIVE"]:
            print(f"   LDS bank-conflict share       {d['SQ_LDS_BANK_CONFLICT'] / d['SQ_LDS_IDX_ACTIVE']:.3f}")


def traffic(tag, wl, words, kernel, mode=0):
    """Default mode: per k_expand_fast dispatch (average).  -r / -s / -s -r (mode > 0): the
    expansion is k_expand_fast beside the mode engine's item kernels, so the traffic of the
    step (1 step, 0 warmup: one expansion) is the sum over all the matched dispatches."""
    sys.path.insert(0, ROOT)
    from bench import kernel_src_sha
    vals = {}
    for grp in ("WRITE_SIZE", "FETCH_SIZE"):
        f = glob.glob(os.path.join(ROOT, "gpurun_out", f"pmct_{tag}_{grp}", "run_counter_collection.csv"))[0]
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Counter_Name"] == grp]
        vals[grp] = sum(v) if mode else sum(v) / len(v)  # KiB per dispatch / per step
    write_b = vals["WRITE_SIZE"] * 1024
    fetch_b = vals["FETCH_SIZE"] * 1024 * 2
    out = {"workload": wl, "words": words, "kernel": kernel, "kernel_src_sha": kernel_src_sha(), "mode": mode,
           "write_size_kib": vals["WRITE_SIZE"], "fetch_size_kib": vals["FETCH_SIZE"],
           "bytes_per_launch": write_b + fetch_b, "write_bytes": write_b, "fetch_bytes_corrected": fetch_b,
           "note": "rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE in separate passes; KiB; FETCH_SIZE x2 (gfx950)"}
    if mode:
        out["note"] += "; summed over the step's dispatches (k_expand_fast + mode-engine item kernels)"
    with open(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_{wl}{'_mode%d' % mode if mode else ''}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "mix":
        mix(sys.argv[2])
    elif sys.argv[1] == "traffic":
        traffic(sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5] if len(sys.argv) > 5 else "k_expand_fast",
                int(sys.argv[6]) if len(sys.argv) > 6 else 0)
    else:
        raise SystemExit(__doc__)
