"""Summarise tools/gpu_digest_prof.sh output for one algorithm into
gpurun_out/pmc_digest_<algo>_c5.json (int ops per candidate, VALU busy, kernel time)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import MODE_NAMES, digest_src_sha  # noqa: E402


def breakdown(algos):
    """tools/gpu.sh dabl: VALU wave instructions per candidate of k_expand_fast_<algo> in the
    product build and the FX_DABL variants (1 no MD rounds, 2 no probe, 3 neither) ->
    MD rounds = full - dabl1, probe = full - dabl2, expansion + ring = dabl3."""
    out = os.path.join(ROOT, "gpurun_out")
    for algo in algos.split():
        per = {}
        for v in ("cur", "dabl1", "dabl2", "dabl3"):
            f = glob.glob(os.path.join(out, "dabl_%s_%s" % (algo, v), "run_counter_collection.csv"))
            valu = sum(float(r["Counter_Value"]) for r in csv.DictReader(open(f[0])) if r["Counter_Name"] == "SQ_INSTS_VALU")
            cands = None
            for line in open(os.path.join(out, "dabl_%s_%s.log" % (algo, v))):
                if line.startswith("{"):
                    cands = json.loads(line)["config"]["candidates_per_gpu_step"]
            per[v] = valu * 64 / cands  # int lane-ops per candidate
        res = {"algo": algo, "kernel": "k_expand_fast_" + algo, "kernel_src_sha": digest_src_sha(),
               "int_ops_per_cand": per["cur"], "md_rounds": per["cur"] - per["dabl1"],
               "probe": per["cur"] - per["dabl2"], "expansion_ring_and_loop": per["dabl3"],
               "variants": per,
               "note": "SQ_INSTS_VALU x 64 / candidates of one C5 step (2M words, 1M targets); FX_DABL variant builds: "
                       "1 = MD rounds replaced by a 4-op stand-in, 2 = probe replaced by a never-true test, 3 = both"}
        json.dump(res, open(os.path.join(out, "digest_breakdown_%s_c5.json" % algo), "w"), indent=1)
        print(json.dumps(res))


if sys.argv[1] == "breakdown":
    breakdown(sys.argv[2])
    sys.exit(0)
algo, words = sys.argv[1], int(sys.argv[2])
kname = sys.argv[3] if len(sys.argv) > 3 else "k_digest_stream"
out = os.path.join(ROOT, "gpurun_out")


def counters(d):
    f = glob.glob(os.path.join(out, d, "run_counter_collection.csv"))
    tot = {}
    if not f:
        return tot
    for r in csv.DictReader(open(f[0])):
        tot.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return tot


c1, c2 = counters("dpmc1_" + algo), counters("dpmc2_" + algo)
bench = None
for line in open(os.path.join(out, "dpmc1_%s.log" % algo)):
    if line.startswith("{"):
        bench = json.loads(line)
cands = bench["config"]["candidates_per_gpu_step"]
stats = list(csv.DictReader(open(glob.glob(os.path.join(out, "dprof_" + algo, "run_kernel_stats.csv"))[0])))
# (kname "a+b": the digest stage's kernels, a = the first; their VALU counters summed)
dig = next((r for r in stats if kname.split("+")[0] in r["Name"]), None)
valu = sum(c1.get("SQ_INSTS_VALU", [0]))
mode = next((k for k, v in MODE_NAMES.items() if v == bench["config"].get("mode")), 0)
mn = int(bench["config"].get("table_min", 0))
res = {
    "workload": "c5", "words": words, "algo": algo, "kernel": kname, "kernel_src_sha": digest_src_sha(),
    "mode": mode, "min": mn,
    "candidates_per_step": cands,
    "valu_wave_insts_per_cand": valu / cands,
    "int_ops_per_cand": valu * 64 / cands,
    "salu_insts_per_cand": sum(c1.get("SQ_INSTS_SALU", [0])) / cands,
    "valu_busy_pct": (sum(c2["VALUBusy"]) / len(c2["VALUBusy"])) if c2.get("VALUBusy") else None,
    "valu_utilization_pct": (sum(c2["VALUUtilization"]) / len(c2["VALUUtilization"])) if c2.get("VALUUtilization") else None,
    "active_valu_per_wave_cycle": sum(c1.get("SQ_ACTIVE_INST_VALU", [0])) / max(1.0, sum(c1.get("SQ_WAVE_CYCLES", [1]))),
    "kernel_avg_us": float(dig["AverageNs"]) / 1e3 if dig else None,
    "kernel_calls": int(dig["Calls"]) if dig else None,
    # SQ_ACTIVE_INST_VALU counts quad-cycles per wave (MI355X_MICROARCH.md): / instructions =
    # a wave's residency per VALU instruction (~1 quad-cycle: one wave alone issues every 4
    # cycles), NOT the SIMD's issue cost (2 or 4 cycles by opcode: profiles/r06_mb_valu.txt)
    "active_valu_quad_cycles_per_inst": sum(c1.get("SQ_ACTIVE_INST_VALU", [0])) / max(1.0, valu),
    # effective shader clock over the profiled dispatches (GRBM_GUI_ACTIVE sums the 8 XCDs;
    # MI355X_MICROARCH.md 'DVFS give-back'), from the kernel's average duration in the
    # kernel-trace pass of the same workload
    "dispatches_counted": len(c1.get("GRBM_GUI_ACTIVE", [])),
    # (one kernel only: a "+" stage mixes the durations of different kernels)
    "eff_clock_ghz": (sum(c1["GRBM_GUI_ACTIVE"]) / 8.0 / (len(c1["GRBM_GUI_ACTIVE"]) * float(dig["AverageNs"])))
                     if dig and c1.get("GRBM_GUI_ACTIVE") and "+" not in kname else None,
    "note": "SQ_INSTS_VALU summed over the %s dispatches of one step (1 step, 0 warmup; the "
            "planted-target setup adds ~1e6 candidates); int_ops = wave instructions x 64 lanes" % kname,
}
tag = kname.replace("+", "_").replace("*", "") + ("_m%d_min%d" % (mode, mn) if mode else "")
json.dump(res, open(os.path.join(out, "pmc_digest_%s_%s_c5.json" % (algo, tag)), "w"), indent=1)
print(json.dumps(res))
