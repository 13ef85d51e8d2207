#!/usr/bin/env python3
"""bench.py -- candidates/s of the hashcat -a 5 table expansion hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3] [--words N]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One "step" = one full pass of the hot path over one batch already resident in HBM:
keyspace (k_keyspace_*) -> prefix scans -> chunk plan -> expansion (k_expand_fast [+ k_expand_slow, k_expand_b])
into an HBM output buffer, i.e. a5x_expand_device() of include/a5x.h.  The default
workload is BASELINE.json configs[2]: czech.table + german.table over a synthetic
[a-z] list (len U[6,12]) of 10M words per GPU.  Multi-GPU (north_star (e)): ONE
global list of 10M x N words (synth.global_words) is split across the N ranks by
balanced output-byte prefix -- each rank keyspaces an equal word-count block, then
one all-gather of block totals + one all-reduce(MIN) give a5x_partition's split
(dist.distributed_split) -- and every rank expands its shard with no data-path
collective; the other collectives are the barrier and the max/sum timing reductions.

Prints ONE JSON line (rank 0) with the driver's fields plus "roofline" (expansion
kernel: algorithmic bytes = sum(len(cand)+1) per launch / average launch time from
HIP events on the library stream) and "cpu_baseline" (oracle/a5_oracle.c run with
the reference's goroutine/channel/writer structure on a bounded sample).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


MODE_NAMES = {0: "processWord (default)", 1: "processWordReverse (-r)", 2: "processWordSubstituteAll (-s)",
              3: "processWordSubstituteAllReverse (-s -r)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", help="c1 c2 c2a c3 c4 c5 (hashcat_a5_table_generator_amd/synth.py)")
    ap.add_argument("--words", type=int, default=10_000_000,
                    help="words per GPU: the global list has words x N words, split by output bytes")
    ap.add_argument("--min", type=int, default=0)
    ap.add_argument("--max", type=int, default=15)
    ap.add_argument("--mode", type=int, default=0, choices=(0, 1, 2, 3),
                    help="0 processWord (headline), 1 -r, 2 -s, 3 -s -r (main.go:80-92)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-words", type=int, default=120_000)
    ap.add_argument("--verify", action="store_true", help="digest-check the last step against the C oracle")
    ap.add_argument("--digest", default="none", choices=("none", "md5", "ntlm"),
                    help="fused expansion + digest + lookup (SURVEY 8(a) a8, configs[4]); use with --workload c5")
    ap.add_argument("--targets", type=int, default=1_000_000, help="target digests for --digest (planted + random)")
    ap.add_argument("--scratch-gb", type=float, default=8.0, help="device scratch for the --digest range loop")
    return ap.parse_args()


class Dist:
    def __init__(self, n_gpus: int):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            torch.cuda.set_device(self.local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            self.dist, self.torch = dist, torch
        if n_gpus != self.world and self.rank == 0:
            log(f"note: --gpus {n_gpus} but WORLD_SIZE={self.world}; using WORLD_SIZE")

    def barrier(self):
        if self.dist:
            self.dist.barrier()
            self.torch.cuda.synchronize()

    def reduce(self, x: float, op: str) -> float:
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device="cuda")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


SEED = 0x5A5


PARALLELISM = ("partition: one global list of words_per_gpu x {world} words, split over {world} rank(s) by "
               "balanced output-byte prefix (a5x_partition semantics: all-gather of block totals + all-reduce MIN); "
               "no data-path collective")


def shard_for_rank(args, D, ctx):
    """This rank's shard of ONE global list of words_per_gpu x N words (north_star (e),
    main.go:70-95 data parallelism): every rank keyspaces an equal word-count block,
    and the balanced split by output bytes (a5x_partition semantics) comes from one
    all-gather of block totals + one all-reduce(MIN) (dist.distributed_split).  Returns
    (tables, data, offs, (w0, w1))."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, dist as hd, synth
    n_total = args.words * D.world
    b0, b1 = hd.block_bounds(n_total, D.world, D.rank)
    tables, (bd, bo) = synth.global_words(args.workload, b0, b1, seed=SEED)
    if D.world == 1:
        return tables, bd, bo, (0, n_total)
    ctx.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
    dw, do = DeviceBuffer.from_array(ctx, bd), DeviceBuffer.from_array(ctx, bo)
    lp = DeviceBuffer(ctx, (b1 - b0 + 1) * 8)
    ctx.keyspace_device(dw.ptr, do.ptr, b1 - b0, args.mode, args.min, args.max, d_byte_off=lp.ptr)
    split = hd.distributed_split(D.dist, lp.to_array(np.uint64, count=b1 - b0 + 1), b0, n_total, D.world, "nccl")
    for b in (dw, do, lp):
        b.free()
    ctx.clear_table()
    w0, w1 = int(split[D.rank]), int(split[D.rank + 1])
    _, (data, offs) = synth.global_words(args.workload, w0, w1, seed=SEED)
    return tables, data, offs, (w0, w1)


def kernel_src_sha() -> str:
    """sha256 of every source under csrc/: a committed PMC profile counts only for the
    exact sources it was measured on."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(ROOT, "hashcat_a5_table_generator_amd", "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith((".h", ".hip", ".cpp")):
            with open(os.path.join(d, f), "rb") as fh:
                h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


digest_src_sha = kernel_src_sha


def digest_profile(algo: str, words: int, kernel: str):
    """VALU evidence of the digest kernel for THESE sources (tools/gpu_digest_prof.sh), else None."""
    sha = digest_src_sha()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_digest_*.json")), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except Exception:
            continue
        if (d.get("algo") == algo and d.get("words") == words and d.get("kernel_src_sha") == sha
                and d.get("kernel") == kernel):
            d["_file"] = os.path.relpath(f, ROOT)
            return d
    return None


def latest_profile_traffic(workload: str, words: int):
    """HBM bytes per expansion launch from a committed rocprofv3 --pmc pass
    (tools/gpu_pmc_traffic.sh) of THESE kernel sources on this workload and size, else None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    sha = kernel_src_sha()
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except Exception:
            continue
        if (d.get("workload") == workload and d.get("words") == words and d.get("kernel_src_sha") == sha
                and d.get("bytes_per_launch")):
            return d
    return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """Host threads for the CPU baseline: every core this process may use, capped at the
    GPU box's per-GPU CPU share (16; nproc there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(tables, args):
    """The reference algorithm restated in C (oracle/a5_oracle.c) with main.go:58-98's
    structure -- one worker per word from a pool, every candidate sent on a 1000-slot
    channel, one writer with a 4 KiB buffer -- timed at 1 thread and at all host threads."""
    from oracle import c_oracle as co
    from hashcat_a5_table_generator_amd import synth
    t = co.CTable([os.path.join(ROOT, "tests", "golden", "tables", x + ".table") for x in tables])
    fd = os.open(os.devnull, os.O_WRONLY)
    runs = []
    nmax = cpu_threads()
    for th in sorted({1, nmax}):
        nwords = args.cpu_sample_words
        _, (data, offs) = synth.config_words(args.workload, nwords, seed=0xC0FFEE)
        t0 = time.perf_counter()
        c, b = t.run_pipeline(data, offs, args.mode, args.min, args.max, th, fd)
        dt = time.perf_counter() - t0
        runs.append({"threads": th, "value": c / dt, "seconds": dt, "candidates": c})
        log(f"cpu baseline threads={th}: {c / dt / 1e6:.2f} Mcand/s ({dt:.2f} s)")
    os.close(fd)
    best = max(runs, key=lambda r: r["value"])
    return {"value": best["value"], "unit": "candidates/s", "cores": best["threads"], "kind": "port",
            "cpu_model": cpu_model(), "runs": runs,
            "sample": f"{args.cpu_sample_words} words of workload {args.workload} (seed 0xC0FFEE) to /dev/null; "
                      f"C restatement of main.go (oracle/a5_oracle.c) with its goroutine pool, 1000-slot channel "
                      f"(lock-free ring; a blocked sender or receiver spins briefly, then parks on a futex like a goroutine) and one 4 KiB writer; best of 1 and "
                      f"{nmax} worker thread(s) ({cpu_model()})"}


def digest_cpu_baseline(tables, args):
    """Reference algorithm restated in C (oracle/a5_oracle.c) + per-candidate digest on one host core."""
    from oracle import c_oracle as co
    from oracle import digest_oracle as dg
    from hashcat_a5_table_generator_amd import synth
    t = co.CTable([os.path.join(ROOT, "tests", "golden", "tables", x + ".table") for x in tables])
    nwords = max(50, args.cpu_sample_words // (50 if args.digest == "md5" else 2000))
    _, (data, offs) = synth.config_words(args.workload, nwords, seed=0xC0FFEE)
    f = dg.ALGOS[0 if args.digest == "md5" else 1]
    t0 = time.perf_counter()
    out, _ = t.expand_batch(data, offs, args.mode, args.min, args.max)
    n = 0
    for line in bytes(out).split(b"\n")[:-1]:
        f(line)
        n += 1
    dt = time.perf_counter() - t0
    log(f"cpu digest baseline: {n / dt / 1e6:.3f} Mcand/s ({dt:.2f} s)")
    return {"value": n / dt, "unit": "candidates/s", "cores": 1, "kind": "port",
            "sample": f"{nwords} words of workload {args.workload} (seed 0xC0FFEE): {n} candidates; C restatement "
                      f"of main.go expansion + {'hashlib MD5' if args.digest == 'md5' else 'RFC 1320 MD4 in Python (NTLM)'}"
                      f" per candidate, 1 thread"}


def digest_roofline(args, tc, ms_dig, ms_exp):
    """Digest stage: VALU-bound.  achieved = integer lane-ops/s of the digest kernel (int
    ops per candidate from the committed PMC profile of these sources x candidates /
    stage time); peak = 256 CUs x 4 SIMDs x 32 lanes/cycle x 2.4 GHz 32-bit VALU ops (a
    wave64 VALU instruction issues over 2 cycles: MI355X_MICROARCH.md; = the 157.3 TF f32
    FMA peak / 2).  Fused path (default mode): k_expand_fast_md5 / k_expand_fast_ntlm
    expand, hash and probe in one kernel, so the stage time is the expansion time."""
    fused = ms_dig < 1e-3
    kernel = f"k_expand_fast_{args.digest}" if fused else "k_digest_stream"
    ms_stage = ms_exp if fused else ms_dig
    prof = digest_profile(args.digest, args.words, kernel)
    peak = 256 * 4 * 32 * 2.4e9 / 1e12  # Tops/s
    r = {"bound": "valu", "kernel": kernel + ("" if fused else f"<{args.digest}>"), "fused": fused,
         "unit": "Tops/s (int32 lane ops)", "peak": peak, "ms_digest_per_step": ms_stage if not fused else 0.0,
         "ms_expand_per_step": ms_exp, "digest_cand_per_s": tc / (ms_stage * 1e-3), "achieved": None, "frac": None,
         "profile": None}
    if prof:
        ach = prof["int_ops_per_cand"] * tc / (ms_stage * 1e-3) / 1e12
        r.update(achieved=ach, frac=ach / peak, int_ops_per_cand=prof["int_ops_per_cand"],
                 valu_busy_pct=prof.get("valu_busy_pct"), valu_utilization_pct=prof.get("valu_utilization_pct"),
                 profile=f"{prof['_file']} (kernel_src_sha {prof['kernel_src_sha'][:12]})")
    return r


def run_digest(args, D):
    """Fused expansion + MD5/NTLM + target lookup over a resident batch (configs[4] shape)."""
    from hashcat_a5_table_generator_amd import ALGO_MD5, ALGO_NTLM, Context, DeviceBuffer, pack_words, synth
    algo = ALGO_MD5 if args.digest == "md5" else ALGO_NTLM
    ctx = Context(D.local)
    tables, data, offs, (w0, w1) = shard_for_rank(args, D, ctx)
    n = len(offs) - 1
    ctx.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
    dw = DeviceBuffer.from_array(ctx, data)
    do = DeviceBuffer.from_array(ctx, offs)
    tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, n, args.mode, args.min, args.max)
    # planted targets: one candidate of each of 1000 sampled words, digested by the device
    rng = np.random.default_rng(0xD16E57 + D.rank)
    sample = sorted(set(int(x) for x in rng.integers(0, n, size=1000)))
    sw = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in sample]
    cands = ctx.expand_words(sw, args.mode, args.min, args.max)
    planted = [(w, int(rng.integers(0, len(c)))) for w, c in zip(sample, cands) if c]
    lines = b"".join(cands[sample.index(w)][k] + b"\n" for w, k in planted)
    lb = DeviceBuffer.from_array(ctx, np.frombuffer(lines, dtype=np.uint8))
    db = DeviceBuffer(ctx, 16 * len(planted) + 16)
    ctx.digest_lines_device(algo, lb.ptr, len(lines), db.ptr, len(planted))
    pd = db.to_array(count=16 * len(planted)).reshape(-1, 16)
    rand = rng.integers(0, 256, size=(max(0, args.targets - len(planted)), 16), dtype=np.uint8)
    ctx.set_targets(algo, np.concatenate([pd, rand]))
    scratch = int(args.scratch_gb * (1 << 30))
    log(f"rank {D.rank}: {n} words -> {tc} candidates, {tb / 1e9:.2f} GB; {args.targets} targets "
        f"({len(planted)} planted)")

    def step():
        return ctx.expand_digest_device(dw.ptr, do.ptr, n, args.mode, args.min, args.max, scratch_bytes=scratch,
                                        hit_cap=1 << 20)

    for _ in range(args.warmup):
        step()
    D.barrier()
    t0 = time.perf_counter()
    res = [step() for _ in range(args.steps)]
    D.barrier()
    dt = time.perf_counter() - t0
    hits, st = res[-1]
    got = {(w, c) for w, c, _ in hits}
    missing = [p for p in planted if p not in got]
    if missing:
        raise SystemExit(f"digest lookup lost {len(missing)} planted hits, e.g. {missing[:3]}")
    dt_max = D.reduce(dt, "max")
    cands_all = D.reduce(float(tc) * args.steps, "sum")
    hits_all = D.reduce(float(len(hits)), "sum")
    ms_dig = float(np.mean([s["ms_total"] - s["ms_keyspace"] - s["ms_expand"] for _, s in res]))
    ms_exp = float(np.mean([s["ms_expand"] for _, s in res]))
    if D.rank == 0:
        desc = synth.CONFIGS[args.workload][3]
        res_line = {
            "metric": "candidates/sec (whole node) at 1/2/4/8 MI355X + % HBM write roofline",
            "value": cands_all / dt_max, "unit": "candidates/s", "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt_max / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8/u32", "data": "synthetic",
            "config": {"workload": f"{args.workload}: {desc} + fused {args.digest.upper()} lookup (configs[4])",
                       "tables": tables, "words_per_gpu": n, "candidates_per_gpu_step": tc, "bytes_per_gpu_step": tb,
                       "targets": args.targets, "planted": len(planted), "hits_all_ranks": hits_all,
                       "mode": MODE_NAMES[args.mode], "table_min": args.min, "table_max": args.max,
                       "scratch_bytes": scratch,
                       "parallelism": PARALLELISM.format(world=D.world) + "; hit counts all-reduced"},
            "roofline": digest_roofline(args, tc, ms_dig, ms_exp),
            "cpu_baseline": None if args.no_cpu_baseline else digest_cpu_baseline(tables, args),
        }
        print(json.dumps(res_line), flush=True)
    D.barrier()
    ctx.close()
    D.close()


def main():
    args = parse()
    D = Dist(args.gpus)
    if args.digest != "none":
        return run_digest(args, D)
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, synth

    ctx = Context(D.local)
    tables, data, offs, (w0, w1) = shard_for_rank(args, D, ctx)
    n = len(offs) - 1
    ctx.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
    dw = DeviceBuffer.from_array(ctx, data)
    do = DeviceBuffer.from_array(ctx, offs)
    tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, n, args.mode, args.min, args.max)
    log(f"rank {D.rank}: {ctx.device_name}: words [{w0}, {w1}) -> {tc} candidates, {tb / 1e9:.2f} GB")
    out = DeviceBuffer(ctx, max(tb, 16))
    boff = DeviceBuffer(ctx, (n + 1) * 8)

    def step():
        return ctx.expand_device(dw.ptr, do.ptr, n, out.ptr, tb, args.mode, args.min, args.max, d_byte_off=boff.ptr)

    for _ in range(args.warmup):
        step()
    D.barrier()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(step())
    D.barrier()
    dt = time.perf_counter() - t0
    dt_max = D.reduce(dt, "max")
    cands_all = D.reduce(float(tc) * args.steps, "sum")
    ms_exp = float(np.mean([s["ms_expand"] for s in stats]))
    ms_ks = float(np.mean([s["ms_keyspace"] for s in stats]))
    launches = stats[-1]["expand_launches"]
    ms_exp_max = D.reduce(ms_exp, "max")

    if args.verify:
        from oracle import c_oracle as co
        dig = DeviceBuffer(ctx, n * 32)
        ctx.digest_device(out.ptr, boff.ptr, 0, n, dig.ptr)
        got = dig.to_array(np.uint64).reshape(n, 4)
        want = co.CTable([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables]
                         ).digest_batch(data, offs, args.mode, args.min, args.max)
        bad = int((got != want).any(axis=1).sum())
        log(f"verify: {bad} mismatching words of {n}")
        if bad:
            raise SystemExit(f"verification failed on {bad} words")

    if D.rank == 0:
        achieved = tb / (ms_exp * 1e-3) / 1e9  # GB/s, algorithmic bytes per launch / launch time
        prof = latest_profile_traffic(args.workload, n) if args.mode == 0 and D.world == 1 else None
        traffic = None
        if prof:
            traffic = prof["bytes_per_launch"]
        desc = synth.CONFIGS[args.workload][3]
        res = {
            "metric": "candidates/sec (whole node) at 1/2/4/8 MI355X + % HBM write roofline",
            "value": cands_all / dt_max,
            "unit": "candidates/s",
            "n_gpus": D.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": f"{args.workload}: {desc}",
                "tables": tables,
                "words_per_gpu": n,
                "candidates_per_gpu_step": tc,
                "bytes_per_gpu_step": tb,
                "table_min": args.min,
                "table_max": args.max,
                "mode": MODE_NAMES[args.mode],
                "parallelism": PARALLELISM.format(world=D.world),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": ("k_expand_fast+k_expand_slow+k_expand_b (launched when present)" if args.mode == 0
                           else "k_mode_items (expansion pass)"),
                "ms_per_launch": ms_exp,
                "ms_per_launch_max_rank": ms_exp_max,
                "ms_keyspace_scan_plan": ms_ks,
                "words_slow_path": int(stats[-1]["words_slow"]),
                "words_big_path": int(stats[-1]["words_pass_b"]),
                "algorithmic_bytes_per_launch": tb,
            },
            "cpu_baseline": None,
        }
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(tables, args)
        print(json.dumps(res), flush=True)
    D.barrier()
    for b in (out, boff, dw, do):
        b.free()
    ctx.close()
    D.close()


if __name__ == "__main__":
    main()
