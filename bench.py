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
    ap.add_argument("--backend", default=os.environ.get("A5X_DIST_BACKEND", "nccl"), choices=("nccl", "gloo"),
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo: CPU collectives)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on device 0 (multi-rank tests on a one-GPU box)")
    ap.add_argument("--steady-batches", type=int, default=4,
                    help="also time this many batches through two contexts on two host threads (batch k+1's "
                         "keyspace under batch k's expansion): the steady-state line; 0 = off")
    ap.add_argument("--stdout", action="store_true",
                    help="the reference's own output path (main.go:58-68): the CLI replica's stdout to /dev/null "
                         "and to a pipe, and a5x_expand into a host sink (PCIe-inclusive rates, never `value` of "
                         "the headline line)")
    ap.add_argument("--dump", default=None,
                    help="directory: per-rank per-word digests (expansion) / gathered hits (--digest) for tests")
    return ap.parse_args()


class Dist:
    """One process per GPU (torchrun env).  backend "nccl" is RCCL over xGMI on ROCm;
    "gloo" runs the same collectives on the host (CPU tests, several ranks on one GPU)."""

    def __init__(self, n_gpus: int, backend: str = "nccl", same_device: bool = False):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        if n_gpus != self.world:  # (launch_ranks sets WORLD_SIZE = --gpus; a launcher must agree)
            raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={self.world} from the launcher")
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.device = 0 if same_device else self.local  # the GPU this rank drives
        self.backend = backend
        self.dist = None
        # (A5X_FORCE_DIST=1 under torchrun: the process group and every collective of the
        # multi-rank path also at WORLD_SIZE=1 -- an RCCL rehearsal on a one-GPU box)
        if self.world > 1 or os.environ.get("A5X_FORCE_DIST") == "1":
            import torch
            import torch.distributed as dist
            if backend == "nccl":
                torch.cuda.set_device(self.device)
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.device))
            else:
                dist.init_process_group(backend)
            self.dist, self.torch = dist, torch

    def barrier(self):
        if self.dist:
            self.dist.barrier()
            self.torch.cuda.synchronize()

    def reduce(self, x: float, op: str) -> float:
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device="cuda" if self.backend == "nccl" else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


SEED = 0x5A5


PARALLELISM = ("partition: one global list of words_per_gpu x {world} words, split over {world} rank(s) by "
               "balanced output-byte prefix (a5x_partition semantics: all-gather of block totals + all-reduce MIN); "
               "no data-path collective")


def shard_for_rank(args, D, ctx, intra_word=True):
    """This rank's shard of ONE global list of words_per_gpu x N words (north_star (e),
    main.go:70-95 data parallelism): every rank keyspaces an equal word-count block, and
    the balanced split by output bytes comes from one all-gather of block totals + one
    all-reduce(MIN).  intra_word: the split points are candidates, found
    exactly on the device (a5x_split_device / a5x_locate_device), so a word larger than a
    rank's share is cut inside (dist.candidate_split) -- the expansion and the fused digest
    alike (run_digest); else word boundaries (dist.distributed_split, a5x_partition
    semantics: only --verify, which checks whole words per rank).
    Returns (tables, data, offs, (w0, w1), (cand_begin, cand_count, shard_bytes)) -- candidates
    of the local batch [w0, w1); (0, None, None) = all of them."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, dist as hd, synth
    n_total = args.words * D.world
    b0, b1 = hd.block_bounds(n_total, D.world, D.rank)
    tables, (bd, bo) = synth.global_words(args.workload, b0, b1, seed=SEED)
    if D.dist is None:
        return tables, bd, bo, (0, n_total), (0, None, None)
    ctx.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
    dw, do = DeviceBuffer.from_array(ctx, bd), DeviceBuffer.from_array(ctx, bo)
    lp = DeviceBuffer(ctx, (b1 - b0 + 1) * 8)
    tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, b1 - b0, args.mode, args.min, args.max, d_byte_off=lp.ptr)
    if intra_word:
        def split_fn(targets):
            g, w, c = ctx.split_device(dw.ptr, do.ptr, b1 - b0, targets, args.mode, args.min, args.max)
            return g, w, c, ctx.locate_device(dw.ptr, do.ptr, b1 - b0, g, args.mode, args.min, args.max)
        split = hd.candidate_split(D.dist, tc, tb, b0, n_total, D.world, split_fn, D.backend)
        w0, w1, c0, ncand, _, nbytes = hd.shard_of(split, D.rank)
    else:
        ws = hd.distributed_split(D.dist, lp.to_array(np.uint64, count=b1 - b0 + 1), b0, n_total, D.world, D.backend)
        w0, w1, c0, ncand, nbytes = int(ws[D.rank]), int(ws[D.rank + 1]), 0, None, None
    for b in (dw, do, lp):
        b.free()
    ctx.clear_table()
    _, (data, offs) = synth.global_words(args.workload, w0, w1, seed=SEED)
    return tables, data, offs, (w0, w1), (c0, ncand, nbytes)


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


def digest_profile(algo: str, words: int, kernel: str, mode: int = 0, mn: int = 0):
    """VALU evidence of the digest kernel (tools/gpu.sh digestprof): the profile of THESE
    sources when committed, else the newest one for the same kernel, size and mode,
    flagged (its int ops per candidate are those of the profiled sources)."""
    sha = digest_src_sha()
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_digest_*.json")), key=os.path.getmtime, reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except Exception:
            continue
        if (d.get("algo") == algo and d.get("words") == words and d.get("kernel") == kernel
                and d.get("mode", 0) == mode and d.get("min", 0) == (mn if mode else d.get("min", 0))):
            d["_file"] = os.path.relpath(f, ROOT)
            d["_sha_match"] = d.get("kernel_src_sha") == sha
            if d["_sha_match"]:
                return d
            best = best or d
    return best


def latest_profile_traffic(workload: str, words: int, mode: int = 0):
    """HBM bytes per expansion launch (-r / -s / -s -r: per expansion, k_expand_fast and the
    mode-engine item kernels beside it summed) from a committed rocprofv3 --pmc pass
    (tools/gpu.sh traffic) of THESE kernel sources on this workload, size and mode, else None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    sha = kernel_src_sha()
    for f in reversed(files):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except Exception:
            continue
        if (d.get("workload") == workload and d.get("words") == words and d.get("kernel_src_sha") == sha
                and d.get("mode", 0) == mode and d.get("bytes_per_launch")):
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
    """Every core this process may use: its CPU affinity, capped by the cgroup CPU quota
    (on the GPU box the affinity lists the whole machine, 256 CPUs, but cpu.max grants 16:
    256 workers on 16 CPUs of quota ran the C port at 0.05 Mcand/s)."""
    try:
        n = max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_quota() -> str:
    """The cgroup CPU quota (cpu.max), if one limits this process."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        return "none" if q == "max" else f"{int(q) / int(p):g} CPUs"
    except (OSError, ValueError):
        return "unknown"


def thread_counts() -> list:
    """1 worker, the GPU box's per-GPU share (16) and all cores the process may use."""
    n = cpu_threads()
    return sorted({1, min(16, n), n})


def cpu_baseline(tables, args):
    """The reference algorithm restated in C (oracle/a5_oracle.c) with main.go:58-98's
    structure -- one worker per word from a pool, every candidate sent on a 1000-slot
    channel, one writer with a 4 KiB buffer -- timed at 1 thread, 16 threads and every core
    the process may use (all runs reported; value = the best)."""
    from oracle import c_oracle as co
    from hashcat_a5_table_generator_amd import synth
    t = co.CTable([os.path.join(ROOT, "tests", "golden", "tables", x + ".table") for x in tables])
    fd = os.open(os.devnull, os.O_WRONLY)
    runs = []
    for th in thread_counts():
        # with several workers the one shared channel (the reference's) serialises them and
        # every extra worker only adds contention (16 workers: ~1/5 of the 1-worker rate on
        # the GPU box): the pools get half the sample, shrinking further past 16 workers, so
        # every run stays within ~10-30 s (the rate, not the sample, is reported)
        nwords = args.cpu_sample_words if th == 1 else max(2000, args.cpu_sample_words * 8 // max(16, th))
        _, (data, offs) = synth.config_words(args.workload, nwords, seed=0xC0FFEE)
        t0 = time.perf_counter()
        c, b = t.run_pipeline(data, offs, args.mode, args.min, args.max, th, fd)
        dt = time.perf_counter() - t0
        runs.append({"threads": th, "value": c / dt, "seconds": dt, "candidates": c, "words": nwords})
        log(f"cpu baseline threads={th}: {c / dt / 1e6:.2f} Mcand/s ({dt:.2f} s, {nwords} words)")
    os.close(fd)
    best = max(runs, key=lambda r: r["value"])
    return {"value": best["value"], "unit": "candidates/s", "cores": best["threads"], "kind": "port",
            "cpu_model": cpu_model(), "cpu_affinity": cpu_threads(), "cpu_quota": cpu_quota(), "runs": runs,
            "sample": f"{args.cpu_sample_words} words of workload {args.workload} (seed 0xC0FFEE; worker pools "
                      f"{args.cpu_sample_words} x 8 / max(16, workers)) to /dev/null; "
                      f"C restatement of main.go (oracle/a5_oracle.c) with its goroutine pool, 1000-slot channel "
                      f"(lock-free ring; a blocked sender or receiver spins briefly, then parks on a futex like a "
                      f"goroutine) and one 4 KiB writer; runs at {[r['threads'] for r in runs]} worker thread(s), "
                      f"the best reported ({cpu_model()}, affinity {cpu_threads()} CPUs, quota {cpu_quota()})"}


def digest_cpu_baseline(tables, args, targets):
    """The reference expansion restated in C (oracle/a5_oracle.c) with every candidate
    digested (MD5 / NTLM = MD4 of Go's UTF-16LE, in C) and probed in the same target set,
    one word per worker task (main.go:77-93's goroutines), timed at 1 thread, 16 and every
    core the process may use."""
    from oracle import c_oracle as co
    from hashcat_a5_table_generator_amd import synth
    t = co.CTable([os.path.join(ROOT, "tests", "golden", "tables", x + ".table") for x in tables])
    # sample sized for ~10 s per run on the EPYC host (one thread: cpu_sample_words / 2 words;
    # a pool: 4 x cpu_sample_words), the words a prefix of one seeded stream
    nw1, nwp = max(50, args.cpu_sample_words // 2), max(50, args.cpu_sample_words * 4)
    _, (data_all, offs_all) = synth.config_words(args.workload, max(nw1, nwp), seed=0xC0FFEE)
    algo = 0 if args.digest == "md5" else 1
    runs = []
    for th in thread_counts():
        nwords = nw1 if th == 1 else nwp
        offs = offs_all[:nwords + 1]
        data = data_all[:int(offs[-1])]
        t0 = time.perf_counter()
        n, hits = t.digest_run(data, offs, args.mode, args.min, args.max, algo, targets, th)
        dt = time.perf_counter() - t0
        runs.append({"threads": th, "value": n / dt, "seconds": dt, "candidates": n, "hits": hits, "words": nwords})
        log(f"cpu digest baseline threads={th}: {n / dt / 1e6:.3f} Mcand/s ({dt:.2f} s)")
    best = max(runs, key=lambda r: r["value"])
    return {"value": best["value"], "unit": "candidates/s", "cores": best["threads"], "kind": "port", "runs": runs,
            "cpu_model": cpu_model(), "cpu_affinity": cpu_threads(), "cpu_quota": cpu_quota(),
            "sample": f"{nw1} words (1 thread) / {nwp} words (pools) of workload {args.workload} (seed 0xC0FFEE): C restatement of main.go's "
                      f"expansion + {args.digest.upper()} in C ({'RFC 1321' if algo == 0 else 'RFC 1320 MD4 of Go UTF-16LE'})"
                      f" + probe of the same {len(targets)} targets per candidate; runs at {[r['threads'] for r in runs]}"
                      f" thread(s), the best reported"}


def digest_mix_cycles(algo: str):
    """Mean SIMD issue cycles per VALU wave-instruction of the MD5 / MD4 compression
    (profiles/r06_digest_isa_mix.json: tools/isa_mix.py prices every opcode of md5_block /
    md4_block by the issue costs measured in profiles/r06_mb_valu.txt -- 2 cycles for
    v_add_u32 / v_xor_b32 / v_bitop3_b32, 4 for v_add3_u32 / v_alignbit_b32 / v_bfi_b32 /
    v_perm_b32 ...).  None when the file is absent."""
    f = os.path.join(ROOT, "profiles", "r06_digest_isa_mix.json")
    try:
        d = json.load(open(f))
        return d["md5_block" if algo == "md5" else "md4_block"]["mean_issue_cycles"]
    except (OSError, KeyError, ValueError):
        return None


def digest_roofline(args, tc, ms_dig, ms_exp, ms_ks, ms_step):
    """Digest stage: VALU-bound.  achieved = integer lane-ops/s of the digest kernel (int
    ops per candidate from the PMC profile (tools/gpu.sh digestprof: SQ_INSTS_VALU x 64 /
    candidates) x candidates / stage time).  Three peaks, all 256 CUs x 4 SIMDs at 2.4 GHz:
      * peak (frac): the nominal VALU rate, one wave64 instruction per 2 cycles per SIMD
        (32 lanes / cycle, MI355X_MICROARCH.md) = 78.6 T int32 lane-ops/s;
      * peak_vop3 (frac_vop3): every instruction at the half rate (4 cycles) of the VOP3
        integer ops the rounds lean on = 39.3 T;
      * peak_mix (frac_mix): the MD core's own mix, 64 lanes per (mean issue cycles) per SIMD
        (digest_mix_cycles: 2.80 cycles for MD5, 2.94 for MD4; profiles/r06_mb_valu.txt has the
        per-opcode costs, measured with every line live).
    SQ_ACTIVE_INST_VALU is in quad-cycles per wave: ACTIVE / INSTS is a wave's residency per
    instruction (~1 quad-cycle = 4 cycles), not the SIMD's issue cost.  Fused path (default
    mode): k_expand_fast_md5 / k_expand_fast_ntlm expand, hash and probe in one kernel, so the
    stage time is the expansion time.  The step's time is accounted as keyspace + stage
    (+ two-pass digest) + the rest (host)."""
    fused = ms_dig < 1e-3
    # (-r / -s / -s -r: the FAST-probe and virtual words hash in k_expand_fast_<algo>, the
    # rest in the mode engine's k_mode_digest_* beside it -- ops summed over both)
    kernel = ((f"k_expand_fast_{args.digest}" if args.mode == 0 else f"k_expand_fast_{args.digest}+k_mode_digest_*")
              if fused else "k_digest_stream")
    ms_stage = ms_exp if fused else ms_dig
    prof = digest_profile(args.digest, args.words, kernel, args.mode, args.min)
    peak = 256 * 4 * 32 * 2.4e9 / 1e12  # Tops/s: the nominal VALU rate (2 cycles per wave64 instruction)
    mixc = digest_mix_cycles(args.digest)
    peak_mix = 256 * 4 * 64 * 2.4e9 / mixc / 1e12 if mixc else None
    r = {"bound": "valu", "kernel": kernel + ("" if fused else f"<{args.digest}>"), "fused": fused,
         "unit": "Tops/s (int32 lane ops)", "peak": peak, "peak_vop3": peak / 2, "peak_mix": peak_mix,
         "mix_issue_cycles_per_inst": mixc,
         "ms_digest_per_step": ms_stage if not fused else 0.0,
         "ms_expand_per_step": ms_exp, "ms_keyspace_per_step": ms_ks, "ms_step": ms_step,
         "ms_step_unaccounted": ms_step - ms_ks - ms_exp - (0.0 if fused else ms_dig),
         "digest_cand_per_s": tc / (ms_stage * 1e-3), "achieved": None, "frac": None, "profile": None}
    if prof:
        r.update(profile=f"{prof['_file']} (kernel_src_sha {prof['kernel_src_sha'][:12]}"
                         f"{'' if prof['_sha_match'] else ', an earlier source revision'})")
        if prof["_sha_match"]:  # int ops per candidate count only for the sources they were measured on
            ach = prof["int_ops_per_cand"] * tc / (ms_stage * 1e-3) / 1e12
            r.update(achieved=ach, frac=ach / peak, frac_vop3=ach / (peak / 2),
                     frac_mix=(ach / peak_mix) if peak_mix else None, int_ops_per_cand=prof["int_ops_per_cand"],
                     valu_busy_pct=prof.get("valu_busy_pct"), valu_utilization_pct=prof.get("valu_utilization_pct"),
                     active_valu_quad_cycles_per_inst=prof.get("active_valu_quad_cycles_per_inst",
                                                               (prof.get("valu_cycles_per_inst") or 0) / 4 or None),
                     eff_clock_ghz=prof.get("eff_clock_ghz"))
            if prof.get("eff_clock_ghz") and peak_mix:  # the mix peak at the clock the chip held
                pk = peak_mix * prof["eff_clock_ghz"] / 2.4
                r.update(peak_mix_at_eff_clock=pk, frac_mix_at_eff_clock=ach / pk)
        else:
            r.update(frac_from_stale_profile=True, stale_int_ops_per_cand=prof["int_ops_per_cand"])
    return r


def plant_targets(args, D, ctx, data, offs, w0, algo, skip_first=False):
    """Targets of the C5 lookup: one candidate of each sampled word of the GLOBAL list
    (every stride-th global word index, candidate chosen by a generator seeded with that
    index, so the planted set does not depend on how the list is sharded), digested on
    the device; each rank plants the sampled words of its shard and one all-gather
    (dist.gather_rows_u64 to every rank via all-gather) gives every rank the same
    target set, plus the same random digests.  Returns (planted [(global word, cand)],
    target digests (n, 16) u8)."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, dist as hd
    n = len(offs) - 1
    stride = max(1, (args.words * D.world) // 1000)
    first = (w0 + (1 if skip_first else 0) + stride - 1) // stride * stride
    sample = list(range(first - w0, n, stride))
    sw = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in sample]
    cands = ctx.expand_words(sw, args.mode, args.min, args.max)
    mine = [(w0 + w, int(np.random.default_rng(w0 + w).integers(0, len(c)))) for w, c in zip(sample, cands) if c]
    lines = b"".join(cands[sample.index(g - w0)][k] + b"\n" for g, k in mine)
    rows = np.zeros((len(mine), 4), dtype=np.uint64)
    if mine:
        lb = DeviceBuffer.from_array(ctx, np.frombuffer(lines, dtype=np.uint8))
        db = DeviceBuffer(ctx, 16 * len(mine) + 16)
        ctx.digest_lines_device(algo, lb.ptr, len(lines), db.ptr, len(mine))
        dig = db.to_array(count=16 * len(mine)).reshape(-1, 16)
        rows = hd.hits_to_rows([(g, k, bytes(dig[i])) for i, (g, k) in enumerate(mine)])
    allrows = rows
    if D.dist is not None:  # every rank gets every rank's planted rows (an all-gather)
        allrows = _allgather_rows(D, rows, hd.allgather_u64(D.dist, [len(rows)], D.backend)[:, 0])
    planted = hd.rows_to_hits(allrows)
    pd = np.frombuffer(b"".join(d for _, _, d in planted), dtype=np.uint8).reshape(-1, 16)
    rng = np.random.default_rng(0xD16E57)  # the same random digests on every rank
    rand = rng.integers(0, 256, size=(max(0, args.targets - len(planted)), 16), dtype=np.uint8)
    return [(w, c) for w, c, _ in planted], np.concatenate([pd, rand])


def _allgather_rows(D, rows, counts):
    """Every rank's (n_r, 4) u64 rows on every rank (all-gather, padded to the largest n_r)."""
    from hashcat_a5_table_generator_amd import dist as hd
    m = int(counts.max())
    pad = np.zeros((max(m, 1), 4), dtype=np.uint64)
    pad[: len(rows)] = rows
    flat = hd.allgather_u64(D.dist, pad.reshape(-1), D.backend)
    return np.concatenate([flat[r].reshape(-1, 4)[: int(counts[r])] for r in range(D.world)])


def run_digest(args, D):
    """Fused expansion + MD5/NTLM + target lookup over a resident batch (configs[4]
    shape).  Multi-GPU (north_star (e)): every rank looks up its shard against the same
    target set; the hit counts are all-reduced and the hit records -- word indices
    rebased from the shard to the global list -- are gathered on rank 0, which checks
    that every planted (global word, candidate) was found."""
    from hashcat_a5_table_generator_amd import ALGO_MD5, ALGO_NTLM, Context, DeviceBuffer, dist as hd, synth
    algo = ALGO_MD5 if args.digest == "md5" else ALGO_NTLM
    ctx = Context(D.device)
    # (shards cut inside words at candidate split points, SURVEY 8(e) e1: each rank digests
    # the candidates [cb, ce) of its local word range, a5x_expand_digest_range_device)
    tables, data, offs, (w0, w1), (cb, ncand, nbytes) = shard_for_rank(args, D, ctx)
    n = len(offs) - 1
    ctx.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
    dw = DeviceBuffer.from_array(ctx, data)
    do = DeviceBuffer.from_array(ctx, offs)
    tc_all, tb_all = ctx.keyspace_device(dw.ptr, do.ptr, n, args.mode, args.min, args.max)
    bytes_per_rank = [tb_all if nbytes is None else nbytes] if D.dist is None else [
        int(x) for x in hd.allgather_u64(D.dist, [tb_all if nbytes is None else nbytes], D.backend)[:, 0]]
    ce = tc_all if ncand is None else cb + ncand
    tc = ce - cb
    rng = None if (cb, ce) == (0, tc_all) else (cb, ce)
    # (a word cut between two ranks is planted by the rank holding its start)
    planted, targets = plant_targets(args, D, ctx, data, offs, w0, algo, skip_first=cb > 0)
    ctx.set_targets(algo, targets)
    scratch = int(args.scratch_gb * (1 << 30))
    log(f"rank {D.rank}: words [{w0}, {w1}) candidates [{cb}, {ce}) of the local batch -> {tc} candidates; "
        f"{len(targets)} targets ({len(planted)} planted over all ranks)")

    def step():
        if rng is None:
            return ctx.expand_digest_device(dw.ptr, do.ptr, n, args.mode, args.min, args.max, scratch_bytes=scratch,
                                            hit_cap=1 << 20)
        return ctx.expand_digest_device(dw.ptr, do.ptr, n, args.mode, args.min, args.max, scratch_bytes=scratch,
                                        hit_cap=1 << 20, cand_begin=rng[0], cand_end=rng[1])

    for _ in range(args.warmup):
        step()
    D.barrier()
    t0 = time.perf_counter()
    res = [step() for _ in range(args.steps)]
    D.barrier()
    dt = time.perf_counter() - t0
    hits, st = res[-1]
    gathered = hd.gather_rows_u64(D.dist, hd.hits_to_rows(hits, word_base=w0), D.backend)  # rank 0: all ranks' hits
    dt_max = D.reduce(dt, "max")
    cands_all = D.reduce(float(tc) * args.steps, "sum")
    hits_all = D.reduce(float(len(hits)), "sum")
    ms_dig = float(np.mean([s["ms_total"] - s["ms_keyspace"] - s["ms_expand"] for _, s in res]))
    ms_exp = float(np.mean([s["ms_expand"] for _, s in res]))
    ms_ks = float(np.mean([s["ms_keyspace"] for _, s in res]))
    if D.rank == 0:
        got = {(w, c) for w, c, _ in hd.rows_to_hits(gathered)}
        missing = [p for p in planted if p not in got]
        if missing and not os.environ.get("A5X_BENCH_NO_HITCHECK"):  # (set only for ablation builds)
            raise SystemExit(f"digest lookup lost {len(missing)} planted hits, e.g. {missing[:3]}")
        if len(gathered) != int(hits_all):
            raise SystemExit(f"gathered {len(gathered)} hit records, ranks report {int(hits_all)}")
        if args.dump:
            os.makedirs(args.dump, exist_ok=True)
            np.save(os.path.join(args.dump, "hits.npy"), gathered)
        desc = synth.CONFIGS[args.workload][3]
        res_line = {
            "metric": "candidates/sec (whole node) at 1/2/4/8 MI355X + % HBM write roofline",
            "value": cands_all / dt_max, "unit": "candidates/s", "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt_max / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8/u32", "data": "synthetic",
            "config": {"workload": f"{args.workload}: {desc} + fused {args.digest.upper()} lookup (configs[4])",
                       "tables": tables, "words_per_gpu": n, "candidates_per_gpu_step": tc,
                       "candidate_range": [cb, ce], "bytes_per_rank": bytes_per_rank, "targets": len(targets), "planted": len(planted), "hits_all_ranks": hits_all,
                       "hits_gathered_on_rank0": len(gathered),
                       "mode": MODE_NAMES[args.mode], "table_min": args.min, "table_max": args.max,
                       "scratch_bytes": scratch,
                       "parallelism": PARALLELISM.format(world=D.world) + "; one target set on every rank (planted "
                                      "digests all-gathered); hit counts all-reduced, hit records gathered on rank 0 "
                                      "with global word indices"},
            "roofline": digest_roofline(args, tc, ms_dig, ms_exp, ms_ks, dt_max / args.steps * 1e3),
            "cpu_baseline": None if args.no_cpu_baseline else digest_cpu_baseline(tables, args, targets),
        }
        print(json.dumps(res_line), flush=True)
    D.barrier()
    ctx.close()
    D.close()


def steady_state(args, D, tables, tb1, n1):
    """Whole-job throughput over a stream of batches: ``--steady-batches`` batches (words
    disjoint from the headline batch and across ranks) already resident in HBM, run
    through two contexts on two host threads, so batch k + 1's keyspace overlaps batch
    k's expansion on the device (the CLI's pipeline, csrc/a5x_cli.cpp).  Batches are
    sized so the two output buffers stay <= 100 GB.  Returns the steady-state record."""
    import threading
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, synth
    nb = args.steady_batches
    wpb = max(1, min(n1, int(n1 * 50e9 / max(tb1, 1))))
    base = (D.world + D.rank * nb) * args.words  # past every rank's headline words
    batches = []
    ctxs = [Context(D.device) for _ in range(2)]
    paths = [os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables]
    for c in ctxs:
        c.load_tables(paths)
    for i in range(nb):
        _, (bd, bo) = synth.global_words(args.workload, base + i * wpb, base + (i + 1) * wpb, seed=SEED)
        batches.append((DeviceBuffer.from_array(ctxs[i & 1], bd), DeviceBuffer.from_array(ctxs[i & 1], bo)))
    sizes = [ctxs[i & 1].keyspace_device(batches[i][0].ptr, batches[i][1].ptr, wpb, 0, args.min, args.max)
             for i in range(nb)]
    outs = [DeviceBuffer(ctxs[t], max(16, max(sz[1] for i, sz in enumerate(sizes) if (i & 1) == t)))
            for t in range(min(2, nb))]
    errs = []

    def run(t):
        try:
            for i in range(t, nb, 2):
                dw, do = batches[i]
                ctxs[t].expand_device(dw.ptr, do.ptr, wpb, outs[t].ptr, sizes[i][1], 0, args.min, args.max)
        except Exception as e:  # noqa: BLE001 -- reported after the join
            errs.append(e)

    def all_batches():
        th = [threading.Thread(target=run, args=(t,)) for t in range(min(2, nb))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            raise errs[0]

    all_batches()  # warmup
    D.barrier()
    t0 = time.perf_counter()
    all_batches()
    D.barrier()
    dt = D.reduce(time.perf_counter() - t0, "max")
    cands = D.reduce(float(sum(c for c, _ in sizes)), "sum")
    nbytes = D.reduce(float(sum(b for _, b in sizes)), "sum")
    for dw, do in batches:
        dw.free()
        do.free()
    for o in outs:
        o.free()
    for c in ctxs:
        c.close()
    log(f"steady state: {nb} batches x {wpb} words, {dt * 1e3 / nb:.2f} ms/batch, "
        f"{nbytes / dt / 1e9:.0f} GB/s all ranks")
    return {"batches": nb, "words_per_batch": wpb, "contexts": 2, "value": cands / dt, "unit": "candidates/s",
            "ms_per_batch": dt * 1e3 / nb, "bytes_per_s": nbytes / dt,
            "frac": nbytes / dt / D.world / (HBM_PEAK_GBS * 1e9),
            "note": "whole job (keyspace + scan + plan + expansion) per batch, two contexts on two host threads: "
                    "batch k+1's keyspace overlaps batch k's expansion; frac = algorithmic bytes / wall / GPUs / 8 TB/s"}


PCIE_GBS = 64.0  # PCIe 5.0 x16, one direction, theoretical (MI355X host link)


def run_stdout(args, D):
    """Throughput of the drop-in's stdout path at the C3 shape: the CLI replica
    (a5x_generator: streamed dictionary, two-context batch pipeline, 4 MiB stdio
    buffer) writing "cand\n" to /dev/null and into a pipe drained by ``wc -c``, and
    a5x_expand (double-buffered pinned D2H) handing every span to a no-op host sink.
    Every byte crosses PCIe; the fraction is against 64 GB/s.  The CLI runs first, as
    a child process, before this process touches the GPU."""
    import ctypes
    import subprocess
    import tempfile
    from hashcat_a5_table_generator_amd import synth
    from hashcat_a5_table_generator_amd.build import CLI
    tables, (data, offs) = synth.config_words(args.workload, args.words, seed=SEED)
    n = len(offs) - 1
    tpaths = [os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables]
    body = bytes(data[: int(offs[-1])])
    lens = np.diff(offs.astype(np.int64))
    # the dictionary file: the words, one per line
    ends = np.cumsum(lens)
    text = bytearray(len(body) + n)
    src = np.frombuffer(body, dtype=np.uint8)
    dst = np.frombuffer(text, dtype=np.uint8)
    pos = np.arange(len(body)) + np.repeat(np.arange(n), lens)
    dst[pos] = src
    dst[ends + np.arange(n)] = 10
    runs = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        dpath = os.path.join(td, "dict.txt")
        with open(dpath, "wb") as f:
            f.write(text)
        cmd = [CLI, dpath] + sum((["-t", t] for t in tpaths), []) + ["-m", str(args.min), "-x", str(args.max)]
        tl = {}
        for name, shell in (("cli_devnull", None), ("cli_pipe_wc", " | wc -c")):
            best = None
            for _ in range(2):
                t0 = time.perf_counter()
                if shell is None:
                    r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                       env=dict(os.environ, A5X_CLI_TIMELINE="1"))
                    # the CLI's own clock (ms since main): first byte streamed, last batch written
                    ev = [ln.split("]", 1) for ln in r.stderr.decode(errors="replace").splitlines()
                          if ln.startswith("[tl")]
                    ts = [float(a[3:]) for a, b in ev if "streaming" in b]
                    te = [float(a[3:]) for a, b in ev if "all batches written" in b]
                    if ts and te and (not tl or te[0] - ts[0] < tl["stream_ms"]):
                        tl = {"first_byte_ms": ts[0], "stream_ms": te[0] - ts[0], "main_to_end_ms": te[0]}
                else:
                    r = subprocess.run(["bash", "-o", "pipefail", "-c", " ".join(cmd) + shell], stdout=subprocess.PIPE,
                                       stderr=subprocess.PIPE)
                dt = time.perf_counter() - t0
                if r.returncode:
                    raise SystemExit(f"{name}: {r.stderr.decode(errors='replace')[-500:]}")
                best = dt if best is None else min(best, dt)
            runs[name] = best
            if shell:
                runs["pipe_bytes"] = int(r.stdout.split()[0])
    from hashcat_a5_table_generator_amd import Context, _lib
    ctx = Context(D.device)
    ctx.load_tables(tpaths)
    tc, tb = ctx.keyspace(data, offs, args.mode, args.min, args.max)
    tc, tb = int(tc.sum()), int(tb.sum())
    cb = _lib.SINK(lambda u, p, k: 0)
    st = _lib.Stats()
    lib_t = None
    for _ in range(3):
        t0 = time.perf_counter()
        ctx._chk(ctx._L.a5x_expand(ctx.h, data.ctypes.data, offs.ctypes.data, n, args.mode, args.min, args.max, cb,
                                   None, ctypes.byref(st)))
        dt = time.perf_counter() - t0
        lib_t = dt if lib_t is None else min(lib_t, dt)
    ctx.close()
    if "pipe_bytes" in runs and runs["pipe_bytes"] != tb:
        raise SystemExit(f"CLI wrote {runs['pipe_bytes']} bytes, keyspace says {tb}")

    def rec(t):
        return {"seconds": t, "candidates_per_s": tc / t, "GB_per_s": tb / t / 1e9, "pcie_frac": tb / t / 1e9 / PCIE_GBS}
    desc = synth.CONFIGS[args.workload][3]
    line = {"metric": "candidates/sec through the stdout path (main.go:58-68), PCIe-inclusive", "value": tc / runs["cli_devnull"],
            "unit": "candidates/s", "n_gpus": 1, "higher_is_better": True, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.workload}: {desc}", "words": n, "candidates": tc, "bytes": tb,
                       "dict_bytes": len(text), "pcie_peak_GBps": PCIE_GBS},
            "cli_devnull": rec(runs["cli_devnull"]), "cli_pipe_wc": rec(runs["cli_pipe_wc"]),
            "cli_devnull_timeline": dict(tl, stream_GB_per_s=tb / (tl["stream_ms"] * 1e-3) / 1e9,
                                         main_to_end_GB_per_s=tb / (tl["main_to_end_ms"] * 1e-3) / 1e9,
                                         note="the CLI's own clock (A5X_CLI_TIMELINE): from main() / from its first "
                                              "streamed byte to the last batch written; the wall rate above adds "
                                              "process start and exit") if tl else None,
            "a5x_expand_host_sink": rec(lib_t),
            "note": "a5x_generator <dict> -t ... > /dev/null (and | wc -c): file read, batches of 4M words through "
                    "two contexts, pinned double-buffered D2H, fwrite; a5x_expand: the same D2H into a no-op C sink"}
    print(json.dumps(line), flush=True)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """``bench.py --gpus N`` with no launcher (WORLD_SIZE unset): this process starts N
    child ranks of itself -- RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1
    and a free MASTER_PORT, i.e. what ``torch.distributed.run --nproc-per-node N`` gives
    them -- relays rank 0's stdout (the one JSON line) and returns non-zero if any rank
    fails (the others are then terminated).  The parent never touches the GPU: the ranks
    initialise it, one process per GPU (main.go:70-95's data parallelism over words, here
    over devices)."""
    import subprocess
    import tempfile
    port = _free_port()
    procs = []
    # rank 0's stdout goes to a temporary file, read after the ranks exit: a PIPE read only
    # then could fill (~64 KiB) and block rank 0 while the others wait at a collective
    out0 = tempfile.TemporaryFile()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out0 if r == 0 else sys.stderr.fileno()))
    log(f"launched {n} ranks (pids {[p.pid for p in procs]}, master 127.0.0.1:{port})")
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            if p.poll() is not None:
                live.remove(p)
                if p.returncode and not rc:
                    rc = p.returncode
                    log(f"rank {procs.index(p)} exited with {p.returncode}; stopping the other ranks")
                    for q in live:
                        q.terminate()
        if live:
            time.sleep(0.2)
    out0.seek(0)
    out = out0.read().decode(errors="replace")
    out0.close()
    sys.stdout.write(out)
    sys.stdout.flush()
    return rc if rc > 0 else (1 if rc else 0)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus))
    probe = os.environ.get("A5X_LAUNCH_PROBE")  # (tests: the rank environment, before any GPU work)
    if probe:
        if probe == "fail" and os.environ.get("RANK") == "1":
            raise SystemExit(3)
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                         "MASTER_PORT")}), flush=True)
        return
    D = Dist(args.gpus, args.backend, args.same_device)
    if args.stdout:
        return run_stdout(args, D)
    if args.digest != "none":
        return run_digest(args, D)
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, synth

    ctx = Context(D.device)
    # (--verify checks whole words against the oracle on every rank: word-boundary shards)
    tables, data, offs, (w0, w1), (cb, ncand, _) = shard_for_rank(args, D, ctx, intra_word=not args.verify)
    n = len(offs) - 1
    ctx.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
    dw = DeviceBuffer.from_array(ctx, data)
    do = DeviceBuffer.from_array(ctx, offs)
    tc_all, tb_all = ctx.keyspace_device(dw.ptr, do.ptr, n, args.mode, args.min, args.max)
    ce = tc_all if ncand is None else cb + ncand
    rb, re_ = (0, tb_all) if (cb, ce) == (0, tc_all) else \
        (int(x) for x in ctx.locate_device(dw.ptr, do.ptr, n, [cb, ce], args.mode, args.min, args.max))
    tc, tb = ce - cb, re_ - rb  # this rank's candidates / bytes (the shard may cut words)
    log(f"rank {D.rank}: {ctx.device_name}: words [{w0}, {w1}) candidates [{cb}, {ce}) of the local batch -> "
        f"{tc} candidates, {tb / 1e9:.2f} GB")
    out = DeviceBuffer(ctx, max(tb, 16))
    boff = DeviceBuffer(ctx, (n + 1) * 8)

    def step():
        return ctx.expand_device(dw.ptr, do.ptr, n, out.ptr, tb, args.mode, args.min, args.max, cand_begin=cb,
                                 cand_end=ce, d_byte_off=boff.ptr)

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
    bytes_per_rank = [tb] if D.dist is None else \
        [int(x) for x in __import__("hashcat_a5_table_generator_amd.dist", fromlist=["x"]).allgather_u64(
            D.dist, [tb], D.backend)[:, 0]]
    ms_exp = float(np.mean([s["ms_expand"] for s in stats]))
    ms_ks = float(np.mean([s["ms_keyspace"] for s in stats]))
    launches = stats[-1]["expand_launches"]
    ms_exp_max = D.reduce(ms_exp, "max")

    if args.verify or args.dump:
        # per-word digests of this rank's bytes [rb, re_) of the local stream (a cut word:
        # the part this rank wrote; digests are sums, so the parts add up across ranks)
        bo_h = boff.to_array(np.uint64, count=n + 1)
        cut = DeviceBuffer.from_array(ctx, (np.clip(bo_h, rb, re_) - np.uint64(rb)).astype(np.uint64))
        dig = DeviceBuffer(ctx, n * 32)
        ctx.digest_device(out.ptr, cut.ptr, 0, n, dig.ptr)
        got = dig.to_array(np.uint64).reshape(n, 4)
        cut.free()
        if args.dump:  # this rank's shard: per-word digests of words [w0, w1) of the global list
            os.makedirs(args.dump, exist_ok=True)
            np.save(os.path.join(args.dump, f"digest_{w0}_{w1}.npy"), got)
    if args.verify and (cb, ce) != (0, tc_all):
        raise SystemExit("--verify checks whole batches (one rank); the multi-rank check is tests/test_gpu_dist.py")
    if args.verify:
        from oracle import c_oracle as co
        want = co.CTable([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables]
                         ).digest_batch(data, offs, args.mode, args.min, args.max)
        bad = int((got != want).any(axis=1).sum())
        log(f"verify: {bad} mismatching words of {n}")
        if bad:
            raise SystemExit(f"verification failed on {bad} words")

    out.free()
    steady = steady_state(args, D, tables, tb, n) if args.steady_batches > 0 and args.mode == 0 else None

    if D.rank == 0:
        achieved = tb / (ms_exp * 1e-3) / 1e9  # GB/s, algorithmic bytes per launch / launch time
        prof = latest_profile_traffic(args.workload, n, args.mode) if D.world == 1 else None
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
                "bytes_per_rank": bytes_per_rank,
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
                           else "k_expand_fast (-r FAST words) + k_mode_items_* (the other words), one stream each"
                           if args.mode == 1 else
                           "k_expand_fast (FAST-probe and virtual words) + k_mode_items_* (the other words), one stream each"),
                "ms_per_launch": ms_exp,
                "ms_per_launch_max_rank": ms_exp_max,
                "ms_keyspace_scan_plan": ms_ks,
                "words_slow_path": int(stats[-1]["words_slow"]),
                "words_big_path": int(stats[-1]["words_pass_b"]),
                "algorithmic_bytes_per_launch": tb,
            },
            "cpu_baseline": None,
            "steady_state": steady,
        }
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(tables, args)
        print(json.dumps(res), flush=True)
    D.barrier()
    for b in (boff, dw, do):
        b.free()
    ctx.close()
    D.close()


if __name__ == "__main__":
    main()
