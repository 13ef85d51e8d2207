"""Multi-rank path on the GPU: bench.py's own sharding driven by two ranks (gloo
collectives, both ranks on device 0 of the one-GPU box) through liba5x.

north_star (e): ONE global word list, split across ranks by balanced output-byte prefix
(each rank keyspaces an equal word-count block on its device; dist.distributed_split),
every rank expands (or expands + digests + looks up) its shard with no data-path
collective; hit records are gathered on rank 0 with global word indices.  The
concatenated per-word digests and the gathered hits must equal a single-rank run over
the same global list (main.go:77: words are independent).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(world, args, dump):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--backend", "gloo",
               "--same-device", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--dump", str(dump), *args]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=300)
        assert p.returncode == 0, e[-3000:]
        outs.append(o)
    return json.loads(outs[0].strip().splitlines()[-1])


def _digests(dump):
    """Per-word digests of the whole list from the ranks' dumps.  Shards are candidate
    ranges (dist.candidate_split): a word cut between two ranks appears in both dumps with
    the digest of each rank's part -- {count, bytes, sum h, sum h^2} add up (mod 2^64)."""
    parts = []
    for f in os.listdir(dump):
        if f.startswith("digest_"):
            w0, w1 = (int(x) for x in f[len("digest_"):-len(".npy")].split("_"))
            parts.append((w0, w1, np.load(os.path.join(dump, f))))
    parts.sort()
    # contiguous, overlapping by at most the one cut word
    assert all(b[0] in (a[1], a[1] - 1) for a, b in zip(parts, parts[1:])), [(a, b) for a, b, _ in parts]
    lo, hi = parts[0][0], max(p[1] for p in parts)
    acc = np.zeros((hi - lo, 4), dtype=np.uint64)
    for w0, w1, d in parts:
        acc[w0 - lo:w1 - lo] += d
    return lo, hi, acc


@pytest.mark.parametrize("wl,mode", [("c3", 0), ("c5", 1), ("c5", 3)])
def test_two_ranks_expand_equals_one_rank(tmp_path, wl, mode):
    """2 ranks x 30k words per rank == 1 rank x 60k words, per-word digests: C3 in the
    default mode, C5 in -r (FAST-probe words) and -s -r (piece engine + FAST probe)."""
    args = ["--workload", wl, "--mode", str(mode), "--steady-batches", "0"]
    r2 = _bench(2, args + ["--words", "30000"], tmp_path / "w2")
    r1 = _bench(1, args + ["--words", "60000"], tmp_path / "w1")
    a0, a1, d2 = _digests(tmp_path / "w2")
    b0, b1, d1 = _digests(tmp_path / "w1")
    assert (a0, a1) == (b0, b1) == (0, 60000)
    assert np.array_equal(d2, d1)
    assert r2["n_gpus"] == 2 and r2["config"]["candidates_per_gpu_step"] > 0
    # every rank's candidates sum to the single-rank run's (value = all ranks' candidates / time)
    assert int(d2[:, 0].sum()) == r1["config"]["candidates_per_gpu_step"]


def test_two_ranks_cut_huge_words(tmp_path):
    """SURVEY 8(e) e1 / VERDICT r3: a list whose 24-letter words (2^24 - 1 candidates, ~0.6 GB
    each) are larger than a rank's share: the split points are candidates found on the
    device (a5x_split_device), the ranks' shard bytes differ by < 1 %, and the per-word
    digests (cut words summed over their two parts) equal the single-rank run."""
    args = ["--workload", "c4h", "--steady-batches", "0"]
    r2 = _bench(2, args + ["--words", "30000"], tmp_path / "w2")
    r1 = _bench(1, args + ["--words", "60000"], tmp_path / "w1")
    a0, a1, d2 = _digests(tmp_path / "w2")
    b0, b1, d1 = _digests(tmp_path / "w1")
    assert (a0, a1) == (b0, b1) == (0, 60000)
    assert np.array_equal(d2, d1)
    shares = r2["config"]["bytes_per_rank"]
    assert max(shares) / min(shares) < 1.01, shares
    assert int(d2[:, 0].sum()) == r1["config"]["candidates_per_gpu_step"]


@pytest.mark.parametrize("algo", ["md5", "ntlm"])
def test_two_ranks_digest_hits_gathered(tmp_path, algo):
    """C5 words, fused digest + lookup: the hits gathered on rank 0 (global word indices)
    equal the single-rank run's over the same global list and target set."""
    args = ["--workload", "c5", "--digest", algo, "--targets", "20000"]
    r2 = _bench(2, args + ["--words", "20000"], tmp_path / "h2")
    r1 = _bench(1, args + ["--words", "40000"], tmp_path / "h1")
    h2 = np.load(tmp_path / "h2" / "hits.npy")
    h1 = np.load(tmp_path / "h1" / "hits.npy")
    assert len(h1) >= r1["config"]["planted"] > 0
    key = lambda h: sorted(map(tuple, h.tolist()))
    assert key(h2) == key(h1)
    assert r2["config"]["hits_gathered_on_rank0"] == len(h1) and r2["config"]["planted"] == r1["config"]["planted"]


@pytest.mark.parametrize("wl,mode", [("c3", 0), ("c5", 3)])
def test_rccl_world1_rehearsal(tmp_path, wl, mode):
    """The RCCL branch (backend nccl: process group with device_id, cuda-tensor all-gather /
    all-reduce, candidate-granular split) under torchrun at WORLD_SIZE=1 (A5X_FORCE_DIST):
    per-word digests equal the plain single-process run -- the N>1 code path executed on
    the one-GPU box (the driver runs N = 2..8 on a full node)."""
    args = ["--workload", wl, "--mode", str(mode), "--steady-batches", "0", "--words", "60000",
            "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
    d1 = tmp_path / "rccl"
    env = dict(os.environ, A5X_FORCE_DIST="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--dump", str(d1), *args]
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert r["n_gpus"] == 1 and r["config"]["candidates_per_gpu_step"] > 0
    _bench(1, ["--workload", wl, "--mode", str(mode), "--steady-batches", "0", "--words", "60000"], tmp_path / "plain")
    a0, a1, dr = _digests(d1)
    b0, b1, dp = _digests(tmp_path / "plain")
    assert (a0, a1) == (b0, b1) == (0, 60000)
    assert np.array_equal(dr, dp)


def test_bench_gpus_2_without_launcher(tmp_path):
    """``bench.py --gpus 2`` with no torchrun starts its own two ranks (gloo, both
    on device 0 here), reports n_gpus 2, and their per-word digests equal a one-rank run."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    args = ["--workload", "c3", "--steady-batches", "0", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--same-device",
           "--words", "20000", "--dump", str(tmp_path / "w2"), *args]
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    r2 = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert r2["n_gpus"] == 2
    _bench(1, ["--workload", "c3", "--steady-batches", "0", "--words", "40000"], tmp_path / "w1")
    a0, a1, d2 = _digests(tmp_path / "w2")
    b0, b1, d1 = _digests(tmp_path / "w1")
    assert (a0, a1) == (b0, b1) == (0, 40000)
    assert np.array_equal(d2, d1)


def test_two_ranks_digest_cut_huge_words(tmp_path):
    """the fused digest cuts words too -- 24-letter words (2^24 - 1
    candidates each) larger than a rank's share are split at candidates
    (a5x_expand_digest_range_device), the ranks' shard bytes differ by < 1 %, and the hits
    gathered on rank 0 equal the single-rank run's."""
    args = ["--workload", "c4h", "--digest", "md5", "--targets", "20000"]
    r2 = _bench(2, args + ["--words", "30000"], tmp_path / "h2")
    r1 = _bench(1, args + ["--words", "60000"], tmp_path / "h1")
    h2 = np.load(tmp_path / "h2" / "hits.npy")
    h1 = np.load(tmp_path / "h1" / "hits.npy")
    assert len(h1) >= r1["config"]["planted"] > 0
    key = lambda h: sorted(map(tuple, h.tolist()))
    assert key(h2) == key(h1)
    shares = r2["config"]["bytes_per_rank"]
    assert max(shares) / min(shares) < 1.01, shares  # (word-granular shards could not: a word is ~20 % of one)
