"""Multi-rank path on CPU (gloo, world_size 2): balanced shards + counter all-reduce.

Per rank, the oracle (C restatement) digests its shard; the all-reduced totals must
equal the single-process totals -- the same reduction bench.py and the product use
over RCCL on GPUs (no data-path collective: words are independent, main.go:77)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

WORKER = r"""
import os, sys, json
sys.path.insert(0, {root!r})
import numpy as np
from hashcat_a5_table_generator_amd import dist as D, synth
from oracle import c_oracle as co
dist, rank, world, _ = D.init_from_env("gloo")
tables, (data, offs) = synth.config_words("c3", 3000, seed=11)
t = co.CTable([os.path.join({root!r}, "tests", "golden", "tables", x + ".table") for x in tables])
dig = t.digest_batch(data, offs, 0, 0, 15, nthreads=1)
prefix = np.zeros(len(offs), dtype=np.uint64); prefix[1:] = np.cumsum(dig[:, 1])
w0, w1 = D.shard_bounds(prefix, world, rank)
sd, so = D.shard_words(data, offs, w0, w1)
mine = t.digest_batch(sd, so, 0, 0, 15, nthreads=1)
tot = D.allreduce_u64(dist, [mine[:, 0].sum(), mine[:, 1].sum(), mine[:, 2].sum(dtype=np.uint64), w1 - w0], "gloo")
ref = [dig[:, 0].sum(), dig[:, 1].sum(), dig[:, 2].sum(dtype=np.uint64), len(offs) - 1]
out = dict(rank=rank, shard=[w0, w1], bytes=int(mine[:, 1].sum()), ok=[int(a) == int(b) for a, b in zip(tot, ref)])
print(json.dumps(out), flush=True)
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_two_ranks_shard_and_reduce(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), A5X_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e[-2000:]
        outs.append(o.strip().splitlines()[-1])
    import json
    res = sorted((json.loads(x) for x in outs), key=lambda d: d["rank"])
    assert all(all(r["ok"]) for r in res), res
    # contiguous, covering shards, balanced by output bytes
    assert res[0]["shard"][0] == 0 and res[0]["shard"][1] == res[1]["shard"][0] and res[1]["shard"][1] == 3000
    b0, b1 = res[0]["bytes"], res[1]["bytes"]
    assert abs(b0 - b1) / (b0 + b1) < 0.05


SPLIT_WORKER = r"""
import os, sys, json
sys.path.insert(0, {root!r})
import numpy as np
from hashcat_a5_table_generator_amd import dist as D, synth, partition
from oracle import c_oracle as co
dist, rank, world, _ = D.init_from_env("gloo")
n = {n}
tables, (data, offs) = synth.global_words("c3", 0, n, seed=23)
# this rank's equal-count block: its keyspace prefix (bytes per word; the C oracle stands
# in for the keyspace kernel on CPU) -> distributed split
b0, b1 = D.block_bounds(n, world, rank)
t = co.CTable([os.path.join({root!r}, "tests", "golden", "tables", x + ".table") for x in tables])
sd, so = D.shard_words(data, offs, b0, b1)
lp = np.zeros(b1 - b0 + 1, dtype=np.uint64); lp[1:] = np.cumsum(t.digest_batch(sd, so, 0, 0, 15, nthreads=1)[:, 1])
split = D.distributed_split(dist, lp, b0, n, world, "gloo")
# rank 0 checks against a5x_partition over the whole prefix
ok = True
if rank == 0:
    full = np.zeros(n + 1, dtype=np.uint64); full[1:] = np.cumsum(t.digest_batch(data, offs, 0, 0, 15, nthreads=1)[:, 1])
    ok = bool(np.array_equal(split, partition(full, world)))
print(json.dumps(dict(rank=rank, split=[int(x) for x in split], ok=ok)), flush=True)
dist.destroy_process_group()
"""


def _run_ranks(tmp_path, src, world):
    script = tmp_path / f"w{world}.py"
    script.write_text(src)
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), A5X_DIST_BACKEND="gloo")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e[-2000:]
        outs.append(o.strip().splitlines()[-1])
    import json
    return sorted((json.loads(x) for x in outs), key=lambda d: d["rank"])


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_split_equals_global_partition(tmp_path, world):
    """north_star (e): each rank keyspaces only its equal-count block; an all-gather of
    block totals + all-reduce(MIN) gives exactly a5x_partition over the global prefix."""
    res = _run_ranks(tmp_path, SPLIT_WORKER.format(root=ROOT, n=4000), world)
    assert all(r["ok"] for r in res), res
    assert all(r["split"] == res[0]["split"] for r in res), res
    s = res[0]["split"]
    assert s[0] == 0 and s[-1] == 4000 and s == sorted(s)


def test_global_words_slices_are_consistent(monkeypatch):
    from hashcat_a5_table_generator_amd import synth
    monkeypatch.setattr(synth, "GLOBAL_BLOCK", 1000)  # slices that cross block seeds
    _, (d, o) = synth.global_words("c4", 0, 2500, seed=5)
    _, (d2, o2) = synth.global_words("c4", 700, 1900, seed=5)
    assert bytes(d[int(o[700]):int(o[1900])]) == bytes(d2[:int(o2[-1])])
    assert np.array_equal(np.diff(o[700:1901].astype(np.int64)), np.diff(o2.astype(np.int64)))


def test_partition_properties():
    from hashcat_a5_table_generator_amd import partition
    rng = np.random.default_rng(0)
    w = rng.integers(0, 1000, size=1000).astype(np.uint64)
    prefix = np.zeros(1001, dtype=np.uint64)
    prefix[1:] = np.cumsum(w)
    for parts in (1, 2, 3, 8, 64):
        s = partition(prefix, parts)
        assert s[0] == 0 and s[-1] == 1000 and np.all(np.diff(s.astype(np.int64)) >= 0)
        total = int(prefix[-1])
        for r in range(1, parts):
            # split r starts at the first word whose start offset reaches r/parts of the total
            assert int(prefix[s[r]]) >= total * r // parts
            assert s[r] == 0 or int(prefix[s[r] - 1]) < -(-total * r // parts)


GATHER_WORKER = r"""
import os, sys, json
sys.path.insert(0, {root!r})
import numpy as np
from hashcat_a5_table_generator_amd import dist as D
dist, rank, world, _ = D.init_from_env("gloo")
# rank r found r + 1 hits (rank 1 none at all, to cover an empty contribution) in its
# shard [w0, w0 + 1000): local word indices, mapped to global ones by the shard base
n = 0 if rank == 1 else rank + 2
rng = np.random.default_rng(rank)
hits = [(int(rng.integers(0, 1000)), int(rng.integers(0, 1 << 40)), rng.bytes(16)) for _ in range(n)]
rows = D.hits_to_rows(hits, word_base=1000 * rank)
got = D.gather_rows_u64(dist, rows, "gloo")
ok = True
if rank == 0:
    want = []
    for r in range(world):
        m = 0 if r == 1 else r + 2
        g = np.random.default_rng(r)
        want += [(int(g.integers(0, 1000)) + 1000 * r, int(g.integers(0, 1 << 40)), g.bytes(16)) for _ in range(m)]
    ok = D.rows_to_hits(got) == want
else:
    ok = got is None
print(json.dumps(dict(rank=rank, ok=bool(ok))), flush=True)
dist.destroy_process_group()
"""


@pytest.mark.parametrize("world", [2, 3])
def test_hit_gather_global_word_indices(tmp_path, world):
    """north_star (e) "gather hits": every rank's hit records, word indices rebased from
    its shard to the global list, arrive on rank 0 in rank order (empty ranks included)."""
    res = _run_ranks(tmp_path, GATHER_WORKER.format(root=ROOT), world)
    assert all(r["ok"] for r in res), res


HUGE_WORKER = r"""
import hashlib, os, sys, json
sys.path.insert(0, {root!r})
import numpy as np
from hashcat_a5_table_generator_amd import dist as D
from oracle import c_oracle as co
dist, rank, world, _ = D.init_from_env("gloo")
# ONE global list: length-10 [a-z] words and three 20-letter words (2^20 - 1 candidates,
# ~32 MB each under qwerty-cyrillic: each larger than a rank's share of the ~110 MB)
rng = np.random.default_rng(3)
words = [bytes(rng.integers(97, 123, size=10, dtype=np.uint8)) for _ in range(600)]
for k, at in enumerate((5, 250, 251)):
    words.insert(at, bytes(rng.integers(97, 123, size=20, dtype=np.uint8)))
n = len(words)
t = co.CTable([os.path.join({root!r}, "tests", "golden", "tables", "qwerty-cyrillic.table")])

def stream(ws):
    # the oracle's stream of words ws and the first byte of every candidate (its own,
    # deterministic candidate order stands in for the device's in this CPU test)
    data, offs = co.pack_words(ws)
    out, wb = t.expand_batch(data, offs, 0, 0, 15)
    buf = np.frombuffer(out, dtype=np.uint8)
    nl = np.flatnonzero(buf == 10)
    starts = np.concatenate([[0], nl[:-1] + 1]).astype(np.uint64)
    cnt = np.zeros(len(ws) + 1, dtype=np.int64)
    pos, k = 0, 0
    for i, b in enumerate(wb):  # candidates per word from the per-word bytes
        e = pos + int(b)
        k2 = int(np.searchsorted(starts, np.uint64(e), side="left"))
        cnt[i + 1] = cnt[i] + (k2 - k)
        pos, k = e, k2
    return out, starts, cnt

b0, b1 = D.block_bounds(n, world, rank)
out, starts, cnt = stream(words[b0:b1])

def split_fn(targets):
    g = np.searchsorted(starts, targets, side="left").astype(np.uint64)
    w = np.searchsorted(cnt, g.astype(np.int64), side="right") - 1
    w = np.minimum(w, b1 - b0)
    c = g.astype(np.int64) - cnt[w]
    b = np.array([int(starts[x]) if x < len(starts) else len(out) for x in g], dtype=np.uint64)
    return g, w, c, b

split = D.candidate_split(dist, len(starts), len(out), b0, n, world, split_fn, "gloo")
w0, w1, c0, ncand, bstart, nbytes = D.shard_of(split, rank)
sout, sstarts, _ = stream(words[w0:w1])
lo = int(sstarts[c0]) if c0 < len(sstarts) else len(sout)
hi = int(sstarts[c0 + ncand]) if c0 + ncand < len(sstarts) else len(sout)
piece = sout[lo:hi]
rows = D.allgather_u64(dist, [bstart, len(piece), int.from_bytes(hashlib.sha256(piece).digest()[:7], "little")],
                       "gloo")
ok = len(piece) == nbytes
if rank == 0:
    full, _, _ = stream(words)
    pos = 0
    for r in range(world):
        s, L, h = (int(x) for x in rows[r])
        ok = ok and s == pos and int.from_bytes(hashlib.sha256(full[s:s + L]).digest()[:7], "little") == h
        pos += L
    ok = ok and pos == len(full)
sizes = [int(x) for x in rows[:, 1]]
print(json.dumps(dict(rank=rank, ok=bool(ok), sizes=sizes, split=split.tolist())), flush=True)
dist.destroy_process_group()
"""


@pytest.mark.parametrize("world", [2, 3])
def test_candidate_split_cuts_huge_words(tmp_path, world):
    """SURVEY 8(e) e1 / VERDICT r3: words larger than a rank's share are split inside at the
    candidate whose first byte reaches the rank's byte target, so shards stay balanced
    (max/min bytes < 1.01) where a word-granular split cannot be; the ranks' pieces tile the
    single-rank stream exactly (byte ranges and contents)."""
    res = _run_ranks(tmp_path, HUGE_WORKER.format(root=ROOT), world)
    assert all(r["ok"] for r in res), res
    sizes = res[0]["sizes"]
    assert max(sizes) / min(sizes) < 1.01, sizes
    split = res[0]["split"]
    assert any(c > 0 for c in split[2]), split  # at least one split falls inside a word


def _bench_cmd(*args):
    return [sys.executable, os.path.join(ROOT, "bench.py"), *args]


def test_bench_gpus_n_launches_n_ranks():
    """``bench.py --gpus 3`` with no launcher starts 3 ranks itself (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* as torch.distributed.run sets them) and relays rank 0's stdout
    line only; the parent touches no GPU (A5X_LAUNCH_PROBE: the ranks stop before it)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run(_bench_cmd("--gpus", "3"), env=dict(env, A5X_LAUNCH_PROBE="1"), stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    import json
    r0 = json.loads(lines[0])
    assert r0["RANK"] == "0" and r0["LOCAL_RANK"] == "0" and r0["WORLD_SIZE"] == "3"
    assert r0["MASTER_ADDR"] == "127.0.0.1" and int(r0["MASTER_PORT"]) > 0
    others = [json.loads(ln) for ln in p.stderr.splitlines() if ln.startswith("{")]
    assert sorted(o["RANK"] for o in others) == ["1", "2"]
    assert {o["MASTER_PORT"] for o in others} == {r0["MASTER_PORT"]}


def test_bench_launch_fails_if_a_rank_fails():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run(_bench_cmd("--gpus", "2"), env=dict(env, A5X_LAUNCH_PROBE="fail"), stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=120)
    assert p.returncode != 0
    assert "rank 1 exited with 3" in p.stderr


def test_bench_refuses_gpus_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    p = subprocess.run(_bench_cmd("--gpus", "3", "--backend", "gloo"), env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=120)
    assert p.returncode != 0 and "--gpus 3 but WORLD_SIZE=2" in p.stderr
