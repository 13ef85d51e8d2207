"""Multi-GPU sharding for the expansion path.

Words are independent (the reference runs one goroutine per word,
main.go:77-93), so a node-level run is: split the word list into balanced
contiguous shards (by output bytes from the keyspace pass, or by word count),
expand each shard on its own GPU with no data-path communication, and reduce
only the tiny per-rank totals (candidate count, bytes, multiset digest) --
an all-reduce of a few u64 over RCCL (or gloo on CPU).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np

from .engine import partition


def shard_bounds(prefix: np.ndarray, world: int, rank: int) -> Tuple[int, int]:
    """Word range [w0, w1) of ``rank`` for a balanced split of ``prefix`` (n+1 offsets)."""
    split = partition(prefix, world)
    return int(split[rank]), int(split[rank + 1])


def block_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Equal word-count block [b0, b1) of ``rank``: the words whose keyspace it computes."""
    return n * rank // world, n * (rank + 1) // world


def distributed_split(dist, local_prefix: np.ndarray, b0: int, n: int, world: int,
                      backend: str = "nccl") -> np.ndarray:
    """Balanced split of ONE global word list without any rank holding its whole prefix.

    Rank r has computed the exclusive byte prefix of its equal-count block [b0, b1)
    (``local_prefix``, b1 - b0 + 1 entries, from the keyspace pass).  One all-gather of
    the block totals gives every block's global base; every rank then searches its own
    block for each target and one all-reduce(MIN) of the W + 1 candidates yields the
    split.  The result equals ``a5x_partition`` (engine.partition) over the global
    prefix: split[r] = first word whose global start offset >= total * r // W."""
    lp = np.asarray(local_prefix, dtype=np.uint64)
    totals = allgather_u64(dist, [int(lp[-1])], backend)[:, 0]
    base = int(totals[:dist_rank(dist)].sum()) if world > 1 else 0
    total = int(totals.sum())
    cand = np.full(world + 1, n, dtype=np.uint64)
    cand[0] = 0
    for r in range(1, world):
        t = total * r // world - base  # target relative to this block's base
        if t <= int(lp[-1]):
            # first local index with prefix >= t (index len-1 = the block's end = next block's start)
            i = int(np.searchsorted(lp, np.uint64(max(t, 0)), side="left"))
            cand[r] = b0 + i
    return allreduce_min_u64(dist, cand, backend)


INF_U63 = (1 << 63) - 1


def candidate_split(dist, block_cands: int, block_bytes: int, b0: int, n: int, world: int, split_fn,
                    backend: str = "nccl") -> np.ndarray:
    """Balanced split of ONE global candidate stream at CANDIDATE granularity (SURVEY 8(e)
    e1: split points are (word, intra-word index)): the reference serialises a word on one
    goroutine (main.go:77-93), so a word larger than a rank's share would cap a word-only
    split; here such a word is cut inside.

    Rank r holds the keyspace of its equal-count block [b0, b1) (``block_cands`` /
    ``block_bytes`` totals).  One all-gather of the block totals gives the global bases;
    the owner of byte target t_r = total * r // W (the block whose bytes hold it) finds the
    first candidate starting at or after t_r with ``split_fn(local_targets) -> (g, w, c, b)``
    (block-local candidate, word, candidate in word, first byte: ``Context.split_device`` +
    ``locate_device`` on the GPU) and one all-reduce(MIN) shares the answers.

    Returns a (4, W + 1) u64 array: global candidate g_r, global word w_r, candidate in that
    word c_r and global byte b_r of every split; rank r's shard is candidates [g_r, g_r+1),
    i.e. words w_r .. w_r+1 (the last one only when c_r+1 > 0) from candidate c_r of w_r."""
    tot = allgather_u64(dist, [block_cands, block_bytes], backend)  # (world, 2)
    rank = dist_rank(dist)
    cbase, bbase = int(tot[:rank, 0].sum()), int(tot[:rank, 1].sum())
    T, TB = int(tot[:, 0].sum()), int(tot[:, 1].sum())
    out = np.full((4, world + 1), INF_U63, dtype=np.uint64)
    out[:, 0] = 0
    out[:, world] = (T, n, 0, TB)
    mine = [r for r in range(1, world) if TB and bbase <= TB * r // world < bbase + block_bytes]
    if mine:
        g, w, c, b = split_fn(np.array([TB * r // world - bbase for r in mine], dtype=np.uint64))
        for k, r in enumerate(mine):
            out[:, r] = (cbase + int(g[k]), b0 + int(w[k]), int(c[k]), bbase + int(b[k]))
    if not TB:  # no output at all: every split at the end
        out[:, 1:world] = np.array([[T], [n], [0], [TB]], dtype=np.uint64)
    return allreduce_min_u64(dist, out.reshape(-1), backend).reshape(4, world + 1)


def shard_of(split: np.ndarray, rank: int):
    """Rank's shard from ``candidate_split``: (first word, end word (exclusive), candidate
    in the first word where the shard starts, candidates, first global byte, bytes)."""
    g0, g1 = int(split[0, rank]), int(split[0, rank + 1])
    w0, c0 = int(split[1, rank]), int(split[2, rank])
    w1 = int(split[1, rank + 1]) + (1 if int(split[2, rank + 1]) > 0 else 0)
    return w0, max(w1, w0), c0, g1 - g0, int(split[3, rank]), int(split[3, rank + 1]) - int(split[3, rank])


def dist_rank(dist) -> int:
    return dist.get_rank() if dist is not None and dist.is_initialized() else 0


def shard_words(data: np.ndarray, offs: np.ndarray, w0: int, w1: int) -> Tuple[np.ndarray, np.ndarray]:
    """The packed sub-batch of words [w0, w1) (bytes re-based to 0, 16-byte pad kept)."""
    b0, b1 = int(offs[w0]), int(offs[w1])
    sub = np.zeros(b1 - b0 + 16, dtype=np.uint8)
    sub[: b1 - b0] = data[b0:b1]
    return sub, (offs[w0:w1 + 1] - offs[w0]).astype(np.uint64)


def init_from_env(backend: Optional[str] = None):
    """torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).

    backend: "nccl" (RCCL over xGMI on ROCm) for GPU ranks, "gloo" for CPU tests;
    default from A5X_DIST_BACKEND or nccl.  Returns (dist, rank, world, local_rank)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = backend or os.environ.get("A5X_DIST_BACKEND", "nccl")
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return dist, rank, world, local


def allreduce_u64(dist, values, backend: str = "nccl") -> np.ndarray:
    """Sum a small vector of u64 counters across ranks (exact: split into 32-bit halves)."""
    import torch
    v = np.asarray(values, dtype=np.uint64)
    halves = np.stack([v & np.uint64(0xFFFFFFFF), v >> np.uint64(32)]).astype(np.int64)
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.from_numpy(halves).to(dev)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    h = t.cpu().numpy().astype(np.uint64)
    return (h[0] + (h[1] << np.uint64(32))).astype(np.uint64)


def _world(dist) -> int:
    return dist.get_world_size() if dist is not None and dist.is_initialized() else 1


def _to_halves(v: np.ndarray) -> np.ndarray:
    return np.stack([v & np.uint64(0xFFFFFFFF), v >> np.uint64(32)]).astype(np.int64)


def _from_halves(h: np.ndarray) -> np.ndarray:
    h = h.astype(np.uint64)
    return (h[..., 0, :] + (h[..., 1, :] << np.uint64(32))).astype(np.uint64)


def allgather_u64(dist, values, backend: str = "nccl") -> np.ndarray:
    """(world, k) array of every rank's k u64 values (exact: 32-bit halves)."""
    import torch
    v = np.asarray(values, dtype=np.uint64)
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.from_numpy(_to_halves(v)).to(dev)
    world = _world(dist)
    if world == 1:
        return v.reshape(1, -1)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return np.stack([_from_halves(o.cpu().numpy()) for o in outs])


def allreduce_min_u64(dist, values, backend: str = "nccl") -> np.ndarray:
    """Element-wise MIN of u64 vectors across ranks (values < 2^63)."""
    import torch
    v = np.asarray(values, dtype=np.uint64)
    if _world(dist) == 1:
        return v.copy()
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.from_numpy(v.astype(np.int64)).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return t.cpu().numpy().astype(np.uint64)


def gather_rows_u64(dist, rows, backend: str = "nccl", dst: int = 0):
    """Concatenation, in rank order, of every rank's (n_r, k) u64 rows, on rank ``dst``
    (other ranks get None): one all-gather of the row counts, then one all-gather of
    the rows padded to the largest count (exact: 32-bit halves).  The hit gather of
    north_star (e): each rank's hit records (global word, candidate, digest) -> rank 0."""
    import torch
    r = np.asarray(rows, dtype=np.uint64)
    k = r.shape[1] if r.ndim == 2 else 0
    world = _world(dist)
    if world == 1:
        return r.reshape(-1, k)
    counts = allgather_u64(dist, [r.shape[0]], backend)[:, 0].astype(np.int64)
    m = int(counts.max())
    pad = np.zeros((max(m, 1), k), dtype=np.uint64)
    pad[: r.shape[0]] = r
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.from_numpy(_to_halves(pad.reshape(-1))).to(dev)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    if dist.get_rank() != dst:
        return None
    parts = [_from_halves(o.cpu().numpy()).reshape(-1, k)[: int(c)] for o, c in zip(outs, counts)]
    return np.concatenate(parts) if parts else np.zeros((0, k), dtype=np.uint64)


def hits_to_rows(hits, word_base: int = 0) -> np.ndarray:
    """[(word, cand, digest16)] -> (n, 4) u64 rows {word + word_base, cand, digest lo, digest hi}."""
    out = np.zeros((len(hits), 4), dtype=np.uint64)
    for i, (w, c, d) in enumerate(hits):
        out[i, 0] = w + word_base
        out[i, 1] = c
        out[i, 2] = int.from_bytes(d[:8], "little")
        out[i, 3] = int.from_bytes(d[8:], "little")
    return out


def rows_to_hits(rows):
    """Inverse of hits_to_rows: [(word, cand, digest16)]."""
    return [(int(r[0]), int(r[1]), int(r[2]).to_bytes(8, "little") + int(r[3]).to_bytes(8, "little")) for r in rows]
