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
