"""Proof/path sharding across the GPUs of one node, and the single verdict exchange.

Units of work (proofs, authentication paths) are independent, so each rank verifies its own
shard with no data-path collective.  The only exchange is the verdict:
  * ``all_ok(local_ok)``        — RCCL/gloo all-reduce(MIN) of one byte: the block/batch verdict
                                   (the AND at neptune-core/src/protocol/consensus/transaction/
                                   validity/proof_collection.rs:388 and block validity 1.d,
                                   block/mod.rs:796-804).
  * ``gather_verdicts(...)``    — all-gather of per-unit verdict bytes (per-transaction results).
The reference verifies proofs strictly one after another (proof_collection.rs:342-385,
state/mod.rs:2226-2272); sharding is what the batch boundary adds.
"""
from __future__ import annotations

import heapq
from typing import List, Sequence

import numpy as np


def lpt_shard(costs: Sequence[float], world: int) -> List[List[int]]:
    """Greedy longest-processing-time assignment of units to ranks (deterministic: ties by
    index).  Returns, per rank, the sorted unit indices it owns."""
    if world < 1:
        raise ValueError("world >= 1")
    order = sorted(range(len(costs)), key=lambda i: (-float(costs[i]), i))
    heap = [(0.0, r) for r in range(world)]
    heapq.heapify(heap)
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + float(costs[i]), r))
    return [sorted(s) for s in out]


def contiguous_shard(n: int, world: int, rank: int) -> range:
    """Equal contiguous shard (uniform-cost units such as config-2 paths)."""
    per = (n + world - 1) // world
    return range(min(n, rank * per), min(n, (rank + 1) * per))


def _device_for(dist):
    import torch
    backend = dist.get_backend()
    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")


def all_ok(local_ok: bool, dist) -> bool:
    """Batch verdict across ranks: one all-reduce(MIN) of one byte."""
    import torch
    t = torch.tensor([1 if local_ok else 0], dtype=torch.uint8, device=_device_for(dist))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def gather_verdicts(local: np.ndarray, shards: List[List[int]], n: int, dist) -> np.ndarray:
    """All-gather per-unit verdict bytes; ``shards`` is the assignment every rank agrees on."""
    import torch
    dev = _device_for(dist)
    width = max(len(s) for s in shards) if shards else 0
    buf = torch.zeros(width, dtype=torch.uint8, device=dev)
    buf[: len(local)] = torch.from_numpy(np.ascontiguousarray(local, dtype=np.uint8)).to(dev)
    outs = [torch.zeros(width, dtype=torch.uint8, device=dev) for _ in shards]
    dist.all_gather(outs, buf)
    full = np.zeros(n, dtype=np.uint8)
    for r, s in enumerate(shards):
        if s:
            full[np.asarray(s, dtype=np.int64)] = outs[r][: len(s)].cpu().numpy()
    return full
