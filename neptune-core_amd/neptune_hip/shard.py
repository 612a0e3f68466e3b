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


def on_rank0(fn, dist, key: str = "nhip_rank0_leg", timeout_s: float = 900.0):
    """Run ``fn()`` on rank 0 alone (e.g. one process driving every GPU of the node through
    nhip_group_stream) while the other ranks wait on the HOST, at the rendezvous store, not in a
    collective whose kernel would spin on the GPUs rank 0 drives.  Returns fn's result on rank 0 and
    None elsewhere; rank 0 releases the others even if fn raises (the exception then propagates on
    rank 0).  Without ``dist`` it is just ``fn()``."""
    if dist is None:
        return fn()
    from datetime import timedelta
    store = dist.distributed_c10d._get_default_store()
    if dist.get_rank() != 0:
        store.wait([key], timedelta(seconds=timeout_s))
        return None
    try:
        return fn()
    finally:
        store.set(key, "1")


def agreed_max(vals, dist, fast=None):
    """All-reduce(MAX) of the float list `vals` that every rank completes the same way.

    `fast(vals)` (e.g. one RCCL all-reduce over xGMI on a group made for it, its result synchronized
    to the host INSIDE the call, so a device-side fault raises there) is tried first; then one host
    all-reduce(MIN) of a per-rank success flag on the default (gloo) group decides for every rank
    at once: all succeeded -> the fast result; any failed -> every rank reduces on the host group.
    So a fault on one rank can never leave the ranks issuing different collectives.  Returns
    (values, fast_used, this rank's error or None)."""
    import torch
    res, err = None, None
    if fast is not None:
        try:
            res = [float(x) for x in fast(list(vals))]
        except Exception as e:  # noqa: BLE001 - any fault of the fast path falls back, on every rank
            res, err = None, f"{type(e).__name__}: {e}"[:300]
    flag = torch.tensor([1 if res is not None else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 1:
        return res, True, None
    t = torch.tensor([float(x) for x in vals], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()], False, err


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


class VerdictExchange:
    """The per-step verdict exchange of a sharded batch as ONE collective, posted without waiting.

    Every rank all-gathers ``[local_ok, verdict bytes of its shard (padded to the widest shard)]``;
    the batch verdict is the MIN of the leading bytes (what ``all_ok``'s all-reduce(MIN) gives) and
    the job's verdict vector is scattered from the rest (what ``gather_verdicts`` gives), so one
    collective replaces the pair.  ``post`` enqueues the exchange on a ring of ``depth``
    preallocated buffers and returns at once; ``complete`` returns the oldest posted exchange's
    ``(batch_ok, verdicts)``.  A caller keeps at most ``depth`` exchanges posted (bench.py: post step
    k, complete step k - depth + 1), so a slow collective never stalls the launch of the next GPU
    step.

    RCCL ("nccl") form: the verdict bytes go through pinned host buffers; post enqueues the copy in,
    the all_gather_into_tensor, the stream's wait for it and the copy out on torch's current stream
    and records an event, all without blocking the host; complete waits on that event only.  (Round
    5: the blocking pageable copies of the first form cost a 512-proof rank ~5% of its rate, the
    host stalling on each step's exchange instead of relaunching the GPU's next step.)
    """

    def __init__(self, shards: List[List[int]], n: int, dist, depth: int = 2):
        import torch
        self.dist = dist
        self.n = n
        self.depth = max(2, int(depth))
        self.dev = _device_for(dist)
        self.world = dist.get_world_size()
        self.width = 1 + (max(len(s) for s in shards) if shards else 0)
        self.index = [np.asarray(s, dtype=np.int64) for s in shards]
        # gloo has no all_gather_into_tensor: per-rank views of the flat receive buffer instead
        self.flat = self.dev.type == "cuda"
        self.send = [torch.zeros(self.width, dtype=torch.uint8, device=self.dev) for _ in range(self.depth)]
        self.recv = [torch.zeros(self.world * self.width, dtype=torch.uint8, device=self.dev)
                     for _ in range(self.depth)]
        if self.flat:
            self.send_host = [torch.zeros(self.width, dtype=torch.uint8).pin_memory() for _ in range(self.depth)]
            self.recv_host = [torch.zeros(self.world * self.width, dtype=torch.uint8).pin_memory()
                              for _ in range(self.depth)]
            self.done = [torch.cuda.Event() for _ in range(self.depth)]
        self.pending: List[tuple] = []
        self.slot = 0

    def post(self, local_ok: bool, local: np.ndarray) -> None:
        import torch
        if len(self.pending) >= self.depth:
            raise RuntimeError(f"VerdictExchange: complete() the oldest exchange before posting a {self.depth + 1}th")
        s = self.slot
        self.slot = (s + 1) % self.depth
        host = self.send_host[s].numpy() if self.flat else np.zeros(self.width, dtype=np.uint8)
        host[:] = 0
        host[0] = 1 if local_ok else 0
        host[1:1 + len(local)] = np.asarray(local, dtype=np.uint8)
        if self.flat:
            self.send[s].copy_(self.send_host[s], non_blocking=True)
            work = self.dist.all_gather_into_tensor(self.recv[s], self.send[s], async_op=True)
            work.wait()  # the current stream waits for the collective; the host does not
            self.recv_host[s].copy_(self.recv[s], non_blocking=True)
            self.done[s].record()
            self.pending.append((s, None))
        else:
            self.send[s].copy_(torch.from_numpy(host))
            work = self.dist.all_gather(list(self.recv[s].view(self.world, self.width)), self.send[s], async_op=True)
            self.pending.append((s, work))

    def complete(self):
        s, work = self.pending.pop(0)
        if self.flat:
            self.done[s].synchronize()
            got = self.recv_host[s].numpy().reshape(self.world, self.width).copy()
        else:
            work.wait()
            got = self.recv[s].view(self.world, self.width).numpy().copy()
        full = np.zeros(self.n, dtype=np.uint8)
        for r, idx in enumerate(self.index):
            if len(idx):
                full[idx] = got[r, 1:1 + len(idx)]
        return bool(got[:, 0].min()), full


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
