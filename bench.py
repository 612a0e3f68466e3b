#!/usr/bin/env python3
"""bench.py — BASELINE.json config 2 on MI355X: synthetic 2^20 Tip5 Merkle authentication
paths of depth 20 per GPU, verified with MTree::verify semantics
(neptune-core/src/protocol/consensus/block/pow.rs:162-180) by the hand-written HIP kernel
behind include/neptune_hip.h.

One step = one batch pass of the hot path: verify every resident path
(nhip_mtree_verify_dev), reduce the per-path verdicts to the batch verdict on the device
(nhip_verdicts_all_dev) and, for N > 1, AND the batch verdicts of all ranks with one RCCL
all-reduce(MIN) over xGMI (the path's only exchange step).  Paths are
sharded by rank (weak scaling: every rank owns its own 2^20-path batch).

Inputs are resident in HBM before the timed region.  The rank-0/N=1 CPU baseline is the C
restatement (oracle/tip5_oracle.c) on the host cores, timed on a bounded sample of the same
workload (the reference `triton_vm`/twenty-first Rust code cannot be built here: no Rust
toolchain, crates not vendored — SURVEY.md §8c).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))

P = (1 << 64) - (1 << 32) + 1
# Algorithmic VALU work of one Tip5 permutation in 32-bit VALU lane-ops: a fixed analytic count of
# a minimal implementation: per round S-box 64 + x^7 672 + MDS 512+160 + ARK 96.
TIP5_VALU_OPS_PER_PERM = 5 * 1504
# gfx950: 256 CUs x 4 SIMD x 32 lanes x 2.4 GHz (wave64 VALU issues over 2 cycles on SIMD-32)
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9
# algorithmic HBM bytes per path: leaf (40) + index (8) + depth siblings (40 each) + verdict (1)
def path_bytes(depth: int) -> int:
    return 40 + 8 + 40 * depth + 1


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the latest committed rocprofv3 PMC passes
    (profiles/LATEST -> profiles/<tag>/pmc_{fetch,write}_counter_collection.csv), raw
    (FETCH_SIZE + WRITE_SIZE) x 1024; None when absent."""
    import csv
    try:
        tag = open(os.path.join(ROOT, "profiles", "LATEST")).read().strip()
        tot = 0.0
        for part, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
            vals = [float(r["Counter_Value"]) for r in
                    csv.DictReader(open(os.path.join(ROOT, "profiles", tag, f"pmc_{part}_counter_collection.csv")))
                    if kernel in r["Kernel_Name"] and r["Counter_Name"] == ctr]
            tot += sum(vals) / len(vals) * 1024
        return tot, tag
    except (OSError, ZeroDivisionError, KeyError):
        return None, None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_batch(rng, log2_leaves: int, ctx, corrupt_frac: float):
    """Synthetic tree on the device, paths gathered on the host, all uploaded once."""
    n = 1 << log2_leaves
    depth = log2_leaves
    leafs = rng.integers(0, P, size=(n, 5), dtype=np.uint64)
    d_leafs = ctx.upload(leafs)
    d_nodes = ctx.alloc(n * 40)
    ctx.mtree_build_dev(d_leafs, n, d_nodes)
    nodes = d_nodes.download(np.uint64, (n, 5))
    idx = rng.permutation(n).astype(np.int64)  # paths in random leaf order
    paths = np.empty((n, depth, 5), dtype=np.uint64)
    paths[:, 0] = leafs[idx ^ 1]
    running = idx + n
    for k in range(1, depth):
        running >>= 1
        paths[:, k] = nodes[running ^ 1]
    elements = leafs[idx].copy()
    expect = np.ones(n, dtype=np.uint8)
    n_bad = int(n * corrupt_frac)
    if n_bad:
        bad = rng.choice(n, size=n_bad, replace=False)
        elements[bad, 0] = (elements[bad, 0] + np.uint64(1)) % np.uint64(P)
        expect[bad] = 0
    batch = {
        "n": n, "depth": depth, "root": nodes[1].copy(), "idx": idx.astype(np.uint64),
        "elements": elements, "paths": paths, "expect": expect,
        "d_root": ctx.upload(nodes[1]), "d_idx": ctx.upload(idx.astype(np.uint64)),
        "d_el": ctx.upload(elements), "d_paths": ctx.upload(paths), "d_v": ctx.alloc(n),
    }
    d_leafs.free()
    d_nodes.free()
    return batch


def cpu_baseline(batch, target_s: float, threads: int):
    """C restatement on the host cores over a bounded sample of the same paths."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle as C  # oracle: CPU baseline leg only
    depth = batch["depth"]
    # calibrate on a small slice, then size the sample for ~target_s seconds
    m = 2048
    t = time.perf_counter()
    C.mtree_verify_batch(batch["root"], batch["idx"][:m], batch["elements"][:m], batch["paths"][:m].reshape(-1),
                         depth, nthreads=threads)
    dt = time.perf_counter() - t
    m = int(min(batch["n"], max(m, m * target_s / max(dt, 1e-6))))
    t = time.perf_counter()
    v = C.mtree_verify_batch(batch["root"], batch["idx"][:m], batch["elements"][:m],
                             batch["paths"][:m].reshape(-1), depth, nthreads=threads)
    dt = time.perf_counter() - t
    assert (v == batch["expect"][:m]).all(), "CPU baseline verdicts disagree with the expected verdicts"
    return {"value": m * depth / dt, "unit": "Tip5 perms/s", "cores": threads, "kind": "port",
            "sample": f"{m} of the {batch['n']} depth-{depth} paths of this batch ({m * depth} permutations), "
                      f"C restatement oracle/tip5_oracle.c, {threads} POSIX threads, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log2-leaves", type=int, default=20)
    ap.add_argument("--corrupt-frac", type=float, default=0.01)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    import neptune_hip as nh

    ctx = nh.Context(local_rank)
    rng = np.random.default_rng(0xC2 + rank)
    t0 = time.time()
    batch = make_batch(rng, args.log2_leaves, ctx, args.corrupt_frac)
    n, depth = batch["n"], batch["depth"]
    log(f"[rank {rank}] batch ready: {n} paths, depth {depth}, {time.time() - t0:.1f}s")

    from neptune_hip import shard

    def step(timed: bool):
        if timed:
            ctx.timing(True)
        ctx.mtree_verify_dev(batch["d_root"], 1, batch["d_idx"], batch["d_el"], batch["d_paths"], depth, n,
                             batch["d_v"])
        if timed:
            ctx.timing(False)
        ok = ctx.verdicts_all_dev(batch["d_v"], n)
        if dist is not None:
            ok = shard.all_ok(ok, dist)  # the one exchange: RCCL all-reduce(MIN) of the batch verdict
        return ok

    def barrier_sync():
        ctx.synchronize()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        step(False)
    ctx.timing_read(reset=True)
    barrier_sync()
    t_start = time.perf_counter()
    batch_ok = None
    for _ in range(args.steps):
        batch_ok = step(True)
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    kern_ms, launches = ctx.timing_read(reset=True)

    # correctness of the measured work: per-path verdicts equal the expected ones
    v = batch["d_v"].download(np.uint8, (n,))
    correct = bool((v == batch["expect"]).all())
    if dist is not None:
        import torch
        t = torch.tensor([elapsed, 0.0 if correct else 1.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, any_bad = float(t[0].item()), float(t[1].item())
        correct = any_bad == 0.0
    if not correct:
        log("ERROR: verdicts differ from expected")
    perms_per_step = world * n * depth
    value = perms_per_step * args.steps / elapsed
    kern_avg_s = kern_ms / max(launches, 1) / 1e3
    achieved = n * depth * TIP5_VALU_OPS_PER_PERM / kern_avg_s
    traffic, traffic_tag = pmc_traffic("k_mtree_verify")
    res = {
        "metric": "Tip5 permutations/s verifying synthetic Merkle authentication paths (BASELINE config 2)",
        "value": value,
        "unit": "Tip5 perms/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64 (Goldilocks mod p)",
        "data": "synthetic (seeded uniform canonical leaves, one 2^20-leaf tree per rank, 1% corrupted leaves)",
        "config": {"workload": f"BASELINE config 2: 2^{args.log2_leaves} Tip5 Merkle auth paths of depth {depth} per GPU "
                               "(MTree::verify, pow.rs:162-180) + batch verdict AND (+ RCCL MIN all-reduce for N>1)",
                   "paths_per_gpu": n, "depth": depth, "parallelism": f"path-sharded x{world}"},
        "paths_per_s": world * n * args.steps / elapsed,
        "verdicts_correct": correct,
        "batch_verdict": batch_ok,
        "roofline": {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_LANE_OPS / 1e12,
                     "unit": "T VALU lane-ops/s", "frac": achieved / VALU_PEAK_LANE_OPS, "traffic": traffic,
                     "traffic_unit": "bytes per launch (FETCH_SIZE+WRITE_SIZE, raw; see DESIGN.md §3)",
                     "traffic_profile": traffic_tag,
                     "kernel": "k_mtree_verify", "kernel_avg_ms": kern_avg_s * 1e3,
                     "valu_ops_per_perm": TIP5_VALU_OPS_PER_PERM,
                     "hbm_algorithmic_GBps": n * path_bytes(depth) / kern_avg_s / 1e9},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(batch, args.cpu_seconds, args.cpu_threads)
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0 if correct else 1


if __name__ == "__main__":
    sys.exit(main())
