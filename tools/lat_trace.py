#!/usr/bin/env python3
"""Resident-batch runs of N proofs (default 1: a block's SingleProof-sized call) repeated REPS
times, for a rocprofv3 kernel trace of the small-batch latency path.
Usage: python tools/lat_trace.py [n_proofs=1] [reps=20]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
import bench  # noqa: E402
import neptune_hip as nh  # noqa: E402
import neptune_hip.stark as NS  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    air_words, pool = bench.load_pool()
    ctx = nh.Context(0)
    air = NS.Air([int(w) for w in air_words])
    if n == 1:
        e = pool[16]
        claims, proofs = [e["claim"]], [e["proof"]]
    else:
        claims, proofs, _ = bench.make_batch(pool, max(1, n // 8), 0.0, 1)
    b = NS.Batch(ctx, air, NS.Stark.default(), [NS.Claim(*c) for c in claims], proofs)
    ts = []
    for r in range(reps + 3):
        t = time.perf_counter()
        v, ok = b.run()
        if r >= 3:
            ts.append((time.perf_counter() - t) * 1e3)
        assert ok
    st = b.stats()
    b.close()
    print({"proofs": len(proofs), "run_ms_median": round(float(np.median(ts)), 3),
           "device_ms": round(st["ms_device_total"], 3), "fs_ms": round(st["ms_fiat_shamir"], 3), "merkle_ms": round(st["ms_merkle"], 3)}, flush=True)


if __name__ == "__main__":
    main()
