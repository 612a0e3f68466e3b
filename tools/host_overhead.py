#!/usr/bin/env python3
"""Host time of one step's bookkeeping for small resident batches: nhip_batch_launch (enqueue of
every phase) and nhip_batch_stats, against the device step time.  Usage: python tools/host_overhead.py"""
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
    air_words, pool = bench.load_pool()
    ctx = nh.Context(0)
    air = NS.Air([int(w) for w in air_words])
    for n_coll in (1, 8, 64):
        claims, proofs, _ = bench.make_batch(pool, n_coll, 0.0, 1)
        b = NS.Batch(ctx, air, NS.Stark.default(), [NS.Claim(*c) for c in claims], proofs)
        tl, tw, ts = [], [], []
        for r in range(30):
            t0 = time.perf_counter()
            b.launch()
            t1 = time.perf_counter()
            b.wait()
            t2 = time.perf_counter()
            b.stats()
            t3 = time.perf_counter()
            if r >= 5:
                tl.append(t1 - t0)
                tw.append(t2 - t1)
                ts.append(t3 - t2)
        b.close()
        print(f"{len(proofs)} proofs: launch {np.median(tl) * 1e3:.3f} ms, wait {np.median(tw) * 1e3:.3f} ms, "
              f"stats {np.median(ts) * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
