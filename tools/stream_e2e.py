#!/usr/bin/env python3
"""End-to-end rate from host memory with two alternating batches (nhip_batch_refill): each
refill (host decode + one upload) overlaps the other batch's device run.  Marshaling is done
once up front (a Rust caller hands the C ABI its buffers directly).
Usage: python tools/stream_e2e.py [batches=12] [collections per batch=256]"""
import ctypes
import json
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
from neptune_hip import _lib  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    coll = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    air_words, pool = bench.load_pool()
    ctx = nh.Context(0)
    air = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default()
    params = stark.c()
    data = [bench.make_batch(pool, coll, 0.05, 0xE0 + i) for i in range(2)]
    ms = [NS._Marshal([NS.Claim(*c) for c in d[0]], d[1]) for d in data]
    batches = [NS.Batch(ctx, air, stark, [NS.Claim(*c) for c in d[0]], d[1]) for d in data]
    lib = ctx.lib

    def refill(b, m):
        _lib.check(lib.nhip_batch_refill(ctx.handle, b.handle, air.handle, ctypes.byref(params), m.claims, m.proofs,
                                         m.n), "nhip_batch_refill")

    for b in batches:  # warm: device memory sized, streams created
        b.run()
    n = ms[0].n
    ctx.synchronize()
    t = time.perf_counter()
    cur, nxt = 0, 1
    refill(batches[cur], ms[0])
    batches[cur].launch()
    ok = True
    for i in range(1, nb):
        refill(batches[nxt], ms[i % 2])
        v, _ = batches[cur].wait()
        ok = ok and bool((v.astype(bool) == data[(i - 1) % 2][2]).all())
        batches[nxt].launch()
        cur, nxt = nxt, cur
    v, _ = batches[cur].wait()
    ok = ok and bool((v.astype(bool) == data[(nb - 1) % 2][2]).all())
    dt = time.perf_counter() - t
    st = batches[0].stats()
    res = {"batches": nb, "proofs_per_batch": n, "seconds": dt, "proofs_per_s": nb * n / dt,
           "decode_ms": st["ms_decode"], "upload_ms": st["ms_upload"], "device_ms": st["ms_device_total"],
           "verdicts_correct": ok}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
