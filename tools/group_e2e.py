#!/usr/bin/env python3
"""End-to-end rate of one-shot verify calls from host memory (decode + upload + device + verdicts):
nhip_verify_batch on one context vs nhip_group_verify_batch on groups of K contexts on device 0
(several members on one GPU overlap one member's host decode / upload with another's device run).
Marshaling is done once up front (a Rust caller hands the C ABI its buffers directly).
Usage: python tools/group_e2e.py [calls=6] [collections per call=256] [members=1,2,4]"""
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
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    coll = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    members = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4").split(",")]
    air_words, pool = bench.load_pool()
    air = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default()
    params = stark.c()
    claims, proofs, expect = bench.make_batch(pool, coll, 0.05, 0xE5)
    m = NS._Marshal([NS.Claim(*c) for c in claims], proofs)
    n = m.n
    out = {"proofs_per_call": n, "calls": calls}
    for k in members:
        v = np.zeros(n, dtype=np.uint8)
        ok = ctypes.c_uint8(0)
        if k == 1:
            ctx = nh.Context(0)
            call = lambda: _lib.check(ctx.lib.nhip_verify_batch(ctx.handle, air.handle, ctypes.byref(params), m.claims,
                                                               m.proofs, n, v, None), "nhip_verify_batch")
            closer = ctx
        else:
            g = NS.Group([0] * k)
            call = lambda: _lib.check(g.lib.nhip_group_verify_batch(g.handle, air.handle, ctypes.byref(params),
                                                                   m.claims, m.proofs, n, v, ctypes.byref(ok)),
                                      "nhip_group_verify_batch")
            closer = g
        call()  # warm: scratch sized, streams created, AIR uploaded
        t = time.perf_counter()
        for _ in range(calls):
            call()
        dt = time.perf_counter() - t
        assert (v.astype(bool) == np.asarray(expect)).all(), "verdicts differ"
        out[f"members_{k}"] = {"ms_per_call": dt / calls * 1e3, "proofs_per_s": n * calls / dt}
        closer.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
