#!/usr/bin/env python3
"""Call latency of the drop-in entry point (`nhip_verify_batch` from host buffers: decode, upload,
device phases, verdict copy, free) for small batches: 1 proof (a block's SingleProof), 8 proofs
(one ProofCollection), 64 and 256 proofs; plus the device-resident run alone.  Reports the C-call
time (Python marshaling excluded) per batch size, median of repeated calls after a warmup.
Usage: python tools/latency.py [reps=20]"""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    air_words, pool = bench.load_pool()
    ctx = nh.Context(0)
    air = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default()
    out = {}
    for n_coll, label in ((None, "1 proof (h=16)"), (1, "8 proofs (1 collection)"), (8, "64 proofs"), (32, "256 proofs")):
        if n_coll is None:
            e = pool[16]
            claims, proofs = [e["claim"]], [e["proof"]]
        else:
            claims, proofs, _ = bench.make_batch(pool, n_coll, 0.0, 1)
        m = NS._Marshal([NS.Claim(*c) for c in claims], proofs)
        v = np.zeros(max(m.n, 1), dtype=np.uint8)
        params = stark.c()
        stats = _lib.Stats()
        ts = []
        for r in range(reps + 3):
            t = time.perf_counter()
            _lib.check(ctx.lib.nhip_verify_batch(ctx.handle, air.handle, ctypes.byref(params), m.claims, m.proofs, m.n,
                                                 v, ctypes.byref(stats)), "nhip_verify_batch")
            if r >= 3:
                ts.append((time.perf_counter() - t) * 1e3)
        assert v[:m.n].all()
        b = NS.Batch(ctx, air, stark, [NS.Claim(*c) for c in claims], proofs)
        rs = []
        for r in range(reps + 3):
            t = time.perf_counter()
            b.run()
            if r >= 3:
                rs.append((time.perf_counter() - t) * 1e3)
        b.close()
        out[label] = {"verify_batch_ms": round(float(np.median(ts)), 3), "resident_run_ms": round(float(np.median(rs)), 3),
                      "decode_ms": round(stats.ms_decode, 3), "upload_ms": round(stats.ms_upload, 3),
                      "device_ms": round(stats.ms_device_total, 3)}
        print(label, out[label], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
