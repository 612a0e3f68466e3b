"""The N = 8 rank's 512-proof share of config 4 (bench.py's share_n8) in other launch shapes: streams per
batch, batches in flight, graph replay.  Usage: python tools/share_probe.py [steps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "neptune-core_amd"), ROOT, os.path.join(ROOT, "oracle")]
os.environ["GPU_MAX_HW_QUEUES"] = "22"  # the bench's budget (the boxes export 4)
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
pool4 = bench.load_pool4()
air_words = pool4["air"]
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import stark_ref as S  # noqa: E402  (AIR descriptor construction only)
air_words = np.asarray(S.bloat_air(S.AirCircuit.from_words([int(w) for w in air_words]), 24000).to_words(), dtype=np.uint64)
claims, proofs, expect, _, _, _ = bench.make_config4(pool4, 4096, 0.01, 8, 0)
dcl, dpr = bench.device_form(claims, proofs, True)
import neptune_hip as nh  # noqa: E402
import neptune_hip.stark as NS  # noqa: E402
with nh.Context(0) as ctx:
    gair = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default().montgomery()
    ncl = [NS.Claim(*c) for c in dcl]
    for streams, R, graph in ((2, 10, False), (1, 20, False), (1, 20, True), (2, 10, True), (1, 16, True), (2, 8, False)):
        ring = [NS.Batch(ctx, gair, stark, ncl, dpr).set_streams(streams).set_graph(graph) for _ in range(R)]
        bench.pipelined(ring, 5, R, expect)
        ctx.synchronize()
        rates = []
        for rep in range(2):
            dt, ok = bench.pipelined(ring, steps, R, expect)
            rates.append(len(dpr) * steps / dt)
            assert ok
        for b in ring:
            b.close()
        print(f"streams {streams} inflight {R} graph {graph}: {[round(r) for r in rates]} proofs/s ({steps} steps)", flush=True)
