"""One proof alone (bench.py's config-1 substitute, resident): launch-to-verdict latency per launch shape
(streams, graph replay).  Usage: python tools/lone_probe.py [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "neptune-core_amd"), ROOT, os.path.join(ROOT, "oracle")]
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
pool4 = bench.load_pool4()
import stark_ref as S  # noqa: E402  (AIR descriptor construction only)
air_words = [int(w) for w in S.bloat_air(S.AirCircuit.from_words([int(w) for w in pool4["air"]]), 24000).to_words()]
claim, proof, samples, indices = bench.config1_case(air_words)
import neptune_hip as nh  # noqa: E402
import neptune_hip.stark as NS  # noqa: E402
dcl, dpr = bench.device_form([claim], [proof], True)
with nh.Context(0) as ctx:
    gair = NS.Air(air_words)
    stark = NS.Stark.default().montgomery()
    for streams, graph in ((2, False), (1, False), (1, True), (2, False)):
        b = NS.Batch(ctx, gair, stark, [NS.Claim(*dcl[0])], [dpr[0]]).set_streams(streams).set_graph(graph)
        for _ in range(10):
            v, _ = b.run()
        xs, idx, fail = b.transcript(0)
        ok = bool(v[0]) and fail == 0 and xs == samples and idx == indices
        ms = []
        for _ in range(reps):
            t = time.perf_counter()
            v, _ = b.run()
            ms.append((time.perf_counter() - t) * 1e3)
        b.close()
        print(json.dumps({"streams": streams, "graph": graph, "ok": ok, "median_ms": float(np.median(ms)),
                          "p10_ms": float(np.percentile(ms, 10)), "p90_ms": float(np.percentile(ms, 90))}), flush=True)
