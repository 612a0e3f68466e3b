"""Batch launches replayed from a captured HIP graph: prepare (captured there), runs, refill, runs,
one stream, runs, launch timing on / off; verdicts, transcripts and phase stats at every step."""
import json
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "neptune-core_amd"), ROOT, os.path.join(ROOT, "oracle")]
import bench  # noqa: E402
import neptune_hip as nh  # noqa: E402
import neptune_hip.stark as NS  # noqa: E402

air_words, pool = bench.load_pool()
hs = sorted(pool)
claims = [NS.Claim(*pool[h]["claim"]) for h in hs]
proofs = [pool[h]["proof"] for h in hs]
with nh.Context(0) as ctx:
    gair = NS.Air([int(w) for w in air_words])
    st = NS.Stark.default()
    b = NS.Batch(ctx, gair, st, claims, proofs)
    v0, _ = b.run()  # direct: the phase split
    print("direct", b.stats()["ms_device_total"], flush=True)
    b.set_graph(True)
    steps = [("run", None)] * 3 + [("refill", None)] + [("run", None)] * 3 + [("streams1", None)] + \
        [("run", None)] * 2 + [("timing", True)] + [("run", None)] + [("timing", False)] + [("run", None)] * 2
    ref = None
    for i, (what, arg) in enumerate(steps):
        try:
            if what == "run":
                v, ok = b.run()
                s = b.stats()
                xs, idx, fail = b.transcript(0)
                key = (list(map(bool, v)), len(xs), idx[:4])
                ref = ref or key
                print(i, "run", key == ref, ok, round(s["ms_device_total"], 3), round(s["ms_fiat_shamir"], 3), flush=True)
            elif what == "refill":
                b.refill(claims[::-1], proofs[::-1])
                ref = None
                print(i, "refill ok", flush=True)
            elif what == "streams1":
                b.set_streams(1)
                print(i, "streams1 ok", flush=True)
            elif what == "timing":
                b.set_launch_timing(arg)
                print(i, "timing", arg, flush=True)
        except Exception:
            print(i, what, "FAILED", traceback.format_exc().splitlines()[-1], flush=True)
            raise
    b.close()
    # a group stream slot: prepare, then refills
    with NS.Group([0, 0]) as g, NS.GroupStream(g, gair, st) as gs:
        for k in range(4):
            try:
                r = gs.submit(list(zip(claims, proofs)))
                print("group submit", k, None if r is None else all(r[0]), flush=True)
            except Exception:
                print("group submit", k, "FAILED", traceback.format_exc().splitlines()[-1], flush=True)
                raise
        print("group finish", gs.finish()[1], flush=True)
