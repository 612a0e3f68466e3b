"""bench.py's queue leg alone (the coalescing queue, config-4 proofs, one proof per call): closed loop
and open-loop Poisson arrivals, library-measured latency.  Run it against the A/B build with
NHIP_QUEUE_SLOTS to compare slot counts.  Usage: python tools/queue_probe.py [callers]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "neptune-core_amd"), ROOT, os.path.join(ROOT, "oracle")]
os.environ["GPU_MAX_HW_QUEUES"] = "22"  # the bench's budget (the boxes export 4)
import bench  # noqa: E402

callers = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pool4 = bench.load_pool4()
import stark_ref as S  # noqa: E402  (AIR descriptor construction only)
air_words = np.asarray(S.bloat_air(S.AirCircuit.from_words([int(w) for w in pool4["air"]]), 24000).to_words(),
                       dtype=np.uint64)
claims, proofs, expect, _, _, _ = bench.make_config4(pool4, 4096, 0.01, 1, 0)
dcl, dpr = bench.device_form(claims, proofs, True)
import neptune_hip as nh  # noqa: E402
import neptune_hip.stark as NS  # noqa: E402
with nh.Context(0) as ctx:
    gair = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default().montgomery()
    q = bench.queue_leg(ctx, gair, stark, dcl, dpr, expect, callers)
out = {"slots": os.environ.get("NHIP_QUEUE_SLOTS", "default"), "closed": round(q["value"]),
       "closed_latency_ms": q["latency_ms"], "proofs_per_batch": round(q["proofs_per_batch"], 1),
       "per_batch_ms": q["per_batch_ms"], "correct": q["verdicts_correct"],
       "open": [(o["offered"], round(o["achieved"]), o["latency_ms"], round(o["proofs_per_batch"], 1))
                for o in q["open_loop"]]}
print(json.dumps(out), flush=True)
