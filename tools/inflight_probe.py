"""Where the time of many small batches in flight goes (config 5's N = 8 share: 8 height-23 proofs
per batch, R in flight, one stream per batch): host time inside launch / wait / stats against the
wall time.  Usage: python tools/inflight_probe.py [proofs] [inflight] [steps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "neptune-core_amd"), ROOT]
import bench  # noqa: E402
import neptune_hip as nh  # noqa: E402
import neptune_hip.stark as NS  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
R = int(sys.argv[2]) if len(sys.argv) > 2 else 20
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 400
air_kind = sys.argv[4] if len(sys.argv) > 4 else "synthetic"  # or triton-size (bench.py's default AIR)
mont = len(sys.argv) > 5 and sys.argv[5] == "montgomery"
z = np.load(os.path.join(ROOT, "tests", "golden", "deep_fri.npz"))
meta = json.loads(bytes(z["meta"]).decode())["cases"]["23"]
claim = NS.Claim(meta["digest"], meta["version"], meta["input"], meta["output"])
proof = z["proof_23"]
air_words, _ = bench.load_pool()
if air_kind == "triton-size":
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import stark_ref as S  # AIR descriptor construction only
    air_words = S.bloat_air(S.AirCircuit.from_words([int(w) for w in air_words]), 24000).to_words()
if mont:
    claim = NS.montgomery_claim(claim)
    proof = NS.to_montgomery(proof)
with nh.Context(0) as ctx:
    gair = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default().montgomery() if mont else NS.Stark.default()
    ring = [NS.Batch(ctx, gair, stark, [claim] * n, [np.array(proof, copy=True) for _ in range(n)]).set_streams(
        1 if n <= 64 else 2) for _ in range(R)]
    for rep in range(2):
        tl = tw = 0.0
        dev = 0.0
        phase = {}
        q, launched = [], 0
        ctx.synchronize()
        t0 = time.perf_counter()
        for i in range(min(R, steps)):
            a = time.perf_counter(); ring[i].launch(); tl += time.perf_counter() - a
            q.append(i); launched += 1
        while q:
            i = q.pop(0)
            a = time.perf_counter(); v, ok = ring[i].wait(); tw += time.perf_counter() - a
            stt = ring[i].stats()
            dev += stt["ms_device_total"]
            for kk, vv in stt.items():
                if kk.startswith("ms_") and isinstance(vv, float):
                    phase[kk] = phase.get(kk, 0.0) + vv
            if launched < steps:
                a = time.perf_counter(); ring[i].launch(); tl += time.perf_counter() - a
                q.append(i); launched += 1
        wall = time.perf_counter() - t0
        print(json.dumps({"air": air_kind, "mont": mont, "proofs": n, "inflight": R, "steps": steps, "proofs_per_s": n * steps / wall,
                          "wall_ms_per_step": wall / steps * 1e3, "launch_ms_per_step": tl / steps * 1e3,
                          "wait_ms_per_step": tw / steps * 1e3,
                          "other_host_ms_per_step": (wall - tl - tw) / steps * 1e3,
                          "device_latency_ms_per_step": dev / steps,
                          "phase_ms_per_batch": {kk: round(vv / steps, 4) for kk, vv in phase.items()}}), flush=True)
    for b in ring:
        b.close()
