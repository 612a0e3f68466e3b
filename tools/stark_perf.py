#!/usr/bin/env python3
"""GPU timing of the batched STARK verifier on synthetic proofs with Stark::default()-shaped
parameters.  Usage: python tools/stark_perf.py [--heights 16,10,11,12,12,11,9,9] [--collections 256]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("oracle", "neptune-core_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402

import stark_prover_fast as F  # noqa: E402
import stark_ref as S  # noqa: E402
import neptune_hip as nh  # noqa: E402
import neptune_hip.stark as NS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--heights", default="16,10,11,12,12,11,9,9")
ap.add_argument("--collections", type=int, default=256)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
heights = [int(h) for h in a.heights.split(",")]
params = S.StarkParams()
air, recipe = S.synth_air(params, seed=1)
pool = {}
for lph in sorted(set(heights)):
    claim = ([lph, 2, 3, 4, 5], 0, [lph] * 5, [])
    t = time.time()
    proof, _ = F.prove(params, air, recipe, claim, lph, seed=lph)
    print(f"proved lph={lph}: {len(proof)} words in {time.time() - t:.1f}s", flush=True)
    pool[lph] = (claim, proof)
ctx = nh.Context(0)
gair = NS.Air(air.to_words())
stark = NS.Stark.default()
sel = [pool[h] for _ in range(a.collections) for h in heights]
n = len(sel)
t = time.time()
b = NS.Batch(ctx, gair, stark, [NS.Claim(*c) for c, _ in sel], [p for _, p in sel])
print(f"prepare {n} proofs: {time.time() - t:.2f}s", flush=True)
v, ok = b.run()
assert v.all(), "all proofs must verify"
times = []
for _ in range(a.reps):
    t = time.time()
    b.run()
    times.append(time.time() - t)
dt = min(times)
st = b.stats()
perms = st["tip5_perms_static"] + st["tip5_perms_merkle"]
print(f"n={n}: {dt * 1e3:.2f} ms/batch -> {n / dt:.0f} proofs/s; perms/proof {perms / n:.0f}, "
      f"{perms / dt:.3e} perms/s; device phases (ms): fs {st['ms_fiat_shamir']:.2f} rows {st['ms_row_hash']:.2f} "
      f"merkle {st['ms_merkle']:.2f} ood {st['ms_ood_air']:.2f} fri {st['ms_fri']:.2f} deep {st['ms_deep']:.2f} "
      f"total {st['ms_device_total']:.2f}; decode {st['ms_decode']:.1f} upload {st['ms_upload']:.1f}", flush=True)
