#!/usr/bin/env python3
"""Quick GPU timing of the batched STARK verifier on synthetic full-size-parameter proofs
(oracle prover, small padded heights).  Usage: python tools/stark_perf.py [log2_ph ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("oracle", "neptune-core_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402

import stark_prover as SP  # noqa: E402
import stark_ref as S  # noqa: E402
import neptune_hip as nh  # noqa: E402
import neptune_hip.stark as NS  # noqa: E402

lphs = [int(a) for a in sys.argv[1:]] or [6, 8]
params = S.StarkParams()
air, recipe = S.synth_air(params, seed=1)
pool = []
for lph in lphs:
    for s in range(2):
        claim = ([s + 1, 2, 3, 4, lph], 0, [s] * 4, [lph])
        t = time.time()
        proof, _ = SP.prove(params, air, recipe, claim, lph, seed=1000 * lph + s)
        print(f"proved lph={lph} seed={s}: {len(proof)} words in {time.time() - t:.1f}s", flush=True)
        pool.append((claim, proof))
ctx = nh.Context(0)
gair = NS.Air(air.to_words())
print("air", gair.info())
stark = NS.Stark.default()
for n in (64, 512, 2048):
    sel = [pool[i % len(pool)] for i in range(n)]
    b = NS.Batch(ctx, gair, stark, [NS.Claim(*c) for c, _ in sel], [p for _, p in sel])
    v, ok = b.run()
    assert v.all(), "all proofs must verify"
    t = time.time()
    reps = 5
    for _ in range(reps):
        b.run()
    dt = (time.time() - t) / reps
    st = b.stats()
    print(f"n={n}: {dt * 1e3:.2f} ms/batch -> {n / dt:.0f} proofs/s; device phases (ms): "
          f"fs {st['ms_fiat_shamir']:.2f} rows {st['ms_row_hash']:.2f} merkle {st['ms_merkle']:.2f} "
          f"ood {st['ms_ood_air']:.2f} fri {st['ms_fri']:.2f} deep {st['ms_deep']:.2f} total {st['ms_device_total']:.2f}; "
          f"decode {st['ms_decode']:.1f} upload {st['ms_upload']:.1f}", flush=True)
    del b
