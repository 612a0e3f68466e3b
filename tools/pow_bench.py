#!/usr/bin/env python3
"""PoW Tip5 throughput on one GPU: guesser-buffer preprocess (pow.rs:365-469, 7 x 2^h permutations)
at the given heights and batched guessing (pow.rs:471-507).  Prints one JSON line per height.
Usage: python tools/pow_bench.py [--heights 20,24,27,29] [--nonces 1048576]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "neptune-core_amd"))
import neptune_hip as nh  # noqa: E402
from neptune_hip.pow import Pow, PowMastPaths  # noqa: E402

P = (1 << 64) - (1 << 32) + 1
ap = argparse.ArgumentParser()
ap.add_argument("--heights", default="20,24,27,29")
ap.add_argument("--nonces", type=int, default=1 << 20)
a = ap.parse_args()
rng = np.random.default_rng(0x90)
d = lambda: tuple(int(x) for x in rng.integers(0, P, size=5, dtype=np.uint64))  # noqa: E731
mast = PowMastPaths([d(), d(), d()], [d(), d()], [d()])
prev = d()
ctx = nh.Context(0)
for h in [int(x) for x in a.heights.split(",")]:
    Pow.preprocess(ctx, min(h, 12), mast, False, prev).close()  # warm up
    t = time.perf_counter()
    buf = Pow.preprocess(ctx, h, mast, False, prev)
    dt = time.perf_counter() - t
    perms = 7 * (1 << h) - 1
    picker = buf.index_picker_preimage(mast)
    nonces = rng.integers(0, P, size=(a.nonces, 5), dtype=np.uint64)
    target = (P - 1,) * 4 + (1 << 40,)
    Pow.guess(ctx, buf, mast, picker, nonces[:1024], target)
    t = time.perf_counter()
    _, _, ok = Pow.guess(ctx, buf, mast, picker, nonces, target)
    dg = time.perf_counter() - t
    print(json.dumps({"workload": "pow preprocess (HardforkAlpha)", "merkle_tree_height": h,
                      "preprocess_s": dt, "preprocess_perms": perms, "perms_per_s": perms / dt,
                      "buffer_GB": 2 * (1 << h) * 40 / 1e9, "guess_nonces": a.nonces, "guess_s": dg,
                      "guesses_per_s": a.nonces / dg, "guess_perms_per_nonce": 63 + 10 + h,  # indices + fast_mast_hash (pow.rs:219-222)
                      "successes": int(ok.sum())}), flush=True)
    buf.close()
