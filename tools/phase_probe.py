"""Phase split of small config-5 batches (height-23 proofs, tests/golden/deep_fri.npz), run one at a
time after warm-up runs: where a lone small batch's device time goes.  Usage:
python tools/phase_probe.py [proofs ...]   (NHIP_LIB selects a library variant)"""
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

sizes = [int(x) for x in sys.argv[1:]] or [8, 64]
z = np.load(os.path.join(ROOT, "tests", "golden", "deep_fri.npz"))
meta = json.loads(bytes(z["meta"]).decode())["cases"]["23"]
claim = NS.Claim(meta["digest"], meta["version"], meta["input"], meta["output"])
proof = z["proof_23"]
air_words, _ = bench.load_pool()
with nh.Context(0) as ctx:
    gair = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default()
    for n in sizes:
        b = NS.Batch(ctx, gair, stark, [claim] * n, [np.array(proof, copy=True) for _ in range(n)])
        b.set_streams(1 if n <= 64 else 2)
        rows = []
        for r in range(8):
            t = time.perf_counter()
            v, ok = b.run()
            wall = (time.perf_counter() - t) * 1e3
            st = b.stats()
            rows.append({k[3:]: round(st[k], 3) for k in ("ms_device_decode", "ms_fiat_shamir", "ms_row_hash",
                                                          "ms_merkle", "ms_ood_air", "ms_fri", "ms_deep",
                                                          "ms_device_total")})
            rows[-1]["wall"] = round(wall, 3)
            assert ok
        b.close()
        for r, x in enumerate(rows):
            print(n, r, x, flush=True)
