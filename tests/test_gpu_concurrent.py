"""One context driven from many host threads at once, as neptune-core drives `triton_vm::verify`
(concurrent tokio tasks, verifier.rs:60-63, peer_loop.rs:1342): 12 threads each call
nhip_verify_batch on their own small batches (accepting and mutated proofs, malformed streams,
claim tampering) while 2 threads run device-resident batches (nhip_batch_launch / wait) and 2 hash
with Tip5 on the same context.  Every result equals the same call made alone, and the expected
verdicts."""
import os
import threading

import numpy as np
import pytest

import stark_ref as S
import tip5_ref as T

pytestmark = pytest.mark.gpu


def _pool():
    import json
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_pool.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    out = []
    for h in meta["heights"]:
        c = meta["claims"][str(h)]
        out.append(((c["digest"], c["version"], c["input"], c["output"]), z[f"proof_{h}"], meta["main_rows"][str(h)]))
    return z["air"], out


def _batch(pool, seed):
    rng = np.random.default_rng(seed)
    pairs, expect = [], []
    for claim, proof, (lo, hi) in pool:
        kind = int(rng.integers(0, 4))
        p, c, ok = proof, claim, True
        if kind == 1:  # a revealed row word
            p = proof.copy()
            pos = int(rng.integers(lo, hi))
            p[pos] = np.uint64((int(p[pos]) + 1) % S.P)
            ok = False
        elif kind == 2:  # a truncated stream
            p = proof[: int(rng.integers(1, proof.size))]
            ok = False
        elif kind == 3:  # the claim's output changed
            c = (claim[0], claim[1], claim[2], list(claim[3]) + [int(rng.integers(1, 1 << 30))])
            ok = False
        pairs.append((c, p))
        expect.append(ok)
    return pairs, expect


def test_one_context_many_threads(ctx):
    import neptune_hip.stark as NS
    air_w, pool = _pool()
    air = NS.Air([int(w) for w in air_w])
    stark = NS.Stark.default()
    jobs = [_batch(pool, 100 + t) for t in range(12)]
    alone = [NS.verify_batch(ctx, air, stark, [(NS.Claim(*c), p) for c, p in pairs]) for pairs, _ in jobs]
    for (pairs, expect), got in zip(jobs, alone):
        assert got == expect
    resident = NS.Batch(ctx, air, stark, [NS.Claim(*c) for c, _, _ in pool], [p for _, p, _ in pool])
    want_res, _ = resident.run()
    rng = np.random.default_rng(7)
    rows = [[int(x) for x in rng.integers(0, T.P, size=int(n), dtype=np.uint64)] for n in rng.integers(1, 40, size=64)]
    want_hash = ctx.hash_varlen(rows=rows)
    errors, results = [], {}

    def verifier(t):
        try:
            pairs, _ = jobs[t]
            for rep in range(3):
                got = NS.verify_batch(ctx, air, stark, [(NS.Claim(*c), p) for c, p in pairs])
                results[(t, rep)] = got == alone[t]
        except Exception as exc:  # noqa: BLE001 - reported below
            errors.append(repr(exc))

    def resident_runner(t):
        try:
            b = NS.Batch(ctx, air, stark, [NS.Claim(*c) for c, _, _ in pool], [p for _, p, _ in pool])
            for rep in range(4):
                b.launch()
                v, _ = b.wait()
                results[("res", t, rep)] = list(v) == list(want_res)
            b.close()
        except Exception as exc:  # noqa: BLE001
            errors.append(repr(exc))

    def hasher(t):
        try:
            for rep in range(6):
                out = ctx.hash_varlen(rows=rows)
                results[("hash", t, rep)] = bool((np.asarray(out) == np.asarray(want_hash)).all())
        except Exception as exc:  # noqa: BLE001
            errors.append(repr(exc))

    threads = [threading.Thread(target=verifier, args=(t,)) for t in range(12)]
    threads += [threading.Thread(target=resident_runner, args=(t,)) for t in range(2)]
    threads += [threading.Thread(target=hasher, args=(t,)) for t in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    resident.close()
    assert not errors, errors
    assert len(results) == 12 * 3 + 2 * 4 + 2 * 6
    assert all(results.values()), [k for k, v in results.items() if not v]
