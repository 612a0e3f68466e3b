"""Several GPUs from one process (nhip_group_*): a batch sharded over the members verifies to
exactly the verdicts of one context's nhip_verify_batch (and of the expected mutations), in the
caller's order.  On a one-GPU box the group has several contexts on device 0, which exercises the
sharding, the concurrent member threads and the verdict merge."""
import os

import numpy as np
import pytest

import stark_ref as S

pytestmark = pytest.mark.gpu


def _pool():
    import json as _json
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_pool.npz"))
    meta = _json.loads(bytes(z["meta"]).decode())
    out = []
    for h in meta["heights"]:
        c = meta["claims"][str(h)]
        out.append(((c["digest"], c["version"], c["input"], c["output"]), z[f"proof_{h}"], meta["main_rows"][str(h)]))
    return z["air"], out


def _batch(seed, copies):
    """Pool proofs in a shuffled order, every third one with a flipped MainRows word."""
    air_w, pool = _pool()
    rng = np.random.default_rng(seed)
    pairs, expect = [], []
    for k in range(copies):
        for claim, proof, (lo, hi) in pool:
            p = proof.copy()
            bad = (len(pairs) % 3) == 2
            if bad:
                pos = int(rng.integers(lo, hi))
                p[pos] = np.uint64((int(p[pos]) + 1) % S.P)
            pairs.append((claim, p))
            expect.append(not bad)
    order = rng.permutation(len(pairs))
    return air_w, [pairs[i] for i in order], [expect[i] for i in order]


@pytest.mark.parametrize("members", [2, 3])
def test_group_matches_single_context(ctx, members):
    import neptune_hip.stark as NS
    air_w, pairs, expect = _batch(0x6A + members, 4)
    air = NS.Air([int(w) for w in air_w])
    stark = NS.Stark.default()
    claims = [(NS.Claim(*c), p) for c, p in pairs]
    single = NS.verify_batch(ctx, air, stark, claims)
    assert single == expect
    with NS.Group([ctx.device] * members) as g:
        assert len(g) == members
        v, ok = NS.verify_batch_group(g, air, stark, claims)
        assert v == single and ok is False
        # the accepting subset: all_ok true; repeated calls reuse the members' scratch
        good = [cp for cp, e in zip(claims, expect) if e]
        v2, ok2 = NS.verify_batch_group(g, air, stark, good)
        assert v2 == [True] * len(good) and ok2 is True
        # fewer proofs than members, and an empty batch
        v3, ok3 = NS.verify_batch_group(g, air, stark, claims[:1])
        assert v3 == single[:1] and ok3 == single[0]
        assert NS.verify_batch_group(g, air, stark, []) == ([], True)


def test_group_from_mask_covers_visible_devices():
    import torch
    import neptune_hip.stark as NS
    with NS.Group(mask=0) as g:
        assert len(g) == torch.cuda.device_count()


def test_verifier_mirror_over_a_group(ctx):
    """verifier.rs-shaped mirror (`Verifier.verify_batch`, one call per ProofCollection /
    mempool batch) backed by a group instead of one context: same verdicts."""
    import neptune_hip.stark as NS
    from neptune_hip.verifier import Verifier
    air_w, pairs, expect = _batch(0x77, 2)
    air = NS.Air([int(w) for w in air_w])
    claims = [(NS.Claim(*c), p) for c, p in pairs]
    with NS.Group([ctx.device, ctx.device]) as g:
        assert Verifier(g, air).verify_batch(claims) == expect == Verifier(ctx, air).verify_batch(claims)
