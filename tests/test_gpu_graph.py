"""Resident batches replayed from a captured HIP graph (nhip_batch_set_graph): every verdict and every
Fiat-Shamir sample equal the direct launch's (and so the oracle's, which the other GPU tests hold the
direct launch to), through refills with other proofs, a change to one stream, launch timing on and
off, and 8 batches in flight relaunched 40 times; a replayed launch reports no phase split, a timed
one does.  Reference semantics per proof: triton_vm::verify at verifier.rs:60-63."""
import numpy as np
import pytest

import bench
import stark_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pool():
    air_words, pool = bench.load_pool()
    hs = sorted(pool)
    claims = [pool[h]["claim"] for h in hs]
    proofs = [np.asarray(pool[h]["proof"], dtype=np.uint64) for h in hs]
    bad = proofs[2].copy()
    lo, hi = pool[hs[2]]["main_rows"]
    bad[(lo + hi) // 2] = np.uint64((int(bad[(lo + hi) // 2]) + 1) % S.P)
    return [int(w) for w in air_words], claims + [claims[2]], proofs + [bad]


def _all(b, n):
    v, ok = b.run()
    return [bool(x) for x in v], ok, [b.transcript(i) for i in range(n)]


def test_graph_replay_equals_direct_launch(ctx, pool):
    import neptune_hip.stark as NS
    air_words, claims, proofs = pool
    gair = NS.Air(air_words)
    st = NS.Stark.default()
    cl = [NS.Claim(*c) for c in claims]
    direct = NS.Batch(ctx, gair, st, cl, proofs)
    want = _all(direct, len(proofs))
    assert want[0] == [True] * 5 + [False] and want[1] is False
    assert direct.stats()["ms_device_total"] > 0
    g = NS.Batch(ctx, gair, st, cl, proofs).set_graph(True)
    for _ in range(3):
        assert _all(g, len(proofs)) == want
        assert g.stats()["ms_device_total"] == 0.0  # replayed: no phase split
    g.set_launch_timing(True)
    assert _all(g, len(proofs)) == want and g.stats()["ms_device_total"] > 0  # timed: direct
    g.set_launch_timing(False)
    assert _all(g, len(proofs)) == want
    # refilled with other proofs: captured again at the next launch
    rc, rp = cl[::-1], proofs[::-1]
    direct.refill(rc, rp)
    want_r = _all(direct, len(rp))
    g.refill(rc, rp)
    for _ in range(2):
        assert _all(g, len(rp)) == want_r
    g.set_streams(1)
    direct.set_streams(1)
    assert _all(g, len(rp)) == _all(direct, len(rp)) == want_r
    g.set_graph(False)
    assert _all(g, len(rp)) == want_r and g.stats()["ms_device_total"] > 0
    direct.close()
    g.close()


def test_graph_batches_in_flight(ctx, pool):
    import neptune_hip.stark as NS
    air_words, claims, proofs = pool
    gair = NS.Air(air_words)
    st = NS.Stark.default()
    cl = [NS.Claim(*c) for c in claims]
    want = [True] * 5 + [False]
    ring = [NS.Batch(ctx, gair, st, cl, proofs).set_graph(True) for _ in range(8)]
    dt, ok = bench.pipelined(ring, 40, 8, np.array(want))
    assert ok
    for b in ring:
        b.close()
    with pytest.raises(Exception):
        big = NS.Batch(ctx, gair, st, cl * 180, proofs * 180)  # 1,080 proofs: past the graph cap
        try:
            big.set_graph(True)
        finally:
            big.close()
