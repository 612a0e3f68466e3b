"""The streaming group (nhip_group_stream_*): batch after batch over every member, each member's
share of batch k staged and uploaded while its share of batch k - 1 runs, as bootstrap import
(state/mod.rs:2226-2272) and block batches (peer_loop.rs:315-323) verify one batch after another.
Here the members are several contexts on GPU 0.  Every batch's verdicts arrive one submit later (the
last at finish), in the caller's order, equal to the expected ones, in both input forms; empty
batches, a batch smaller than the member count, a single-member group stream, and eight members
(the driver's node: eight member threads, each with its share of the node's CPUs for its copy
threads) too."""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def batches():
    pool4 = bench.load_pool4()
    claims, proofs, expect, _, _, _ = bench.make_config4(pool4, 1024, 0.02, 1, 0)
    # 4 batches of 256 in a shuffled order (heights mixed), then 3 proofs, an empty batch, 7 proofs
    order = np.random.default_rng(0xB5).permutation(len(proofs))
    cut = [(0, 256), (256, 512), (512, 768), (768, 1024), (0, 3), (0, 0), (100, 107)]
    out = []
    for lo, hi in cut:
        idx = order[lo:hi]
        out.append(([claims[i] for i in idx], [proofs[i] for i in idx], expect[idx]))
    return pool4["air"], out


@pytest.mark.parametrize("members,mont", [(2, False), (3, True), (1, True), (8, True)])
def test_group_stream_verdicts(batches, members, mont):
    import neptune_hip.stark as NS
    air_words, bs = batches
    air = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default().montgomery() if mont else NS.Stark.default()
    got = []
    with NS.Group([0] * members) as g, NS.GroupStream(g, air, stark) as st:
        for claims, proofs, _ in bs:
            cl = [NS.Claim(*c) for c in claims]
            if mont:
                cl = [NS.montgomery_claim(c) for c in cl]
                proofs = [NS.to_montgomery(p) for p in proofs]
            r = st.submit(list(zip(cl, proofs)))
            if r is not None:
                got.append(r)
        got.append(st.finish())
        stats = st.stats()
    assert len(got) == len(bs)
    for (v, ok), (_, _, expect) in zip(got, bs):
        assert v == [bool(x) for x in expect]
        assert ok == bool(expect.all())
    assert stats["proofs"] == sum(len(b[1]) for b in bs) and stats["ms_device"] > 0


@pytest.mark.parametrize("sizes", [(64,), (3, 7, 300), (1, 256)])
def test_group_stream_growing_last_share(batches, sizes):
    """One submit then finish, and batches that grow so the last share is larger than every share
    before it: each member's verdict buffer is sized to the share it reads back (the round-4 advisor
    finding: the buffer was sized to the previous share, and finish wrote past it)."""
    import neptune_hip.stark as NS
    air_words, bs = batches
    air = NS.Air([int(w) for w in air_words])
    stark = NS.Stark.default()
    pool_c = [c for b in bs[:4] for c in b[0]]
    pool_p = [p for b in bs[:4] for p in b[1]]
    pool_e = np.concatenate([b[2] for b in bs[:4]])
    got, want, at = [], [], 0
    with NS.Group([0, 0]) as g, NS.GroupStream(g, air, stark) as st:
        for n in sizes:
            cl = [NS.Claim(*c) for c in pool_c[at:at + n]]
            r = st.submit(list(zip(cl, pool_p[at:at + n])))
            want.append(pool_e[at:at + n])
            at += n
            if r is not None:
                got.append(r)
        got.append(st.finish())
    assert len(got) == len(sizes)
    for (v, ok), expect in zip(got, want):
        assert v == [bool(x) for x in expect]
        assert ok == bool(expect.all())
