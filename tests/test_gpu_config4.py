"""BASELINE config 4, the north-star workload: 4,096 transaction proofs with log2
padded heights drawn from the ProofCollection member mix (seed 0xC4), drawn from 256 distinct
accepting proofs (oracle/pool4.py: distinct claims and seeds, each with its oracle transcript), 1%
corrupted, verified
(1) in one nhip_verify_batch call, (2) through nhip_group_verify_batch with 2 and 3 member
contexts (the in-process multi-GPU path, LPT-sharded; here all members share GPU 0), and (3) as
a device-resident batch whose Fiat-Shamir transcripts are compared with the oracle's for every
accepting proof of the batch (each of the 256 distinct proofs at 16 batch positions).  Every verdict equals the expected one (reference: proof_collection.rs:342-388,
block_program.rs:51-65; the per-proof verdicts are what block validation gathers)."""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu
TOTAL = 4096


@pytest.fixture(scope="module")
def c4():
    pool4 = bench.load_pool4()
    assert len(pool4["proofs"]) == 256 and len({tuple(c[0]) for c in pool4["claims"]}) == 256
    claims, proofs, expect, srcs, shards, expect_all = bench.make_config4(pool4, TOTAL, 0.01, 1, 0)
    assert len(proofs) == TOTAL and (~expect).sum() == round(0.01 * TOTAL)
    assert (expect == expect_all[shards[0]]).all()
    assert len(set(srcs)) == 256
    return pool4["air"], pool4, claims, proofs, expect, srcs


def test_config4_one_call(ctx, c4):
    import neptune_hip.stark as NS
    air_words, _, claims, proofs, expect, _ = c4
    gair = NS.Air([int(w) for w in air_words])
    got = NS.verify_batch(ctx, gair, NS.Stark.default(), [(NS.Claim(*c), p) for c, p in zip(claims, proofs)])
    assert got == [bool(x) for x in expect]


@pytest.mark.parametrize("members", [2, 3])
def test_config4_group(c4, members):
    import neptune_hip.stark as NS
    air_words, _, claims, proofs, expect, _ = c4
    gair = NS.Air([int(w) for w in air_words])
    with NS.Group([0] * members) as g:
        assert len(g) == members
        got, ok = NS.verify_batch_group(g, gair, NS.Stark.default(),
                                        [(NS.Claim(*c), p) for c, p in zip(claims, proofs)])
    assert got == [bool(x) for x in expect] and ok is False
    # the split the group used is balanced by proof length (LPT)
    member_of = np.array(NS.group_shard(proofs, members))
    lens = np.array([len(p) for p in proofs], dtype=np.float64)
    loads = [lens[member_of == m].sum() for m in range(members)]
    assert max(loads) / min(loads) < 1.01


def test_config4_transcripts_vs_oracle(ctx, c4):
    """Every accepting proof's transcript against its pool entry's oracle transcript: 256 distinct
    transcripts, each at ~16 batch positions (offsets, claim staging and scratch slots differ)."""
    import neptune_hip.stark as NS
    air_words, pool4, claims, proofs, expect, srcs = c4
    gair = NS.Air([int(w) for w in air_words])
    b = NS.Batch(ctx, gair, NS.Stark.default(), [NS.Claim(*c) for c in claims], proofs)
    v, ok = b.run()
    assert [bool(x) for x in v] == [bool(x) for x in expect] and not ok
    checked = set()
    for i in np.flatnonzero(expect):
        xs, idx, fail = b.transcript(int(i))
        want_xs, want_idx = pool4["transcripts"][srcs[i]]
        assert fail == 0 and xs == want_xs and idx == want_idx, (int(i), srcs[i])
        checked.add(srcs[i])
    assert len(checked) == 256
    for i in np.flatnonzero(~expect)[:8]:
        assert b.transcript(int(i))[2] != 0
    b.close()


def test_config4_shuffled_order(ctx, c4):
    """The batch in a random order (the heights mixed, as a node's batch arrives): the library
    verifies it in shape-grouped device order (stark_host.cpp batch_prepare) and maps every verdict
    and transcript back to the caller's index."""
    import neptune_hip.stark as NS
    air_words, pool4, claims, proofs, expect, srcs = c4
    order = np.random.default_rng(0x5F).permutation(len(proofs))
    gair = NS.Air([int(w) for w in air_words])
    b = NS.Batch(ctx, gair, NS.Stark.default(), [NS.Claim(*claims[i]) for i in order], [proofs[i] for i in order])
    v, ok = b.run()
    assert [bool(x) for x in v] == [bool(expect[i]) for i in order] and not ok
    for pos in range(0, len(order), 37):
        i = int(order[pos])
        xs, idx, fail = b.transcript(pos)
        if expect[i]:
            want_xs, want_idx = pool4["transcripts"][srcs[i]]
            assert fail == 0 and xs == want_xs and idx == want_idx, (pos, i)
        else:
            assert fail != 0, (pos, i)
    b.close()
    got = NS.verify_batch(ctx, gair, NS.Stark.default(), [(NS.Claim(*claims[i]), proofs[i]) for i in order])
    assert got == [bool(expect[i]) for i in order]
