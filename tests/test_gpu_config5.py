"""BASELINE config 5 at its full size: 64 proofs at log2 padded height 23 (FRI
domain 2^26, 17 FRI rounds, seeds 0xC5 + i from the constant-codeword synthetic prover), verified
(1) in one nhip_verify_batch call with 4 mutated copies beside them, (2) through
nhip_group_verify_batch with 2 member contexts (the in-process multi-GPU split; here both members
share GPU 0), and (3) as the two rank shards bench.py's config 5 uses at 2 ranks.  Every verdict
equals the expected one, and the Fiat-Shamir transcripts of 2 sampled proofs equal the oracle's
(reference: verifier.rs:60-63 per proof; the batch AND of block validation, block/mod.rs:796-804)."""
import numpy as np
import pytest

import bench
import stark_ref as S
import tip5_ref as T

pytestmark = pytest.mark.gpu
TOTAL = 64
LOG2_PH = 23


@pytest.fixture(scope="module")
def c5():
    air_words, _ = bench.load_pool()
    claims, proofs, expect, shards, _ = bench.make_config5(air_words, TOTAL, LOG2_PH, 1, 0)
    assert len(proofs) == TOTAL and expect.all() and shards == [list(range(TOTAL))]
    return air_words, claims, proofs


def _mutants(claims, proofs):
    out = []
    for i, frac in ((3, 0.2), (17, 0.5), (40, 0.8), (63, 0.999)):
        m = np.array(proofs[i], dtype=np.uint64)
        pos = int(len(m) * frac)
        m[pos] = np.uint64((int(m[pos]) + 1) % S.P)
        out.append((claims[i], m))
    return out


def test_config5_one_call_with_mutants(ctx, c5):
    import neptune_hip.stark as NS
    air_words, claims, proofs = c5
    gair = NS.Air([int(w) for w in air_words])
    bad = _mutants(claims, proofs)
    pairs = [(NS.Claim(*c), p) for c, p in zip(claims, proofs)] + [(NS.Claim(*c), p) for c, p in bad]
    got = NS.verify_batch(ctx, gair, NS.Stark.default(), pairs)
    assert got == [True] * TOTAL + [False] * len(bad)


def test_config5_group_of_two(c5):
    import neptune_hip.stark as NS
    air_words, claims, proofs = c5
    gair = NS.Air([int(w) for w in air_words])
    with NS.Group([0, 0]) as g:
        got, ok = NS.verify_batch_group(g, gair, NS.Stark.default(),
                                        [(NS.Claim(*c), p) for c, p in zip(claims, proofs)])
    assert got == [True] * TOTAL and ok is True
    member_of = NS.group_shard(proofs, 2)
    assert sorted(set(member_of)) == [0, 1]


def test_config5_rank_shards_and_transcripts(ctx, c5):
    import neptune_hip.stark as NS
    T.use_c_backend()
    air_words, claims, proofs = c5
    gair = NS.Air([int(w) for w in air_words])
    seen = []
    for rank in range(2):
        rc, rp, rexp, shards, expect_all = bench.make_config5(air_words, TOTAL, LOG2_PH, 2, rank)
        assert shards[rank] == list(range(rank * TOTAL // 2, (rank + 1) * TOTAL // 2)) and expect_all.all()
        # the shard's proofs are the full run's proofs for those indices
        for j, i in enumerate(shards[rank]):
            assert np.array_equal(np.asarray(rp[j]), np.asarray(proofs[i]))
        b = NS.Batch(ctx, gair, NS.Stark.default(), [NS.Claim(*c) for c in rc], rp)
        v, ok = b.run()
        assert [bool(x) for x in v] == [True] * len(rp) and ok
        if rank == 1:
            params = S.StarkParams()
            air = S.AirCircuit.from_words([int(w) for w in air_words])
            for j in (0, len(rp) - 1):
                tr = {}
                assert S.verify(params, air, rc[j], [int(w) for w in rp[j]], tr)
                want_xs = [tuple(x) for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals]
                want_idx = [x for tag, vals in tr["sponge_samples"] if tag == "fri_indices" for x in vals]
                xs, idx, fail = b.transcript(j)
                assert fail == 0 and xs == want_xs and idx == want_idx, j
        b.close()
        seen += shards[rank]
    assert seen == list(range(TOTAL))
