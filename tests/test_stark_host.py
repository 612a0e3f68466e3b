"""CPU tests of the STARK layer: the oracle against its golden fixture, the reference's reject
cases, and the library's host-side proof-stream decoder (no GPU) against the oracle's structural
decode on many malformed variants."""
import json
import os

import numpy as np
import pytest

import stark_ref as S
import tip5_ref as T

GOLD = os.path.join(os.path.dirname(__file__), "golden", "stark_tiny.json")


@pytest.fixture(scope="module")
def tiny():
    g = json.load(open(GOLD))
    params = S.StarkParams(**g["params"])
    return g, params


def _claim(c):
    return (c["digest"], c["version"], c["input"], c["output"])


def _air_obj(g, params):
    air, _ = S.synth_air(params, num_sampled=g["num_sampled"], seed=g["seed"])
    assert [str(w) for w in air.to_words()] == g["air"]
    return air


def test_oracle_accepts_golden_and_reproduces_transcript(tiny):
    g, params = tiny
    air = _air_obj(g, params)
    for case in g["cases"]:
        proof = [int(w) for w in case["proof"]]
        tr = {}
        assert S.verify(params, air, _claim(case["claim"]), proof, tr)
        samples = [[str(c) for c in x] for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals]
        assert samples == case["samples"]


def test_reference_reject_cases(tiny):
    """verifier.rs:95-118 (5-word bogus proof = hash_varlen(claim.encode())), neptune_proof.rs:118-133
    (empty proof, all zeros of length 65 as used at block/mod.rs:2059), mock encodings [0], [1]."""
    g, params = tiny
    air = _air_obj(g, params)
    claim = _claim(g["cases"][0]["claim"])
    bogus = T.hash_varlen(S.encode_claim(*claim))
    for proof in ([], bogus, [0] * 65, [0], [1]):
        assert S.verify(params, air, claim, proof) is False
        assert S.structure_ok(params, proof) is False


def _mutations(proof):
    n = len(proof)
    out = [proof[:-1], proof + [0], proof[:n // 2]]
    for pos in list(range(0, min(n, 40))) + list(range(40, n, max(1, n // 97))):
        for delta in (1, P_MINUS_1):
            m = list(proof)
            m[pos] = (m[pos] + delta) % S.P
            out.append(m)
    return out


P_MINUS_1 = S.P - 1


def test_host_decoder_matches_oracle_structure(tiny):
    import neptune_hip.stark as NS
    g, params = tiny
    air_w = [int(w) for w in g["air"]]
    air = NS.Air(air_w)
    info = air.info()
    assert info["constraints"] == oracle_constraints(g, params)
    stark = NS.Stark(num_collinearity_checks=8, num_main=24, num_aux=9)
    oracle_air = _air_obj(g, params)
    n_checked = 0
    for case in g["cases"]:
        c = case["claim"]
        claim = NS.Claim(c["digest"], c["version"], c["input"], c["output"])
        proof = [int(w) for w in case["proof"]]
        assert NS.proof_decodes(air, stark, claim, proof) is True
        for m in _mutations(proof):
            assert NS.proof_decodes(air, stark, claim, m) == S.structure_ok(params, m), len(m)
            n_checked += 1
    assert n_checked > 300
    bogus = T.hash_varlen(S.encode_claim(*_claim(g["cases"][0]["claim"])))
    for proof in ([], bogus, [0] * 65, [0], [1]):
        assert NS.proof_decodes(air, stark, NS.Claim([1, 2, 3, 4, 5]), proof) is False


def test_air_descriptor_validation():
    import neptune_hip.stark as NS
    from neptune_hip import NhipError
    params = S.StarkParams(num_main=24, num_aux=9, num_collinearity_checks=8)
    air, _ = S.synth_air(params, seed=7)
    w = air.to_words()
    NS.Air(w)
    bad = list(w)
    bad[0] = 0
    with pytest.raises(NhipError):
        NS.Air(bad)
    # the challenge layout is triton-air's: exactly Challenges::SAMPLE_COUNT = 59 sampled challenges
    for k in (16, 55, 58, 60):
        bad = list(w)
        bad[3] = k
        with pytest.raises(NhipError):
            NS.Air(bad)
    bad = list(w)
    # forward reference in an op node -> rejected
    first_op = next(i for i, nd in enumerate(air.nodes) if nd[0] in (S.OP_ADD, S.OP_SUB, S.OP_MUL))
    bad[9 + 4 * first_op + 1] = len(air.nodes) + 5
    with pytest.raises(NhipError):
        NS.Air(bad)
    with pytest.raises(NhipError):
        NS.Air(w[:-1])


def oracle_constraints(g, params):
    return _air_obj(g, params).num_constraints


def test_montgomery_word_helpers():
    """neptune_hip.stark.to_montgomery is twenty-first's in-memory form x * 2^64 mod p (any u64 read
    mod p) and from_montgomery its inverse."""
    import neptune_hip.stark as NS
    rng = np.random.default_rng(0x4D)
    xs = [0, 1, 2, S.P - 1, S.P, S.P + 1, (1 << 64) - 1, 1 << 32, (1 << 32) - 1] + \
        [int(v) for v in rng.integers(0, 1 << 63, size=200, dtype=np.uint64)] + \
        [int(v) | (1 << 63) for v in rng.integers(0, 1 << 63, size=200, dtype=np.uint64)]
    m = NS.to_montgomery(xs)
    for x, w in zip(xs, m):
        assert int(w) == (x % S.P) * (1 << 64) % S.P
    assert [int(v) for v in NS.from_montgomery(m)] == [x % S.P for x in xs]


def test_host_decoder_montgomery_form(tiny):
    """nhip_proof_decodes with input_form = Montgomery: every golden proof and every structural /
    payload mutant (given as the same field elements in Montgomery words) decodes exactly as in the
    canonical form; raw Montgomery words >= p (w + p, the same element) decode too."""
    import neptune_hip.stark as NS
    g, params = tiny
    air = NS.Air([int(w) for w in g["air"]])
    can = NS.Stark(num_collinearity_checks=8, num_main=24, num_aux=9)
    mont = can.montgomery()
    n = 0
    for case in g["cases"]:
        c = case["claim"]
        claim = NS.Claim(c["digest"], c["version"], c["input"], c["output"])
        mclaim = NS.montgomery_claim(claim)
        proof = [int(w) for w in case["proof"]]
        mp = [int(w) for w in NS.to_montgomery(proof)]
        assert NS.proof_decodes(air, mont, mclaim, mp) is True
        # the canonical words read as Montgomery words are other elements: the structure breaks
        assert NS.proof_decodes(air, mont, mclaim, proof) is False
        hi = [w + S.P if w < (1 << 64) - S.P else w for w in mp]
        assert NS.proof_decodes(air, mont, mclaim, hi) is True
        for m in _mutations(proof):
            mm = [int(w) for w in NS.to_montgomery(m)]
            assert NS.proof_decodes(air, mont, mclaim, mm) == NS.proof_decodes(air, can, claim, m)
            n += 1
    assert n > 300
    for proof in ([], [0] * 65, [0], [1]):
        assert NS.proof_decodes(air, mont, NS.Claim([1, 2, 3, 4, 5]), proof) is False
    bad = dataclasses_replace(can, input_form=2)
    with pytest.raises(Exception):
        NS.proof_decodes(air, bad, NS.Claim([1, 2, 3, 4, 5]), [])


def dataclasses_replace(obj, **kw):
    import dataclasses
    return dataclasses.replace(obj, **kw)
