"""The proof-stream decode on the device (k_decode, proof_codec.hpp): every batch run walks the raw
proof words in HBM.  Parity: its FAIL_DECODE bit equals the host walk (nhip_proof_decodes) and
the oracle's structural decode (stark_ref.structure_ok) on the mutation corpus of the CPU tests;
words given as u64 >= p decode and verify as BFieldElement::new would reduce them; a FRI
polynomial padded with zero coefficients is accepted (its degree is unchanged) and one with a
non-zero coefficient above the bound is rejected, as the oracle does."""
import json
import os

import numpy as np
import pytest

import stark_ref as S
import tip5_ref as T
from test_stark_host import _mutations

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "stark_tiny.json")
FAIL_DECODE = 1


def _ns():
    import neptune_hip.stark as NS
    return NS


@pytest.fixture(scope="module")
def tiny():
    g = json.load(open(GOLD))
    params = S.StarkParams(**g["params"])
    air, _ = S.synth_air(params, num_sampled=g["num_sampled"], seed=g["seed"])
    NS = _ns()
    return g, params, air, NS.Air([int(w) for w in g["air"]]), NS.Stark(num_collinearity_checks=8, num_main=24,
                                                                       num_aux=9)


def _claim_t(c):
    return (c["digest"], c["version"], c["input"], c["output"])


def test_device_decode_matches_host_and_oracle(ctx, tiny):
    NS = _ns()
    g, params, air, gair, stark = tiny
    claims, proofs = [], []
    for case in g["cases"]:
        claim = NS.Claim(*_claim_t(case["claim"]))
        proof = [int(w) for w in case["proof"]]
        for m in [proof] + _mutations(proof):
            claims.append(claim)
            proofs.append(m)
    assert len(proofs) > 300
    b = NS.Batch(ctx, gair, stark, claims, proofs)
    v, _ = b.run()
    for i, (c, p) in enumerate(zip(claims, proofs)):
        _, _, fail = b.transcript(i)
        host = NS.proof_decodes(gair, stark, c, p)
        assert (fail & FAIL_DECODE == 0) == host == S.structure_ok(params, p), i
        if not host:
            assert v[i] == 0
    b.close()


def test_non_canonical_words_reduce_mod_p(ctx, tiny):
    """Every word < 2^32 - 1 (all counts, lengths, discriminants, the padded height, small values)
    given as w + p, and every 7th word of the rest left alone: BFieldElement::new semantics, so the
    verdicts and Fiat-Shamir transcripts are the canonical proof's."""
    NS = _ns()
    g, params, air, gair, stark = tiny
    claims, proofs, canon = [], [], []
    for case in g["cases"]:
        proof = [int(w) for w in case["proof"]]
        lifted = [w + S.P if w < (1 << 64) - S.P else w for w in proof]
        assert sum(a != b for a, b in zip(lifted, proof)) > 20
        claims += [NS.Claim(*_claim_t(case["claim"]))] * 2
        proofs += [proof, lifted]
        canon.append(proof)
    b = NS.Batch(ctx, gair, stark, claims, proofs)
    v, ok = b.run()
    assert list(v) == [1] * len(proofs) and ok
    for i in range(0, len(proofs), 2):
        assert b.transcript(i) == b.transcript(i + 1)
    b.close()


def _item_spans(proof):
    """(start, end) of every item's words (discriminant .. end) in the proof encoding."""
    n = proof[1]
    pos, out = 2, []
    for _ in range(n):
        ln = proof[pos]
        out.append((pos + 1, pos + 1 + ln))
        pos += 1 + ln
    return out


def _with_poly(proof, coeffs):
    """The proof with its FriPolynomial item replaced by `coeffs` (XFE triples), raw encoding."""
    spans = _item_spans(proof)
    kinds = [proof[a] for a, _ in spans]
    a, e = spans[kinds.index(S.FRI_POLYNOMIAL)]
    body = [len(coeffs)] + [c for x in coeffs for c in x]
    item = [S.FRI_POLYNOMIAL, len(body)] + body
    enc = proof[1:a - 1] + [len(item)] + item + proof[e:]
    return [len(enc)] + enc


def test_fri_polynomial_padding_and_degree(ctx, tiny):
    NS = _ns()
    g, params, air, gair, stark = tiny
    case = g["cases"][2]
    claim_t = _claim_t(case["claim"])
    proof = [int(w) for w in case["proof"]]
    items = S.decode_proof(proof, params)
    poly = next(p for k, p in items if k == S.FRI_POLYNOMIAL)
    padded = _with_poly(proof, list(poly) + [(0, 0, 0)] * 200)
    zero_as_p = _with_poly(proof, list(poly) + [(S.P, 0, S.P)] * 3)  # non-canonical zeros
    high = _with_poly(proof, list(poly) + [(0, 0, 0)] * 150 + [(1, 0, 0)])
    cases = [proof, padded, zero_as_p, high]
    want = [S.verify(params, air, claim_t, p) for p in cases]
    assert want == [True, True, True, False]
    got = NS.verify_batch(ctx, gair, stark, [(NS.Claim(*claim_t), p) for p in cases])
    assert got == want
