"""Stark parameters other than Stark::default() through the same C ABI: Stark::new(security_level,
log2_of_fri_expansion_factor) sets the FRI expansion factor and num_collinearity_checks =
security_level / log2 expansion (triton-vm's Stark::new; oracle/stark_ref.py StarkParams).  Covered:
(160, 1) -> 160 checks at expansion 2 (the 256-thread Merkle plan, one DEEP chunk per row),
(160, 3) -> 53 checks at expansion 8, (256, 1) -> 256 checks (MAX_CHECKS, a full plan workgroup).
Per parameter set: the synthetic prover's accepting proof verifies with every Fiat-Shamir sample
and FRI index equal to the oracle's, and mutations (a revealed row, an authentication digest, a FRI
response leaf, the claim's input) give the C oracle's verdicts."""
import numpy as np
import pytest

import stark_prover as SP
import stark_ref as S

pytestmark = pytest.mark.gpu

PARAMS = [(160, 1), (160, 3), (256, 1)]


def _oracle_samples(params, air, claim, proof):
    tr = {}
    ok = S.verify(params, air, claim, proof, tr)
    samples = [tuple(x) for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals]
    indices = [v for tag, vals in tr["sponge_samples"] if tag == "fri_indices" for v in vals]
    return ok, samples, indices


def _item_spans(proof, params):
    """(kind, first payload word, end) of every proof item of a well-formed stream."""
    spans, at = [], 2
    for _ in range(int(proof[1])):
        ln = int(proof[at])
        spans.append((int(proof[at + 1]), at + 2, at + 1 + ln))
        at += 1 + ln
    return spans


@pytest.mark.parametrize("sec,log2_exp", PARAMS)
def test_non_default_stark_params(ctx, sec, log2_exp):
    import coracle as C
    import neptune_hip.stark as NS
    params = S.StarkParams(security_level=sec, log2_fri_expansion=log2_exp)
    k = params.num_collinearity_checks
    air, recipe = S.synth_air(params, seed=1)
    claim = ([3, 1, 4, 1, 5], 0, [9, 2, 6], [5, 3])
    proof, _ = SP.prove(params, air, recipe, claim, 4, seed=sec + log2_exp)
    proof = [int(w) for w in proof]
    ok_o, samples, indices = _oracle_samples(params, air, claim, proof)
    assert ok_o
    spans = _item_spans(proof, params)
    kinds = [kd for kd, _, _ in spans]
    muts = []
    for kind in (S.MAIN_ROWS, S.AUTH_STRUCTURE, S.FRI_RESPONSE):
        _, lo, hi = spans[kinds.index(kind)]
        m = list(proof)
        pos = (lo + hi) // 2
        m[pos] = (m[pos] + 1) % S.P
        muts.append((claim, m))
    bad_claim = (claim[0], claim[1], claim[2] + [7], claim[3])
    cases = [(claim, proof)] + muts + [(bad_claim, proof)]
    stark = NS.Stark(sec, log2_exp, k, params.num_main, params.num_aux, params.num_quotient_segments)
    gair = NS.Air(air.to_words())
    b = NS.Batch(ctx, gair, stark, [NS.Claim(*c) for c, _ in cases], [p for _, p in cases])
    v, _ = b.run()
    xs, idx, fail = b.transcript(0)
    assert fail == 0 and xs == samples and idx == indices and len(idx) == k
    want = C.stark_verify_batch(air.to_words(), params, [c for c, _ in cases], [p for _, p in cases], threads=8)
    assert [bool(x) for x in v] == [bool(x) for x in want]
    assert list(v) == [1, 0, 0, 0, 0]
    b.close()
