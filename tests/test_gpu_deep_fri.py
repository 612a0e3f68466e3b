"""Deep FRI with non-zero values on the GPU: accepting proofs at log2 padded
heights 17, 20 and 23 (tests/golden/deep_fri.npz, the sparse synthetic prover: non-zero codewords
in every one of the 11 / 14 / 16 folding rounds, a non-empty last polynomial, distinct main rows),
so k_fri's round-indexed domain points and k_deep at those heights are checked with values that a
wrong point, round or weight would change (the constant-codeword proofs of config 5 fold zeros).

Each proof's verdict and Fiat-Shamir transcript (every squeezed sample, the FRI indices) equal the
oracle's (stored with the fixture), and mutants of every late FRI round's response, of the last
codeword and of the last polynomial get the C oracle's verdict (reference: triton_vm::verify at
verifier.rs:60-63)."""
import json
import os

import numpy as np
import pytest

import coracle as C
import stark_ref as S

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "golden", "deep_fri.npz")
POOL = os.path.join(os.path.dirname(__file__), "golden", "c3_pool.npz")


@pytest.fixture(scope="module")
def deep():
    z = np.load(FIX)
    meta = json.loads(bytes(z["meta"]).decode())
    air_words = [int(w) for w in np.load(POOL)["air"]]
    cases = []
    for h in meta["heights"]:
        m = meta["cases"][str(h)]
        claim = (m["digest"], m["version"], m["input"], m["output"])
        cases.append((h, claim, z[f"proof_{h}"], [tuple(int(c) for c in x) for x in z[f"samples_{h}"]],
                      [int(i) for i in z[f"indices_{h}"]], m["info"]))
    return air_words, cases


def _item_spans(proof, params):
    """(kind, first payload word, end) of every proof item, in stream order."""
    items = S.decode_proof([int(w) for w in proof], params)
    spans, pos = [], 2
    for k, _ in items:
        ln = int(proof[pos])
        spans.append((k, pos + 1, pos + 1 + ln))
        pos += 1 + ln
    return spans


def _mutants(proof, params, rng):
    spans = _item_spans(proof, params)
    fri = [s for s in spans if s[0] == S.FRI_RESPONSE]
    targets = [s for s in spans if s[0] in (S.FRI_CODEWORD, S.FRI_POLYNOMIAL)] + fri[-5:]
    out = []
    for _, lo, hi in targets:
        for pos in (hi - 1, lo + (hi - lo) // 2, int(rng.integers(lo + 1, hi))):
            m = np.array(proof, dtype=np.uint64)
            m[pos] = np.uint64((int(m[pos]) + 1) % S.P)
            out.append(m)
    return out


def test_deep_fri_verdicts_transcripts_and_mutants(ctx, deep):
    import neptune_hip.stark as NS
    air_words, cases = deep
    params = S.StarkParams()
    gair = NS.Air(air_words)
    stark = NS.Stark.default()
    rng = np.random.default_rng(0xDF)
    claims, proofs = [], []
    for h, claim, proof, _, _, info in cases:
        assert info["last_poly_degree"] > 0 and info["fri_rounds"] >= 11
        claims.append(claim)
        proofs.append(proof)
    n_good = len(proofs)
    for h, claim, proof, _, _, _ in cases:
        for m in _mutants(proof, params, rng):
            claims.append(claim)
            proofs.append(m)
    want = [bool(x) for x in C.stark_verify_batch(air_words, params, claims, proofs, threads=8)]
    assert want[:n_good] == [True] * n_good and not all(want[n_good:])
    b = NS.Batch(ctx, gair, stark, [NS.Claim(*c) for c in claims], proofs)
    v, ok = b.run()
    assert [bool(x) for x in v] == want
    for i, (h, _, _, samples, indices, _) in enumerate(cases):
        xs, idx, fail = b.transcript(i)
        assert fail == 0, h
        assert xs == samples, h
        assert idx == indices, h
    b.close()
