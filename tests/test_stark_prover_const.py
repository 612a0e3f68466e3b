"""The constant-codeword synthetic prover (oracle/stark_prover_const.py) makes accepting proofs at
any padded height, including BASELINE config 5's 2^23, and single-word mutations of them reject
(Python and C restatements of the verifier agree).  CPU only."""
import numpy as np

import coracle as C
import stark_prover_const as K
import stark_ref as S
import tip5_ref as T


def test_const_proofs_accept_and_mutations_reject():
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    rng = np.random.default_rng(0xC5)
    claims, proofs = [], []
    for lph in (8, 14, 23):
        claim = ([lph, 5, 4, 3, 2], 0, [lph, 1], [7])
        proof, tr = K.prove(params, air, recipe, claim, lph, seed=lph)
        assert S.verify(params, air, claim, proof)
        assert S.structure_ok(params, proof)
        claims.append(claim)
        proofs.append(proof)
        for _ in range(6):
            m = list(proof)
            pos = int(rng.integers(2, len(m)))
            m[pos] = (m[pos] + 1) % T.P
            claims.append(claim)
            proofs.append(m)
    want = [S.verify(params, air, c, p) for c, p in zip(claims, proofs)]
    got = [bool(x) for x in C.stark_verify_batch(air.to_words(), params, claims, proofs, threads=4)]
    assert got == want
    assert want[0] and want[7] and want[14]
