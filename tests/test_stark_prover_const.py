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


def _config1_case():
    """BASELINE config 1 substitute: one SingleProof-shaped proof, log2 padded
    height 21, seed 0xC1.  The claim has SingleProof's shape (`single_proof.rs:295-304`: input =
    the 5-word kernel MAST hash reversed, output empty); the program digest is synthetic (the
    SingleProof program hash needs tasm-lib, absent here)."""
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    rng = np.random.default_rng(0xC1)
    kernel_mast_hash = [int(x) for x in rng.integers(0, T.P, size=5, dtype=np.uint64)]
    program_digest = [int(x) for x in rng.integers(0, T.P, size=5, dtype=np.uint64)]
    claim = (program_digest, 0, kernel_mast_hash[::-1], [])
    proof, tr = K.prove(params, air, recipe, claim, 21, seed=0xC1)
    return params, air, claim, proof


def test_config1_singleproof_cpu():
    T.use_c_backend()
    params, air, claim, proof = _config1_case()
    assert S.verify(params, air, claim, proof)
    rng = np.random.default_rng(0xC1 + 1)
    claims, proofs = [claim], [proof]
    for pos in [2, len(proof) // 2, len(proof) - 1] + [int(x) for x in rng.integers(2, len(proof), size=3)]:
        m = list(proof)
        m[pos] = (m[pos] + 1) % T.P
        claims.append(claim)
        proofs.append(m)
    wrong_claim = (claim[0], claim[1], claim[2][::-1], [])  # un-reversed MAST hash
    claims.append(wrong_claim)
    proofs.append(proof)
    want = [S.verify(params, air, c, p) for c, p in zip(claims, proofs)]
    got = [bool(x) for x in C.stark_verify_batch(air.to_words(), params, claims, proofs, threads=4)]
    assert got == want
    assert want[0] and not any(want[1:])
