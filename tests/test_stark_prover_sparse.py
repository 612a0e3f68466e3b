"""The sparse synthetic prover (oracle/stark_prover_sparse.py) makes accepting proofs whose FRI is
non-degenerate (non-zero codewords in every round, a non-empty last polynomial) at any padded
height; single-word mutations reject, and the Python and C restatements of the verifier agree.
CPU only (the deep heights' GPU parity is tests/test_gpu_deep_fri.py)."""
import numpy as np

import coracle as C
import stark_prover_sparse as SP
import stark_ref as S
import tip5_ref as T


def _items(params, proof):
    return S.decode_proof(proof, params)


def test_sparse_proofs_accept_with_nonzero_fri_and_mutations_reject():
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    rng = np.random.default_rng(0x5A)
    claims, proofs = [], []
    for lph in (8, 13, 17):
        claim = ([lph, 9, 8, 7, 6], 0, [lph], [1, 2])
        proof, _, info = SP.prove(params, air, recipe, claim, lph, seed=0x5A + lph)
        assert S.verify(params, air, claim, proof)
        items = _items(params, proof)
        by = {}
        for k, p in items:
            by.setdefault(k, []).append(p)
        last_poly = by[S.FRI_POLYNOMIAL][0]
        assert S.xpoly_degree(last_poly) == info["last_poly_degree"] > 0  # non-empty last polynomial
        for auth, leaves in by[S.FRI_RESPONSE]:  # every round reveals non-zero codeword values
            assert all(x != (0, 0, 0) for x in leaves)
        assert len({tuple(r) for r in by[S.MAIN_ROWS][0]}) > 1  # rows differ (last column)
        claims.append(claim)
        proofs.append(proof)
        for _ in range(5):
            m = list(proof)
            pos = int(rng.integers(2, len(m)))
            m[pos] = (m[pos] + 1) % T.P
            claims.append(claim)
            proofs.append(m)
    want = [S.verify(params, air, c, p) for c, p in zip(claims, proofs)]
    got = [bool(x) for x in C.stark_verify_batch(air.to_words(), params, claims, proofs, threads=4)]
    assert got == want
    assert want[0] and want[6] and want[12]
    assert not any(want[1:6]) and not any(want[7:12]) and not any(want[13:18])


def test_sparse_column_is_unconstrained():
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    col = recipe.unconstrained_main[-1]
    assert col == params.num_main - 1
    for op, a, b, c in air.nodes:
        if op == S.OP_INPUT and a in (S.INPUT_MAIN_CURR, S.INPUT_MAIN_NEXT):
            assert b != col
