"""The fast synthetic prover (oracle/stark_prover_fast.py, test-data generator for the large
BASELINE configs) produces proofs the oracle verifier accepts, with the same item sequence as the
small prover, and every single-word corruption of one is rejected by the oracle."""
import numpy as np

import stark_prover_fast as F
import stark_ref as S


def _setup():
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    return params, air, recipe


def test_fast_prover_accepted_by_oracle():
    params, air, recipe = _setup()
    for lph, claim in [(3, ([1, 2, 3, 4, 5], 0, [7], [])), (5, ([9, 9, 9, 9, 9], 0, [], [4, 4]))]:
        proof, _ = F.prove(params, air, recipe, claim, lph, seed=lph)
        assert S.structure_ok(params, proof)
        assert S.verify(params, air, claim, proof) is True
        # bound to the claim
        assert S.verify(params, air, (claim[0], claim[1], claim[2], claim[3] + [1]), proof) is False


def test_fast_prover_corruptions_rejected():
    params, air, recipe = _setup()
    claim = ([3, 1, 4, 1, 5], 0, [], [])
    proof, _ = F.prove(params, air, recipe, claim, 4, seed=11)
    rng = np.random.default_rng(5)
    for pos in rng.integers(2, len(proof), size=6).tolist():
        m = list(proof)
        m[pos] = (m[pos] + 1) % S.P
        assert S.verify(params, air, claim, m) is False
