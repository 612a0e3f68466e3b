"""tests/golden/config1.npz (BASELINE config 1's substitute, tests/golden/make_config1.py) on the
CPU: the C oracle accepts it and rejects a payload mutant and the claim with the kernel MAST hash
not reversed (single_proof.rs:295-304's claim shape); its FRI is non-degenerate (15 rounds, a last
polynomial of degree 122, the sparse polynomial's top degree near the trace length)."""
import json
import os

import numpy as np

import coracle as C
import stark_ref as S

FIX = os.path.join(os.path.dirname(__file__), "golden", "config1.npz")


def test_config1_fixture_verdicts_and_shape():
    z = np.load(FIX)
    m = json.loads(bytes(z["meta"]).decode())
    assert m["log2_padded_height"] == 21 and m["input"] == m["kernel_mast_hash"][::-1] and m["output"] == []
    info = m["info"]
    assert info["fri_rounds"] == 15 and info["last_poly_degree"] > 0 and max(info["f_degrees"]) > (1 << 21)
    params = S.StarkParams()
    air, _ = S.synth_air(params, seed=m["air_seed"])
    claim = (m["digest"], m["version"], m["input"], m["output"])
    proof = [int(w) for w in z["proof"]]
    mutated = list(proof)
    mutated[len(proof) // 3] = (mutated[len(proof) // 3] + 1) % S.P
    unreversed = (m["digest"], m["version"], m["kernel_mast_hash"], m["output"])
    v = C.stark_verify_batch(air.to_words(), params, [claim, claim, unreversed], [proof, mutated, proof], threads=3)
    assert [bool(x) for x in v] == [True, False, False]
    assert len(z["indices"]) == params.num_collinearity_checks and len(z["samples"]) > 100
