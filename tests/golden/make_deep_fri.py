"""Regenerate tests/golden/deep_fri.npz: accepting proofs with a non-degenerate FRI at large padded
heights (Stark::default(), the c3 pool's synthetic AIR), from the sparse synthetic prover
(oracle/stark_prover_sparse.py): every FRI codeword non-zero, a non-empty last polynomial, the main
rows distinct.  Heights 17, 20 and 23 (BASELINE config 5's height: FRI domain 2^26, 16 folding
rounds).  Each proof is checked by the oracle verifier before it is written, with its Fiat-Shamir
transcript (every squeezed sample and the FRI indices) stored beside it for the GPU parity test
(tests/test_gpu_deep_fri.py).  Self-generated (parity of the STARK layer is unpinned).

Usage: python tests/golden/make_deep_fri.py   (a few minutes; ~25 GB of host memory at height 23)
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import stark_prover_sparse as SP  # noqa: E402
import stark_ref as S  # noqa: E402
import tip5_ref as T  # noqa: E402

HEIGHTS = [17, 20, 23]
AIR_SEED = 1  # the c3 pool's AIR (tests/golden/make_bench_pool.py)


def main():
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=AIR_SEED)
    arrays = {}
    meta = {"air_seed": AIR_SEED, "heights": HEIGHTS, "cases": {}}
    for lph in HEIGHTS:
        t = time.time()
        claim = ([0xDF, lph, 1, 2, 3], 0, [lph, 0xDF], [lph * 3])
        proof, _, info = SP.prove(params, air, recipe, claim, lph, seed=0xDF00 + lph)
        tr = {}
        assert S.verify(params, air, claim, proof, tr), lph
        samples = [list(x) for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals]
        indices = [v for tag, vals in tr["sponge_samples"] if tag == "fri_indices" for v in vals]
        arrays[f"proof_{lph}"] = np.array(proof, dtype=np.uint64)
        arrays[f"samples_{lph}"] = np.array(samples, dtype=np.uint64)
        arrays[f"indices_{lph}"] = np.array(indices, dtype=np.uint64)
        meta["cases"][str(lph)] = {"digest": claim[0], "version": claim[1], "input": claim[2], "output": claim[3],
                                   "info": info}
        print(f"lph {lph}: {len(proof)} words, {info}, {time.time() - t:.0f} s", flush=True)
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "deep_fri.npz"), **arrays)


if __name__ == "__main__":
    main()
