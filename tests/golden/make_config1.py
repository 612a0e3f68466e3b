"""Regenerate tests/golden/config1.npz: BASELINE config 1's substitute, one SingleProof-shaped
proof at log2 padded height 21 (FRI domain 2^24, 15 folding rounds) with a NON-degenerate FRI: the
sparse synthetic prover (oracle/stark_prover_sparse.py) makes every FRI codeword non-zero, the last
polynomial non-empty and the main rows distinct (the constant-codeword prover used before folded
zeros).  The claim is single_proof.rs:295-304's shape: input = a 5-word kernel MAST hash reversed,
output empty, a synthetic program digest (seed 0xC1).  The proof is checked by the oracle verifier
before it is written, with its Fiat-Shamir transcript (every squeezed sample, the FRI indices)
stored beside it for tests/test_gpu_stark.py::test_config1_singleproof_gpu and bench.py's
config1_latency.  Self-generated (parity of the STARK layer is unpinned).

Usage: python tests/golden/make_config1.py   (about a minute; ~8 GB of host memory)
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

LOG2_PH = 21
AIR_SEED = 1  # the c3 pool's AIR (tests/golden/make_bench_pool.py)
SEED = 0xC1


def main():
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=AIR_SEED)
    rng = np.random.default_rng(SEED)
    kernel_mast_hash = [int(x) for x in rng.integers(0, S.P, size=5, dtype=np.uint64)]
    program_digest = [int(x) for x in rng.integers(0, S.P, size=5, dtype=np.uint64)]
    claim = (program_digest, 0, kernel_mast_hash[::-1], [])
    t = time.time()
    proof, _, info = SP.prove(params, air, recipe, claim, LOG2_PH, seed=SEED)
    tr = {}
    assert S.verify(params, air, claim, proof, tr)
    samples = [list(x) for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals]
    indices = [v for tag, vals in tr["sponge_samples"] if tag == "fri_indices" for v in vals]
    meta = {"air_seed": AIR_SEED, "log2_padded_height": LOG2_PH, "seed": SEED, "kernel_mast_hash": kernel_mast_hash,
            "digest": claim[0], "version": claim[1], "input": claim[2], "output": claim[3], "info": info}
    np.savez_compressed(os.path.join(HERE, "config1.npz"), proof=np.array(proof, dtype=np.uint64),
                        samples=np.array(samples, dtype=np.uint64), indices=np.array(indices, dtype=np.uint64),
                        meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8))
    print(f"lph {LOG2_PH}: {len(proof)} words, {info}, {time.time() - t:.0f} s", flush=True)


if __name__ == "__main__":
    main()
