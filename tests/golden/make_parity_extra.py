"""Regenerate the full-size parity fixtures of round 6 (TEST DATA GENERATOR, self-generated: the
STARK layer's parity is unpinned):

  * tests/golden/config5_distinct.npz — 4 DISTINCT accepting proofs at log2 padded height 23
    (BASELINE config 5's height: FRI domain 2^26, 16 folding rounds) from the sparse synthetic
    prover (oracle/stark_prover_sparse.py: non-zero codewords in every FRI round, a non-empty last
    polynomial), each with its own claim and seed;
  * tests/golden/pool4_fast.npz — 16 config-4-shaped proofs at log2 padded heights 9-12 (4 each)
    from the full synthetic prover (oracle/stark_prover_fast.py: EVERY main / aux column a
    low-degree polynomial, not the sparse prover's one non-constant column), distinct claims and
    seeds.

Every proof is verified by both oracle restatements (oracle/stark_ref.py, oracle/stark_oracle.c)
before it is written, and the Python oracle's Fiat-Shamir transcript (every squeezed sample, the
FRI indices) is stored beside it for the GPU transcript comparison (tests/test_gpu_parity_extra.py).

Usage: python tests/golden/make_parity_extra.py [config5|pool4|all]
       (height 23: a few minutes and ~25 GB of host memory per proof, made one at a time)
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import coracle as C  # noqa: E402
import stark_prover_fast as F  # noqa: E402
import stark_prover_sparse as SP  # noqa: E402
import stark_ref as S  # noqa: E402
import tip5_ref as T  # noqa: E402

AIR_SEED = 1  # the c3 pool's AIR (tests/golden/make_bench_pool.py)
C5_HEIGHT, C5_COUNT = 23, 4
FAST_HEIGHTS = [9, 10, 11, 12]
FAST_PER_HEIGHT = 4


def _transcript(params, air, claim, proof):
    tr = {}
    assert S.verify(params, air, claim, [int(w) for w in proof], tr), "rejected by the Python oracle"
    samples = np.array([list(x) for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals],
                       dtype=np.uint64)
    indices = np.array([v for tag, vals in tr["sponge_samples"] if tag == "fri_indices" for v in vals],
                       dtype=np.uint64)
    return samples, indices


def _save(path, air, entries, extra_meta):
    """entries: (claim, proof, samples, indices, info) -> one npz of concatenated arrays."""
    claims = [e[0] for e in entries]
    proofs = [np.asarray(e[1], dtype=np.uint64) for e in entries]
    ok = C.stark_verify_batch([int(w) for w in air.to_words()], S.StarkParams(), claims, proofs, threads=8)
    assert all(bool(x) for x in ok), "rejected by the C oracle"

    def offs(xs):
        o = np.zeros(len(xs) + 1, dtype=np.uint64)
        o[1:] = np.cumsum([len(x) for x in xs])
        return o

    meta = dict(extra_meta, claims=[{"digest": c[0], "version": c[1], "input": c[2], "output": c[3]} for c in claims],
                info=[e[4] for e in entries])
    np.savez_compressed(path, words=np.concatenate(proofs), offsets=offs(proofs),
                        samples=np.concatenate([e[2] for e in entries]), sample_offsets=offs([e[2] for e in entries]),
                        indices=np.concatenate([e[3] for e in entries]), index_offsets=offs([e[3] for e in entries]),
                        meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8))


def config5(params, air, recipe):
    entries = []
    for i in range(C5_COUNT):
        t = time.time()
        claim = ([0xC5, C5_HEIGHT, i, 0xD15, 7 * i + 1], 0, [i, C5_HEIGHT, 0xC5][: 1 + i % 3], [i * 3 + 1][: i % 2])
        proof, _, info = SP.prove(params, air, recipe, claim, C5_HEIGHT, seed=0xC5D0 + i)
        samples, indices = _transcript(params, air, claim, proof)
        entries.append((claim, proof, samples, indices, dict(info, log2_ph=C5_HEIGHT, prover="sparse")))
        print(f"config5 {i}: {len(proof)} words, {info}, {time.time() - t:.0f} s", flush=True)
    _save(os.path.join(HERE, "config5_distinct.npz"), air, entries, {"air_seed": AIR_SEED})


def pool4(params, air, recipe):
    entries = []
    for h in FAST_HEIGHTS:
        for j in range(FAST_PER_HEIGHT):
            t = time.time()
            claim = ([h, j, 0xFA57, (j * 7919) % 65521, 0x5EED], 0, [h * 100 + j + k for k in range(j % 5)],
                     [j * 31 + k for k in range(j % 3)])
            proof = F.prove(params, air, recipe, claim, h, seed=(0xFA << 16) + (h << 8) + j)
            proof = proof[0] if isinstance(proof, tuple) else proof
            samples, indices = _transcript(params, air, claim, proof)
            entries.append((claim, proof, samples, indices, {"log2_ph": h, "prover": "fast"}))
            print(f"pool4 fast h{h} j{j}: {len(proof)} words, {time.time() - t:.0f} s", flush=True)
    _save(os.path.join(HERE, "pool4_fast.npz"), air, entries, {"air_seed": AIR_SEED})


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=AIR_SEED)
    if which in ("pool4", "all"):
        pool4(params, air, recipe)
    if which in ("config5", "all"):
        config5(params, air, recipe)


if __name__ == "__main__":
    main()
