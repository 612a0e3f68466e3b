"""Regenerate tests/golden/c3_pool.npz: the proof pool of BASELINE config 3 (one accepting synthetic
proof per ProofCollection member padded height {16, 10, 11, 12, 12, 11, 9, 9} -> distinct heights
9..12 and 16) with Stark::default()-shaped parameters, the synthetic AIR they are proven against,
and per proof the word range of its MainRows payload (where bench.py flips one word to make a
collection reject).  Proofs come from the oracle's fast synthetic prover and are checked by the
oracle verifier before they are written; bench.py and the GPU tests only read this data file.

Usage: python tests/golden/make_bench_pool.py   (about a minute)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import stark_prover_fast as F  # noqa: E402
import stark_ref as S  # noqa: E402
import tip5_ref as T  # noqa: E402

HEIGHTS = [9, 10, 11, 12, 16]
AIR_SEED = 1


def item_payload_range(proof, kind, params):
    items = S.decode_proof(proof, params)
    pos = 2
    for k, _ in items:
        ln = proof[pos]
        if k == kind:
            return pos + 1, pos + 1 + ln
        pos += 1 + ln
    raise ValueError("item kind absent")


def main():
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=AIR_SEED)
    arrays = {"air": np.array(air.to_words(), dtype=np.uint64)}
    meta = {"air_seed": AIR_SEED, "heights": HEIGHTS, "claims": {}, "main_rows": {}}
    for lph in HEIGHTS:
        claim = ([lph, 0xC3, 3, 4, 5], 0, [lph] * 5, [lph + 1])
        proof, _ = F.prove(params, air, recipe, claim, lph, seed=0xC3 + lph)
        assert S.verify(params, air, claim, proof), lph
        arrays[f"proof_{lph}"] = np.array(proof, dtype=np.uint64)
        meta["claims"][str(lph)] = {"digest": claim[0], "version": claim[1], "input": claim[2], "output": claim[3]}
        meta["main_rows"][str(lph)] = list(item_payload_range(proof, S.MAIN_ROWS, params))
        print(f"lph {lph}: {len(proof)} words", flush=True)
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez(os.path.join(HERE, "c3_pool.npz"), **arrays)


if __name__ == "__main__":
    main()
