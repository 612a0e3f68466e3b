"""Regenerate tests/golden/stark_tiny.json: a small synthetic AIR (oracle.stark_ref.synth_air) and
accepting proofs from the oracle's synthetic prover, with the oracle's Fiat-Shamir transcripts.
Self-generated (parity of the STARK layer is unpinned); Tip5 underneath is pinned
by the reference KATs."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import stark_prover as SP  # noqa: E402
import stark_ref as S  # noqa: E402

TINY = dict(num_main=24, num_aux=9, num_collinearity_checks=8)


def main():
    params = S.StarkParams(**TINY)
    air, recipe = S.synth_air(params, num_sampled=S.CHALLENGE_SAMPLE_COUNT, seed=7)
    cases = []
    for lph, claim in [(3, ([1, 2, 3, 4, 5], 0, [7, 8, 9], [10])), (4, ([9, 9, 9, 9, 9], 0, [], [3, 1, 4])),
                       (6, ([5, 4, 3, 2, 1], 0, [2] * 12, []))]:
        proof, _ = SP.prove(params, air, recipe, claim, lph, seed=100 + lph)
        tr = {}
        assert S.verify(params, air, claim, proof, tr)
        samples = [list(x) for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals]
        indices = [v for tag, vals in tr["sponge_samples"] if tag == "fri_indices" for v in vals]
        cases.append({"log2_padded_height": lph, "claim": {"digest": claim[0], "version": claim[1],
                                                           "input": claim[2], "output": claim[3]},
                      "proof": [str(w) for w in proof], "samples": [[str(c) for c in x] for x in samples],
                      "fri_indices": indices})
    out = {"params": TINY, "air": [str(w) for w in air.to_words()], "num_sampled": S.CHALLENGE_SAMPLE_COUNT, "seed": 7, "cases": cases}
    json.dump(out, open(os.path.join(HERE, "stark_tiny.json"), "w"))
    print("wrote stark_tiny.json", sum(len(c["proof"]) for c in cases), "proof words")


if __name__ == "__main__":
    main()
