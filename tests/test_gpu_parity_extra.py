"""Full-size parity data of round 6 (self-generated, the STARK layer stays unpinned past
Tip5: DESIGN.md §4), compared transcript for transcript with the oracle on the GPU:

  * tests/golden/config5_distinct.npz: 4 DISTINCT accepting proofs at BASELINE config 5's log2 padded
    height 23 (FRI domain 2^26, 16 folding rounds, sparse synthetic prover: non-zero codewords in every
    round, non-empty last polynomial), each with its own claim and seed;
  * authentication-structure mutants of those proofs: a word of a main / aux / quotient
    AuthenticationStructure item (two per item).  Fiat-Shamir does not
    absorb these items, so the transcript stays the accepting proof's and only the Merkle check can
    reject; the 26-level trees climb per tree from the level with <= 4,096 hash ops
    (k_mp_climb from a start level) by default, and level by level with that form off
    (nhip_set_climb_from_ops(0)): both reject, as the C oracle does;
  * tests/golden/pool4_fast.npz: 16 config-4-shaped proofs (heights 9-12) from the FULL synthetic
    prover (every column a low-degree polynomial), plus a MainRows mutant per height.
Each batch runs on two streams (the library default) and on one stream (the bench's form for small
batches: the sponge replay and the row hashing then share one launch, k_fs_rows_small).
Reference: triton_vm::verify at verifier.rs:60-63, one proof at a time."""
import json
import os

import numpy as np
import pytest

import coracle as C
import stark_ref as S

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
POOL = os.path.join(GOLD, "c3_pool.npz")


def _load(name):
    z = np.load(os.path.join(GOLD, name))
    meta = json.loads(bytes(z["meta"]).decode())
    w, o = z["words"], z["offsets"]
    smp, so, idx, io = z["samples"], z["sample_offsets"], z["indices"], z["index_offsets"]
    out = []
    for i, c in enumerate(meta["claims"]):
        out.append({"claim": (c["digest"], c["version"], c["input"], c["output"]),
                    "proof": np.asarray(w[int(o[i]):int(o[i + 1])], dtype=np.uint64),
                    "samples": [tuple(int(v) for v in x) for x in smp[int(so[i]):int(so[i + 1])]],
                    "indices": [int(v) for v in idx[int(io[i]):int(io[i + 1])]], "info": meta["info"][i]})
    return out


@pytest.fixture(scope="module")
def air_words():
    return [int(w) for w in np.load(POOL)["air"]]


def _spans(proof, params):
    items = S.decode_proof([int(w) for w in proof], params)
    out, pos = [], 2
    for k, _ in items:
        ln = int(proof[pos])
        out.append((k, pos + 1, pos + 1 + ln))
        pos += 1 + ln
    return out


def _run(ctx, air_words, cases, extra=(), streams=2):
    import neptune_hip.stark as NS
    claims = [c["claim"] for c in cases] + [c for c, _ in extra]
    proofs = [c["proof"] for c in cases] + [p for _, p in extra]
    b = NS.Batch(ctx, NS.Air(air_words), NS.Stark.default(), [NS.Claim(*c) for c in claims], proofs)
    b.set_streams(streams)
    v, _ = b.run()
    tr = [b.transcript(i) for i in range(len(proofs))]
    b.close()
    return [bool(x) for x in v], tr, claims, proofs


@pytest.mark.parametrize("streams", [2, 1])
def test_config5_distinct_height23_transcripts(ctx, air_words, streams):
    cases = _load("config5_distinct.npz")
    assert len(cases) == 4 and len({tuple(c["proof"][:64].tolist()) for c in cases}) == 4
    assert all(c["info"]["log2_ph"] == 23 and c["info"]["last_poly_degree"] > 0 for c in cases)
    got, tr, _, _ = _run(ctx, air_words, cases, streams=streams)
    assert got == [True] * 4
    for c, (xs, idx, fail) in zip(cases, tr):
        assert fail == 0 and xs == c["samples"] and idx == c["indices"]


def _auth_mutants(case, params):
    """Two words of each authentication structure (main, aux, quotient): one inside the first
    digests, the structure's last word.  (A FRI response's words start with structural lengths,
    which the decoder rejects before any Merkle check: covered by test_gpu_decode_fuzz.)"""
    sp = _spans(case["proof"], params)
    out = []
    auths = [s for s in sp if s[0] == S.AUTH_STRUCTURE]
    assert len(auths) == 3
    for k, (_, lo, hi) in enumerate(auths):
        out += [lo + 1 + (7 + 5 * k) % max(1, hi - lo - 1), hi - 1]
    res = []
    for pos in out:
        m = case["proof"].copy()
        m[pos] = np.uint64((int(m[pos]) + 1) % S.P)
        res.append((case["claim"], m))
    return res


@pytest.mark.parametrize("climb_from,streams", [(-1, 2), (0, 2), (-1, 1)])
def test_auth_structure_mutants_reject_with_and_without_climb_from(ctx, air_words, climb_from, streams):
    import neptune_hip._lib as L
    lib = L.load()
    cases = _load("config5_distinct.npz")[:2]
    params = S.StarkParams()
    extra = []
    for c in cases:
        extra += _auth_mutants(c, params)
    assert lib.nhip_set_climb_from_ops(climb_from) == 0
    try:
        got, tr, claims, proofs = _run(ctx, air_words, cases, extra, streams)
    finally:
        assert lib.nhip_set_climb_from_ops(-1) == 0
    want = [bool(x) for x in C.stark_verify_batch(air_words, params, claims, proofs, threads=8)]
    assert got == want and want[:2] == [True, True] and not any(want[2:])
    # Fiat-Shamir never saw the mutated word: each mutant's samples are its source proof's
    per = len(extra) // len(cases)
    for j in range(len(extra)):
        src = cases[j // per]
        xs, idx, fail = tr[2 + j]
        assert fail != 0 and xs == src["samples"] and idx == src["indices"], j


@pytest.mark.parametrize("streams", [2, 1])
def test_pool4_fast_prover_transcripts_and_mutants(ctx, air_words, streams):
    cases = _load("pool4_fast.npz")
    assert len(cases) == 16 and {c["info"]["log2_ph"] for c in cases} == {9, 10, 11, 12}
    params = S.StarkParams()
    extra = []
    for c in cases[::4]:  # one MainRows mutant per height
        (_, lo, hi), = [s for s in _spans(c["proof"], params) if s[0] == S.MAIN_ROWS]
        m = c["proof"].copy()
        m[(lo + hi) // 2] = np.uint64((int(m[(lo + hi) // 2]) + 1) % S.P)
        extra.append((c["claim"], m))
    got, tr, claims, proofs = _run(ctx, air_words, cases, extra, streams)
    want = [bool(x) for x in C.stark_verify_batch(air_words, params, claims, proofs, threads=8)]
    assert got == want == [True] * 16 + [False] * 4
    for c, (xs, idx, fail) in zip(cases, tr):
        assert fail == 0 and xs == c["samples"] and idx == c["indices"]
