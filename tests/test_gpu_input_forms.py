"""Both input forms of the STARK entry points (nhip_stark_params.input_form): canonical values and
twenty-first's in-memory Montgomery words, the form the Rust drop-in hands over without a copy
(`Proof(Vec<BFieldElement>)`, verifier.rs:61, neptune_proof.rs:42-44).  The same proofs in either
form give identical verdicts and Fiat-Shamir transcripts (equal to the oracle's), mutants given as
the same field elements give the same verdicts, raw Montgomery words >= p read mod p, and the
device decoder survives every structural word set to boundary raw values in Montgomery form (each
verdict equal to the C oracle's on the element values)."""
import numpy as np
import pytest

import bench
import stark_ref as S
from test_gpu_decode_fuzz import FAIL_DECODE, _boundary_values, _structural_positions

pytestmark = pytest.mark.gpu
TOTAL = 512


@pytest.fixture(scope="module")
def c4():
    pool4 = bench.load_pool4()
    claims, proofs, expect, srcs, _, _ = bench.make_config4(pool4, TOTAL, 0.01, 1, 0)
    return pool4, claims, proofs, expect, srcs


def _mont(NS, claims, proofs):
    return [NS.montgomery_claim(NS.Claim(*c)) for c in claims], [NS.to_montgomery(p) for p in proofs]


def test_forms_give_identical_verdicts_and_transcripts(ctx, c4):
    import neptune_hip.stark as NS
    pool4, claims, proofs, expect, srcs = c4
    air = NS.Air([int(w) for w in pool4["air"]])
    can = NS.Stark.default()
    mclaims, mproofs = _mont(NS, claims, proofs)
    a = NS.Batch(ctx, air, can, [NS.Claim(*c) for c in claims], proofs)
    b = NS.Batch(ctx, air, can.montgomery(), mclaims, mproofs)
    va, _ = a.run()
    vb, _ = b.run()
    assert [bool(x) for x in va] == [bool(x) for x in vb] == [bool(x) for x in expect]
    seen = set()
    for i in range(TOTAL):
        ta, tb = a.transcript(i), b.transcript(i)
        assert ta == tb, i
        if expect[i] and srcs[i] not in seen:
            want_xs, want_idx = pool4["transcripts"][srcs[i]]
            assert tb[2] == 0 and tb[0] == want_xs and tb[1] == want_idx, i
            seen.add(srcs[i])
    assert len(seen) >= 200
    a.close()
    b.close()


def test_montgomery_mutants_and_noncanonical_words(ctx, c4):
    """Payload words of each height's proofs changed (+1, p - 1, a random element) in Montgomery
    form reject exactly as the canonical mutants do; w + p (the same element, raw word >= p) on every
    word that allows it accepts; the canonical words passed as Montgomery words reject."""
    import neptune_hip.stark as NS
    pool4, claims, proofs, expect, srcs = c4
    air = NS.Air([int(w) for w in pool4["air"]])
    can = NS.Stark.default()
    rng = np.random.default_rng(0x3F)
    cl, pr = [], []
    picks = [int(np.flatnonzero((np.asarray(srcs) == s) & expect)[0]) for s in sorted(set(srcs))[::16]]
    for i in picks:
        p = proofs[i]
        for _ in range(6):
            m = p.copy()
            pos = int(rng.integers(10, len(p)))
            delta = [1, S.P - 1, int(rng.integers(1, 1 << 63))][int(rng.integers(0, 3))]
            m[pos] = np.uint64((int(m[pos]) + delta) % S.P)
            cl.append(claims[i])
            pr.append(m)
    got_can = NS.verify_batch(ctx, air, can, [(NS.Claim(*c), p) for c, p in zip(cl, pr)])
    mcl, mpr = _mont(NS, cl, pr)
    got_mont = NS.verify_batch(ctx, air, can.montgomery(), list(zip(mcl, mpr)))
    assert got_can == got_mont and not all(got_can)
    # raw words >= p: the same elements
    hi = []
    for i in picks:
        w = NS.to_montgomery(proofs[i])
        lift = w < np.uint64((1 << 64) - S.P)
        hi.append(np.where(lift, w + np.uint64(S.P), w).astype(np.uint64))
    mcl = [NS.montgomery_claim(NS.Claim(*claims[i])) for i in picks]
    assert NS.verify_batch(ctx, air, can.montgomery(), list(zip(mcl, hi))) == [True] * len(picks)
    # canonical words read as Montgomery words are other elements
    assert NS.verify_batch(ctx, air, can.montgomery(), [(mcl[0], proofs[picks[0]])]) == [False]


def test_structural_fuzz_montgomery_form(ctx):
    """The device decoder in Montgomery form: every structural word of the smallest pool proof set
    to boundary RAW values (so its element value is that raw word * 2^-64); verdicts equal the C
    oracle's on the element values, FAIL_DECODE equals the host walk in the same form."""
    import json
    import os

    import coracle as C
    import neptune_hip.stark as NS
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_pool.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    air_w = z["air"]
    h = sorted(meta["heights"])[0]
    c = meta["claims"][str(h)]
    claim = (c["digest"], c["version"], c["input"], c["output"])
    proof = z[f"proof_{h}"]
    mproof = NS.to_montgomery(proof)
    variants = [mproof]
    for p in _structural_positions(proof):
        for v in _boundary_values(int(mproof[p])):
            m = mproof.copy()
            m[p] = np.uint64(v)
            variants.append(m)
    assert len(variants) > 500
    air = NS.Air([int(w) for w in air_w])
    stark = NS.Stark.default().montgomery()
    mclaim = NS.montgomery_claim(NS.Claim(*claim))
    b = NS.Batch(ctx, air, stark, [mclaim] * len(variants), variants)
    got, _ = b.run()
    values = [NS.from_montgomery(m) for m in variants]
    want = C.stark_verify_batch(air_w, S.StarkParams(), [claim] * len(values), values, threads=16)
    assert [bool(x) for x in got] == [bool(x) for x in want]
    for i, m in enumerate(variants):
        _, _, fail = b.transcript(i, max_xfe=1)
        assert (fail & FAIL_DECODE == 0) == NS.proof_decodes(air, stark, mclaim, m), i
    b.close()
    assert bool(got[0])
