"""The C restatement of the verifier (oracle/stark_oracle.c, the CPU baseline of bench.py) agrees
with the Python restatement (oracle/stark_ref.py) on accepting proofs, the reference's reject
cases and mutations, and its fast permutation (twenty-first MDS arithmetic) with the reference-form
one.  CPU only."""
import json
import os

import numpy as np

import coracle as C
import stark_ref as S
import tip5_ref as T

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_fast_permutation_matches_reference_form():
    rng = np.random.default_rng(11)
    st = rng.integers(0, T.P, size=(3000, 16), dtype=np.uint64)
    st[:8] = np.uint64(T.P - 1)
    st[8:16] = 0
    raw = np.array([[T.to_mont(int(x)) for x in row] for row in st], dtype=np.uint64)
    avx2 = C.set_mds_avx2(True)
    try:
        for form in ([True, False] if avx2 else [False]):  # the MDS sums in AVX2 and scalar
            assert C.set_mds_avx2(form) == form
            a, b = C.permutation_raw_pair(raw)
            assert (a == b).all()
    finally:
        C.set_mds_avx2(avx2)


def _tiny():
    g = json.load(open(os.path.join(GOLD, "stark_tiny.json")))
    params = S.StarkParams(**g["params"])
    air, _ = S.synth_air(params, num_sampled=g["num_sampled"], seed=g["seed"])
    claims = [(c["claim"]["digest"], c["claim"]["version"], c["claim"]["input"], c["claim"]["output"])
              for c in g["cases"]]
    proofs = [[int(w) for w in c["proof"]] for c in g["cases"]]
    return g, params, air, claims, proofs


def test_tiny_golden_and_reject_cases_match_python_oracle():
    T.use_c_backend()
    g, params, air, claims, proofs = _tiny()
    cl = claims[0]
    bogus = T.hash_varlen(S.encode_claim(*cl))
    rejects = [[], bogus, [0] * 65, [0], [1]]
    wrong = [(cl[0], cl[1], cl[2], list(cl[3]) + [1]), (cl[0], cl[1], [5] + list(cl[2]), cl[3]),
             ([1, 1, 1, 1, 1], cl[1], cl[2], cl[3]), (cl[0], 1, cl[2], cl[3])]
    all_claims = claims + [cl] * len(rejects) + wrong
    all_proofs = proofs + rejects + [proofs[0]] * len(wrong)
    v = C.stark_verify_batch(g["air"], params, all_claims, all_proofs, threads=4)
    want = [S.verify(params, air, c, p) for c, p in zip(all_claims, all_proofs)]
    assert [bool(x) for x in v] == want
    assert want[:3] == [True] * 3 and not any(want[3:])


def test_tiny_mutations_match_python_oracle():
    T.use_c_backend()
    g, params, air, claims, proofs = _tiny()
    rng = np.random.default_rng(3)
    mc, mp = [], []
    for _ in range(120):
        i = int(rng.integers(0, len(proofs)))
        p = list(proofs[i])
        pos = int(rng.integers(0, len(p)))
        p[pos] = (p[pos] + int(rng.integers(1, 4))) % T.P if rng.integers(0, 4) else int(rng.integers(0, 2 ** 63)) * 2 + 1
        mc.append(claims[i])
        mp.append(p)
    v = C.stark_verify_batch(g["air"], params, mc, mp, threads=4)
    want = [S.verify(params, air, c, p) for c, p in zip(mc, mp)]
    assert [bool(x) for x in v] == want


def test_pool_proofs_match_python_oracle():
    T.use_c_backend()
    z = np.load(os.path.join(GOLD, "c3_pool.npz"))
    meta = json.loads(bytes(z["meta"]).decode())
    params = S.StarkParams()
    air = S.AirCircuit.from_words([int(w) for w in z["air"]])
    claims, proofs = [], []
    for h in meta["heights"][:3]:
        c = meta["claims"][str(h)]
        claim = (c["digest"], c["version"], c["input"], c["output"])
        p = [int(w) for w in z[f"proof_{h}"]]
        lo, hi = meta["main_rows"][str(h)]
        bad = list(p)
        bad[(lo + hi) // 2] = (bad[(lo + hi) // 2] + 1) % T.P
        claims += [claim, claim]
        proofs += [p, bad]
    v = C.stark_verify_batch(z["air"], params, claims, proofs, threads=4)
    assert [bool(x) for x in v] == [True, False] * 3
    assert S.verify(params, air, claims[0], proofs[0]) and not S.verify(params, air, claims[1], proofs[1])
