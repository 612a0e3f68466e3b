"""Oracle pinning (CPU): the Python and C restatements against the reference's own
known-answer vectors, and against each other."""
import json
import os

import numpy as np

import tip5_ref as T
import coracle as C
from blake3_min import blake3_short


def test_blake3_known_answers():
    assert blake3_short(b"").hex() == "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"
    assert blake3_short(b"abc").hex() == "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"


def test_lookup_table_is_permutation_and_prefix():
    assert sorted(T.LOOKUP_TABLE) == list(range(256))
    assert T.LOOKUP_TABLE[:9] == [0, 7, 26, 63, 124, 215, 85, 254, 214]


def _kat_v(golden_dir):
    return json.load(open(os.path.join(golden_dir, "kat_v.json")))["vectors"]


def test_kat_v_python_oracle(golden_dir):
    """KAT-V: Tip5::hash_varlen — neptune-core/src/state/wallet/mod.rs:1379-1383."""
    for v in _kat_v(golden_dir):
        d = T.hash_varlen([int(x) for x in v["input"]])
        assert T.digest_to_hex(d) == v["digest_hex"], v["index"]


def test_kat_v_c_oracle(golden_dir):
    vs = _kat_v(golden_dir)
    data = np.array([int(x) for v in vs for x in v["input"]], dtype=np.uint64)
    off = np.arange(0, 5 * len(vs) + 1, 5, dtype=np.uint64)
    out = C.hash_varlen_batch(data, off)
    for k, v in enumerate(vs):
        assert T.digest_to_hex([int(x) for x in out[k]]) == v["digest_hex"]


def _kat_f(golden_dir):
    sol = json.load(open(os.path.join(golden_dir, "precalculated_pow_solution.json")))
    root = T.digest_from_hex(sol["root"])
    A = [T.digest_from_hex(h) for h in sol["path_a"]]
    B = [T.digest_from_hex(h) for h in sol["path_b"]]
    return root, A, B


def _kat_f_candidates(hp, A, B):
    out = []
    for order in (0, 1):
        n26 = hp(B[26], A[26]) if order == 0 else hp(A[26], B[26])
        for b27 in (0, 1):
            n27 = hp(A[27], n26) if b27 else hp(n26, A[27])
            for b28 in (0, 1):
                n28 = hp(A[28], n27) if b28 else hp(n27, A[28])
                out.append(((order, b27, b28), list(n28)))
    return out


def test_kat_f_python_and_c(golden_dir):
    """KAT-F: hash_pair + MTree child order — test_data/precalculated_pow_solution.json,
    semantics pow.rs:162-180.  Paths coincide at levels 27-28 and split at 26, so exactly
    one of 8 (order, bit27, bit28) climbs must reproduce the committed root."""
    root, A, B = _kat_f(golden_dir)
    assert [k for k in range(29) if A[k] == B[k]] == [27, 28]
    hits_py = [k for k, r in _kat_f_candidates(T.hash_pair, A, B) if r == root]
    hp_c = lambda l, r: [int(x) for x in C.hash_pair(np.array(l, np.uint64), np.array(r, np.uint64))]
    hits_c = [k for k, r in _kat_f_candidates(hp_c, A, B) if r == root]
    assert hits_py == hits_c == [(1, 1, 0)]


def test_c_and_python_oracles_agree():
    rng = np.random.default_rng(7)
    s = rng.integers(0, 2**64 - 2**32, size=(24, 16), dtype=np.uint64)
    cp = C.permutation_batch(s)
    pp = np.array([T.permutation([int(x) for x in r]) for r in s], dtype=np.uint64)
    assert (cp == pp).all()
    leafs = rng.integers(0, 2**63, size=(32, 5), dtype=np.uint64)
    nodes = C.mtree_build(leafs)
    pn = T.mtree_build([[int(x) for x in l] for l in leafs])
    assert (np.array(pn[1:], dtype=np.uint64) == nodes[1:]).all()


def test_oracle_matches_golden(golden_dir):
    g = json.load(open(os.path.join(golden_dir, "tip5_golden.json")))
    for c in g["permutation"]:
        assert [str(v) for v in T.permutation([int(x) for x in c["in"]])] == c["out"]
    for c in g["hash_varlen"]:
        data = np.array([int(x) for x in c["in"]] or [0], dtype=np.uint64)
        off = np.array([0, len(c["in"])], dtype=np.uint64)
        assert [str(int(x)) for x in C.hash_varlen_batch(data, off)[0]] == c["out"]


def test_c_oracle_mtree_verify_semantics():
    rng = np.random.default_rng(3)
    n, depth = 64, 6
    leafs = rng.integers(0, 2**63, size=(n, 5), dtype=np.uint64)
    nodes = C.mtree_build(leafs)
    lp = [[int(x) for x in l] for l in leafs]
    nd = [[int(x) for x in r] for r in nodes]
    idx = np.arange(n, dtype=np.uint64)
    paths = np.array([T.mtree_path(lp, nd, i) for i in range(n)], dtype=np.uint64)
    v = C.mtree_verify_batch(nodes[1], idx, leafs, paths, depth, nthreads=4)
    assert v.all()
    # strict '>' bound: index == 2^depth is climbed (as index 0), index > 2^depth rejected early
    assert C.mtree_verify_batch(nodes[1], np.array([n], np.uint64), leafs[:1], paths[:1], depth)[0] == 1
    assert C.mtree_verify_batch(nodes[1], np.array([n + 1], np.uint64), leafs[:1], paths[:1], depth)[0] == 0
    assert T.mtree_verify(nd[1], n, T.mtree_path(lp, nd, 0), lp[0]) is True
