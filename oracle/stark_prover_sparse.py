"""Sparse synthetic STARK prover: non-degenerate FRI at any padded height — TEST DATA GENERATOR ONLY.

Same proof structure and Fiat-Shamir order as stark_prover_fast.py / stark_prover_const.py (and the
verifier oracle/stark_ref.py).  Every column is constant, as in the constant prover, except the
synthetic AIR's unconstrained main column (SynthRecipe.unconstrained_main, the row's last word):
that one is a sparse polynomial f(X) = sum_m a_m X^(d_m) with a few random degrees d_m < the
randomized trace length, one of them near the top.  Then

  * every constraint still holds identically (no constraint reads the column), so the quotient
    segments are zero, as in the constant prover;
  * the DEEP codeword is w_c * (wd0 (f(x) - f(z)) / (x - z) + wd1 (f(x) - f(z w)) / (x - z w)) — non-zero
    at every point, of degree ~ the trace length, so every FRI round folds non-zero values with its
    own alpha and domain points, the last codeword is non-constant and the last polynomial is
    non-empty (degree up to first_max_degree >> R);
  * the main rows differ only in their last Tip5 absorption chunk, so a leaf costs one permutation
    from the shared prefix state (oracle_hash_varlen_resume); the aux and quotient trees are the
    constant prover's O(height) trees.

Cost is O(N) vector work and ~4N Tip5 permutations for a FRI domain of N points, so the proofs
reach BASELINE config 5's log2 padded height 23 (N = 2^26) in about a minute and heights <= 16 in
well under a second of C time; this is what makes the distinct-proof pools of config 4 and the
deep-FRI fixtures (tests/golden/make_deep_fri.py) affordable.  Checked by the oracle verifier
(accept, and mutations reject) in tests/test_stark_prover_sparse.py.
"""
from __future__ import annotations

import ctypes
from typing import Dict

import numpy as np

import stark_prover_const as K
import stark_prover_fast as F
import stark_ref as S
import tip5_ref as T
from field_ref import P, X_ZERO, interpolate_subgroup_x, lift, primitive_root_of_unity, xadd, xmul, xpow, xscale

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_bound = False


def _lib():
    global _bound
    L = F.lib()
    if not _bound:
        L.oracle_sponge_absorb_chunks.argtypes = [_u64p, ctypes.c_size_t, _u64p]
        L.hash_rows_tail.argtypes = [_u64p, _u64p, ctypes.c_size_t, ctypes.c_size_t, _u64p, ctypes.c_int]
        L.hash_rows_tail.restype = ctypes.c_int
        _bound = True
    return L


def _sparse_eval(terms, xs_offset: int, gen: int, n: int) -> np.ndarray:
    """f(o g^i) for i < n, f = sum a X^d: each monomial is a geometric sequence."""
    out = np.zeros(n, dtype=np.uint64)
    for a, d in terms:
        mono = F.vgeom(pow(xs_offset, d, P), pow(gen, d, P), n)
        _lib().vec_axpy(mono, int(a) % P, out, n, F.THREADS)
    return out


def _sparse_at(terms, x):
    acc = X_ZERO
    for a, d in terms:
        acc = xadd(acc, xscale(xpow(x, d), a))
    return acc


def prove(params: S.StarkParams, air: S.AirCircuit, recipe: S.SynthRecipe, claim, log2_ph: int, seed: int = 1,
          n_terms: int = 4):
    assert recipe.unconstrained_main, "the AIR needs an unconstrained main column (stark_ref.synth_air)"
    rng = S._SplitMix(seed)
    ph = 1 << log2_ph
    w_tr = primitive_root_of_unity(ph)
    dom = params.fri_domain(ph)
    N = dom.length
    h = N.bit_length() - 1
    Tlen = N // params.fri_expansion_factor
    M, A, nseg = params.num_main, params.num_aux, params.num_quotient_segments
    col = recipe.unconstrained_main[-1]
    assert col == M - 1
    # f: one term near the top degree (so the last FRI polynomial is non-empty), the rest spread
    degs = [Tlen - 1 - rng.below(max(1, Tlen // 8))] + [rng.below(Tlen) for _ in range(n_terms - 1)]
    terms = [(1 + rng.below(P - 1), d) for d in degs]

    ps = S.ProofStream(params)
    digest, version, inp, out = claim
    ps.absorb_words(S.encode_claim(digest, version, inp, out))
    ps.enqueue(S.LOG2_PADDED_HEIGHT, log2_ph)

    target_of = {(t["aux"], t["col"]): i for i, t in enumerate(recipe.targets)}
    free = {c: rng.fe() for c in recipe.free_columns}
    memo: Dict[tuple, tuple] = {}

    def col_value(is_aux: bool, c: int, chal):
        key = (is_aux, c)
        if key in memo:
            return memo[key]
        if not is_aux and c in free:
            v = lift(free[c])
        else:
            t = recipe.targets[target_of[key]]
            acc = t["coef"]
            for kind, idx in t["factors"]:
                if kind == S.INPUT_CHALLENGE:
                    acc = xmul(acc, chal[idx])
                else:
                    assert not (kind in (S.INPUT_MAIN_CURR, S.INPUT_MAIN_NEXT) and idx == col)
                    acc = xmul(acc, col_value(kind in (S.INPUT_AUX_CURR, S.INPUT_AUX_NEXT), idx, chal))
            if t["lin"] is not None:
                lk, li = t["lin"]
                assert not (lk == S.INPUT_MAIN_CURR and li == col)
                acc = xadd(acc, xmul(t["lin_coef"], col_value(lk == S.INPUT_AUX_CURR, li, chal)))
            v = acc
        memo[key] = v
        return v

    # ---- main table: constant columns + f in the last column
    main_vals = [col_value(False, c, None) for c in range(M)]
    main_row = [v[0] for v in main_vals]
    xs = F.vgeom(dom.offset, dom.generator, N)
    fx = _sparse_eval(terms, dom.offset, dom.generator, N)
    n_pre = (M - 1) // 10  # full rate chunks before the one holding the last column
    s0 = np.zeros(16, dtype=np.uint64)
    _lib().oracle_sponge_absorb_chunks(np.ascontiguousarray(np.array(main_row[:10 * n_pre] or [0], dtype=np.uint64)),
                                       n_pre, s0)
    tail_const = main_row[10 * n_pre:M - 1]
    tail = np.empty((len(tail_const) + 1, N), dtype=np.uint64)
    for j, v in enumerate(tail_const):
        tail[j] = v
    tail[-1] = fx
    main_leaf = np.zeros((N, 5), dtype=np.uint64)
    assert _lib().hash_rows_tail(s0, tail, tail.shape[0], N, main_leaf, F.THREADS) == 0
    del tail
    main_nodes = F._tree(main_leaf)
    ps.enqueue(S.MERKLE_ROOT, [int(x) for x in main_nodes[1]])
    sampled = ps.sample_scalars(air.num_sampled, "challenges")
    chal = S.derive_challenges(sampled, claim)
    aux_vals = [col_value(True, j, chal) for j in range(A)]
    aux_levels = K._const_tree(T.hash_varlen([c for v in aux_vals for c in v]), h)
    ps.enqueue(S.MERKLE_ROOT, aux_levels[h])
    ps.sample_scalars(air.num_constraints, "quotient_weights")
    q_levels = K._const_tree(T.hash_varlen([0] * (3 * nseg)), h)
    ps.enqueue(S.MERKLE_ROOT, q_levels[h])
    z = ps.sample_scalars(1, "ood_point")[0]
    z_next = xscale(z, w_tr)
    fz, fzn = _sparse_at(terms, z), _sparse_at(terms, z_next)
    mc = list(main_vals)
    mn = list(main_vals)
    mc[col], mn[col] = fz, fzn
    for kind, payload in ((S.OOD_MAIN_ROW, mc), (S.OOD_AUX_ROW, aux_vals), (S.OOD_MAIN_ROW, mn),
                          (S.OOD_AUX_ROW, aux_vals), (S.OOD_QUOT_SEGMENTS, [X_ZERO] * nseg)):
        ps.enqueue(kind, payload)
    w = ps.sample_scalars(M + A + nseg + params.num_deep, "lincomb_weights")
    w_c, w_deep = w[col], w[-params.num_deep:]
    # ---- DEEP codeword: the constant columns cancel against the OOD rows exactly
    t0 = F.xv_mul(F.xv_sub(F.xv_from_b(fx), tuple(F.vconst(c, N) for c in fz)), F.xv_inv_of_x_minus(xs, z))
    t1 = F.xv_mul(F.xv_sub(F.xv_from_b(fx), tuple(F.vconst(c, N) for c in fzn)), F.xv_inv_of_x_minus(xs, z_next))
    deep = F.xv_add(F.xv_mul_const(t0, xmul(w_c, w_deep[0])), F.xv_mul_const(t1, xmul(w_c, w_deep[1])))
    del t0, t1, xs
    # ---- FRI (as stark_prover_fast)
    R = params.fri_num_rounds(N)
    cws, trees = [deep], []
    dom_r = dom
    half_inv2 = pow(2, P - 2, P)
    for r in range(R + 1):
        leaves = F._digests_of_xfe(cws[r])
        nodes = F._tree(leaves)
        trees.append((leaves, nodes))
        ps.enqueue(S.MERKLE_ROOT, [int(x) for x in (nodes[1] if leaves.shape[0] > 1 else leaves[0])])
        if r < R:
            alpha = ps.sample_scalars(1, f"fri_alpha_{r}")[0]
            n = dom_r.length
            hh = n // 2
            xr = F.vgeom(dom_r.offset, dom_r.generator, hh)
            inv2x = F.vinv(F.vscale(xr, 2))
            a = tuple(x[:hh] for x in cws[r])
            b = tuple(x[hh:] for x in cws[r])
            even = tuple(F.vscale(x, half_inv2) for x in F.xv_add(a, b))
            odd = F.xv_scale_b(F.xv_sub(a, b), inv2x)
            cws.append(F.xv_add(even, F.xv_mul_const(odd, alpha)))
            dom_r = dom_r.halve()
    last = [(int(cws[R][0][i]), int(cws[R][1][i]), int(cws[R][2][i])) for i in range(cws[R][0].size)]
    ps.enqueue(S.FRI_CODEWORD, last)
    ps.enqueue(S.FRI_POLYNOMIAL, interpolate_subgroup_x(last))
    k = params.num_collinearity_checks
    idx = ps.sample_indices(N, k, "fri_indices")

    def resp(r, indices):
        leaves, nodes = trees[r]
        auth = S.auth_structure(nodes, leaves, leaves.shape[0], indices)
        return (auth, [(int(cws[r][0][i]), int(cws[r][1][i]), int(cws[r][2][i])) for i in indices])

    ps.enqueue(S.FRI_RESPONSE, resp(0, list(idx)))
    for r in range(R):
        n = cws[r][0].size
        ps.enqueue(S.FRI_RESPONSE, resp(r, [(i + n // 2) % n for i in idx]))
    ps.sample_scalars(1, "fri_last_indeterminate")
    rows = []
    for i in idx:
        row = list(main_row)
        row[col] = int(fx[i])
        rows.append(row)
    ps.enqueue(S.MAIN_ROWS, rows)
    ps.enqueue(S.AUTH_STRUCTURE, S.auth_structure(main_nodes, main_leaf, N, idx))
    ps.enqueue(S.AUX_ROWS, [list(aux_vals)] * k)
    ps.enqueue(S.AUTH_STRUCTURE, K._const_auth(aux_levels, h, idx))
    ps.enqueue(S.QUOT_SEGMENTS_ELEMENTS, [[X_ZERO] * nseg] * k)
    ps.enqueue(S.AUTH_STRUCTURE, K._const_auth(q_levels, h, idx))
    info = {"f_degrees": degs, "fri_rounds": R, "last_codeword_len": len(last),
            "last_poly_degree": S.xpoly_degree(interpolate_subgroup_x(last))}
    return S.encode_proof(ps.items, params), ps.transcript, info
