"""Synthetic STARK prover for the oracle's verifier — TEST DATA GENERATOR ONLY.

Produces proofs in the triton-vm 1.0 proof-stream structure restated in stark_ref.py, for a
synthetic AIR from `stark_ref.synth_air` (which also returns the construction recipe used here).
Column polynomials are built so that every constraint C satisfies C = Z_type * r with known r, so
the quotient is known in closed form and the proofs are genuinely accepting: Fiat-Shamir order,
OOD quotient identity, DEEP combination, FRI and all Merkle authentications hold.  Mutations of
the encoded proof give rejecting proofs.

Neither the product path nor the verifier imports this module.
"""
from __future__ import annotations

import math
from typing import List, Sequence

import numpy as np

import coracle as CO
from field_ref import (P, X_ONE, X_ZERO, Domain, binv, bpoly_mul, coset_evaluate_b, coset_evaluate_x,
                       interpolate_subgroup_x, lift, xpoly_mul, primitive_root_of_unity, xadd, xbatch_inv, xmul, xpoly_eval,
                       xpow, xscale, xsub)
import stark_ref as S


def _padd(a, b, is_x):
    n = max(len(a), len(b))
    z = X_ZERO if is_x else 0
    a = list(a) + [z] * (n - len(a))
    b = list(b) + [z] * (n - len(b))
    if is_x:
        return [xadd(x, y) for x, y in zip(a, b)]
    return [(x + y) % P for x, y in zip(a, b)]


def _to_x(poly):
    return [x if isinstance(x, tuple) else lift(x) for x in poly]


def _xpoly_mul_b(xp, bp):
    """XFE-coefficient poly times BFE-coefficient poly."""
    cols = [bpoly_mul([c[k] for c in xp], bp) for k in range(3)]
    return list(zip(cols[0], cols[1], cols[2]))


def _eval_poly_at_x(poly, z):
    acc = X_ZERO
    for c in reversed(poly):
        cc = c if isinstance(c, tuple) else lift(c)
        acc = xadd(xmul(acc, z), cc)
    return acc


class _Rng(S._SplitMix):
    pass


def zerofier_poly(ctype, ph, w):
    w_inv = binv(w)
    if ctype == S.C_INIT:
        return [P - 1, 1]
    if ctype == S.C_CONS:
        return [P - 1] + [0] * (ph - 1) + [1]
    if ctype == S.C_TERM:
        return [(P - w_inv) % P, 1]
    # (X^ph - 1) / (X - w^-1) = sum_k a^(ph-1-k) X^k, a = w^-1
    return [pow(w_inv, ph - 1 - k, P) for k in range(ph)]


def prove(params: S.StarkParams, air: S.AirCircuit, recipe: S.SynthRecipe, claim, log2_ph: int, seed: int = 1):
    rng = _Rng(seed)
    ph = 1 << log2_ph
    Tlen = params.randomized_trace_len(ph)
    w_tr = primitive_root_of_unity(ph)
    fri_dom = params.fri_domain(ph)
    N = fri_dom.length
    tree_h = int(math.log2(N))
    M, A = params.num_main, params.num_aux
    ps = S.ProofStream(params)
    digest, version, inp, out = claim
    ps.absorb_words(S.encode_claim(digest, version, inp, out))
    ps.enqueue(S.LOG2_PADDED_HEIGHT, log2_ph)

    def rand_b(n):
        return [rng.fe() for _ in range(n)]

    def rand_x(n):
        return [(rng.fe(), rng.fe(), rng.fe()) for _ in range(n)]

    def shift(poly, is_x):  # p(X) -> p(w X)
        out_, s = [], 1
        for c in poly:
            out_.append(xscale(c, s) if is_x else c * s % P)
            s = s * w_tr % P
        return out_

    main: List[list] = [None] * M
    aux: List[list] = [None] * A
    free_deg = max(1, Tlen // 4 - 1)
    for c in recipe.free_columns:
        main[c] = rand_b(free_deg)
    quot_r = {}

    def operand_poly(op, chal):
        kind, idx = op
        if kind == S.INPUT_MAIN_CURR:
            return main[idx], False
        if kind == S.INPUT_MAIN_NEXT:
            return shift(main[idx], False), False
        if kind == S.INPUT_AUX_CURR:
            return aux[idx], True
        if kind == S.INPUT_AUX_NEXT:
            return shift(aux[idx], True), True
        return [chal[idx]], True

    def build(ti, chal):
        t = recipe.targets[ti]
        Z = zerofier_poly(t["type"], ph, w_tr)
        rdeg = Tlen - (len(Z) - 1)
        prod, is_x = [t["coef"]], True
        for f in t["factors"]:
            fp, fx = operand_poly(f, chal)
            prod = xpoly_mul(prod, _to_x(fp)) if fx else _xpoly_mul_b(prod, fp)
        if t["lin"] is not None:
            lp, lx = operand_poly(t["lin"], chal)
            prod = _padd(prod, xpoly_mul([t["lin_coef"]], _to_x(lp)), True)
        if t["aux"]:
            r = rand_x(rdeg)
            poly = _padd(prod, _xpoly_mul_b(r, Z), True)
            aux[t["col"]] = poly
        else:
            r = rand_b(rdeg)
            assert all(c[1] == 0 and c[2] == 0 for c in prod), "main target must stay in the base field"
            poly = _padd([c[0] for c in prod], bpoly_mul(r, Z), False)
            main[t["col"]] = poly
            r = [lift(c) for c in r]
        assert len(poly) <= Tlen
        quot_r[ti] = r

    for ti, t in enumerate(recipe.targets):
        if not t["aux"]:
            build(ti, None)
    # main codewords on the FRI domain, rows -> leaves -> root
    main_cw = [coset_evaluate_b(main[c], fri_dom) for c in range(M)]
    main_rows = np.array(main_cw, dtype=np.uint64).T.copy()  # N x M
    main_leaf = CO.hash_varlen_batch(main_rows.reshape(-1), np.arange(0, N * M + 1, M, dtype=np.uint64))
    main_nodes = S.merkle_nodes(main_leaf)
    ps.enqueue(S.MERKLE_ROOT, [int(x) for x in main_nodes[1]])
    sampled = ps.sample_scalars(air.num_sampled, "challenges")
    chal = S.derive_challenges(sampled, claim)
    for ti, t in enumerate(recipe.targets):
        if t["aux"]:
            build(ti, chal)
    aux_cw = [coset_evaluate_x(aux[j], fri_dom) for j in range(A)]
    aux_rows = np.array([[c for j in range(A) for c in aux_cw[j][i]] for i in range(N)], dtype=np.uint64)
    aux_leaf = CO.hash_varlen_batch(aux_rows.reshape(-1), np.arange(0, N * 3 * A + 1, 3 * A, dtype=np.uint64))
    aux_nodes = S.merkle_nodes(aux_leaf)
    ps.enqueue(S.MERKLE_ROOT, [int(x) for x in aux_nodes[1]])
    quot_w = ps.sample_scalars(air.num_constraints, "quotient_weights")
    # quotient Q = sum w_i q_i in verifier constraint order
    order = []
    for ctype in range(4):
        for ti, t in enumerate(recipe.targets):
            if t["type"] == ctype:
                order.append([(ti, X_ONE)])
        for cb in recipe.combos:
            if cb["type"] == ctype:
                order.append([(cb["a"], X_ONE), (cb["b"], cb["lam"])])
    assert len(order) == air.num_constraints
    Q = [X_ZERO] * Tlen
    for wi, terms in zip(quot_w, order):
        for ti, lam in terms:
            sc = xmul(wi, lam)
            for k, c in enumerate(quot_r[ti]):
                Q[k] = xadd(Q[k], xmul(sc, c))
    nseg = params.num_quotient_segments
    segs = [[Q[j * nseg + k] for j in range(Tlen // nseg)] for k in range(nseg)]
    seg_cw = [coset_evaluate_x(s, fri_dom) for s in segs]
    q_rows = np.array([[c for k in range(nseg) for c in seg_cw[k][i]] for i in range(N)], dtype=np.uint64)
    q_leaf = CO.hash_varlen_batch(q_rows.reshape(-1), np.arange(0, N * 3 * nseg + 1, 3 * nseg, dtype=np.uint64))
    q_nodes = S.merkle_nodes(q_leaf)
    ps.enqueue(S.MERKLE_ROOT, [int(x) for x in q_nodes[1]])
    z = ps.sample_scalars(1, "ood_point")[0]
    z_next = xscale(z, w_tr)
    z_pow = xpow(z, nseg)
    mc = [_eval_poly_at_x(main[c], z) for c in range(M)]
    ac = [_eval_poly_at_x(aux[j], z) for j in range(A)]
    mn = [_eval_poly_at_x(main[c], z_next) for c in range(M)]
    an = [_eval_poly_at_x(aux[j], z_next) for j in range(A)]
    qs = [_eval_poly_at_x(s, z_pow) for s in segs]
    ps.enqueue(S.OOD_MAIN_ROW, mc)
    ps.enqueue(S.OOD_AUX_ROW, ac)
    ps.enqueue(S.OOD_MAIN_ROW, mn)
    ps.enqueue(S.OOD_AUX_ROW, an)
    ps.enqueue(S.OOD_QUOT_SEGMENTS, qs)
    nw = M + A + nseg + params.num_deep
    w = ps.sample_scalars(nw, "lincomb_weights")
    w_main, w_aux = w[:M], w[M:M + A]
    w_quot, w_deep = w[M + A:M + A + nseg], w[-params.num_deep:]

    def lin(mrow, arow):
        acc = X_ZERO
        for wi, v in zip(w_main, mrow):
            acc = xadd(acc, xscale(wi, int(v)) if not isinstance(v, tuple) else xmul(wi, v))
        for wi, v in zip(w_aux, arow):
            acc = xadd(acc, xmul(wi, v))
        return acc

    o_curr = lin(mc, ac)
    o_next = lin(mn, an)
    o_q = X_ZERO
    for wi, v in zip(w_quot, qs):
        o_q = xadd(o_q, xmul(wi, v))
    xs = fri_dom.values()
    inv0 = xbatch_inv([xsub(lift(x), z) for x in xs])
    inv1 = xbatch_inv([xsub(lift(x), z_next) for x in xs])
    inv2 = xbatch_inv([xsub(lift(x), z_pow) for x in xs])
    deep = []
    for i in range(N):
        mav = lin(main_rows[i], [aux_cw[j][i] for j in range(A)])
        qv = X_ZERO
        for k in range(nseg):
            qv = xadd(qv, xmul(w_quot[k], seg_cw[k][i]))
        t0 = xmul(xsub(mav, o_curr), inv0[i])
        t1 = xmul(xsub(mav, o_next), inv1[i])
        t2 = xmul(xsub(qv, o_q), inv2[i])
        deep.append(xadd(xadd(xmul(t0, w_deep[0]), xmul(t1, w_deep[1])), xmul(t2, w_deep[2])))
    # FRI
    R = params.fri_num_rounds(N)
    cws, trees, doms = [deep], [], [fri_dom]
    for r in range(R + 1):
        leaves = np.array([S.xfe_digest(x) for x in cws[r]], dtype=np.uint64)
        nodes = S.merkle_nodes(leaves) if len(cws[r]) > 1 else leaves
        trees.append((leaves, nodes))
        ps.enqueue(S.MERKLE_ROOT, [int(x) for x in (nodes[1] if len(cws[r]) > 1 else leaves[0])])
        if r < R:
            alpha = ps.sample_scalars(1, f"fri_alpha_{r}")[0]
            dom, cw = doms[r], cws[r]
            n = dom.length
            half = n // 2
            dx = dom.values()
            ax_inv = xbatch_inv([lift(2 * dx[i] % P) for i in range(half)])
            nxt = []
            for i in range(half):
                # line through (x, a), (-x, b) at alpha:  (a+b)/2 + alpha (a-b)/(2x)
                a_, b_ = cw[i], cw[i + half]
                even = xscale(xadd(a_, b_), binv(2))
                odd = xmul(xsub(a_, b_), ax_inv[i])
                nxt.append(xadd(even, xmul(alpha, odd)))
            cws.append(nxt)
            doms.append(dom.halve())
    last = cws[R]
    ps.enqueue(S.FRI_CODEWORD, last)
    ps.enqueue(S.FRI_POLYNOMIAL, interpolate_subgroup_x(last))
    k = params.num_collinearity_checks
    idx = ps.sample_indices(N, k, "fri_indices")

    def resp(r, indices):
        leaves, nodes = trees[r]
        n = len(cws[r])
        auth = S.auth_structure(nodes, leaves, n, indices)
        return (auth, [cws[r][i] for i in indices])

    ps.enqueue(S.FRI_RESPONSE, resp(0, [i % N for i in idx]))
    for r in range(R):
        n = len(cws[r])
        ps.enqueue(S.FRI_RESPONSE, resp(r, [(i + n // 2) % n for i in idx]))
    ps.sample_scalars(1, "fri_last_indeterminate")
    ps.enqueue(S.MAIN_ROWS, [[int(x) for x in main_rows[i]] for i in idx])
    ps.enqueue(S.AUTH_STRUCTURE, S.auth_structure(main_nodes, main_leaf, N, idx))
    ps.enqueue(S.AUX_ROWS, [[aux_cw[j][i] for j in range(A)] for i in idx])
    ps.enqueue(S.AUTH_STRUCTURE, S.auth_structure(aux_nodes, aux_leaf, N, idx))
    ps.enqueue(S.QUOT_SEGMENTS_ELEMENTS, [[seg_cw[kk][i] for kk in range(nseg)] for i in idx])
    ps.enqueue(S.AUTH_STRUCTURE, S.auth_structure(q_nodes, q_leaf, N, idx))
    return S.encode_proof(ps.items, params), ps.transcript
