"""Fast synthetic STARK prover (large padded heights) — TEST DATA GENERATOR ONLY.

Same proof structure and Fiat-Shamir order as stark_prover.py, but every column is evaluated
pointwise on the FRI domain with vectorised C helpers (vec_oracle.c): free main columns are random
polynomials of low degree DF, each target column is t = F(sources) + Z_type * r with r of low
degree DR, so codewords, OOD values and the quotient need no interpolation.  Degrees stay far below
the STARK bounds, so the proofs are genuinely accepting (checked against the oracle verifier in
tests/test_stark_prover_fast.py); verification cost does not depend on the degrees.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

import coracle as CO
import stark_ref as S
from field_ref import (P, X_ONE, X_ZERO, binv, interpolate_subgroup_x, lift, primitive_root_of_unity, xadd, xmul,
                       xpow, xscale, xsub)

_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_sz = ctypes.c_size_t
_L = None
THREADS = int(os.environ.get("NHIP_PROVER_THREADS", str(min(16, os.cpu_count() or 1))))


def lib():
    global _L
    if _L is None:
        L = CO.lib()
        for name, args in {
            "vec_mul": [_u64p, _u64p, _u64p, _sz, ctypes.c_int],
            "vec_add": [_u64p, _u64p, _u64p, _sz, ctypes.c_int],
            "vec_sub": [_u64p, _u64p, _u64p, _sz, ctypes.c_int],
            "vec_scale": [_u64p, ctypes.c_uint64, _u64p, _sz, ctypes.c_int],
            "vec_axpy": [_u64p, ctypes.c_uint64, _u64p, _sz, ctypes.c_int],
            "vec_geom": [ctypes.c_uint64, ctypes.c_uint64, _u64p, _sz],
            "vec_horner": [_u64p, _sz, _u64p, _u64p, _sz, ctypes.c_int],
            "vec_batch_inv": [_u64p, _u64p, _sz],
            "vec_xlincomb": [_u64p, _sz, ctypes.c_int, _u64p, _u64p, _u64p, _u64p, _sz, ctypes.c_int],
            "hash_rows_planes": [_u64p, _sz, _sz, _u64p, ctypes.c_int],
            "mtree_build_mt": [_u64p, _sz, _u64p, ctypes.c_int],
        }.items():
            getattr(L, name).argtypes = args
        _L = L
    return _L


# ------------------------------------------------------------------ base vectors (canonical u64)
def vmul(a, b):
    o = np.empty_like(a); lib().vec_mul(a, b, o, a.size, THREADS); return o


def vadd(a, b):
    o = np.empty_like(a); lib().vec_add(a, b, o, a.size, THREADS); return o


def vsub(a, b):
    o = np.empty_like(a); lib().vec_sub(a, b, o, a.size, THREADS); return o


def vscale(a, c):
    o = np.empty_like(a); lib().vec_scale(a, int(c) % P, o, a.size, THREADS); return o


def vconst(c, n):
    return np.full(n, int(c) % P, dtype=np.uint64)


def vgeom(start, ratio, n):
    o = np.empty(n, dtype=np.uint64); lib().vec_geom(int(start) % P, int(ratio) % P, o, n); return o


def vhorner(coeffs, xs):
    c = np.ascontiguousarray(np.asarray([int(v) % P for v in coeffs], dtype=np.uint64))
    o = np.empty_like(xs); lib().vec_horner(c, c.size, xs, o, xs.size, THREADS); return o


def vinv(a):
    o = np.empty_like(a); lib().vec_batch_inv(np.ascontiguousarray(a), o, a.size); return o


# ------------------------------------------------------------------ XFE vectors: tuple of 3 arrays
def xv_from_b(b):
    z = np.zeros_like(b)
    return (b, z, z.copy())


def xv_add(a, b):
    return tuple(vadd(x, y) for x, y in zip(a, b))


def xv_sub(a, b):
    return tuple(vsub(x, y) for x, y in zip(a, b))


def xv_scale_b(a, bvec):
    return tuple(vmul(x, bvec) for x in a)


def xv_mul_const(a, c):
    """XFE vector a times XFE constant c."""
    c0, c1, c2 = c
    a0, a1, a2 = a
    r0 = vscale(a0, c0)
    r1 = vadd(vscale(a0, c1), vscale(a1, c0))
    r2 = vadd(vadd(vscale(a0, c2), vscale(a1, c1)), vscale(a2, c0))
    r3 = vadd(vscale(a1, c2), vscale(a2, c1))
    r4 = vscale(a2, c2)
    return (vsub(r0, r3), vsub(vadd(r1, r3), r4), vadd(r2, r4))


def xv_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    r0 = vmul(a0, b0)
    r1 = vadd(vmul(a0, b1), vmul(a1, b0))
    r2 = vadd(vadd(vmul(a0, b2), vmul(a1, b1)), vmul(a2, b0))
    r3 = vadd(vmul(a1, b2), vmul(a2, b1))
    r4 = vmul(a2, b2)
    return (vsub(r0, r3), vsub(vadd(r1, r3), r4), vadd(r2, r4))


def xv_inv_of_x_minus(xs, z):
    """1 / (x - z) for BFE vector xs and XFE constant z (adjugate formula, batched det inverse)."""
    a0 = vsub(xs, vconst(z[0], xs.size))
    a1c, a2c = (-z[1]) % P, (-z[2]) % P
    s = vadd(a0, vconst(a2c, xs.size))           # a0 + a2
    d = (a1c - a2c) % P                            # a1 - a2 (constant)
    C00 = vsub(vmul(s, s), vconst(d * a1c, xs.size))
    C01 = vsub(vconst(d * a2c, xs.size), vscale(s, a1c))
    C02 = vsub(vconst(a1c * a1c, xs.size), vscale(s, a2c))
    det = vsub(vsub(vmul(a0, C00), vscale(C01, a2c)), vscale(C02, a1c))
    di = vinv(det)
    return (vmul(C00, di), vmul(C01, di), vmul(C02, di))


def horner_x(coeffs, x):
    acc = X_ZERO
    for c in reversed(coeffs):
        cc = c if isinstance(c, tuple) else lift(c)
        acc = xadd(xmul(acc, x), cc)
    return acc


def _digests_of_xfe(v3):
    n = v3[0].size
    leaves = np.zeros((n, 5), dtype=np.uint64)
    leaves[:, 0], leaves[:, 1], leaves[:, 2] = v3
    return leaves


def _tree(leaves):
    n = leaves.shape[0]
    if n == 1:
        return leaves.copy()
    nodes = np.zeros((n, 5), dtype=np.uint64)
    lib().mtree_build_mt(np.ascontiguousarray(leaves), n, nodes, THREADS)
    return nodes


def _hash_planes(planes):
    planes = np.ascontiguousarray(planes, dtype=np.uint64)
    n = planes.shape[1]
    out = np.zeros((n, 5), dtype=np.uint64)
    lib().hash_rows_planes(planes, planes.shape[0], n, out, THREADS)
    return out


def prove(params: S.StarkParams, air: S.AirCircuit, recipe: S.SynthRecipe, claim, log2_ph: int, seed: int = 1,
          DF: int = 4, DR: int = 15):
    rng = S._SplitMix(seed)
    ph = 1 << log2_ph
    w_tr = primitive_root_of_unity(ph)
    w_inv = binv(w_tr)
    dom = params.fri_domain(ph)
    N = dom.length
    M, A, nseg = params.num_main, params.num_aux, params.num_quotient_segments
    g = dom.generator
    xs = vgeom(dom.offset, g, N)
    xs_next = vgeom(dom.offset * w_tr, g, N)
    xph = vgeom(pow(dom.offset, ph, P), pow(g, ph, P), N)
    one = vconst(1, N)
    Zc = {S.C_INIT: vsub(xs, one), S.C_CONS: vsub(xph, one), S.C_TERM: vsub(xs, vconst(w_inv, N))}
    Zc[S.C_TRANS] = vmul(Zc[S.C_CONS], vinv(Zc[S.C_TERM]))

    def Z_at(ctype, x):
        if ctype == S.C_INIT:
            return xsub(x, X_ONE)
        if ctype == S.C_CONS:
            return xsub(xpow(x, ph), X_ONE)
        if ctype == S.C_TERM:
            return xsub(x, lift(w_inv))
        return xmul(xsub(xpow(x, ph), X_ONE), S.xinv(xsub(x, lift(w_inv))))

    ps = S.ProofStream(params)
    digest, version, inp, out = claim
    ps.absorb_words(S.encode_claim(digest, version, inp, out))
    ps.enqueue(S.LOG2_PADDED_HEIGHT, log2_ph)

    free = {c: [rng.fe() for _ in range(DF + 1)] for c in recipe.free_columns}
    main_cw = np.zeros((M, N), dtype=np.uint64)
    free_next = {}
    for c, co in free.items():
        main_cw[c] = vhorner(co, xs)
        free_next[c] = vhorner(co, xs_next)
    rpoly = {}
    memo = {}

    def col_value(is_aux, col, x, chal):
        key = (is_aux, col, x)
        if key in memo:
            return memo[key]
        if not is_aux and col in free:
            v = horner_x(free[col], x)
        else:
            ti = target_of[(is_aux, col)]
            t = recipe.targets[ti]
            acc = t["coef"]
            for kind, idx in t["factors"]:
                if kind == S.INPUT_CHALLENGE:
                    acc = xmul(acc, chal[idx])
                else:
                    xx = x if kind in (S.INPUT_MAIN_CURR, S.INPUT_AUX_CURR) else xscale(x, w_tr)
                    acc = xmul(acc, col_value(kind in (S.INPUT_AUX_CURR, S.INPUT_AUX_NEXT), idx, xx, chal))
            if t["lin"] is not None:
                lk, li = t["lin"]
                acc = xadd(acc, xmul(t["lin_coef"], col_value(lk == S.INPUT_AUX_CURR, li, x, chal)))
            acc = xadd(acc, xmul(Z_at(t["type"], x), horner_x(rpoly[ti], x)))
            v = acc
        memo[key] = v
        return v

    target_of = {(t["aux"], t["col"]): i for i, t in enumerate(recipe.targets)}

    def build(ti, chal, aux_cw):
        t = recipe.targets[ti]
        if t["aux"]:
            r = [(rng.fe(), rng.fe(), rng.fe()) for _ in range(DR + 1)]
        else:
            r = [rng.fe() for _ in range(DR + 1)]
        rpoly[ti] = r
        prod = None  # XFE vector or BFE vector (tracked)
        prod_is_x = False
        const = t["coef"]
        for kind, idx in t["factors"]:
            if kind == S.INPUT_CHALLENGE:
                const = xmul(const, chal[idx])
                continue
            if kind == S.INPUT_MAIN_CURR:
                v, vx = main_cw[idx], False
            elif kind == S.INPUT_MAIN_NEXT:
                v, vx = free_next[idx], False
            elif kind == S.INPUT_AUX_CURR:
                v, vx = aux_cw[idx], True
            else:
                raise ValueError("aux next factors are not generated by synth_air")
            if prod is None:
                prod, prod_is_x = v, vx
            elif prod_is_x and vx:
                prod = xv_mul(prod, v)
            elif prod_is_x:
                prod = xv_scale_b(prod, v)
            elif vx:
                prod, prod_is_x = xv_scale_b(v, prod), True
            else:
                prod = vmul(prod, v)
        if prod is None:
            prod, prod_is_x = one, False
        acc = xv_mul_const(prod if prod_is_x else xv_from_b(prod), const)
        if t["lin"] is not None:
            lk, li = t["lin"]
            lv = aux_cw[li] if lk == S.INPUT_AUX_CURR else xv_from_b(main_cw[li])
            acc = xv_add(acc, xv_mul_const(lv, t["lin_coef"]))
        if t["aux"]:
            rv = tuple(vhorner([c[k] for c in r], xs) for k in range(3))
            acc = xv_add(acc, xv_scale_b(rv, Zc[t["type"]]))
            aux_cw[t["col"]] = acc
        else:
            assert not prod_is_x and t["coef"][1] == 0 and t["coef"][2] == 0
            base = acc[0]
            base = vadd(base, vmul(vhorner(r, xs), Zc[t["type"]]))
            main_cw[t["col"]] = base

    for ti, t in enumerate(recipe.targets):
        if not t["aux"]:
            build(ti, None, None)
    main_leaf = _hash_planes(main_cw)
    main_nodes = _tree(main_leaf)
    ps.enqueue(S.MERKLE_ROOT, [int(x) for x in main_nodes[1]])
    sampled = ps.sample_scalars(air.num_sampled, "challenges")
    chal = S.derive_challenges(sampled, claim)
    aux_cw = [None] * A
    for ti, t in enumerate(recipe.targets):
        if t["aux"]:
            build(ti, chal, aux_cw)
    aux_planes = np.zeros((3 * A, N), dtype=np.uint64)
    for j in range(A):
        for k in range(3):
            aux_planes[3 * j + k] = aux_cw[j][k]
    aux_leaf = _hash_planes(aux_planes)
    aux_nodes = _tree(aux_leaf)
    ps.enqueue(S.MERKLE_ROOT, [int(x) for x in aux_nodes[1]])
    quot_w = ps.sample_scalars(air.num_constraints, "quotient_weights")
    order = []
    for ctype in range(4):
        for ti, t in enumerate(recipe.targets):
            if t["type"] == ctype:
                order.append([(ti, X_ONE)])
        for cb in recipe.combos:
            if cb["type"] == ctype:
                order.append([(cb["a"], X_ONE), (cb["b"], cb["lam"])])
    Q = [X_ZERO] * (DR + 1)
    for wi, terms in zip(quot_w, order):
        for ti, lam in terms:
            sc = xmul(wi, lam)
            for k, c in enumerate(rpoly[ti]):
                Q[k] = xadd(Q[k], xmul(sc, c if isinstance(c, tuple) else lift(c)))
    nq = -(-len(Q) // nseg) * nseg
    Q = Q + [X_ZERO] * (nq - len(Q))
    segs = [[Q[j * nseg + k] for j in range(nq // nseg)] for k in range(nseg)]
    seg_cw = [tuple(vhorner([c[kk] for c in s], xs) for kk in range(3)) for s in segs]
    q_planes = np.zeros((3 * nseg, N), dtype=np.uint64)
    for k in range(nseg):
        for kk in range(3):
            q_planes[3 * k + kk] = seg_cw[k][kk]
    q_leaf = _hash_planes(q_planes)
    q_nodes = _tree(q_leaf)
    ps.enqueue(S.MERKLE_ROOT, [int(x) for x in q_nodes[1]])
    z = ps.sample_scalars(1, "ood_point")[0]
    z_next = xscale(z, w_tr)
    z_pow = xpow(z, nseg)
    mc = [col_value(False, c, z, chal) for c in range(M)]
    ac = [col_value(True, j, z, chal) for j in range(A)]
    mn = [col_value(False, c, z_next, chal) for c in range(M)]
    an = [col_value(True, j, z_next, chal) for j in range(A)]
    qs = [horner_x(s, z_pow) for s in segs]
    for kind, payload in ((S.OOD_MAIN_ROW, mc), (S.OOD_AUX_ROW, ac), (S.OOD_MAIN_ROW, mn), (S.OOD_AUX_ROW, an),
                          (S.OOD_QUOT_SEGMENTS, qs)):
        ps.enqueue(kind, payload)
    nw = M + A + nseg + params.num_deep
    w = ps.sample_scalars(nw, "lincomb_weights")
    w_main, w_aux, w_quot, w_deep = w[:M], w[M:M + A], w[M + A:M + A + nseg], w[-params.num_deep:]

    def lin(mrow, arow):
        acc = X_ZERO
        for wi, v in zip(w_main, mrow):
            acc = xadd(acc, xmul(wi, v))
        for wi, v in zip(w_aux, arow):
            acc = xadd(acc, xmul(wi, v))
        return acc

    o_curr, o_next = lin(mc, ac), lin(mn, an)
    o_q = X_ZERO
    for wi, v in zip(w_quot, qs):
        o_q = xadd(o_q, xmul(wi, v))
    mav = [np.zeros(N, dtype=np.uint64) for _ in range(3)]
    wm = np.array([c for x in w_main for c in x], dtype=np.uint64)
    wa = np.array([c for x in w_aux for c in x], dtype=np.uint64)
    lib().vec_xlincomb(np.ascontiguousarray(main_cw), M, 0, wm, mav[0], mav[1], mav[2], N, THREADS)
    lib().vec_xlincomb(aux_planes, A, 1, wa, mav[0], mav[1], mav[2], N, THREADS)
    mav = tuple(mav)
    qv = (np.zeros(N, dtype=np.uint64),) * 3
    for k in range(nseg):
        qv = xv_add(qv, xv_mul_const(seg_cw[k], w_quot[k]))

    def csub(v, c):
        return tuple(vsub(x, vconst(cc, N)) for x, cc in zip(v, c))

    t0 = xv_mul(csub(mav, o_curr), xv_inv_of_x_minus(xs, z))
    t1 = xv_mul(csub(mav, o_next), xv_inv_of_x_minus(xs, z_next))
    t2 = xv_mul(csub(qv, o_q), xv_inv_of_x_minus(xs, z_pow))
    deep = xv_add(xv_add(xv_mul_const(t0, w_deep[0]), xv_mul_const(t1, w_deep[1])), xv_mul_const(t2, w_deep[2]))
    # FRI
    R = params.fri_num_rounds(N)
    cws, trees = [deep], []
    dom_r = dom
    half_inv2 = binv(2)
    for r in range(R + 1):
        leaves = _digests_of_xfe(cws[r])
        nodes = _tree(leaves)
        trees.append((leaves, nodes))
        ps.enqueue(S.MERKLE_ROOT, [int(x) for x in (nodes[1] if leaves.shape[0] > 1 else leaves[0])])
        if r < R:
            alpha = ps.sample_scalars(1, f"fri_alpha_{r}")[0]
            n = dom_r.length
            h = n // 2
            xr = vgeom(dom_r.offset, dom_r.generator, h)
            inv2x = vinv(vscale(xr, 2))
            a = tuple(x[:h].copy() for x in cws[r])
            b = tuple(x[h:].copy() for x in cws[r])
            even = tuple(vscale(x, half_inv2) for x in xv_add(a, b))
            odd = xv_scale_b(xv_sub(a, b), inv2x)
            cws.append(xv_add(even, xv_mul_const(odd, alpha)))
            dom_r = dom_r.halve()
    last = [(int(cws[R][0][i]), int(cws[R][1][i]), int(cws[R][2][i])) for i in range(cws[R][0].size)]
    ps.enqueue(S.FRI_CODEWORD, last)
    ps.enqueue(S.FRI_POLYNOMIAL, interpolate_subgroup_x(last))
    k = params.num_collinearity_checks
    idx = ps.sample_indices(N, k, "fri_indices")

    def resp(r, indices):
        leaves, nodes = trees[r]
        n = leaves.shape[0]
        auth = S.auth_structure(nodes, leaves, n, indices)
        return (auth, [(int(cws[r][0][i]), int(cws[r][1][i]), int(cws[r][2][i])) for i in indices])

    ps.enqueue(S.FRI_RESPONSE, resp(0, list(idx)))
    for r in range(R):
        n = cws[r][0].size
        ps.enqueue(S.FRI_RESPONSE, resp(r, [(i + n // 2) % n for i in idx]))
    ps.sample_scalars(1, "fri_last_indeterminate")
    ps.enqueue(S.MAIN_ROWS, [[int(x) for x in main_cw[:, i]] for i in idx])
    ps.enqueue(S.AUTH_STRUCTURE, S.auth_structure(main_nodes, main_leaf, N, idx))
    ps.enqueue(S.AUX_ROWS, [[(int(aux_cw[j][0][i]), int(aux_cw[j][1][i]), int(aux_cw[j][2][i])) for j in range(A)]
                            for i in idx])
    ps.enqueue(S.AUTH_STRUCTURE, S.auth_structure(aux_nodes, aux_leaf, N, idx))
    ps.enqueue(S.QUOT_SEGMENTS_ELEMENTS, [[(int(seg_cw[kk][0][i]), int(seg_cw[kk][1][i]), int(seg_cw[kk][2][i]))
                                           for kk in range(nseg)] for i in idx])
    ps.enqueue(S.AUTH_STRUCTURE, S.auth_structure(q_nodes, q_leaf, N, idx))
    return S.encode_proof(ps.items, params), ps.transcript
