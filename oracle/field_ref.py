"""Goldilocks base field, cubic extension XFieldElement, domains and polynomials — TEST ORACLE ONLY.

Restates twenty-first 1.0.0 (Cargo.lock:4297):
  * BFieldElement arithmetic mod p = 2^64 - 2^32 + 1 (canonical values here).
  * XFieldElement = F_p[x] / (x^3 - x + 1), coefficients [c0, c1, c2] (unpinned
    beyond the modulus).
  * primitive_root_of_unity(2^k) = 7^((p-1)/2^k) (checked against the recalled table entries
    for 2, 4, 8 and 2^32; unpinned).
  * ArithmeticDomain: offset * generator^i, `halve()` squares both (triton-vm 1.0.0).
Only tests/ and the oracle's own synthetic prover import this.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

P = (1 << 64) - (1 << 32) + 1
GENERATOR = 7

XFE = Tuple[int, int, int]
X_ZERO: XFE = (0, 0, 0)
X_ONE: XFE = (1, 0, 0)


def binv(a: int) -> int:
    if a % P == 0:
        raise ZeroDivisionError("inverse of zero")
    return pow(a, P - 2, P)


def xadd(a: XFE, b: XFE) -> XFE:
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P, (a[2] + b[2]) % P)


def xsub(a: XFE, b: XFE) -> XFE:
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P, (a[2] - b[2]) % P)


def xneg(a: XFE) -> XFE:
    return ((-a[0]) % P, (-a[1]) % P, (-a[2]) % P)


def xmul(a: XFE, b: XFE) -> XFE:
    # (a0 + a1 x + a2 x^2)(b0 + b1 x + b2 x^2) with x^3 = x - 1, x^4 = x^2 - x
    c0 = a[0] * b[0]
    c1 = a[0] * b[1] + a[1] * b[0]
    c2 = a[0] * b[2] + a[1] * b[1] + a[2] * b[0]
    c3 = a[1] * b[2] + a[2] * b[1]
    c4 = a[2] * b[2]
    return ((c0 - c3) % P, (c1 + c3 - c4) % P, (c2 + c4) % P)


def xscale(a: XFE, s: int) -> XFE:
    return (a[0] * s % P, a[1] * s % P, a[2] * s % P)


def lift(b: int) -> XFE:
    return (b % P, 0, 0)


def xpow(a: XFE, e: int) -> XFE:
    r = X_ONE
    while e:
        if e & 1:
            r = xmul(r, a)
        a = xmul(a, a)
        e >>= 1
    return r


def xinv(a: XFE) -> XFE:
    if a == X_ZERO:
        raise ZeroDivisionError("inverse of zero")
    return xpow(a, P ** 3 - 2)


def xbatch_inv(vals: Sequence[XFE]) -> List[XFE]:
    """Montgomery batch inversion (same result as element-wise inverses)."""
    n = len(vals)
    pref = [X_ONE] * (n + 1)
    for i, v in enumerate(vals):
        pref[i + 1] = xmul(pref[i], v)
    inv_all = xinv(pref[n])
    out = [X_ZERO] * n
    for i in range(n - 1, -1, -1):
        out[i] = xmul(inv_all, pref[i])
        inv_all = xmul(inv_all, vals[i])
    return out


def primitive_root_of_unity(n: int) -> int:
    if n < 1 or n & (n - 1) or n > (1 << 32):
        raise ValueError("domain length must be a power of two <= 2^32")
    return pow(GENERATOR, (P - 1) // n, P)


class Domain:
    """triton-vm ArithmeticDomain: {offset * generator^i : i < length}."""

    def __init__(self, length: int, offset: int = 1):
        self.length = length
        self.offset = offset % P
        self.generator = primitive_root_of_unity(length)

    def value(self, i: int) -> int:
        return self.offset * pow(self.generator, i, P) % P

    def values(self) -> List[int]:
        out, x = [], self.offset
        for _ in range(self.length):
            out.append(x)
            x = x * self.generator % P
        return out

    def halve(self) -> "Domain":
        d = Domain(self.length // 2, self.offset * self.offset % P)
        return d


# ------------------------------------------------------------------ polynomials
def bpoly_eval(coeffs: Sequence[int], x: int) -> int:
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % P
    return acc


def xpoly_eval(coeffs: Sequence[XFE], x: XFE) -> XFE:
    acc = X_ZERO
    for c in reversed(coeffs):
        acc = xadd(xmul(acc, x), c)
    return acc


def xpoly_eval_at_b(coeffs: Sequence[XFE], x: int) -> XFE:
    acc = X_ZERO
    for c in reversed(coeffs):
        acc = xadd(xscale(acc, x), c)
    return acc


def bpoly_mul(a: Sequence[int], b: Sequence[int]) -> List[int]:
    if not a or not b:
        return []
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                out[i + j] = (out[i + j] + x * y) % P
    return out


def xpoly_mul(a: Sequence[XFE], b: Sequence[XFE]) -> List[XFE]:
    if not a or not b:
        return []
    out = [X_ZERO] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            out[i + j] = xadd(out[i + j], xmul(x, y))
    return out


def poly_scale_arg(coeffs, s: int, is_x: bool):
    """p(X) -> p(s X)."""
    out, sp = [], 1
    for c in coeffs:
        out.append(xscale(c, sp) if is_x else c * sp % P)
        sp = sp * s % P
    return out


def ntt(vals: List[int], root: int) -> List[int]:
    """Evaluate (in place semantics) the polynomial with coefficients vals at root^i."""
    n = len(vals)
    if n == 1:
        return list(vals)
    ev = ntt(vals[0::2], root * root % P)
    od = ntt(vals[1::2], root * root % P)
    out = [0] * n
    w = 1
    for i in range(n // 2):
        t = w * od[i] % P
        out[i] = (ev[i] + t) % P
        out[i + n // 2] = (ev[i] - t) % P
        w = w * root % P
    return out


def coset_evaluate_b(coeffs: Sequence[int], dom: Domain) -> List[int]:
    c = list(coeffs) + [0] * (dom.length - len(coeffs))
    assert len(c) == dom.length, "polynomial longer than domain"
    c = poly_scale_arg(c, dom.offset, False)
    return ntt(c, dom.generator)


def coset_evaluate_x(coeffs: Sequence[XFE], dom: Domain) -> List[XFE]:
    cols = [coset_evaluate_b([c[k] for c in coeffs], dom) for k in range(3)]
    return list(zip(cols[0], cols[1], cols[2]))


def interpolate_subgroup_x(vals: Sequence[XFE]) -> List[XFE]:
    """Coefficients of the polynomial taking vals[i] at w^i, w = primitive root of len(vals)."""
    n = len(vals)
    w_inv = binv(primitive_root_of_unity(n))
    n_inv = binv(n)
    cols = []
    for k in range(3):
        c = ntt([v[k] for v in vals], w_inv)
        cols.append([x * n_inv % P for x in c])
    return list(zip(cols[0], cols[1], cols[2]))


def barycentric_evaluate(codeword: Sequence[XFE], x: XFE) -> XFE:
    """Value at x of the polynomial interpolating codeword on the subgroup <w> (no offset):
    f(x) = (x^n - 1)/n * sum_i w^i f_i / (x - w^i)  (triton-vm `barycentric_evaluate`)."""
    n = len(codeword)
    w = primitive_root_of_unity(n)
    pts = []
    wi = 1
    for _ in range(n):
        pts.append(wi)
        wi = wi * w % P
    dens = xbatch_inv([xsub(x, lift(g)) for g in pts])
    num = X_ZERO
    den = X_ZERO
    for g, f, d in zip(pts, codeword, dens):
        t = xscale(d, g)
        num = xadd(num, xmul(t, f))
        den = xadd(den, t)
    return xmul(num, xinv(den))


def xpoly_degree(coeffs: Sequence[XFE]) -> int:
    d = len(coeffs) - 1
    while d >= 0 and coeffs[d] == X_ZERO:
        d -= 1
    return d
