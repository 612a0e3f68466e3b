// Cubic extension XFieldElement = F_p[x] / (x^3 - x + 1) on top of the Montgomery Goldilocks
// field (goldilocks.hpp).  Coefficients are raw Montgomery words.  Mirrors twenty-first 1.0.0
// `XFieldElement` (Cargo.lock:4297); multiplication uses x^3 = x - 1, x^4 = x^2 - x.
#pragma once
#include "goldilocks.hpp"

namespace nhip {

struct Xfe {
    uint64_t c0, c1, c2;
};

static constexpr uint64_t MONT_ONE_W = 0x00000000FFFFFFFFull;  // raw word of 1

__host__ __device__ __forceinline__ Xfe x_zero() { return {0, 0, 0}; }
__host__ __device__ __forceinline__ Xfe x_one() { return {MONT_ONE_W, 0, 0}; }
__host__ __device__ __forceinline__ Xfe x_lift(uint64_t b) { return {b, 0, 0}; }

__host__ __device__ __forceinline__ Xfe x_add(Xfe a, Xfe b) {
    return {gl_add(a.c0, b.c0), gl_add(a.c1, b.c1), gl_add(a.c2, b.c2)};
}
__host__ __device__ __forceinline__ Xfe x_sub(Xfe a, Xfe b) {
    return {gl_sub(a.c0, b.c0), gl_sub(a.c1, b.c1), gl_sub(a.c2, b.c2)};
}
__host__ __device__ __forceinline__ Xfe x_scale(Xfe a, uint64_t s) {
    return {mont_mul(a.c0, s), mont_mul(a.c1, s), mont_mul(a.c2, s)};
}
__host__ __device__ __forceinline__ bool x_eq(Xfe a, Xfe b) { return a.c0 == b.c0 && a.c1 == b.c1 && a.c2 == b.c2; }

// Lazily reduced products: montyred is linear, so sum_k mont_mul(a_k, b_k) == the Montgomery
// reduction of sum_k a_k * b_k (mod p).  x_mul forms its nine 128-bit products, adds them per output
// coefficient in 160 bits and reduces three times instead of nine (plus eight modular sums):
// ~200 VALU per product instead of ~230 (gfx950 ISA count).  Negative terms are taken as
// + 2p * 2^64 - t, which leaves the reduction unchanged and keeps the sums non-negative.
struct U128 {
    uint64_t lo, hi;
};
struct U160 {
    uint64_t lo, hi;
    uint32_t top;
};

__host__ __device__ __forceinline__ U128 mul128(uint64_t a, uint64_t b) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
    const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
    const uint64_t v = (uint64_t)a1 * b1 + (t >> 32);
    return {(u << 32) | (uint32_t)p00, v + (u >> 32)};
}

// x + y with the carry out of 128 bits added to x's top word
__host__ __device__ __forceinline__ U160 add160(U160 x, U128 y) {
    unsigned int c0, c1, c2, c3;
    const uint32_t l0 = __builtin_addc((uint32_t)x.lo, (uint32_t)y.lo, 0u, &c0);
    const uint32_t l1 = __builtin_addc((uint32_t)(x.lo >> 32), (uint32_t)(y.lo >> 32), c0, &c1);
    const uint32_t h0 = __builtin_addc((uint32_t)x.hi, (uint32_t)y.hi, c1, &c2);
    const uint32_t h1 = __builtin_addc((uint32_t)(x.hi >> 32), (uint32_t)(y.hi >> 32), c2, &c3);
    return {((uint64_t)l1 << 32) | l0, ((uint64_t)h1 << 32) | h0, x.top + c3};
}
__host__ __device__ __forceinline__ U160 wide(U128 x) { return {x.lo, x.hi, 0u}; }

// x + 2p * 2^64 - y  (non-negative for every y this file forms: y < 2p * 2^64)
__host__ __device__ __forceinline__ U160 sub160_2p(U160 x, U160 y) {
    unsigned int c0, c1, b0, b1, b2, b3;
    // 2p = 2^65 - 2^33 + 2: hi += 2^64 - 2^33 + 2, top += 1
    const uint32_t h0 = __builtin_addc((uint32_t)x.hi, 2u, 0u, &c0);
    const uint32_t h1 = __builtin_addc((uint32_t)(x.hi >> 32), 0xFFFFFFFEu, c0, &c1);
    const uint32_t l0 = __builtin_subc((uint32_t)x.lo, (uint32_t)y.lo, 0u, &b0);
    const uint32_t l1 = __builtin_subc((uint32_t)(x.lo >> 32), (uint32_t)(y.lo >> 32), b0, &b1);
    const uint32_t g0 = __builtin_subc(h0, (uint32_t)y.hi, b1, &b2);
    const uint32_t g1 = __builtin_subc(h1, (uint32_t)(y.hi >> 32), b2, &b3);
    return {((uint64_t)l1 << 32) | l0, ((uint64_t)g1 << 32) | g0, x.top + 1u + c1 - y.top - b3};
}

// (top * 2^128 + hi * 2^64 + lo) * 2^-64 mod p, in [0, p): the high part is folded below 2^64
// (2^64 == 2^32 - 1 mod p), then montyred as in mont_mul, whose result for a high word past p is
// still correct mod p and at most one p above the canonical value.
__host__ __device__ __forceinline__ uint64_t red160(U160 x) {
    const uint64_t tt = ((uint64_t)x.top << 32) - x.top;
    uint64_t h = x.hi + tt;
    if (h < tt) h += GL_EPS;
    const uint32_t xl0 = (uint32_t)x.lo, xl1 = (uint32_t)(x.lo >> 32);
    unsigned int e, br1, br2, c1, c, c2;
    const uint32_t ah = __builtin_addc(xl1, xl0, 0u, &e);
    const uint32_t bl = __builtin_subc(xl0, ah, e, &br1);
    const uint32_t bh = __builtin_subc(ah, 0u, br1, &br2);
    uint32_t rl = __builtin_subc((uint32_t)h, bl, 0u, &c1);
    uint32_t rh = __builtin_subc((uint32_t)(h >> 32), bh, c1, &c);
    const uint32_t m = 0u - c;
    rl = __builtin_subc(rl, m, 0u, &c2);
    rh = rh - c2;
    const uint64_t r = ((uint64_t)rh << 32) | rl;
    return r >= GL_P ? r - GL_P : r;
}

// (a0 + a1 x + a2 x^2)(b0 + b1 x + b2 x^2) with x^3 = x - 1, x^4 = x^2 - x:
//   c0 = a0b0 - (a1b2 + a2b1),  c1 = a0b1 + a1b0 + (a1b2 + a2b1) - a2b2,  c2 = a0b2 + a1b1 + a2b0 + a2b2
__host__ __device__ __forceinline__ Xfe x_mul(Xfe a, Xfe b) {
    // three groups of three products, each group's coefficient reduced before the next group's
    // products are formed: fewer live 128-bit values (k_ood_air 121 -> 97 VGPRs, k_deep_rows8's
    // spill 96 -> 56 bytes per lane), the same instructions.  The 128-bit products with
    // v_mad_u64_u32's carry-out (mad_carry3, tip5_device.hpp: ~180 instead of ~200 VALU per XFE
    // product) measured -1.1% at 4,096 proofs, the OOD kernel's dependent chain longer (ab_r04l).
    const U128 p12 = mul128(a.c1, b.c2), p21 = mul128(a.c2, b.c1), p00 = mul128(a.c0, b.c0);
    const U160 n = add160(wide(p12), p21);  // < 2p^2
    Xfe r;
    r.c0 = red160(sub160_2p(wide(p00), n));
    const U128 p01 = mul128(a.c0, b.c1), p10 = mul128(a.c1, b.c0), p22 = mul128(a.c2, b.c2);
    U160 s1 = add160(add160(wide(p01), p10), U128{n.lo, n.hi});
    s1.top += n.top;
    r.c1 = red160(sub160_2p(s1, wide(p22)));
    const U128 p02 = mul128(a.c0, b.c2), p11 = mul128(a.c1, b.c1), p20 = mul128(a.c2, b.c0);
    r.c2 = red160(add160(add160(add160(wide(p02), p11), p20), p22));
    return r;
}

// x^(2^n) (n successive Montgomery squarings)
__host__ __device__ __forceinline__ uint64_t b_sqn(uint64_t x, int n) {
#pragma unroll 1
    for (int i = 0; i < n; ++i) x = mont_mul(x, x);
    return x;
}

// base-field inverse a^(p-2) (a != 0; 0 -> 0), Montgomery in/out.  Addition chain for
// p - 2 = (2^32 - 2) * 2^32 + (2^32 - 1): 63 squarings + 9 products (square-and-multiply over the
// 63 one-bits of p - 2 would take 125).
__host__ __device__ __forceinline__ uint64_t b_inv(uint64_t a) {
    const uint64_t t2 = mont_mul(mont_mul(a, a), a);         // a^(2^2 - 1)
    const uint64_t t3 = mont_mul(mont_mul(t2, t2), a);       // a^(2^3 - 1)
    const uint64_t t6 = mont_mul(b_sqn(t3, 3), t3);          // a^(2^6 - 1)
    const uint64_t t12 = mont_mul(b_sqn(t6, 6), t6);         // a^(2^12 - 1)
    const uint64_t t15 = mont_mul(b_sqn(t12, 3), t3);        // a^(2^15 - 1)
    const uint64_t t30 = mont_mul(b_sqn(t15, 15), t15);      // a^(2^30 - 1)
    const uint64_t t31 = mont_mul(mont_mul(t30, t30), a);    // a^(2^31 - 1)
    const uint64_t t32m2 = mont_mul(t31, t31);               // a^(2^32 - 2)
    const uint64_t t32 = mont_mul(t32m2, a);                 // a^(2^32 - 1)
    return mont_mul(b_sqn(t32m2, 32), t32);                  // a^(p - 2)
}

__host__ __device__ __forceinline__ uint64_t b_pow(uint64_t a, uint64_t e) {
    uint64_t r = MONT_ONE_W;
    while (e) {
        if (e & 1) r = mont_mul(r, a);
        a = mont_mul(a, a);
        e >>= 1;
    }
    return r;
}

// Inverse via the adjugate of the multiplication matrix (first row of cofactors / determinant).
// Returns zero for zero (caller checks).
__host__ __device__ __forceinline__ Xfe x_inv(Xfe a) {
    const uint64_t s = gl_add(a.c0, a.c2);  // a0 + a2
    const uint64_t d = gl_sub(a.c1, a.c2);  // a1 - a2
    const uint64_t C00 = gl_sub(mont_mul(s, s), mont_mul(d, a.c1));
    const uint64_t C01 = gl_sub(mont_mul(d, a.c2), mont_mul(a.c1, s));
    const uint64_t C02 = gl_sub(mont_mul(a.c1, a.c1), mont_mul(s, a.c2));
    const uint64_t det = gl_sub(gl_sub(mont_mul(a.c0, C00), mont_mul(a.c2, C01)), mont_mul(a.c1, C02));
    const uint64_t di = b_inv(det);
    return {mont_mul(C00, di), mont_mul(C01, di), mont_mul(C02, di)};
}

__host__ __device__ __forceinline__ Xfe x_pow(Xfe a, uint64_t e) {
    Xfe r = x_one();
    while (e) {
        if (e & 1) r = x_mul(r, a);
        a = x_mul(a, a);
        e >>= 1;
    }
    return r;
}

}  // namespace nhip
