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

__host__ __device__ __forceinline__ Xfe x_mul(Xfe a, Xfe b) {
    const uint64_t p00 = mont_mul(a.c0, b.c0);
    const uint64_t c1 = gl_add(mont_mul(a.c0, b.c1), mont_mul(a.c1, b.c0));
    const uint64_t c2 = gl_add(gl_add(mont_mul(a.c0, b.c2), mont_mul(a.c1, b.c1)), mont_mul(a.c2, b.c0));
    const uint64_t c3 = gl_add(mont_mul(a.c1, b.c2), mont_mul(a.c2, b.c1));
    const uint64_t c4 = mont_mul(a.c2, b.c2);
    return {gl_sub(p00, c3), gl_sub(gl_add(c1, c3), c4), gl_add(c2, c4)};
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
