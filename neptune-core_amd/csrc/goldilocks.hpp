// Goldilocks field p = 2^64 - 2^32 + 1 in Montgomery form (R = 2^64), CDNA4 VALU code.
//
// Mirrors twenty-first 1.0.0 `BFieldElement` (crate pinned at /root/reference/Cargo.lock:4297):
// the element is held as its raw Montgomery word r = x * 2^64 mod p, r in [0, p).  Keeping the
// raw word is required by Tip5, whose S-box looks up the raw bytes (see tip5_device.hpp).
//
// All functions are __host__ __device__ so that host-side helpers (descriptor setup, tests of the
// header itself) use the exact same arithmetic; the hot path is the device code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nhip {

static constexpr uint64_t GL_P = 0xFFFFFFFF00000001ull;
static constexpr uint64_t GL_R2 = 0xFFFFFFFE00000001ull;  // 2^128 mod p (to-Montgomery factor)
static constexpr uint64_t GL_EPS = 0xFFFFFFFFull;         // 2^64 mod p

__host__ __device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// twenty-first `montyred`: (xh:xl) < p * 2^64  ->  (xh:xl) * 2^-64 mod p, in [0, p).
__host__ __device__ __forceinline__ uint64_t montyred(uint64_t xl, uint64_t xh) {
    const uint64_t a = xl + (xl << 32);
    const uint64_t e = a < xl ? 1ull : 0ull;
    const uint64_t b = a - (a >> 32) - e;
    const uint64_t r = xh - b;
    return xh < b ? r - GL_EPS : r;
}

// Montgomery product on 32-bit VALU pieces: 4 v_mad_u64_u32 for the 128-bit product,
// then twenty-first's montyred written as explicit carry chains (v_add_co / v_sub_co / subb),
// 14 VALU instructions in total.
__host__ __device__ __forceinline__ uint64_t mont_mul(uint64_t a, uint64_t b) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
    const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
    const uint64_t v = (uint64_t)a1 * b1 + (t >> 32);
    const uint64_t xh = v + (u >> 32);
    const uint32_t xl0 = (uint32_t)p00, xl1 = (uint32_t)u;
    // a = xl + (xl << 32):  a.lo = xl0, a.hi = xl1 + xl0 (carry e)
    unsigned int e, br1, br2, c1, c, c2;
    const uint32_t ah = __builtin_addc(xl1, xl0, 0u, &e);
    // b = a - (a >> 32) - e
    const uint32_t bl = __builtin_subc(xl0, ah, e, &br1);
    const uint32_t bh = __builtin_subc(ah, 0u, br1, &br2);
    // r = xh - b; if borrow: r -= 2^32 - 1
    uint32_t rl = __builtin_subc((uint32_t)xh, bl, 0u, &c1);
    uint32_t rh = __builtin_subc((uint32_t)(xh >> 32), bh, c1, &c);
    const uint32_t m = 0u - c;
    rl = __builtin_subc(rl, m, 0u, &c2);
    rh = rh - c2;
    return ((uint64_t)rh << 32) | rl;
}

__host__ __device__ __forceinline__ uint64_t mont_sqr(uint64_t a) { return mont_mul(a, a); }

// The same product for latency-bound code (one dependent chain per lane: the sponge replay's row
// Tip5).  A carry passed from one VALU instruction to the next through an SGPR pair costs ~14 cycles
// on gfx950 (two mandatory wait states; neptune-core_amd/tools/valu_latency.hip), and montyred above
// has five such links.  Here the sums are 64-bit values (v_mad_u64_u32 / v_lshl_add_u64, no carry
// flags) and only the final sign test goes through VCC.  Exactly montyred's result for any 64-bit
// inputs: with s = l0 + l1 (33 bits, e = s >> 32) and M = s_lo * (2^32 - 1) + l0, twenty-first's
// b = a - (a >> 32) - e equals M - e (>= 0), so r = xh - b = E - M with E = xh + e (no overflow:
// xh <= 2^64 - 2), + p when E < M.  More instructions (22 vs 17), ~half the dependent latency.
__host__ __device__ __forceinline__ uint64_t mont_mul_lat(uint64_t a, uint64_t b) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p00 = (uint64_t)a0 * b0;
    const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
    const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
    const uint64_t v = (uint64_t)a1 * b1 + (t >> 32);
    const uint64_t xh = v + (u >> 32);
    const uint64_t l0 = (uint32_t)p00, l1 = (uint32_t)u;
    const uint64_t sum = l1 + l0;
    const uint64_t M = (uint64_t)(uint32_t)sum * 0xFFFFFFFFull + l0;
    const uint64_t E = (sum >> 32) + xh;
    const bool neg = E < M;
    return (E + ~M) + (neg ? GL_P + 1 : 1ull);
}

// a + b mod p for a, b in [0, p).  The sum a + b < 2p needs one subtraction of p exactly when it
// carries out of 64 bits or is >= p, and s - p == s + (2^32 - 1) mod 2^64, so one select of
// s + EPS does both cases (8 VALU instead of 11: the carry flag is the add's own).
__host__ __device__ __forceinline__ uint64_t gl_add(uint64_t a, uint64_t b) {
    unsigned int c0, c1;
    const uint32_t s0 = __builtin_addc((uint32_t)a, (uint32_t)b, 0u, &c0);
    const uint32_t s1 = __builtin_addc((uint32_t)(a >> 32), (uint32_t)(b >> 32), c0, &c1);
    const uint64_t s = ((uint64_t)s1 << 32) | s0;
    return (c1 || s >= GL_P) ? s + GL_EPS : s;
}

// a - b mod p for a, b in [0, p)
__host__ __device__ __forceinline__ uint64_t gl_sub(uint64_t a, uint64_t b) {
    const uint64_t d = a - b;
    return a < b ? d + GL_P : d;
}

// Any u64 (BFieldElement::new semantics: reduced mod p) -> raw Montgomery word x * 2^64 mod p.
// With x = h * 2^32 + l and 2^64 == 2^32 - 1 (mod p):  x * 2^64 == l * 2^32 - h - l, and that
// integer lies in (-2^33, p - 1], so one conditional + p makes it canonical: the same word as
// mont_mul(x, 2^128 mod p) in ~7 VALU instead of a Montgomery product (tests/test_constants.py
// and the CPU test of this header check the identity).
__host__ __device__ __forceinline__ uint64_t to_mont(uint64_t x) {
    const uint32_t l = (uint32_t)x, h = (uint32_t)(x >> 32);
    const uint64_t s = (uint64_t)h + l;
    const uint64_t t = (uint64_t)l << 32;
    const uint64_t v = t - s;
    return t < s ? v + GL_P : v;
}
__host__ __device__ __forceinline__ uint64_t to_mont_mul(uint64_t x) { return mont_mul(x, GL_R2); }

// Raw Montgomery word -> canonical value (BFieldElement::value()).
__host__ __device__ __forceinline__ uint64_t from_mont(uint64_t r) { return montyred(r, 0); }

// Reduce an 85-bit quantity lo + hi * 2^64 (hi < 2^32) mod p, result in [0, p).
__host__ __device__ __forceinline__ uint64_t reduce96(uint64_t lo, uint32_t hi) {
    // hi * 2^64 == hi * (2^32 - 1)  (mod p)
    const uint64_t t = ((uint64_t)hi << 32) - (uint64_t)hi;
    uint64_t s = lo + t;
    if (s < lo) s += GL_EPS;  // carry out of 2^64
    return s >= GL_P ? s - GL_P : s;
}

}  // namespace nhip
