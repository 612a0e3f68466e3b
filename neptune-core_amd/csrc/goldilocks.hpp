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

__host__ __device__ __forceinline__ uint64_t mont_mul(uint64_t a, uint64_t b) {
    return montyred(a * b, mulhi64(a, b));
}

__host__ __device__ __forceinline__ uint64_t mont_sqr(uint64_t a) { return mont_mul(a, a); }

// a + b mod p for a, b in [0, p)
__host__ __device__ __forceinline__ uint64_t gl_add(uint64_t a, uint64_t b) {
    const uint64_t s = a + b;
    const bool ovf = s < a;
    uint64_t t = ovf ? s + GL_EPS : s;  // wrap: 2^64 == 2^32 - 1 (mod p); cannot overflow again
    return t >= GL_P ? t - GL_P : t;
}

// a - b mod p for a, b in [0, p)
__host__ __device__ __forceinline__ uint64_t gl_sub(uint64_t a, uint64_t b) {
    const uint64_t d = a - b;
    return a < b ? d + GL_P : d;
}

// Any u64 (BFieldElement::new semantics: reduced mod p) -> raw Montgomery word.
__host__ __device__ __forceinline__ uint64_t to_mont(uint64_t x) { return mont_mul(x, GL_R2); }

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
