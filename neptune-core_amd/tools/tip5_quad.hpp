// Tip5 permutation in the "quad" layout: one 16-word state spread over 4 lanes of a wave, the
// circulant MDS on the f64 matrix cores.
//
// Same function as tip5_permute_raw (twenty-first 1.0.0 `Tip5::permutation`, crate pinned at
// /root/reference/Cargo.lock:4297; KAT-V / KAT-F pinned), different mapping onto gfx950:
//
//  * State n of a wave lives in lanes {n, n+16, n+32, n+48}; lane q*16+n holds the 4 words
//    quad_word(q, 0..3) = {q, 4+3q, 5+3q, 6+3q}.  Every lane therefore owns exactly one S-box
//    lookup word (words 0..3) and three x^7 words: no divergence, a quarter of the registers.
//  * MDS: out[i] = sum_j MDS[(i-j)&15] * in[j] on the raw words, as two exact integer products
//    (32-bit halves x 16-bit coefficients, sums < 2^52) done by v_mfma_f64_16x16x4_f64: B[k][n] is
//    lane (k, n)'s slot-r word half, A_r[m][k] = MDS[(sigma(m) - quad_word(k, r)) & 15] with the
//    row permutation sigma chosen so that D's row layout ((lane>>4) + 4*reg) lands output word
//    quad_word(q, reg) in lane q's slot reg - the next round needs no data movement.  The
//    accumulator starts at 2^52, so every partial sum is an integer in [2^52, 2^53) (ulp 1: exact)
//    and the integer is the low 52 bits of the f64's bit pattern.  This replaces 512
//    v_mad_u64_u32 per state-round with 8 MFMAs per 16 states + 16 conversions/masks per lane.
//  * The recombination s = al + ah * 2^32 -> raw word and the round-constant add are the same
//    carry chains as mds_ark(), so every intermediate word is bit-identical to the reference's.
#pragma once
#include "tip5_device.hpp"

namespace nhip {

typedef double f64x4_t __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int quad_word(int q, int slot) { return slot == 0 ? q : 3 + 3 * q + slot; }

__constant__ static uint32_t c_tip5_mds[16] = {61402, 1108,  28750, 33823, 7454,  43244, 53865, 12034,
                                               56951, 27521, 41351, 40901, 12021, 59689, 26798, 17845};

// LDS: byte table + per-(round, slot, q) negated round constants (p - rc, raw).
struct Tip5QuadLds {
    uint8_t lut[256];
    uint64_t nrc[TIP5_ROUNDS][4][4];
};

__device__ __forceinline__ void tip5_quad_lds_init(Tip5QuadLds& lds) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lds.lut[i] = TIP5_LUT[i];
    for (int i = threadIdx.x; i < TIP5_ROUNDS * 16; i += blockDim.x) {
        const int r = i >> 4, slot = (i >> 2) & 3, q = i & 3;
        lds.nrc[r][slot][q] = GL_P - c_tip5_rc_raw[r * 16 + quad_word(q, slot)];
    }
    __syncthreads();
}

// This lane's entries of the 4 A matrices (row m = lane & 15, column k = lane >> 4).
struct Tip5QuadMat {
    double a[4];
};

__device__ __forceinline__ Tip5QuadMat tip5_quad_mat() {
    const int l = threadIdx.x & 63, m = l & 15, k = l >> 4;
    const int row_word = quad_word(m & 3, m >> 2);
    Tip5QuadMat A;
#pragma unroll
    for (int r = 0; r < 4; ++r) A.a[r] = (double)c_tip5_mds[(row_word - quad_word(k, r)) & 15];
    return A;
}

static constexpr double F64_2P52 = 4503599627370496.0;
static constexpr uint64_t LOW52 = (1ull << 52) - 1;

// One permutation.  w: this lane's 4 raw words (slots); q = (lane & 63) >> 4.  All 64 lanes of
// the wave must execute it (the MFMA reads every lane).
__device__ __forceinline__ void tip5_permute_quad(uint64_t w[4], const Tip5QuadMat& A, const Tip5QuadLds& lds,
                                                  uint32_t q) {
#pragma unroll 1
    for (int r = 0; r < TIP5_ROUNDS; ++r) {
        w[0] = split_and_lookup(lds.lut, w[0]);
        {
            uint64_t x2[3], x4[3], x3[3];
            mont_mul_n<3>(w + 1, w + 1, x2);
            mont_mul_n<3>(x2, x2, x4);
            mont_mul_n<3>(w + 1, x2, x3);
            mont_mul_n<3>(x3, x4, w + 1);
        }
        f64x4_t accl = {F64_2P52, F64_2P52, F64_2P52, F64_2P52};
        f64x4_t acch = accl;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#if NHIP_QUAD_NO_MFMA
            accl[s] = (double)(uint32_t)w[s] + A.a[s];
            acch[s] = (double)(uint32_t)(w[s] >> 32);
#else
            accl = __builtin_amdgcn_mfma_f64_16x16x4f64(A.a[s], (double)(uint32_t)w[s], accl, 0, 0, 0);
            acch = __builtin_amdgcn_mfma_f64_16x16x4f64(A.a[s], (double)(uint32_t)(w[s] >> 32), acch, 0, 0, 0);
#endif
        }
        uint64_t al[4], ah[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            al[s] = (uint64_t)__double_as_longlong(accl[s]) & LOW52;
            ah[s] = (uint64_t)__double_as_longlong(acch[s]) & LOW52;
        }
        // recombination + ARK: the carry chains of mds_ark() on 4 words
        uint32_t m1[4], sh[4], rl[4], rh[4], tl[4], th[4];
        unsigned int k[4], b[4], over[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) m1[i] = __builtin_addc((uint32_t)(al[i] >> 32), (uint32_t)ah[i], 0u, &k[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) sh[i] = (uint32_t)(ah[i] >> 32) + k[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) tl[i] = __builtin_subc(0u, sh[i], 0u, &b[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            unsigned int dummy;
            th[i] = __builtin_subc(sh[i], 0u, b[i], &dummy);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) rl[i] = __builtin_addc((uint32_t)al[i], tl[i], 0u, &k[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) rh[i] = __builtin_addc(m1[i], th[i], k[i], &over[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) rl[i] = __builtin_addc(rl[i], 0u - over[i], 0u, &k[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) rh[i] = rh[i] + k[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t nq = lds.nrc[r][i][q];
            rl[i] = __builtin_subc(rl[i], (uint32_t)nq, 0u, &b[i]);
            rh[i] = __builtin_subc(rh[i], (uint32_t)(nq >> 32), b[i], &over[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) rl[i] = __builtin_subc(rl[i], 0u - over[i], 0u, &b[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = ((uint64_t)(rh[i] - b[i]) << 32) | rl[i];
    }
}

}  // namespace nhip
