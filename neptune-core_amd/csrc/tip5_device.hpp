// Tip5 permutation for CDNA4 (gfx950): one 16-word state per lane, held in VGPRs in raw
// Montgomery form; S-box lookup table staged in LDS.
//
// Restates twenty-first 1.0.0 `Tip5::permutation` (crate pinned at /root/reference/Cargo.lock:4297;
// behaviour pinned by KAT-V neptune-core/src/state/wallet/mod.rs:1379-1383 and KAT-F
// neptune-core/test_data/precalculated_pow_solution.json):
//   5 rounds of  { S-box: split-and-lookup of the 8 raw Montgomery LE bytes of state[0..4],
//                          x^7 on state[4..16];
//                  MDS:   out[i] = sum_j MDS[(i-j) & 15] * in[j]   (integer-linear on raw words);
//                  ARK:   state[i] += RC[r*16 + i] }
//
// Sponge conventions used by the kernels (twenty-first `Sponge` for Tip5):
//   FixedLength domain (hash_pair): capacity words state[10..16] = 1 (canonical 1).
//   VariableLength domain (hash_varlen, Fiat-Shamir): state starts all-zero; absorb overwrites
//   state[0..10]; padding appends a single 1 then zeros to a multiple of 10.
#pragma once
#include "goldilocks.hpp"
#include "tip5_constants.h"

namespace nhip {

static constexpr int TIP5_STATE = 16;
static constexpr int TIP5_RATE = 10;
static constexpr int TIP5_ROUNDS = 5;
static constexpr uint64_t MONT_ONE = 0x00000000FFFFFFFFull;  // raw Montgomery word of 1 (= 2^64 mod p)

__constant__ static uint64_t c_tip5_rc_raw[80] = {
#define NHIP_RC(i) TIP5_RC_RAW[i]
    NHIP_RC(0), NHIP_RC(1), NHIP_RC(2), NHIP_RC(3), NHIP_RC(4), NHIP_RC(5), NHIP_RC(6), NHIP_RC(7),
    NHIP_RC(8), NHIP_RC(9), NHIP_RC(10), NHIP_RC(11), NHIP_RC(12), NHIP_RC(13), NHIP_RC(14), NHIP_RC(15),
    NHIP_RC(16), NHIP_RC(17), NHIP_RC(18), NHIP_RC(19), NHIP_RC(20), NHIP_RC(21), NHIP_RC(22), NHIP_RC(23),
    NHIP_RC(24), NHIP_RC(25), NHIP_RC(26), NHIP_RC(27), NHIP_RC(28), NHIP_RC(29), NHIP_RC(30), NHIP_RC(31),
    NHIP_RC(32), NHIP_RC(33), NHIP_RC(34), NHIP_RC(35), NHIP_RC(36), NHIP_RC(37), NHIP_RC(38), NHIP_RC(39),
    NHIP_RC(40), NHIP_RC(41), NHIP_RC(42), NHIP_RC(43), NHIP_RC(44), NHIP_RC(45), NHIP_RC(46), NHIP_RC(47),
    NHIP_RC(48), NHIP_RC(49), NHIP_RC(50), NHIP_RC(51), NHIP_RC(52), NHIP_RC(53), NHIP_RC(54), NHIP_RC(55),
    NHIP_RC(56), NHIP_RC(57), NHIP_RC(58), NHIP_RC(59), NHIP_RC(60), NHIP_RC(61), NHIP_RC(62), NHIP_RC(63),
    NHIP_RC(64), NHIP_RC(65), NHIP_RC(66), NHIP_RC(67), NHIP_RC(68), NHIP_RC(69), NHIP_RC(70), NHIP_RC(71),
    NHIP_RC(72), NHIP_RC(73), NHIP_RC(74), NHIP_RC(75), NHIP_RC(76), NHIP_RC(77), NHIP_RC(78), NHIP_RC(79),
#undef NHIP_RC
};

// K = RC + 2^32 - 1 per round constant: the value mds_ark's folded reduction starts the low MDS
// accumulator with (kept as a table so the addition is not redone on the vector unit every round)
__constant__ static uint64_t c_tip5_rck_raw[80] = {
#define NHIP_RC(i) (TIP5_RC_RAW[i] + 0xFFFFFFFFull)
    NHIP_RC(0), NHIP_RC(1), NHIP_RC(2), NHIP_RC(3), NHIP_RC(4), NHIP_RC(5), NHIP_RC(6), NHIP_RC(7),
    NHIP_RC(8), NHIP_RC(9), NHIP_RC(10), NHIP_RC(11), NHIP_RC(12), NHIP_RC(13), NHIP_RC(14), NHIP_RC(15),
    NHIP_RC(16), NHIP_RC(17), NHIP_RC(18), NHIP_RC(19), NHIP_RC(20), NHIP_RC(21), NHIP_RC(22), NHIP_RC(23),
    NHIP_RC(24), NHIP_RC(25), NHIP_RC(26), NHIP_RC(27), NHIP_RC(28), NHIP_RC(29), NHIP_RC(30), NHIP_RC(31),
    NHIP_RC(32), NHIP_RC(33), NHIP_RC(34), NHIP_RC(35), NHIP_RC(36), NHIP_RC(37), NHIP_RC(38), NHIP_RC(39),
    NHIP_RC(40), NHIP_RC(41), NHIP_RC(42), NHIP_RC(43), NHIP_RC(44), NHIP_RC(45), NHIP_RC(46), NHIP_RC(47),
    NHIP_RC(48), NHIP_RC(49), NHIP_RC(50), NHIP_RC(51), NHIP_RC(52), NHIP_RC(53), NHIP_RC(54), NHIP_RC(55),
    NHIP_RC(56), NHIP_RC(57), NHIP_RC(58), NHIP_RC(59), NHIP_RC(60), NHIP_RC(61), NHIP_RC(62), NHIP_RC(63),
    NHIP_RC(64), NHIP_RC(65), NHIP_RC(66), NHIP_RC(67), NHIP_RC(68), NHIP_RC(69), NHIP_RC(70), NHIP_RC(71),
    NHIP_RC(72), NHIP_RC(73), NHIP_RC(74), NHIP_RC(75), NHIP_RC(76), NHIP_RC(77), NHIP_RC(78), NHIP_RC(79),
#undef NHIP_RC
};

// LDS copy of the byte lookup table, one per workgroup.  256 B = 64 dwords: a random byte
// gather from a wave touches at most 2 distinct dwords per bank for ds_read_u8 (bank = dword % 32).
struct Tip5Lds {
    uint8_t lut[256];
};

// L(x) = (x + 1)^3 - 1 mod 257: twenty-first's tip5::LOOKUP_TABLE, equal to the table TIP5_LUT for
// every x (checked at compile time below).  Computing the entries per thread instead of loading
// them measured within noise in round 3 (-0.9% at 4,096 proofs, +1% at 512): the table load stays.
__host__ __device__ constexpr uint32_t tip5_lut_entry(uint32_t x) {
    return ((((x + 1u) * (x + 1u)) % 257u * (x + 1u)) % 257u + 256u) % 257u;
}
constexpr bool tip5_lut_formula_matches_table() {
    for (uint32_t x = 0; x < 256; ++x)
        if (tip5_lut_entry(x) != TIP5_LUT[x]) return false;
    return true;
}
static_assert(tip5_lut_formula_matches_table(), "L(x) = (x+1)^3 - 1 mod 257 is the Tip5 lookup table");

__device__ __forceinline__ void tip5_lds_init(Tip5Lds& lds) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lds.lut[i] = TIP5_LUT[i];
    __syncthreads();
}

// The four looked-up bytes packed by a shift / or chain.  Packing them with two v_perm_b32 and one
// v_or_b32 instead (16 fewer regular VALU per round) ran config 4 1.4% slower (profiles/r03i).
__device__ __forceinline__ uint32_t lookup4(const uint8_t* __restrict__ lut, uint32_t w) {
    const uint32_t b0 = lut[w & 0xFFu];
    const uint32_t b1 = lut[(w >> 8) & 0xFFu];
    const uint32_t b2 = lut[(w >> 16) & 0xFFu];
    const uint32_t b3 = lut[w >> 24];
    return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}

__device__ __forceinline__ uint64_t split_and_lookup(const uint8_t* __restrict__ lut, uint64_t r) {
    const uint32_t lo = lookup4(lut, (uint32_t)r);
    const uint32_t hi = lookup4(lut, (uint32_t)(r >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t pow7(uint64_t x) {
    const uint64_t x2 = mont_sqr(x);
    const uint64_t x4 = mont_sqr(x2);
    const uint64_t x3 = mont_mul(x, x2);
    return mont_mul(x3, x4);
}

// x -> x^7 on 12 words, NHIP_POW7_GROUP words at a time (stage-interleaved Montgomery
// products: wider groups fill more carry-chain wait states but hold more VGPRs).  3: the Merkle
// level kernel fits 95 VGPRs (5 waves per SIMD instead of 4 at 6), config 4 +1%
// (profiles/r02h/ab_g3/).
#ifndef NHIP_POW7_GROUP
#define NHIP_POW7_GROUP 3
#endif
// u = a1 * b0 + t as a 65-bit sum for three products: u (64 bits) and its carry c (0 / 1), with
// v_mad_u64_u32's carry-out read by v_cndmask two instructions later (gfx950's two wait states).
__device__ __forceinline__ void mad_carry3(const uint32_t* a1, const uint32_t* b0, const uint64_t* t, uint64_t* u,
                                           uint32_t* c) {
    uint64_t g0, g1, g2;
    asm("v_mad_u64_u32 %0, %6, %9, %12, %15\n\t"
        "v_mad_u64_u32 %1, %7, %10, %13, %16\n\t"
        "v_mad_u64_u32 %2, %8, %11, %14, %17\n\t"
        "v_cndmask_b32_e64 %3, 0, 1, %6\n\t"
        "v_cndmask_b32_e64 %4, 0, 1, %7\n\t"
        "v_cndmask_b32_e64 %5, 0, 1, %8"
        : "=&v"(u[0]), "=&v"(u[1]), "=&v"(u[2]), "=v"(c[0]), "=v"(c[1]), "=v"(c[2]), "=&s"(g0), "=&s"(g1),
          "=&s"(g2)
        : "v"(a1[0]), "v"(a1[1]), "v"(a1[2]), "v"(b0[0]), "v"(b0[1]), "v"(b0[2]), "v"(t[0]), "v"(t[1]), "v"(t[2]));
}

// N independent Montgomery products (N a multiple of 3), the same words as mont_mul.  The 128-bit
// product's middle column is summed as u = a1*b0 + t with t = a0*b1 + (p00 >> 32) taken whole
// (u's low half is the product's bits 32..63 as before; its top 33 bits are t's and the old u's
// high halves together), so xh = a1*b1 + (u >> 32, carry): two multiply-adds whose 64-bit addends
// no longer need a 32-bit half zero-extended into a fresh register pair (gfx950 64-bit operands are
// even-aligned pairs: one v_mov each), and no separate xh add.
template <int N>
__device__ __forceinline__ void mont_mul_n_dev(const uint64_t* a, const uint64_t* b, uint64_t* out) {
    static_assert(N % 3 == 0, "groups of three");
    uint64_t p00[N], t[N], u[N], xh[N];
    uint32_t a1[N], b0[N], c[N];
    uint32_t ah[N], e[N], bl[N], bh[N], rl[N], rh[N], c1[N], cc[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        a1[i] = (uint32_t)(a[i] >> 32);
        b0[i] = (uint32_t)b[i];
        p00[i] = (uint64_t)(uint32_t)a[i] * b0[i];
    }
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = (uint64_t)(uint32_t)a[i] * (uint32_t)(b[i] >> 32) + (p00[i] >> 32);
#pragma unroll
    for (int i = 0; i < N; i += 3) mad_carry3(a1 + i, b0 + i, t + i, u + i, c + i);
#pragma unroll
    for (int i = 0; i < N; ++i)
        xh[i] = (uint64_t)a1[i] * (uint32_t)(b[i] >> 32) + (((uint64_t)c[i] << 32) | (uint32_t)(u[i] >> 32));
    // montyred, as mont_mul (stage by stage across the N products)
#pragma unroll
    for (int i = 0; i < N; ++i) ah[i] = __builtin_addc((uint32_t)u[i], (uint32_t)p00[i], 0u, &e[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        unsigned int br1;
        bl[i] = __builtin_subc((uint32_t)p00[i], ah[i], e[i], &br1);
        e[i] = br1;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        unsigned int br2;
        bh[i] = __builtin_subc(ah[i], 0u, e[i], &br2);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) rl[i] = __builtin_subc((uint32_t)xh[i], bl[i], 0u, &c1[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) rh[i] = __builtin_subc((uint32_t)(xh[i] >> 32), bh[i], c1[i], &cc[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        unsigned int c2;
        const uint32_t lo = __builtin_subc(rl[i], 0u - cc[i], 0u, &c2);
        out[i] = ((uint64_t)(rh[i] - c2) << 32) | lo;
    }
}

template <int G>
__device__ __forceinline__ void pow7_mul(const uint64_t* a, const uint64_t* b, uint64_t* out) {
    mont_mul_n_dev<G>(a, b, out);
}

__device__ __forceinline__ void pow7_12(uint64_t* x) {
    constexpr int G = NHIP_POW7_GROUP;
    static_assert(12 % G == 0, "group must divide 12");
#pragma unroll
    for (int g = 0; g < 12; g += G) {
        uint64_t x2[G], x4[G], x3[G];
        pow7_mul<G>(x + g, x + g, x2);
        pow7_mul<G>(x2, x2, x4);
        pow7_mul<G>(x + g, x2, x3);
        pow7_mul<G>(x3, x4, x + g);
    }
}

// MDS + ARK.  Circulant 16x16 with small (< 2^16) coefficients applied to the raw words: each
// word is split into 32-bit halves and the two half-products are accumulated exactly in 64 bits
// (< 2^53) by v_mad_u64_u32; the round constant and the reduction are folded (below).  The
// step-by-step form twenty-first writes (reduce, then add the constant) is kept as the reference
// of tests/native/mds_fold_check.cpp and as the latency forms' mds_reduce_ark_lat.
// Four words of mds_ark's folded reduction: w = sh * (2^32 - 1) + s_lo with the multiply-add's
// carry-out G (bit 64 of the sum), and e = G ? 0 : 2^32 - 1.  Written as assembly because the
// compiler cannot keep v_mad_u64_u32's carry-out as a lane mask; each v_cndmask reads its mask
// three instructions after the multiply-add that wrote it (gfx950 wants two wait states between a
// VALU SGPR write and a VALU read of it).
__device__ __forceinline__ void mds_fold4(const uint32_t* sh, const uint64_t* slo, uint64_t* w, uint32_t* e) {
    uint64_t g0, g1, g2, g3;
    asm("v_mad_u64_u32 %0, %8, %12, -1, %16\n\t"
        "v_mad_u64_u32 %1, %9, %13, -1, %17\n\t"
        "v_mad_u64_u32 %2, %10, %14, -1, %18\n\t"
        "v_mad_u64_u32 %3, %11, %15, -1, %19\n\t"
        "v_cndmask_b32_e64 %4, -1, 0, %8\n\t"
        "v_cndmask_b32_e64 %5, -1, 0, %9\n\t"
        "v_cndmask_b32_e64 %6, -1, 0, %10\n\t"
        "v_cndmask_b32_e64 %7, -1, 0, %11"
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=v"(e[0]), "=v"(e[1]), "=v"(e[2]), "=v"(e[3]),
          "=&s"(g0), "=&s"(g1), "=&s"(g2), "=&s"(g3)
        : "v"(sh[0]), "v"(sh[1]), "v"(sh[2]), "v"(sh[3]), "v"(slo[0]), "v"(slo[1]), "v"(slo[2]), "v"(slo[3]));
}

// MDS + ARK with the round constant folded into the accumulators.  For twenty-first's steps above
// (y = reduce(s), then the field add y + rc), the result is the canonical representative of
// s + rc mod p whenever rc < p - 2^32 + 2, which every Tip5 round constant satisfies: if y >= q
// the add gives y - q = y + rc - p < p, else y + rc < p.  So: accumulate s'' = s + K with
// K = rc + 2^32 - 1 (K starts the low accumulator: every Tip5 constant has K < 2^64 - 2^52, so
// it never overflows), W = s''_lo + s''_hi * (2^32 - 1)
// (= s'' mod p, 65 bits); if W >= 2^64 the result is W - 2^64 (= W - (2^32 - 1) - p, < 2^54),
// else W - (2^32 - 1) (in [0, p): s'' >= 2^32 - 1 keeps W >= 2^32 - 1).  6 VALU instructions per
// word after the accumulation instead of 15 (checked against the step-by-step form for every Tip5
// round constant and 3 x 10^6 other in-range constants: tests/native/mds_fold_check.cpp).
// rc: the round's 16 constants; rck: the same round's K = rc + 2^32 - 1 (c_tip5_rck_raw).
// mds_ark's folded form over the first NIN state words (the others are known constants whose MDS
// contribution the caller has folded into rck, see tip5_hash_pair_digest).
// [OBEG, OEND) != [0, 16): only those outputs are computed (a digest read after the last round,
// or the capacity words a sponge keeps when the next absorb overwrites the rate).
__device__ __forceinline__ uint64_t mds_reduce_fold(uint64_t al, uint64_t ah);
// Outputs I0 .. I0 + N of the folded MDS (accumulate, then reduce four words at a time).
template <int NIN, int I0, int N>
__device__ __forceinline__ void mds_fold_outputs(const uint32_t* lo, const uint32_t* hi,
                                                 const uint64_t* __restrict__ rck, uint64_t* out) {
    uint64_t al[N], ah[N];
#pragma unroll
    for (int o = 0; o < N; ++o) {
        const int i = I0 + o;
        al[o] = rck[i];  // < 2^64 - 2^52 for every Tip5 constant: al never overflows
        ah[o] = 0;
#pragma unroll
        for (int j = 0; j < NIN; ++j) {
            const uint64_t c = TIP5_MDS[(i - j) & 15];
            al[o] += c * lo[j];
            ah[o] += c * hi[j];
        }
    }
    constexpr int N4 = N & ~3;
    uint32_t sh[N4 > 0 ? N4 : 1];
    uint64_t slo[N4 > 0 ? N4 : 1], w[N4 > 0 ? N4 : 1];
    uint32_t e[N4 > 0 ? N4 : 1];
#pragma unroll
    for (int o = 0; o < N4; ++o) {
        unsigned int k;
        const uint32_t m1 = __builtin_addc((uint32_t)(al[o] >> 32), (uint32_t)ah[o], 0u, &k);
        sh[o] = (uint32_t)(ah[o] >> 32) + k;
        slo[o] = ((uint64_t)m1 << 32) | (uint32_t)al[o];
    }
#pragma unroll
    for (int o = 0; o < N4; o += 4) mds_fold4(sh + o, slo + o, w + o, e + o);
#pragma unroll
    for (int o = 0; o < N4; ++o) out[o] = w[o] - e[o];
#pragma unroll
    for (int o = N4; o < N; ++o) out[o] = mds_reduce_fold(al[o], ah[o]);
}

// G < 16: the outputs are finished G at a time, a scheduling barrier between groups, so that only
// one group's accumulators are live (fewer VGPRs at the MDS peak).  NHIP_PAIR_MDS_GROUP: hash_pair
// (the Merkle level kernels); NHIP_SPONGE_MDS_GROUP: the sponge permutations (row hashing).
#ifndef NHIP_PAIR_MDS_GROUP
#define NHIP_PAIR_MDS_GROUP 2
#endif
#ifndef NHIP_SPONGE_MDS_GROUP
#define NHIP_SPONGE_MDS_GROUP 4
#endif
template <int NIN, int OBEG, int OEND, int G>
__device__ __forceinline__ void mds_fold_groups(const uint32_t* lo, const uint32_t* hi,
                                                const uint64_t* __restrict__ rck, uint64_t* out) {
    constexpr int N = (OEND - OBEG) < G ? (OEND - OBEG) : G;
    mds_fold_outputs<NIN, OBEG, N>(lo, hi, rck, out);
    if constexpr (OBEG + N < OEND) {
        __builtin_amdgcn_sched_barrier(0);
        mds_fold_groups<NIN, OBEG + N, OEND, G>(lo, hi, rck, out + N);
    }
}

template <int NIN, int OBEG = 0, int OEND = 16, int G = 16>
__device__ __forceinline__ void mds_ark_fold(uint64_t s[16], const uint64_t* __restrict__ rck) {
    uint32_t lo[NIN], hi[NIN];
#pragma unroll
    for (int j = 0; j < NIN; ++j) {
        lo[j] = (uint32_t)s[j];
        hi[j] = (uint32_t)(s[j] >> 32);
    }
    uint64_t out[OEND - OBEG];
    mds_fold_groups<NIN, OBEG, OEND, G>(lo, hi, rck, out);
#pragma unroll
    for (int o = 0; o < OEND - OBEG; ++o) s[OBEG + o] = out[o];
}

template <int G = NHIP_SPONGE_MDS_GROUP>
__device__ __forceinline__ void mds_ark(uint64_t s[16], const uint64_t* __restrict__ rc,
                                        const uint64_t* __restrict__ rck) {
    (void)rc;
    mds_ark_fold<16, 0, 16, G>(s, rck);
}

// One permutation on a raw Montgomery state.
__device__ __forceinline__ void tip5_permute_raw(uint64_t s[16], const uint8_t* __restrict__ lut) {
#pragma unroll 1
    for (int r = 0; r < TIP5_ROUNDS; ++r) {
#pragma unroll
        for (int i = 0; i < 4; ++i) s[i] = split_and_lookup(lut, s[i]);
        pow7_12(s + 4);
        mds_ark(s, c_tip5_rc_raw + r * 16, c_tip5_rck_raw + r * 16);
    }
}


// FixedLength-domain (hash_pair) round-0 accumulator starts: K = RC + 2^32 - 1 plus the MDS
// contribution of the six capacity words, which enter round 0 as 1 (raw MONT_ONE = 2^32 - 1: low
// half 2^32 - 1, high half 0) and leave its S-box as 1 (1^7 = 1).  The integer sum s of a round is
// the same whichever part of it starts the accumulator, so the words the permutation produces are
// bit-identical to tip5_permute_raw on a state whose words 10..15 are MONT_ONE.
__host__ __device__ constexpr uint64_t tip5_rck0_fixed(int i) {
    uint64_t k = TIP5_RC_RAW[i] + 0xFFFFFFFFull;
    for (int j = 10; j < 16; ++j) k += (uint64_t)TIP5_MDS[(i - j) & 15] * 0xFFFFFFFFull;
    return k;
}
constexpr bool tip5_rck0_fixed_in_range() {  // the accumulator bound mds_ark relies on
    for (int i = 0; i < 16; ++i)
        if (tip5_rck0_fixed(i) >= 0xFFF0000000000000ull || tip5_rck0_fixed(i) < TIP5_RC_RAW[i]) return false;
    return true;
}
static_assert(tip5_rck0_fixed_in_range(), "round-0 FixedLength accumulator start below 2^64 - 2^52");
__constant__ static uint64_t c_tip5_rck0_fixed[16] = {
    tip5_rck0_fixed(0),  tip5_rck0_fixed(1),  tip5_rck0_fixed(2),  tip5_rck0_fixed(3),
    tip5_rck0_fixed(4),  tip5_rck0_fixed(5),  tip5_rck0_fixed(6),  tip5_rck0_fixed(7),
    tip5_rck0_fixed(8),  tip5_rck0_fixed(9),  tip5_rck0_fixed(10), tip5_rck0_fixed(11),
    tip5_rck0_fixed(12), tip5_rck0_fixed(13), tip5_rck0_fixed(14), tip5_rck0_fixed(15),
};

// Tip5::hash_pair's permutation (FixedLength domain) on s[0..10] = left, right digests (raw),
// producing the digest s[0..5] (the rest of the state is not the permutation's: callers read the
// digest only).  The capacity words 10..15 are 1 on entry and are not read.  Round 0 runs x^7 on words 4..9 only and
// the MDS over 10 inputs (the capacity's share is in c_tip5_rck0_fixed); rounds 1-4 as
// tip5_permute_raw, the last of them computing the digest words only.  Round 0: 552 fewer VALU
// instructions (6 x^7 chains of 4 Montgomery products, 6 x 16 x 2 MDS multiply-adds); round 4: ~420
// fewer (11 of 16 MDS outputs).
__device__ __forceinline__ void tip5_hash_pair_digest(uint64_t s[16], const uint8_t* __restrict__ lut) {
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = split_and_lookup(lut, s[i]);
#pragma unroll
    for (int g = 4; g < 10; g += 3) {
        uint64_t x2[3], x4[3], x3[3];
        pow7_mul<3>(s + g, s + g, x2);
        pow7_mul<3>(x2, x2, x4);
        pow7_mul<3>(s + g, x2, x3);
        pow7_mul<3>(x3, x4, s + g);
    }
    mds_ark_fold<10, 0, 16, NHIP_PAIR_MDS_GROUP>(s, c_tip5_rck0_fixed);
#pragma unroll 1
    for (int r = 1; r < TIP5_ROUNDS - 1; ++r) {
#pragma unroll
        for (int i = 0; i < 4; ++i) s[i] = split_and_lookup(lut, s[i]);
        pow7_12(s + 4);
        mds_ark<NHIP_PAIR_MDS_GROUP>(s, c_tip5_rc_raw + r * 16, c_tip5_rck_raw + r * 16);
    }
    // last round: the caller reads the digest s[0..5] only, so the MDS computes those 5 outputs
    // (11 x 16 x 2 multiply-adds and 11 reductions fewer); s[5..16] are left stale
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = split_and_lookup(lut, s[i]);
    pow7_12(s + 4);
    mds_ark_fold<16, 0, 5, NHIP_PAIR_MDS_GROUP>(s, c_tip5_rck_raw + (TIP5_ROUNDS - 1) * 16);
}

// Rounds 0..3 of the permutation, then the last round computing only the state words
// [OBEG, OEND) (the sponge's kept words): hash_varlen's absorbs overwrite the rate s[0..10], so a
// permutation followed by another absorb needs s[10..16] only (<10, 16>: 10 x 16 x 2 multiply-adds
// and 10 reductions fewer), and the one before the digest is read needs s[0..5] (<0, 5>).
__device__ __forceinline__ void tip5_rounds_0_3(uint64_t s[16], const uint8_t* __restrict__ lut) {
#pragma unroll 1
    for (int r = 0; r < TIP5_ROUNDS - 1; ++r) {
#pragma unroll
        for (int i = 0; i < 4; ++i) s[i] = split_and_lookup(lut, s[i]);
        pow7_12(s + 4);
        mds_ark(s, c_tip5_rc_raw + r * 16, c_tip5_rck_raw + r * 16);
    }
}
// The last round's S-box layer; the caller then keeps the MDS outputs it needs
// (tip5_last_mds<OBEG, OEND>).  A caller choosing between two output ranges at run time branches on
// the MDS only: with the whole last round in each branch the row kernel needed ~40 more VGPRs.
__device__ __forceinline__ void tip5_last_sbox(uint64_t s[16], const uint8_t* __restrict__ lut) {
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = split_and_lookup(lut, s[i]);
    pow7_12(s + 4);
}
template <int OBEG, int OEND>
__device__ __forceinline__ void tip5_last_mds(uint64_t s[16]) {
    mds_ark_fold<16, OBEG, OEND, NHIP_SPONGE_MDS_GROUP>(s, c_tip5_rck_raw + (TIP5_ROUNDS - 1) * 16);
}
template <int OBEG, int OEND>
__device__ __forceinline__ void tip5_last_round(uint64_t s[16], const uint8_t* __restrict__ lut) {
    tip5_last_sbox(s, lut);
    tip5_last_mds<OBEG, OEND>(s);
}

}  // namespace nhip

namespace nhip {

// MDS reduction + round-constant add of one word, for the latency-bound row forms below: the same
// steps as mds_ark() (s = al + ah * 2^32; (res, over) = s_lo.overflowing_add(s_hi * (2^32 - 1));
// y = res + over * (2^32 - 1); x1 = y - q with q = p - rc; + p on borrow), written with 64-bit sums
// and two VCC tests instead of carry chains through SGPRs (see mont_mul_lat): nq = -q mod 2^64,
// x1 = y + nq, and the borrow of y - q is x1 > y (q >= 1).  Checked against the step-by-step form
// on 2 x 10^8 random and boundary inputs; the GPU tests compare every sample with the oracle.
__device__ __forceinline__ uint64_t mds_reduce_ark_lat(uint64_t al, uint64_t ah, uint64_t nq) {
    const uint64_t w = (uint64_t)(uint32_t)(al >> 32) + (uint32_t)ah;
    const uint32_t sh = (uint32_t)(ah >> 32) + (uint32_t)(w >> 32);
    const uint64_t slo = ((uint64_t)(uint32_t)w << 32) | (uint32_t)al;
    const uint64_t res = slo + (uint64_t)sh * 0xFFFFFFFFull;
    const uint64_t y = res + (res < slo ? GL_EPS : 0ull);
    const uint64_t x1 = y + nq;
    return x1 + (x1 > y ? GL_P : 0ull);
}

// mds_ark's folded reduction for one word (the row forms): al started at K = rc + 2^32 - 1.  One chain per lane, so the mask read waits out the two wait states itself.
__device__ __forceinline__ uint64_t mds_reduce_fold(uint64_t al, uint64_t ah) {
    unsigned int k;
    const uint32_t m1 = __builtin_addc((uint32_t)(al >> 32), (uint32_t)ah, 0u, &k);
    const uint32_t sh = (uint32_t)(ah >> 32) + k;
    const uint64_t slo = ((uint64_t)m1 << 32) | (uint32_t)al;
    uint64_t w, g;
    uint32_t e;
    asm("v_mad_u64_u32 %0, %2, %3, -1, %4\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %1, -1, 0, %2"
        : "=&v"(w), "=v"(e), "=&s"(g)
        : "v"(sh), "v"(slo));
    return w - e;
}

// LAT = true: the carry-light arithmetic (mont_mul_lat, mds_reduce_ark_lat) for callers bound by one
// permutation's latency (small batches); false: the fewer-instruction carry-chain form for callers
// that share the SIMDs with other work (the sponge replay of large batches, the wide Merkle levels).
// Measured (A/B, tools/ab_latform.sh): carry-light rows cut the one-collection resident verify
// 1.63 -> 1.44 ms but cost 0.7-2% at 512 / 4,096 proofs, whose row-form work is issue-bound.
template <bool LAT>
__device__ __forceinline__ uint64_t mont_mul_sel(uint64_t a, uint64_t b) {
    if constexpr (LAT) return mont_mul_lat(a, b);
    else return mont_mul(a, b);
}

// ---------------------------------------------------------------------------------------------
// "Wide" Tip5: one state spread over a 16-lane DPP row (lane e of the row holds state[e]).
// Used where latency, not throughput, matters (the sequential Fiat-Shamir sponge of one proof):
// a permutation costs ~10x fewer dependent instructions than the lane-per-state form.  The
// circulant MDS becomes 16 row rotations (`row_ror:k`, DPP) with one uniform coefficient MDS[k]
// per rotation: lane e receives state[(e - k) & 15] and out[e] = sum_k MDS[k] * state[e - k].
// ---------------------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ uint32_t row_ror(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + K, 0xF, 0xF, false);
}

template <int K>
__device__ __forceinline__ void mds_term(uint32_t lo, uint32_t hi, uint64_t& al, uint64_t& ah) {
    const uint64_t c = TIP5_MDS[K];
    al += c * row_ror<K>(lo);
    ah += c * row_ror<K>(hi);
}

// s: this lane's state word (raw Montgomery); e: lane index within the row; rc: this lane's 5
// round constants (raw).
template <bool LAT>
__device__ __forceinline__ uint64_t tip5_permute_wide(uint64_t s, uint32_t e, const uint64_t rc[5],
                                                      const uint8_t* __restrict__ lut) {
#pragma unroll
    for (int r = 0; r < TIP5_ROUNDS; ++r) {
        // S-box: split-and-lookup on lanes 0..3, x^7 elsewhere.  Straight-line on every lane (the
        // row runs both paths either way): the LDS lookups are issued first and their latency
        // hides behind the x^7 chain; the lane picks its result at the end.
        {
            const uint64_t lk = split_and_lookup(lut, s);
            const uint64_t x2 = mont_mul_sel<LAT>(s, s);
            const uint64_t x4 = mont_mul_sel<LAT>(x2, x2);
            const uint64_t x3 = mont_mul_sel<LAT>(s, x2);
            const uint64_t x7 = mont_mul_sel<LAT>(x3, x4);
            s = e < 4 ? lk : x7;
        }
        // MDS over the row
        const uint32_t lo = (uint32_t)s, hi = (uint32_t)(s >> 32);
        uint64_t al, ah;
        if constexpr (LAT) {
            al = (uint64_t)TIP5_MDS[0] * lo;
            ah = (uint64_t)TIP5_MDS[0] * hi;
        } else {  // the round constant folded into the sums (mds_reduce_fold)
            al = (uint64_t)TIP5_MDS[0] * lo + (rc[r] + GL_EPS);
            ah = (uint64_t)TIP5_MDS[0] * hi;
        }
        mds_term<1>(lo, hi, al, ah);
        mds_term<2>(lo, hi, al, ah);
        mds_term<3>(lo, hi, al, ah);
        mds_term<4>(lo, hi, al, ah);
        mds_term<5>(lo, hi, al, ah);
        mds_term<6>(lo, hi, al, ah);
        mds_term<7>(lo, hi, al, ah);
        mds_term<8>(lo, hi, al, ah);
        mds_term<9>(lo, hi, al, ah);
        mds_term<10>(lo, hi, al, ah);
        mds_term<11>(lo, hi, al, ah);
        mds_term<12>(lo, hi, al, ah);
        mds_term<13>(lo, hi, al, ah);
        mds_term<14>(lo, hi, al, ah);
        mds_term<15>(lo, hi, al, ah);
        // recombination + ARK, the same words as mds_ark()
        if constexpr (LAT) s = mds_reduce_ark_lat(al, ah, 0ull - (GL_P - rc[r]));
        else s = mds_reduce_fold(al, ah);
    }
    return s;
}

// ---------------------------------------------------------------------------------------------
// "Pair" Tip5 (small batches only: always the carry-light arithmetic): one state on two 16-lane DPP rows (rows 2r and 2r+1 of a wave; lane e of both rows
// holds state[e], so both rows keep the whole state).  The rows split each round's work, which
// cuts the dependent instructions per round by about a quarter (for the sequential Fiat-Shamir
// sponge of small batches, where most SIMDs are idle anyway):
//   * S-box: row h looks up dword h of the lookup words; x2 = x^2 on both rows, then ONE product
//     stream computes x^4 = x2*x2 on row 0 and x^3 = x*x2 on row 1 (operands chosen per row), and
//     x^7 = x^4 * x^3 after one v_permlane16_swap (gfx950) hands each row the other's value;
//   * MDS: row 0 takes rotations 0..7, row 1 rotations 8..15 (its input pre-rotated by 8, per-row
//     coefficients cm[]), the two partial sums are added across the rows with v_permlane16_swap
//     (exact: every partial sum < 2^53), so al / ah are the one-row form's integers;
//   * recombination + ARK as tip5_permute_wide, on both rows.
// cm[j] = MDS[j + 8h]; h = row parity.
// ---------------------------------------------------------------------------------------------
// (row 0's x, row 1's x) of a 64-bit value, on both rows of the pair
__device__ __forceinline__ void row_pair(uint64_t x, uint64_t& r0, uint64_t& r1) {
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)x, (uint32_t)x, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(x >> 32), (uint32_t)(x >> 32), false, false);
    r0 = ((uint64_t)hi[0] << 32) | lo[0];
    r1 = ((uint64_t)hi[1] << 32) | lo[1];
}

template <int K>
__device__ __forceinline__ void mds_term_pair(uint32_t lo, uint32_t hi, uint32_t c, uint64_t& al, uint64_t& ah) {
    al += (uint64_t)c * row_ror<K>(lo);
    ah += (uint64_t)c * row_ror<K>(hi);
}

__device__ __forceinline__ uint64_t tip5_permute_pair(uint64_t s, uint32_t e, uint32_t h, const uint64_t rc[5],
                                                      const uint32_t cm[8], const uint8_t* __restrict__ lut) {
#pragma unroll
    for (int r = 0; r < TIP5_ROUNDS; ++r) {
        // S-box
        const uint32_t lk_mine = lookup4(lut, h ? (uint32_t)(s >> 32) : (uint32_t)s);
        const uint64_t x2 = mont_mul_lat(s, s);
        const uint64_t m = mont_mul_lat(h ? s : x2, x2);  // row 0: x^4, row 1: x^3
        uint64_t mr0, mr1;
        row_pair(m, mr0, mr1);
        const uint64_t x7 = mont_mul_lat(mr0, mr1);
        const auto lk = __builtin_amdgcn_permlane16_swap(lk_mine, lk_mine, false, false);
        s = e < 4 ? (((uint64_t)lk[1] << 32) | lk[0]) : x7;
        // MDS: half of the rotations per row
        const uint32_t lo0 = (uint32_t)s, hi0 = (uint32_t)(s >> 32);
        const uint32_t lo8 = row_ror<8>(lo0), hi8 = row_ror<8>(hi0);
        const uint32_t lo = h ? lo8 : lo0, hi = h ? hi8 : hi0;
        uint64_t al = (uint64_t)cm[0] * lo, ah = (uint64_t)cm[0] * hi;
        mds_term_pair<1>(lo, hi, cm[1], al, ah);
        mds_term_pair<2>(lo, hi, cm[2], al, ah);
        mds_term_pair<3>(lo, hi, cm[3], al, ah);
        mds_term_pair<4>(lo, hi, cm[4], al, ah);
        mds_term_pair<5>(lo, hi, cm[5], al, ah);
        mds_term_pair<6>(lo, hi, cm[6], al, ah);
        mds_term_pair<7>(lo, hi, cm[7], al, ah);
        uint64_t a0, a1, b0, b1;
        row_pair(al, a0, a1);
        row_pair(ah, b0, b1);
        al = a0 + a1;
        ah = b0 + b1;
        // recombination + ARK, the same words as mds_ark()
        s = mds_reduce_ark_lat(al, ah, 0ull - (GL_P - rc[r]));
    }
    return s;
}

// ---------------------------------------------------------------------------------------------
// "Quad" Tip5 (the sponge replay of large batches): one state on the 4 lanes of a DPP quad, lane e
// holding words e, e + 4, e + 8, e + 12 in slots 0..3.  Every lane then has one split-and-lookup
// word (slot 0) and three x^7 words (slots 1..3), so no lane computes an S-box result it throws
// away (the 16-lane row computes both on every lane), and the three x^7 chains are the lane form's
// three-product groups.  MDS: output slot k of lane e is word i = e + 4k; writing the circulant's
// shift as m = 4a + b, the b = 0 terms are the lane's own slots (k - a) & 3 with the uniform
// coefficient MDS[4a]; for b = 1..3 the term is slot (k - a) & 3 of lane (e - b) & 3 when e >= b,
// and slot (k - a - 1) & 3 of that lane when e < b.  With X^b = the lane (e - b) & 3 slots (one
// quad_perm DPP move per dword) the slot is (k - a') & 3 for both cases once the coefficient is
// per lane: cq[b - 1][a'] = MDS[(4a' + b - 4 [e < b]) & 15].  16 terms per output as in the lane
// form (128 multiply-adds per lane and round), then mds_ark's folded reduction four words at a
// time.  Per round and lane ~380 VALU (1,520 per state, 1.08x the lane form's, vs 2,400 for the
// 16-lane row) at a quarter of the lane form's dependent instructions.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void tip5_quad_coefs(uint32_t e, uint32_t cq[3][4]) {
#pragma unroll
    for (int b = 1; b < 4; ++b)
#pragma unroll
        for (int a = 0; a < 4; ++a) cq[b - 1][a] = TIP5_MDS[(4 * a + b - (e < (uint32_t)b ? 4 : 0)) & 15];
}

// lane e of the quad reads lane (e - B) & 3: quad_perm [(0-B)&3, (1-B)&3, (2-B)&3, (3-B)&3]
template <int B>
__device__ __forceinline__ uint32_t quad_from(uint32_t v) {
    constexpr int ctrl = ((0 - B) & 3) | (((1 - B) & 3) << 2) | (((2 - B) & 3) << 4) | (((3 - B) & 3) << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, false);
}

// s: this lane's 4 slots (raw Montgomery); rck: the 80 K = RC + 2^32 - 1 constants (c_tip5_rck_raw
// order, staged in LDS by the caller); e: lane within the quad.
__device__ __forceinline__ void tip5_permute_quad(uint64_t s[4], const uint32_t cq[3][4],
                                                  const uint64_t* __restrict__ rck, uint32_t e,
                                                  const uint8_t* __restrict__ lut) {
#pragma unroll 1
    for (int r = 0; r < TIP5_ROUNDS; ++r) {
        uint64_t al[4], ah[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) al[k] = rck[r * 16 + 4 * k + e];  // LDS, issued before the S-box
        s[0] = split_and_lookup(lut, s[0]);
        {
            uint64_t x2[3], x4[3], x3[3];
            mont_mul_n_dev<3>(s + 1, s + 1, x2);
            mont_mul_n_dev<3>(x2, x2, x4);
            mont_mul_n_dev<3>(s + 1, x2, x3);
            mont_mul_n_dev<3>(x3, x4, s + 1);
        }
        uint32_t lo[4], hi[4], xl[3][4], xh[3][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            lo[k] = (uint32_t)s[k];
            hi[k] = (uint32_t)(s[k] >> 32);
            xl[0][k] = quad_from<1>(lo[k]);
            xh[0][k] = quad_from<1>(hi[k]);
            xl[1][k] = quad_from<2>(lo[k]);
            xh[1][k] = quad_from<2>(hi[k]);
            xl[2][k] = quad_from<3>(lo[k]);
            xh[2][k] = quad_from<3>(hi[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ah[k] = 0;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const uint64_t c = TIP5_MDS[4 * a];
                al[k] += c * lo[(k - a) & 3];
                ah[k] += c * hi[(k - a) & 3];
            }
#pragma unroll
            for (int b = 0; b < 3; ++b)
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    al[k] += (uint64_t)cq[b][a] * xl[b][(k - a) & 3];
                    ah[k] += (uint64_t)cq[b][a] * xh[b][(k - a) & 3];
                }
        }
        // mds_ark's folded reduction (al started at K = RC + 2^32 - 1)
        uint32_t sh[4], e4[4];
        uint64_t slo[4], w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            unsigned int c;
            const uint32_t m1 = __builtin_addc((uint32_t)(al[k] >> 32), (uint32_t)ah[k], 0u, &c);
            sh[k] = (uint32_t)(ah[k] >> 32) + c;
            slo[k] = ((uint64_t)m1 << 32) | (uint32_t)al[k];
        }
        mds_fold4(sh, slo, w, e4);
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] = w[k] - e4[k];
    }
}

}  // namespace nhip
