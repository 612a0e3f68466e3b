// Phase kernels of the batched STARK verifier (see stark.hpp for the phase list).
//
// Conventions: the batch word buffer holds the proof words as the caller gave them (any u64, in the
// batch's input form: canonical values or twenty-first's Montgomery words; every kernel that reads
// it is instantiated for both, MW = Montgomery) and the staged claims in the same form; every load
// of a field element from it goes through word_mont<MW> (proof_codec.hpp), structural words through
// word_value<MW> in the decoder.  Every
// scratch value written by these kernels (samples, row digests, OOD sums) is a raw Montgomery word.  Each failed check ORs a FailBits bit into fail[proof].
#include <hip/hip_ext.h>

#include <atomic>
#include <cstdlib>

#include "../../include/nhip_challenge_id.h"
#include "kernels.hpp"
#include "proof_codec.hpp"
#include "stark.hpp"
#include "tip5_device.hpp"
#include "xfe.hpp"

namespace nhip {

// Wave priority of the latency-bound kernels (decode, the Fiat-Shamir sponge, the Merkle plan,
// the small top Merkle levels, OOD, FRI): their waves share SIMDs with the VALU-bound hashing of
// the same and the other in-flight steps, and the SIMD arbitrates VALU issue by wave priority,
// then age.  Raising it lets a dependent chain issue as soon as it can, while the throughput
// kernels fill the remaining slots.  NHIP_LAT_PRIO (0..3) selects it at build time.
#ifndef NHIP_LAT_PRIO
#define NHIP_LAT_PRIO 2
#endif
__device__ __forceinline__ void latency_priority() {
    if constexpr (NHIP_LAT_PRIO > 0) __builtin_amdgcn_s_setprio(NHIP_LAT_PRIO);
}
// Oldest-first wave priority: the AGE_PRIO_OLDEST oldest batch launches in flight on the device run
// their row hashing and Merkle levels one priority level above their kernel's base (the sponge
// replay keeps its own), so the in-flight steps drift apart (the oldest finishes first) instead of
// moving through their phases in lockstep.  Measured
// (profiles/r05z/ab/age_prio_ab_r05w.txt, 3 alternating repetitions per run): config 4 in the
// driver's 20 steps at 4,096 proofs +1.4%, 2,048 +0.9%, 1,024 and 512 equal, so from
// AGE_PRIO_MIN_PROOFS on.  Raising the sponge replay too (NHIP_AGE_PRIO_FS=1): 512 -1 to -2% (round 5);
// 4,096 +0.6% and 2,048 equal, within the run-to-run spread (round 6, once the quad launch took
// age_sponge: round 5's 4,096 arms were the same code; profiles/r06/ab_age_prio_fs.txt), so it stays off.  g_batches_done counts the
// device's finished batch launches (k_verdicts); a launch's seq is its place in the device's launch
// order.
static constexpr uint32_t AGE_PRIO_OLDEST = 2;
static constexpr uint32_t AGE_PRIO_MIN_PROOFS = 2048;
__device__ uint32_t g_batches_done;
struct AgePrio {
    uint32_t seq, k;
};
__device__ __forceinline__ void age_priority(AgePrio a, int base) {
    bool old = false;
    if (a.k) {  // uniform: a kernel argument
        const uint32_t done = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&g_batches_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        old = (int32_t)(a.seq - done) < (int32_t)a.k;
    }
    switch (base + (old ? 1 : 0)) {
        case 0: break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}
// wave priority of the lane-per-op Merkle level kernel (the level chain is each step's critical
// path once its sponge replay is done; the row hashing has slack)
#ifndef NHIP_MP_PRIO
#define NHIP_MP_PRIO 1
#endif


// an XFE of the batch word buffer as raw Montgomery coefficients (either input form)
template <bool MW>
__device__ __forceinline__ Xfe ld_xfe_w(const uint64_t* __restrict__ w, uint64_t off) {
    return {word_mont<MW>(w[off]), word_mont<MW>(w[off + 1]), word_mont<MW>(w[off + 2])};
}
__device__ __forceinline__ Xfe ld_xfe_raw(const uint64_t* __restrict__ w, uint64_t off) {
    return {w[off], w[off + 1], w[off + 2]};
}
__device__ __forceinline__ void st_xfe_raw(uint64_t* __restrict__ w, uint64_t off, Xfe v) {
    w[off] = v.c0;
    w[off + 1] = v.c1;
    w[off + 2] = v.c2;
}
__device__ __forceinline__ bool x_is_zero(Xfe a) { return (a.c0 | a.c1 | a.c2) == 0; }

// primitive root of unity of order 2^k (raw Montgomery): 7^((p-1) / 2^k)
__device__ __forceinline__ uint64_t root_of_unity(uint32_t log2n) {
    return b_pow(to_mont(7), (GL_P - 1) >> log2n);
}

// ------------------------------------------------------------------ proof-stream decode
// One wave per proof: lane 0 walks the proof stream (decode_stream, proof_codec.hpp: the item
// headers form a dependent chain of ~20-70 wave-uniform loads), writing the descriptor into LDS and
// the Fiat-Shamir program into the proof's slot; the wave then scans the last FRI polynomial for
// its degree (lane-parallel: a prover can pad it with zero coefficients) and copies the descriptor
// out.  Every run of a batch decodes again from the raw words in HBM, so the device phases never
// depend on host-side parsing.  fail[p] is (re)initialised here: FAIL_DECODE or 0.
template <bool MW>
__global__ void __launch_bounds__(64) k_decode(const uint64_t* __restrict__ words, const ProofIn* __restrict__ in,
                                               uint32_t n_proofs, Dims D, uint32_t fs_stride, uint32_t xs_stride,
                                               ProofDesc* __restrict__ desc, FsOp* __restrict__ ops,
                                               uint32_t* __restrict__ fail, unsigned long long* __restrict__ counters) {
    latency_priority();
    __shared__ ProofDesc spd;
    __shared__ uint32_t sfail;
    __shared__ int sdeg;
    const uint32_t p = blockIdx.x, lane = threadIdx.x;
    if (p >= n_proofs) return;
    const ProofIn pin = in[p];
    if (lane == 0) {
        uint64_t perms = 0, perms_lcw = 0;
        const ClaimLoc cl{pin.claim_off, pin.claim_in_n, pin.claim_out_n};
        uint32_t f = decode_stream<MW>(words, pin.off, pin.len, cl, D, spd, ops + (uint64_t)p * fs_stride, perms, perms_lcw);
        if (!f && spd.log2_ph != pin.sized_log2_ph) {  // capacity guard: the batch was sized from the header
            f = FAIL_DECODE;
            spd = ProofDesc{};
            claim_offsets(spd, cl);
        }
        if (!f) {
            atomicAdd(counters + CNT_PERMS_STATIC, (unsigned long long)perms);
            atomicAdd(counters + CNT_PERMS_LCW, (unsigned long long)perms_lcw);
        }
        sfail = f;
        sdeg = -1;
    }
    __syncthreads();
    const uint32_t f = sfail;
    if (!f) {
        // highest non-zero coefficient, 64 coefficients per step from the top (lane 0 = highest)
        int deg = -1;
        for (uint32_t hi = spd.last_poly_n; hi > 0; hi = hi > 64 ? hi - 64 : 0) {
            bool nz = false;
            if (lane < hi) {
                const uint64_t* x = words + spd.last_poly_off + 3ull * (hi - 1 - lane);
                nz = (canon(x[0]) | canon(x[1]) | canon(x[2])) != 0;
            }
            const uint64_t b = __ballot(nz);
            if (b) {
                deg = (int)(hi - (uint32_t)__ffsll((unsigned long long)b));
                break;
            }
        }
        if (lane == 0) sdeg = deg;
    }
    __syncthreads();
    if (lane == 0) {
        if (!f) last_poly_finish(spd, sdeg, D);
        const SampleLayout sl = SampleLayout::of(D.d, spd.R);
        spd.fs_op_off = p * fs_stride;
        spd.xs_off = (uint64_t)p * xs_stride;
        spd.n_xs = f ? 0u : sl.total;
        spd.idx_off = (uint64_t)p * D.d.num_checks;
        fail[p] = f;
    }
    __syncthreads();
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&spd);
    uint64_t* dst = reinterpret_cast<uint64_t*>(desc + p);
    for (uint32_t i = lane; i < sizeof(ProofDesc) / 8; i += 64) dst[i] = src[i];
}

// Same program on the 16-lane "wide" Tip5 (one proof per DPP row, PAIR = false: ~10x lower
// latency per permutation than a lane per proof, which is what a sequential sponge needs), or on
// the two-row "pair" Tip5 (one proof per 32 lanes, PAIR = true: about a quarter fewer dependent
// instructions per permutation again, at ~1.5x the lane-instructions; used for batches small
// enough that the sponge replay is on the critical path with most SIMDs idle).  Both rows of a
// pair hold the same state; only row 0 writes.  (The row form with the carry-light arithmetic was
// measured for the mid sizes and not kept: history §3.)
// (the body, for workgroup bx of the replay's grid: also run by k_fs_rows_small)
template <bool PAIR, bool MW>
__device__ __forceinline__ void fs_replay_wide_body(uint32_t bx, const Tip5Lds& lds, const uint64_t* __restrict__ words,
                                                    const ProofDesc* __restrict__ desc,
                                                    const FsOp* __restrict__ ops, uint32_t n_proofs,
                                                    uint64_t* __restrict__ xs, uint32_t* __restrict__ idx_out,
                                                    const uint32_t* __restrict__ fail) {
    constexpr uint32_t LANES = PAIR ? 32u : 16u;
    const uint32_t e = threadIdx.x & 15u;
    const uint32_t h = PAIR ? (threadIdx.x >> 4) & 1u : 0u;
    const uint32_t g = (bx * blockDim.x + threadIdx.x) / LANES;
    if (g >= n_proofs || fail[g]) return;  // uniform within the proof's lanes
    uint64_t rc[TIP5_ROUNDS];
#pragma unroll
    for (int r = 0; r < TIP5_ROUNDS; ++r) rc[r] = c_tip5_rc_raw[r * 16 + e];
    uint32_t cm[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cm[j] = h ? TIP5_MDS[j + 8] : TIP5_MDS[j];
    auto permute = [&](uint64_t st) {
        if constexpr (PAIR) return tip5_permute_pair(st, e, h, rc, cm, lds.lut);
        else return tip5_permute_wide<false>(st, e, rc, lds.lut);
    };
    const bool writer = h == 0;
    const ProofDesc& d = desc[g];
    uint64_t s = 0;
    uint64_t xcur = d.xs_off * 3;
    uint64_t icur = d.idx_off;
    const uint32_t row_shift = threadIdx.x & (64u - LANES);  // first lane of this proof (row 0) in the wave
    for (uint32_t o = 0; o < d.fs_op_n; ++o) {
        const FsOp op = ops[d.fs_op_off + o];
        if (op.kind == FS_ABSORB) {
            // len / 10 full chunks, then the padded one; each chunk's word is loaded while the
            // previous chunk's permutation runs (the load is off the sponge's critical path)
            const uint64_t* __restrict__ src = words + op.arg;
            const uint32_t len = op.n;
            const uint32_t nchunks = len / TIP5_RATE + 1;
            uint64_t w = (e < TIP5_RATE && e < len) ? src[e] : 0ull;
            for (uint32_t c = 0; c < nchunks; ++c) {
                const uint32_t pos = c * TIP5_RATE;
                const uint64_t cur = w;
                const uint32_t ni = pos + TIP5_RATE + e;
                w = (e < TIP5_RATE && ni < len) ? src[ni] : 0ull;
                if (e < TIP5_RATE) {
                    const uint32_t rem = len - pos;  // >= 10 except in the last chunk
                    s = e < rem ? word_mont<MW>(cur) : (e == rem ? MONT_ONE : 0ull);
                }
                s = permute(s);
            }
        } else if (op.kind == FS_SQUEEZE_X) {
            const uint32_t nwords = 3 * op.n;
            for (uint32_t f = 0; f < nwords; f += TIP5_RATE) {
                if (writer && e < TIP5_RATE && f + e < nwords) xs[xcur + f + e] = s;
                s = permute(s);
            }
            xcur += nwords;
        } else {  // FS_SAMPLE_IDX
            const uint64_t bound = op.arg;
            uint32_t got = 0;
            while (got < op.n) {
                const uint64_t v = from_mont(s);
                s = permute(s);
                const bool valid = e < TIP5_RATE && v != GL_P - 1;
                const uint64_t ball = __ballot(valid);
                const uint32_t bits = (uint32_t)(ball >> row_shift) & 0x3FFu;
                const uint32_t rank = __popc(bits & ((1u << e) - 1u));
                if (writer && valid && got + rank < op.n) idx_out[icur + got + rank] = (uint32_t)((v & 0xFFFFFFFFull) % bound);
                got += __popc(bits);
            }
            icur += op.n;
        }
    }
}
template <bool PAIR, bool MW>
__global__ void __launch_bounds__(256) k_fs_replay_wide(const uint64_t* __restrict__ words,
                                                        const ProofDesc* __restrict__ desc,
                                                        const FsOp* __restrict__ ops, uint32_t n_proofs,
                                                        uint64_t* __restrict__ xs, uint32_t* __restrict__ idx_out,
                                                        const uint32_t* __restrict__ fail, AgePrio age) {
    age_priority(age, NHIP_LAT_PRIO);
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    fs_replay_wide_body<PAIR, MW>(blockIdx.x, lds, words, desc, ops, n_proofs, xs, idx_out, fail);
}

// The same program on the quad Tip5 (tip5_permute_quad: one proof per 4 lanes, ~0.63x the 16-lane
// row's lane-instructions per permutation at ~2.5x its dependent instructions), for large batches
// whose sponge replays run beside the other in-flight step's hashing: the replay then costs fewer
// of the issue slots the hashing needs.  Lane e of a proof's quad holds state words e + 4k (slot k);
// rate word w = e + 4k < 10.  Workgroup size: quad_wg() (how the few replay waves are placed on the
// SIMDs matters more than their count, see there).
#ifndef NHIP_QUAD_PRIO
#define NHIP_QUAD_PRIO NHIP_LAT_PRIO
#endif
template <bool MW>
__global__ void __launch_bounds__(1024) k_fs_replay_quad(const uint64_t* __restrict__ words,
                                                       const ProofDesc* __restrict__ desc,
                                                       const FsOp* __restrict__ ops, uint32_t n_proofs,
                                                       uint64_t* __restrict__ xs, uint32_t* __restrict__ idx_out,
                                                       const uint32_t* __restrict__ fail, AgePrio age) {
    age_priority(age, NHIP_QUAD_PRIO);
    __shared__ Tip5Lds lds;
    __shared__ uint64_t rck[80];
    for (int i = threadIdx.x; i < 80; i += blockDim.x) rck[i] = c_tip5_rck_raw[i];
    tip5_lds_init(lds);  // (its barrier also orders the rck stores)
    const uint32_t e = threadIdx.x & 3u;
    const uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    if (g >= n_proofs || fail[g]) return;  // uniform within the proof's quad
    uint32_t cq[3][4];
    tip5_quad_coefs(e, cq);
    const ProofDesc& d = desc[g];
    uint64_t s[4] = {0, 0, 0, 0};
    uint64_t xcur = d.xs_off * 3;
    uint64_t icur = d.idx_off;
    const uint32_t qb = threadIdx.x & 60u;  // first lane of this quad in its wave
    // slots 0 and 1 are rate words for every lane (words e, 4 + e); slot 2 for lanes 0, 1 (8, 9)
    const bool r2 = e < 2;
    for (uint32_t o = 0; o < d.fs_op_n; ++o) {
        const FsOp op = ops[d.fs_op_off + o];
        if (op.kind == FS_ABSORB) {
            const uint64_t* __restrict__ src = words + op.arg;
            const uint32_t len = op.n;
            const uint32_t nchunks = len / TIP5_RATE + 1;
            uint64_t w0 = e < len ? src[e] : 0ull;
            uint64_t w1 = 4 + e < len ? src[4 + e] : 0ull;
            uint64_t w2 = (r2 && 8 + e < len) ? src[8 + e] : 0ull;
            for (uint32_t c = 0; c < nchunks; ++c) {
                const uint32_t pos = c * TIP5_RATE;
                const uint32_t rem = len - pos;  // >= 10 except in the last chunk
                const uint64_t c0 = w0, c1 = w1, c2 = w2;
                const uint32_t nx = pos + TIP5_RATE;
                w0 = nx + e < len ? src[nx + e] : 0ull;
                w1 = nx + 4 + e < len ? src[nx + 4 + e] : 0ull;
                w2 = (r2 && nx + 8 + e < len) ? src[nx + 8 + e] : 0ull;
                s[0] = e < rem ? word_mont<MW>(c0) : (e == rem ? MONT_ONE : 0ull);
                s[1] = 4 + e < rem ? word_mont<MW>(c1) : (4 + e == rem ? MONT_ONE : 0ull);
                if (r2) s[2] = 8 + e < rem ? word_mont<MW>(c2) : (8 + e == rem ? MONT_ONE : 0ull);
                tip5_permute_quad(s, cq, rck, e, lds.lut);
            }
        } else if (op.kind == FS_SQUEEZE_X) {
            const uint32_t nwords = 3 * op.n;
            for (uint32_t f = 0; f < nwords; f += TIP5_RATE) {
                if (f + e < nwords) xs[xcur + f + e] = s[0];
                if (f + 4 + e < nwords) xs[xcur + f + 4 + e] = s[1];
                if (r2 && f + 8 + e < nwords) xs[xcur + f + 8 + e] = s[2];
                tip5_permute_quad(s, cq, rck, e, lds.lut);
            }
            xcur += nwords;
        } else {  // FS_SAMPLE_IDX: the valid rate words in word order, as k_fs_replay_wide
            const uint64_t bound = op.arg;
            uint32_t got = 0;
            while (got < op.n) {
                const uint64_t v0 = from_mont(s[0]), v1 = from_mont(s[1]), v2 = from_mont(s[2]);
                tip5_permute_quad(s, cq, rck, e, lds.lut);
                const bool ok0 = v0 != GL_P - 1, ok1 = v1 != GL_P - 1, ok2 = r2 && v2 != GL_P - 1;
                const uint64_t b0 = __ballot(ok0), b1 = __ballot(ok1), b2 = __ballot(ok2);
                const uint32_t bits = ((uint32_t)(b0 >> qb) & 0xFu) | (((uint32_t)(b1 >> qb) & 0xFu) << 4) |
                                      (((uint32_t)(b2 >> qb) & 0x3u) << 8);
                auto put = [&](bool ok, uint32_t w, uint64_t v) {
                    const uint32_t rank = __popc(bits & ((1u << w) - 1u));
                    if (ok && got + rank < op.n) idx_out[icur + got + rank] = (uint32_t)((v & 0xFFFFFFFFull) % bound);
                };
                put(ok0, e, v0);
                put(ok1, 4 + e, v1);
                put(ok2, 8 + e, v2);
                got += __popc(bits);
            }
            icur += op.n;
        }
    }
}

// ------------------------------------------------------------------ revealed-row hashing
// grid.y = 0 main, 1 aux, 2 quotient; one lane per (proof, row).
// 5 waves per SIMD: 84 VGPRs, no scratch, with the sponge MDS finished four outputs at a time and
// the last round branching on its MDS only (122-128 VGPRs and 4 waves before): config 4 equal at
// 4,096 proofs, +3.5-5% at 512 (profiles/r03za; 6 waves with pairs: -0.7% at 4,096)
#ifndef NHIP_ROWS_WAVES
#define NHIP_ROWS_WAVES 5
#endif
template <bool MW>
__global__ void __launch_bounds__(256, NHIP_ROWS_WAVES) k_hash_rows(const uint64_t* __restrict__ words, const ProofDesc* __restrict__ desc,
                                                   uint32_t n_proofs, uint32_t k, StarkDims dims,
                                                   uint64_t* __restrict__ dig, const uint32_t* __restrict__ fail,
                                                   AgePrio age) {
    age_priority(age, 0);
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    const uint32_t tree = blockIdx.y;
    const uint32_t width = tree == 0 ? dims.num_main : (tree == 1 ? 3 * dims.num_aux : 3 * dims.num_quot_seg);
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < (uint64_t)n_proofs * k;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = (uint32_t)(t / k), j = (uint32_t)(t % k);
        if (fail[p]) continue;
        const ProofDesc& d = desc[p];
        const uint64_t base = (tree == 0 ? d.main_rows_off : (tree == 1 ? d.aux_rows_off : d.quot_rows_off)) +
                              (uint64_t)j * width;
        const uint64_t* __restrict__ row = words + base;
        uint64_t s[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) s[q] = 0;
        // width / 10 full chunks, then the padded one (always present); the wave's rows are of one
        // tree, so `last` is uniform.  Every permutation but the last is followed by an absorb that
        // overwrites the rate, so its last round computes the capacity words only.
        const uint32_t nchunks = width / TIP5_RATE + 1;
        for (uint32_t c = 0; c < nchunks; ++c) {
            const uint32_t pos = c * TIP5_RATE;
            const bool last = c + 1 == nchunks;
            if (!last) {
#pragma unroll
                for (int q = 0; q < TIP5_RATE; ++q) s[q] = word_mont<MW>(row[pos + q]);
            } else {
                const uint32_t rem = width - pos;
#pragma unroll
                for (int q = 0; q < TIP5_RATE; ++q) {
                    const uint32_t qq = (uint32_t)q;
                    s[q] = qq < rem ? word_mont<MW>(row[pos + qq]) : (qq == rem ? MONT_ONE : 0ull);
                }
            }
            tip5_rounds_0_3(s, lds.lut);
            tip5_last_sbox(s, lds.lut);
            if (!last) tip5_last_mds<10, 16>(s);
            else tip5_last_mds<0, 5>(s);
        }
        uint64_t* __restrict__ o = dig + (((uint64_t)p * 3 + tree) * k + j) * 5;
#pragma unroll
        for (int q = 0; q < 5; ++q) o[q] = s[q];
    }
}

// Small batches: the same row hashing with one 16-lane DPP row per revealed row (tip5_permute_wide,
// carry-light).  The lane form above gives each row one lane, so a main row's 38 absorbs are 38
// dependent lane-form permutations (~7,000 VALU each on one lane): 1.8 ms for config 5's 8 / 64 proofs
// alone, the longest phase of a small batch and the one the Merkle climb waits for.  Here a
// permutation is ~10x fewer dependent instructions (at ~1.7x the lane form's VALU per permutation,
// which a small batch's idle SIMDs absorb); each lane e keeps state word e, lanes 0..9 load the
// chunk's words (10 lanes read a row's 80 contiguous bytes), the next chunk's word is loaded before
// the permutation so its latency hides behind it.  Every digest is the lane form's (same sponge:
// hash_varlen with the rate overwritten per chunk, padding 1 then 0s).
// (the body, for workgroup bx of tree `tree`: also run by k_fs_rows_small)
template <bool MW>
__device__ __forceinline__ void hash_rows_wide_body(uint32_t bx, uint32_t tree, const Tip5Lds& t5,
                                                    const uint64_t* __restrict__ words,
                                                    const ProofDesc* __restrict__ desc, uint32_t n_proofs,
                                                    uint32_t k, StarkDims dims, uint64_t* __restrict__ dig,
                                                    const uint32_t* __restrict__ fail) {
    const uint32_t width = tree == 0 ? dims.num_main : (tree == 1 ? 3 * dims.num_aux : 3 * dims.num_quot_seg);
    const uint32_t e = threadIdx.x & 15u;
    const uint64_t t = ((uint64_t)bx * blockDim.x + threadIdx.x) >> 4;  // uniform within the row
    if (t >= (uint64_t)n_proofs * k) return;
    const uint32_t p = (uint32_t)(t / k), j = (uint32_t)(t % k);
    if (fail[p]) return;
    const ProofDesc& d = desc[p];
    const uint64_t* __restrict__ row =
        words + (tree == 0 ? d.main_rows_off : (tree == 1 ? d.aux_rows_off : d.quot_rows_off)) + (uint64_t)j * width;
    uint64_t rcs[TIP5_ROUNDS];
#pragma unroll
    for (int r = 0; r < TIP5_ROUNDS; ++r) rcs[r] = c_tip5_rc_raw[r * 16 + e];
    const uint32_t nchunks = width / TIP5_RATE + 1;
    auto chunk_word = [&](uint32_t c) -> uint64_t {
        const uint32_t pos = c * TIP5_RATE;
        if (c + 1 < nchunks) return e < TIP5_RATE ? word_mont<MW>(row[pos + e]) : 0ull;
        const uint32_t rem = width - pos;  // the padded chunk: words, then 1, then 0s
        return e < rem ? word_mont<MW>(row[pos + e]) : (e == rem ? MONT_ONE : 0ull);
    };
    uint64_t s = 0, next = chunk_word(0);
    for (uint32_t c = 0; c < nchunks; ++c) {
        if (e < TIP5_RATE) s = next;  // absorb: the rate is overwritten, the capacity kept
        if (c + 1 < nchunks) next = chunk_word(c + 1);
        s = tip5_permute_wide<true>(s, e, rcs, t5.lut);
    }
    if (e < 5) dig[(((uint64_t)p * 3 + tree) * k + j) * 5 + e] = s;
}
template <bool MW>
__global__ void __launch_bounds__(256) k_hash_rows_wide(const uint64_t* __restrict__ words,
                                                        const ProofDesc* __restrict__ desc, uint32_t n_proofs,
                                                        uint32_t k, StarkDims dims, uint64_t* __restrict__ dig,
                                                        const uint32_t* __restrict__ fail) {
    latency_priority();
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);  // includes the barrier: every exit in the body comes after it
    hash_rows_wide_body<MW>(blockIdx.x, blockIdx.y, t5, words, desc, n_proofs, k, dims, dig, fail);
}

// One-stream small batches: the pair-form sponge replay (workgroups [0, fs_blocks)) and the 16-lane
// row hashing (the rest, rows_gx per tree) in ONE launch.  The row hashing needs no Fiat-Shamir
// sample, so it runs beside the replay instead of after it, and the batch's dependent chain is one
// packet shorter (each dependent packet costs ~38 us of a small batch's latency when 20 batches are
// in flight: profiles/r06/ab_pad_packets.txt).  The replay's workgroups come first in dispatch order.
template <bool MW>
__global__ void __launch_bounds__(256) k_fs_rows_small(const uint64_t* __restrict__ words,
                                                       const ProofDesc* __restrict__ desc,
                                                       const FsOp* __restrict__ ops, uint32_t n_proofs,
                                                       uint64_t* __restrict__ xs, uint32_t* __restrict__ idx_out,
                                                       const uint32_t* __restrict__ fail, AgePrio age,
                                                       uint32_t fs_blocks, uint32_t rows_gx, uint32_t k,
                                                       StarkDims dims, uint64_t* __restrict__ dig) {
    const uint32_t bx = blockIdx.x;
    if (bx < fs_blocks) age_priority(age, NHIP_LAT_PRIO);
    else latency_priority();
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    if (bx < fs_blocks) {
        fs_replay_wide_body<true, MW>(bx, lds, words, desc, ops, n_proofs, xs, idx_out, fail);
    } else {
        const uint32_t r = bx - fs_blocks;
        hash_rows_wide_body<MW>(r % rows_gx, r / rows_gx, lds, words, desc, n_proofs, k, dims, dig, fail);
    }
}

// ------------------------------------------------------------------ workgroup helpers
__device__ __forceinline__ void hash_pair_raw(const uint64_t* l, const uint64_t* r, uint64_t* out,
                                              const uint8_t* __restrict__ lut) {
    uint64_t s[16];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        s[q] = l[q];
        s[5 + q] = r[q];
    }
    tip5_hash_pair_digest(s, lut);  // capacity 1: FixedLength domain
#pragma unroll
    for (int q = 0; q < 5; ++q) out[q] = s[q];
}

// ------------------------------------------------------------------ Merkle multi-proofs
// twenty-first MerkleTreeInclusionProof::verify: leaves at (index, digest), the authentication
// structure lists the missing siblings in descending node-index order.  Trees per proof: 0 main,
// 1 aux, 2 quotient, 3 FRI round-0 a-values, 4 + r FRI round-r b-values.
//
// Level-synchronous design: which nodes get hashed, and from which children, depends only on the
// leaf indices and the authentication-structure length.  k_mp_plan sorts and dedupes the leaves
// and climbs the tree on indices alone, appending one hash op per parent node to a global
// per-level op list; k_mp_hash then runs once per level over ALL trees of ALL proofs (one lane per
// op: full waves whatever the tree shapes), and k_mp_roots compares every tree's final node with
// its committed root.  Trees 0-3 open the same leaf indices at the same height, so one plan
// workgroup (grid.y = 0) serves all four; grid.y = 1 + r plans FRI b-tree r.  Child digests are
// referenced by 64-bit source codes (type in the top 2 bits).
enum : uint64_t { MPS_ARENA = 0, MPS_AUTH = 1, MPS_DIG = 2, MPS_XFE = 3 };
static constexpr uint64_t MPS_MASK = (1ull << 62) - 1, MPS_NONE = ~0ull;
__device__ __forceinline__ uint64_t mps(uint64_t type, uint64_t v) { return (type << 62) | v; }

template <bool MW>
__device__ __forceinline__ void mp_load(uint64_t code, const uint64_t* __restrict__ words,
                                        const uint64_t* __restrict__ dig, const uint64_t* __restrict__ arena,
                                        uint64_t o[5]) {
    const uint64_t t = code >> 62, v = code & MPS_MASK;
    if (t == MPS_ARENA || t == MPS_DIG) {
        const uint64_t* s = (t == MPS_ARENA ? arena : dig) + 5 * v;
#pragma unroll
        for (int q = 0; q < 5; ++q) o[q] = s[q];
    } else if (t == MPS_AUTH) {
#pragma unroll
        for (int q = 0; q < 5; ++q) o[q] = word_mont<MW>(words[v + q]);
    } else {  // an XFE leaf of a FRI codeword: digest [c0, c1, c2, 0, 0]
#pragma unroll
        for (int q = 0; q < 3; ++q) o[q] = word_mont<MW>(words[v + q]);
        o[3] = 0;
        o[4] = 0;
    }
}

// exclusive prefix counts of two predicates over the workgroup (<= 4 waves), one barrier pair
__device__ __forceinline__ void wg_count_scan2(bool p0, bool p1, uint32_t& e0, uint32_t& e1, uint32_t& t0,
                                               uint32_t& t1, uint32_t* sh) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6, nw = blockDim.x >> 6;
    const uint64_t b0 = __ballot(p0), b1 = __ballot(p1);
    const uint64_t below = (1ull << lane) - 1ull;
    if (lane == 0) {
        sh[w] = (uint32_t)__popcll(b0);
        sh[4 + w] = (uint32_t)__popcll(b1);
    }
    __syncthreads();
    uint32_t s0 = 0, s1 = 0;
    t0 = 0;
    t1 = 0;
    for (uint32_t q = 0; q < nw; ++q) {
        const uint32_t c0 = sh[q], c1 = sh[4 + q];
        s0 += q < w ? c0 : 0u;
        s1 += q < w ? c1 : 0u;
        t0 += c0;
        t1 += c1;
    }
    __syncthreads();
    e0 = s0 + (uint32_t)__popcll(b0 & below);
    e1 = s1 + (uint32_t)__popcll(b1 & below);
}

__device__ __forceinline__ uint64_t mp_leaf_code(const ProofDesc& d, uint32_t p, uint32_t tree, uint32_t k,
                                                 uint32_t slot) {
    return tree < 3 ? mps(MPS_DIG, ((uint64_t)p * 3 + tree) * k + slot)
                    : mps(MPS_XFE, d.fri[tree == 3 ? 0 : tree - 3].leaves_off + 3ull * slot);
}

template <int B>
struct MpPlanLds {
    uint32_t key[2][B];
    uint64_t src[2][4][B];
    uint32_t order[B];
    uint32_t scan[8];
    uint32_t bad;  // bit t: tree t failed (authentication structure too short)
    uint32_t base, ndup;
};

// (the body, for proof p's tree group grp: also run by k_plan_fri_small)
template <int B>
__device__ __forceinline__ void mp_plan_body(uint32_t p, uint32_t grp, const uint64_t* __restrict__ words,
                                             const ProofDesc* __restrict__ desc, uint32_t n_proofs, uint32_t k,
                                             uint32_t trees_per_proof, const uint64_t* __restrict__ dig,
                                             const uint32_t* __restrict__ idx_all, MpPlan plan,
                                             uint32_t* __restrict__ fail, unsigned long long* __restrict__ perm_counter) {
    __shared__ MpPlanLds<B> L;
    const uint32_t tid = threadIdx.x;
    if (p >= n_proofs) return;
    const ProofDesc& d = desc[p];
    const uint32_t NT = grp == 0 ? 4u : 1u;
    const uint32_t tree0 = grp == 0 ? 0u : 3u + grp;  // tree id of this group's first tree
    if (tid < NT) plan.roots[(uint64_t)p * trees_per_proof + tree0 + tid].code = MPS_NONE;
    if (tid == 0) {
        plan.ndup[(uint64_t)p * (trees_per_proof - 3) + grp] = 0;
        plan.lvl_n[(uint64_t)p * (trees_per_proof - 3) + grp] = 0;
    }
    if (fail[p] & FAIL_DECODE) return;
    if (grp > d.R) return;
    uint32_t h, auth_n[4], fail_bit[4];
    uint64_t root_off[4], auth_off[4];
    if (grp == 0) {
        h = d.log2_N;
        root_off[0] = d.main_root, root_off[1] = d.aux_root, root_off[2] = d.quot_root, root_off[3] = d.fri_root[0];
        auth_off[0] = d.main_auth_off, auth_off[1] = d.aux_auth_off, auth_off[2] = d.quot_auth_off;
        auth_off[3] = d.fri[0].auth_off;
        auth_n[0] = d.main_auth_n, auth_n[1] = d.aux_auth_n, auth_n[2] = d.quot_auth_n, auth_n[3] = d.fri[0].auth_n;
        fail_bit[0] = FAIL_MERKLE_MAIN, fail_bit[1] = FAIL_MERKLE_AUX, fail_bit[2] = FAIL_MERKLE_QUOT;
        fail_bit[3] = FAIL_MERKLE_FRI;
    } else {
        const uint32_t r = grp - 1;
        h = d.log2_N - r;
        root_off[0] = d.fri_root[r];
        auth_off[0] = d.fri[1 + r].auth_off;
        auth_n[0] = d.fri[1 + r].auth_n;
        fail_bit[0] = FAIL_MERKLE_FRI;
    }
    const uint32_t shard = p % MP_SHARDS;
    const uint32_t* __restrict__ idx = idx_all + d.idx_off;
    // ---- leaves (key = node index = leaf index + 2^h; 0 = empty slot)
    uint32_t key = 0u;
    if (tid < k) {
        const uint64_t nl = 1ull << h;
        uint64_t li = idx[tid] % nl;
        if (grp > 0) li = (li + nl / 2) % nl;
        key = (uint32_t)(li + nl);
    }
    L.key[0][tid] = key;
    L.order[tid] = tid;
    if (tid == 0) {
        L.bad = 0;
        L.ndup = 0;
    }
    __syncthreads();
    // ---- bitonic sort (descending) of (key, original slot)
    for (uint32_t size = 2; size <= (uint32_t)B; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            const uint32_t partner = tid ^ stride;
            if (partner > tid) {
                const bool desc_dir = (tid & size) == 0;
                const uint32_t a = L.key[0][tid], b = L.key[0][partner];
                if ((a < b) == desc_dir && a != b) {
                    L.key[0][tid] = b;
                    L.key[0][partner] = a;
                    const uint32_t t = L.order[tid];
                    L.order[tid] = L.order[partner];
                    L.order[partner] = t;
                }
            }
            __syncthreads();
        }
    }
    const uint32_t skey = L.key[0][tid];
    const uint32_t slot = L.order[tid];
    uint64_t scode[4];
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) scode[t] = t < NT ? mp_leaf_code(d, p, tree0 + t, k, slot) : MPS_NONE;
    // duplicate leaf indices: kept once; equal digests are checked by k_mp_roots (the leaf digests
    // are not needed here, so planning does not wait for the row hashes)
    const uint64_t grp_id = (uint64_t)p * (trees_per_proof - 3) + grp;
    bool dup = false;
    if (skey != 0 && tid > 0 && L.key[0][tid - 1] == skey) {
        dup = true;
        const uint32_t j = atomicAdd(&L.ndup, 1u);
        plan.dups[(grp_id * k + j) * 2] = slot;
        plan.dups[(grp_id * k + j) * 2 + 1] = L.order[tid - 1];
    }
    const bool keep = skey != 0 && !dup;
    uint32_t pos, unused_e, m, unused_t;
    wg_count_scan2(keep, false, pos, unused_e, m, unused_t, L.scan);
    if (keep) {
        L.key[0][pos] = skey;
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) L.src[0][t][pos] = scode[t];
    }
    if (tid == 0) plan.ndup[grp_id] = L.ndup;
    __syncthreads();
    // ---- climb on indices; emit one op per parent node and tree
    uint32_t ap = 0, done = 0;
    int cur = 0;
    for (uint32_t lvl = 0; lvl < h; ++lvl) {
        const uint32_t i = tid;
        uint32_t ki = 0;
        bool unpaired = false, owner = false, pair_next = false;
        if (i < m) {
            ki = L.key[cur][i];
            const bool pair_prev = i > 0 && L.key[cur][i - 1] == (ki ^ 1u);
            pair_next = i + 1 < m && L.key[cur][i + 1] == (ki ^ 1u);
            unpaired = !pair_prev && !pair_next;
            owner = !pair_prev;
        }
        uint32_t upos, opos, n_unp, n_own;
        wg_count_scan2(unpaired, owner, upos, opos, n_unp, n_own, L.scan);
        uint32_t bad = L.bad;
        for (uint32_t t = 0; t < NT; ++t)
            if (ap + n_unp > auth_n[t]) bad |= 1u << t;  // authentication structure too short
        const uint64_t sidx = (uint64_t)lvl * MP_SHARDS + shard;
        if (tid == 0) L.base = atomicAdd(plan.counter + sidx, NT * n_own);
        __syncthreads();
        const uint32_t base = L.base;
        if (lvl >= plan.levels || (uint64_t)base + NT * n_own > plan.shard_cap[sidx]) {
            bad = 0xFu;  // capacity guard (cannot trigger with the host's bounds)
            if (tid == 0) L.bad = bad;
            break;  // uniform
        }
        if (tid == 0) {
            plan.lvl_g0[grp_id * plan.levels + lvl] = plan.shard_base[sidx] + base;
            plan.lvl_cnt[grp_id * plan.levels + lvl] = n_own;
        }
        done = lvl + 1;
        if (owner) {
            const uint64_t g0 = plan.shard_base[sidx] + base + opos;
            for (uint32_t t = 0; t < NT; ++t) {
                const uint64_t g = g0 + (uint64_t)t * n_own;
                uint64_t lc = MPS_NONE, rc = MPS_NONE;
                if (!((bad >> t) & 1u)) {
                    const uint64_t mine = L.src[cur][t][i];
                    if (pair_next) {  // i holds 2q+1, i+1 holds 2q
                        lc = L.src[cur][t][i + 1];
                        rc = mine;
                    } else {
                        const uint64_t sib = mps(MPS_AUTH, auth_off[t] + 5ull * (ap + upos));
                        const bool odd = (ki & 1u) != 0;
                        lc = odd ? sib : mine;
                        rc = odd ? mine : sib;
                    }
                }
                plan.ops[2 * g] = lc;
                plan.ops[2 * g + 1] = rc;
                L.src[cur ^ 1][t][opos] = mps(MPS_ARENA, g);
            }
            L.key[cur ^ 1][opos] = ki >> 1;
        }
        if (tid == 0) {
            L.bad = bad;
            uint32_t skipped = 0;
            for (uint32_t t = 0; t < NT; ++t) skipped += ((bad >> t) & 1u) ? n_own : 0u;
            if (skipped && perm_counter) atomicAdd(perm_counter, (unsigned long long)skipped);
        }
        ap += n_unp;
        m = n_own;
        cur ^= 1;
        __syncthreads();
    }
    __syncthreads();
    if (tid == 0) plan.lvl_n[grp_id] = done;
    if (tid < NT) {
        const uint32_t t = tid;
        const bool ok = !((L.bad >> t) & 1u) && m == 1 && L.key[cur][0] == 1u && ap == auth_n[t];
        MpRoot* rec = plan.roots + (uint64_t)p * trees_per_proof + tree0 + t;
        if (ok) {
            rec->code = L.src[cur][t][0];
            rec->root_off = root_off[t];
            rec->fail_bit = fail_bit[t];
        } else {
            atomicOr(&fail[p], fail_bit[t]);
        }
    }
}
template <int B>
__global__ void __launch_bounds__(B) k_mp_plan(const uint64_t* __restrict__ words, const ProofDesc* __restrict__ desc,
                                               uint32_t n_proofs, uint32_t k, uint32_t trees_per_proof,
                                               const uint64_t* __restrict__ dig, const uint32_t* __restrict__ idx_all,
                                               MpPlan plan, uint32_t* __restrict__ fail,
                                               unsigned long long* __restrict__ perm_counter) {
    latency_priority();
    mp_plan_body<B>(blockIdx.x, blockIdx.y, words, desc, n_proofs, k, trees_per_proof, dig, idx_all, plan, fail,
                    perm_counter);
}

// The last FRI codeword's Merkle tree (every node; XFE leaves embedded as [c0, c1, c2, 0, 0]) is
// hashed by the same launches: blocks past the multiproof ops of level l take the level-l parents
// of every proof's last-codeword tree, lane q -> (proof q / (maxL >> (l + 1)), parent q % ...).
// Node v of a proof's tree (heap order, root 1, leaves L..2L-1) lives at lcw[(p * maxL + v) * 5].
struct LcwTree {
    uint64_t* nodes;
    uint32_t max_len;   // max last-codeword length over the batch (power of two)
};

template <bool MW>
__device__ __forceinline__ void lcw_node(const uint64_t* __restrict__ words, const ProofDesc& d,
                                         const uint64_t* __restrict__ mine, uint32_t v, uint32_t L, uint64_t o[5]) {
    if (v >= L) {
        const uint64_t off = d.last_cw_off + 3ull * (v - L);
        o[0] = word_mont<MW>(words[off]);
        o[1] = word_mont<MW>(words[off + 1]);
        o[2] = word_mont<MW>(words[off + 2]);
        o[3] = 0;
        o[4] = 0;
    } else {
#pragma unroll
        for (int q = 0; q < 5; ++q) o[q] = mine[5ull * v + q];
    }
}

// 6 waves per SIMD (<= 80 VGPRs): with hash_pair's MDS finished two outputs at a time
// (NHIP_PAIR_MDS_GROUP) the kernel needs 77 VGPRs and no scratch (5 waves and a 20-byte spill before,
// 109 VGPRs unconstrained).  Config 4 +1.1-1.4% at 4,096 proofs, +2.3-3.4% at 512 (profiles/r03x).
// Batches below MP_SMALL_MAX_PROOFS (kernels.hpp) launch the 7-wave instance (72 VGPRs, a 24-byte
// spill): 512 to 2,048 proofs +1.2-4.3%, 4,096 proofs -0.6% (profiles/r03ze, r03zf).
#ifndef NHIP_MP_WAVES
#define NHIP_MP_WAVES 6
#endif
#ifndef NHIP_MP_WAVES_SMALL
#define NHIP_MP_WAVES_SMALL 7
#endif
template <int WAVES, bool MW>
__global__ void __launch_bounds__(256, WAVES) k_mp_hash(const uint64_t* __restrict__ words, const uint64_t* __restrict__ dig,
                                                 MpPlan plan, uint32_t lvl, uint32_t mp_blocks,
                                                 const ProofDesc* __restrict__ desc, uint32_t n_proofs,
                                                 const uint32_t* __restrict__ fail, LcwTree lcw, AgePrio age) {
    __shared__ Tip5Lds t5;
    __shared__ uint64_t s_base[MP_SHARDS + 1];
    __shared__ uint32_t s_cnt[MP_SHARDS];
    age_priority(age, NHIP_MP_PRIO);
    const bool is_lcw = blockIdx.x >= mp_blocks;  // uniform per block
    if (!is_lcw) {
        if (threadIdx.x < MP_SHARDS) {
            s_base[threadIdx.x] = plan.shard_base[lvl * MP_SHARDS + threadIdx.x];
            s_cnt[threadIdx.x] = plan.counter[lvl * MP_SHARDS + threadIdx.x];
        }
        if (threadIdx.x == 0)
            s_base[MP_SHARDS] = plan.shard_base[(lvl + 1) * MP_SHARDS - 1] + plan.shard_cap[(lvl + 1) * MP_SHARDS - 1];
    }
    tip5_lds_init(t5);  // includes the barrier
    uint64_t s[16];
    uint64_t* o = nullptr;
    bool work = false;
    if (is_lcw) {
        const uint32_t per = lcw.max_len >> (lvl + 1);
        const uint64_t q = (uint64_t)(blockIdx.x - mp_blocks) * blockDim.x + threadIdx.x;
        const uint32_t p = (uint32_t)(q / per), i = (uint32_t)(q % per);
        if (p < n_proofs && !(fail[p] & FAIL_DECODE)) {  // FAIL_DECODE is final once k_decode ran
            const ProofDesc& d = desc[p];
            const uint32_t L = d.last_cw_n;
            if (i < (L >> (lvl + 1))) {
                const uint32_t v = (L >> (lvl + 1)) + i;
                uint64_t* mine = lcw.nodes + (uint64_t)p * lcw.max_len * 5;
                lcw_node<MW>(words, d, mine, 2 * v, L, s);
                lcw_node<MW>(words, d, mine, 2 * v + 1, L, s + 5);
                o = mine + 5ull * v;
                work = true;
            }
        }
    } else {
        const uint64_t g = s_base[0] + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (g < s_base[MP_SHARDS]) {
            uint32_t sh = 0;
#pragma unroll
            for (uint32_t q = 1; q < MP_SHARDS; ++q) sh += g >= s_base[q] ? 1u : 0u;
            if (g - s_base[sh] < s_cnt[sh]) {
                const uint64_t lc = plan.ops[2 * g], rc = plan.ops[2 * g + 1];
                if (lc != MPS_NONE) {  // else: op of a tree that already failed
                    mp_load<MW>(lc, words, dig, plan.arena, s);
                    mp_load<MW>(rc, words, dig, plan.arena, s + 5);
                    o = plan.arena + 5 * g;
                    work = true;
                }
            }
        }
    }
    if (!work) return;
    tip5_hash_pair_digest(s, t5.lut);  // capacity 1: FixedLength domain
#pragma unroll
    for (int q = 0; q < 5; ++q) o[q] = s[q];
}

// Small levels (the last levels of the tallest trees): a lane-per-op permutation is a ~20 us
// dependent instruction chain however few ops there are, so these levels use the 16-lane row
// Tip5 (one op per DPP row, ~8x shorter chain) instead.
template <bool MW>
__device__ __forceinline__ uint64_t mp_load_word(uint64_t code, uint32_t e, const uint64_t* __restrict__ words,
                                                 const uint64_t* __restrict__ dig, const uint64_t* __restrict__ arena) {
    const uint64_t t = code >> 62, v = code & MPS_MASK;
    if (t == MPS_ARENA) return arena[5 * v + e];
    if (t == MPS_DIG) return dig[5 * v + e];
    if (t == MPS_AUTH) return word_mont<MW>(words[v + e]);
    return e < 3 ? word_mont<MW>(words[v + e]) : 0ull;  // XFE leaf [c0, c1, c2, 0, 0]
}

// Word e of a last-codeword tree node v (lcw_node, one word per lane of the row).
template <bool MW>
__device__ __forceinline__ uint64_t lcw_node_word(const uint64_t* __restrict__ words, const ProofDesc& d,
                                                  const uint64_t* __restrict__ mine, uint32_t v, uint32_t L, uint32_t e) {
    if (v >= L) return e < 3 ? word_mont<MW>(words[d.last_cw_off + 3ull * (v - L) + e]) : 0ull;
    return mine[5ull * v + e];
}

// Rows [0, mp_rows) take the multiproof ops of level `lvl`; rows past them the level-`lvl` parents of
// every proof's last-codeword tree (the same mapping as k_mp_hash's lcw blocks, one parent per row).
template <bool MW>
__global__ void __launch_bounds__(256) k_mp_hash_wide(const uint64_t* __restrict__ words,
                                                      const uint64_t* __restrict__ dig, MpPlan plan, uint32_t lvl,
                                                      uint64_t mp_rows, const ProofDesc* __restrict__ desc,
                                                      uint32_t n_proofs, const uint32_t* __restrict__ fail, LcwTree lcw) {
    latency_priority();
    __shared__ Tip5Lds t5;
    __shared__ uint64_t s_base[MP_SHARDS + 1];
    __shared__ uint32_t s_cnt[MP_SHARDS];
    if (threadIdx.x < MP_SHARDS) {
        s_base[threadIdx.x] = plan.shard_base[lvl * MP_SHARDS + threadIdx.x];
        s_cnt[threadIdx.x] = plan.counter[lvl * MP_SHARDS + threadIdx.x];
    }
    if (threadIdx.x == 0)
        s_base[MP_SHARDS] = plan.shard_base[(lvl + 1) * MP_SHARDS - 1] + plan.shard_cap[(lvl + 1) * MP_SHARDS - 1];
    tip5_lds_init(t5);  // includes the barrier
    const uint32_t e = threadIdx.x & 15u;
    const uint64_t row = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    // every test below is uniform within the 16-lane row (one op per row)
    uint64_t s = MONT_ONE;
    uint64_t* o = nullptr;
    if (row < mp_rows) {
        const uint64_t g = s_base[0] + row;
        if (g >= s_base[MP_SHARDS]) return;
        uint32_t sh = 0;
#pragma unroll
        for (uint32_t q = 1; q < MP_SHARDS; ++q) sh += g >= s_base[q] ? 1u : 0u;
        if (g - s_base[sh] >= s_cnt[sh]) return;
        const uint64_t lc = plan.ops[2 * g], rc = plan.ops[2 * g + 1];
        if (lc == MPS_NONE) return;  // op of a tree that already failed
        if (e < 5) s = mp_load_word<MW>(lc, e, words, dig, plan.arena);
        else if (e < 10) s = mp_load_word<MW>(rc, e - 5, words, dig, plan.arena);
        o = plan.arena + 5 * g;
    } else {
        const uint32_t per = lcw.max_len >> (lvl + 1);
        const uint64_t q = row - mp_rows;
        const uint32_t p = (uint32_t)(q / per), i = (uint32_t)(q % per);
        if (p >= n_proofs || (fail[p] & FAIL_DECODE)) return;  // FAIL_DECODE is final once k_decode ran
        const ProofDesc& d = desc[p];
        const uint32_t L = d.last_cw_n;
        if (i >= (L >> (lvl + 1))) return;
        const uint32_t v = (L >> (lvl + 1)) + i;
        uint64_t* mine = lcw.nodes + (uint64_t)p * lcw.max_len * 5;
        if (e < 5) s = lcw_node_word<MW>(words, d, mine, 2 * v, L, e);
        else if (e < 10) s = lcw_node_word<MW>(words, d, mine, 2 * v + 1, L, e - 5);
        o = mine + 5ull * v;
    }
    uint64_t rcs[TIP5_ROUNDS];
#pragma unroll
    for (int r = 0; r < TIP5_ROUNDS; ++r) rcs[r] = c_tip5_rc_raw[r * 16 + e];
    s = tip5_permute_wide<false>(s, e, rcs, t5.lut);
    if (e < 5) o[e] = s;
}

// The last levels of a small batch (a few dozen parents each, e.g. one block's proof): one
// workgroup climbs levels [lvl0, lvl1) itself, 64 rows in flight, with a barrier between levels
// (all of its waves share one CU and its L1, so a parent written at level l is visible to every
// wave at level l + 1).  One launch instead of one per level: the ~9 us dispatch gap between
// dependent launches exceeds the level's own hashing time there.  caps[l - lvl0] = the multiproof
// rows of level l (its capacity, as the per-level launches use).
static constexpr uint32_t MP_TAIL_THREADS = 1024;
struct TailCaps {
    uint32_t cap[MP_TAIL_LEVELS_MAX];
};

template <bool MW>
__global__ void __launch_bounds__(MP_TAIL_THREADS) k_mp_hash_tail(const uint64_t* __restrict__ words,
                                                                 const uint64_t* __restrict__ dig, MpPlan plan,
                                                                 uint32_t lvl0, uint32_t lvl1, TailCaps caps,
                                                                 const ProofDesc* __restrict__ desc, uint32_t n_proofs,
                                                                 const uint32_t* __restrict__ fail, LcwTree lcw) {
    latency_priority();
    __shared__ Tip5Lds t5;
    __shared__ uint64_t s_base[MP_SHARDS + 1];
    __shared__ uint32_t s_cnt[MP_SHARDS];
    tip5_lds_init(t5);
    const uint32_t e = threadIdx.x & 15u;
    const uint32_t row0 = threadIdx.x >> 4;
    constexpr uint32_t ROWS = MP_TAIL_THREADS / 16;
    uint64_t rcs[TIP5_ROUNDS];
#pragma unroll
    for (int r = 0; r < TIP5_ROUNDS; ++r) rcs[r] = c_tip5_rc_raw[r * 16 + e];
    for (uint32_t lvl = lvl0; lvl < lvl1; ++lvl) {
        const bool has_mp = lvl < plan.levels;
        if (has_mp) {
            if (threadIdx.x < MP_SHARDS) {
                s_base[threadIdx.x] = plan.shard_base[lvl * MP_SHARDS + threadIdx.x];
                s_cnt[threadIdx.x] = plan.counter[lvl * MP_SHARDS + threadIdx.x];
            }
            if (threadIdx.x == 0)
                s_base[MP_SHARDS] =
                    plan.shard_base[(lvl + 1) * MP_SHARDS - 1] + plan.shard_cap[(lvl + 1) * MP_SHARDS - 1];
        }
        __syncthreads();  // shard table of this level; parents of the previous level written
        const uint64_t mp_rows = has_mp ? caps.cap[lvl - lvl0] : 0;
        const uint32_t per = lcw.max_len >> (lvl + 1);
        const uint64_t rows = mp_rows + (uint64_t)per * n_proofs;
        for (uint64_t row = row0; row < rows; row += ROWS) {  // uniform within the 16-lane row
            uint64_t st = MONT_ONE;
            uint64_t* o = nullptr;
            if (row < mp_rows) {
                const uint64_t g = s_base[0] + row;
                if (g >= s_base[MP_SHARDS]) continue;
                uint32_t sh = 0;
#pragma unroll
                for (uint32_t q = 1; q < MP_SHARDS; ++q) sh += g >= s_base[q] ? 1u : 0u;
                if (g - s_base[sh] >= s_cnt[sh]) continue;
                const uint64_t lc = plan.ops[2 * g], rc = plan.ops[2 * g + 1];
                if (lc == MPS_NONE) continue;
                if (e < 5) st = mp_load_word<MW>(lc, e, words, dig, plan.arena);
                else if (e < 10) st = mp_load_word<MW>(rc, e - 5, words, dig, plan.arena);
                o = plan.arena + 5 * g;
            } else {
                const uint64_t q = row - mp_rows;
                const uint32_t p = (uint32_t)(q / per), i = (uint32_t)(q % per);
                if (p >= n_proofs || (fail[p] & FAIL_DECODE)) continue;
                const ProofDesc& d = desc[p];
                const uint32_t L = d.last_cw_n;
                if (i >= (L >> (lvl + 1))) continue;
                const uint32_t v = (L >> (lvl + 1)) + i;
                uint64_t* mine = lcw.nodes + (uint64_t)p * lcw.max_len * 5;
                if (e < 5) st = lcw_node_word<MW>(words, d, mine, 2 * v, L, e);
                else if (e < 10) st = lcw_node_word<MW>(words, d, mine, 2 * v + 1, L, e - 5);
                o = mine + 5ull * v;
            }
            st = tip5_permute_wide<true>(st, e, rcs, t5.lut);
            if (e < 5) o[e] = st;
        }
        __syncthreads();  // every parent of this level written before the next level reads it
    }
}

// Small batches: one 1,024-thread workgroup per (proof, tree) climbs that tree's every level
// itself (the plan's per-level op ranges of its group, this tree's share), 64 ops in flight on
// 16-lane rows, a barrier between levels; grid.y = trees_per_proof is each proof's last-codeword
// tree.  One launch replaces the per-level chain, whose ~14 us per level (9 of it dispatch latency)
// is most of a small batch's Merkle phase.  A tree's parents depend only on its own earlier
// levels, its leaves (row digests, done before this launch) and proof words.
static constexpr uint32_t MP_CLIMB_THREADS = 1024;
template <bool MW>
__global__ void __launch_bounds__(MP_CLIMB_THREADS) k_mp_climb(const uint64_t* __restrict__ words,
                                                               const uint64_t* __restrict__ dig, MpPlan plan,
                                                               uint32_t trees_per_proof,
                                                               const ProofDesc* __restrict__ desc, uint32_t n_proofs,
                                                               const uint32_t* __restrict__ fail, LcwTree lcw,
                                                               uint32_t start_lvl) {
    latency_priority();
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const uint32_t p = blockIdx.x, y = blockIdx.y;
    if (p >= n_proofs || (fail[p] & FAIL_DECODE)) return;  // uniform per workgroup
    const uint32_t e = threadIdx.x & 15u, row0 = threadIdx.x >> 4;
    constexpr uint32_t ROWS = MP_CLIMB_THREADS / 16;
    uint64_t rcs[TIP5_ROUNDS];
#pragma unroll
    for (int r = 0; r < TIP5_ROUNDS; ++r) rcs[r] = c_tip5_rc_raw[r * 16 + e];
    if (y == trees_per_proof) {  // the last codeword's tree: every node
        const ProofDesc& d = desc[p];
        const uint32_t L = d.last_cw_n;
        uint64_t* mine = lcw.nodes + (uint64_t)p * lcw.max_len * 5;
        for (uint32_t lvl = start_lvl; (L >> (lvl + 1)) > 0; ++lvl) {
            const uint32_t cnt = L >> (lvl + 1);
            for (uint32_t row = row0; row < cnt; row += ROWS) {  // uniform within the 16-lane row
                const uint32_t v = cnt + row;
                uint64_t st = MONT_ONE;
                if (e < 5) st = lcw_node_word<MW>(words, d, mine, 2 * v, L, e);
                else if (e < 10) st = lcw_node_word<MW>(words, d, mine, 2 * v + 1, L, e - 5);
                st = tip5_permute_wide<true>(st, e, rcs, t5.lut);
                if (e < 5) mine[5ull * v + e] = st;
            }
            __syncthreads();
        }
        return;
    }
    const uint32_t grp = y < 4 ? 0u : y - 3u, sub = y < 4 ? y : 0u;
    const uint64_t grp_id = (uint64_t)p * (trees_per_proof - 3) + grp;
    const uint32_t nl = plan.lvl_n[grp_id];
    for (uint32_t lvl = start_lvl; lvl < nl; ++lvl) {
        const uint64_t g0 = plan.lvl_g0[grp_id * plan.levels + lvl];
        const uint32_t cnt = plan.lvl_cnt[grp_id * plan.levels + lvl];
        for (uint32_t row = row0; row < cnt; row += ROWS) {  // uniform within the 16-lane row
            const uint64_t g = g0 + (uint64_t)sub * cnt + row;
            const uint64_t lc = plan.ops[2 * g], rc = plan.ops[2 * g + 1];
            if (lc == MPS_NONE) continue;  // a tree that already failed
            uint64_t st = MONT_ONE;
            if (e < 5) st = mp_load_word<MW>(lc, e, words, dig, plan.arena);
            else if (e < 10) st = mp_load_word<MW>(rc, e - 5, words, dig, plan.arena);
            st = tip5_permute_wide<true>(st, e, rcs, t5.lut);
            if (e < 5) plan.arena[5 * g + e] = st;
        }
        __syncthreads();
    }
}

// One lane per (proof, tree): duplicate leaf indices carry equal digests, final node == root.
// Lanes n_records.. check the last codeword's Merkle root, one per proof.
// (the body, for record i: also run by k_roots_verdicts_small)
template <bool MW>
__device__ __forceinline__ void mp_roots_body(uint32_t i, const uint64_t* __restrict__ words,
                                              const ProofDesc* __restrict__ desc, const uint64_t* __restrict__ dig,
                                              MpPlan plan, uint32_t n_records, uint32_t trees_per_proof, uint32_t k,
                                              uint32_t* __restrict__ fail, uint32_t n_proofs, LcwTree lcw) {
    if (i >= n_records) {
        const uint32_t p = i - n_records;
        if (p >= n_proofs || (fail[p] & FAIL_DECODE)) return;
        const ProofDesc& d = desc[p];
        uint64_t v[5];
        lcw_node<MW>(words, d, lcw.nodes + (uint64_t)p * lcw.max_len * 5, 1, d.last_cw_n, v);
        bool ok = true;
#pragma unroll
        for (int q = 0; q < 5; ++q) ok &= v[q] == word_mont<MW>(words[d.fri_root[d.R] + q]);
        if (!ok) atomicOr(&fail[p], FAIL_FRI_LAST_ROOT);
        return;
    }
    const MpRoot r = plan.roots[i];
    if (r.code == MPS_NONE) return;
    const uint32_t p = i / trees_per_proof, tree = i - p * trees_per_proof;
    const ProofDesc& d = desc[p];
    const uint64_t grp_id = (uint64_t)p * (trees_per_proof - 3) + (tree < 4 ? 0u : tree - 3);
    const uint32_t nd = plan.ndup[grp_id];
    bool ok = true;
    for (uint32_t j = 0; j < nd; ++j) {
        uint64_t a[5], b[5];
        mp_load<MW>(mp_leaf_code(d, p, tree, k, plan.dups[(grp_id * k + j) * 2]), words, dig, nullptr, a);
        mp_load<MW>(mp_leaf_code(d, p, tree, k, plan.dups[(grp_id * k + j) * 2 + 1]), words, dig, nullptr, b);
#pragma unroll
        for (int q = 0; q < 5; ++q) ok &= a[q] == b[q];
    }
    uint64_t v[5];
    mp_load<MW>(r.code, words, dig, plan.arena, v);
#pragma unroll
    for (int q = 0; q < 5; ++q) ok &= v[q] == word_mont<MW>(words[r.root_off + q]);
    if (!ok) atomicOr(&fail[p], r.fail_bit);
}
template <bool MW>
__global__ void k_mp_roots(const uint64_t* __restrict__ words, const ProofDesc* __restrict__ desc,
                           const uint64_t* __restrict__ dig, MpPlan plan, uint32_t n_records, uint32_t trees_per_proof,
                           uint32_t k, uint32_t* __restrict__ fail, uint32_t n_proofs, LcwTree lcw) {
    mp_roots_body<MW>(blockIdx.x * blockDim.x + threadIdx.x, words, desc, dig, plan, n_records, trees_per_proof, k,
                      fail, n_proofs, lcw);
}

// ------------------------------------------------------------------ XFE block reduction
__device__ Xfe block_sum_xfe(Xfe v, Xfe* sh) {
    const uint32_t tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (uint32_t s = blockDim.x >> 1; s > 0; s >>= 1) {
        if (tid < s) sh[tid] = x_add(sh[tid], sh[tid + s]);
        __syncthreads();
    }
    const Xfe r = sh[0];
    __syncthreads();
    return r;
}

__device__ __forceinline__ Xfe shfl_xor_xfe_fwd(Xfe v, int m) {
    return {(uint64_t)__shfl_xor((long long)v.c0, m), (uint64_t)__shfl_xor((long long)v.c1, m),
            (uint64_t)__shfl_xor((long long)v.c2, m)};
}

// Workgroup sum with one LDS entry per wave (sh[blockDim / 64]); every thread gets the sum.
__device__ Xfe block_sum_xfe_waves(Xfe v, Xfe* sh) {
    const uint32_t tid = threadIdx.x, nw = blockDim.x >> 6;
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v = x_add(v, shfl_xor_xfe_fwd(v, m));
    if ((tid & 63u) == 0) sh[tid >> 6] = v;
    __syncthreads();
    Xfe r = sh[0];
    for (uint32_t w = 1; w < nw; ++w) r = x_add(r, sh[w]);
    __syncthreads();
    return r;
}

// ------------------------------------------------------------------ Challenges::new
// triton-air 1.0 ChallengeId indices (include/nhip_challenge_id.h; public design, unpinned) of the
// sampled indeterminates the derived challenges use
static constexpr uint32_t CH_COMPRESS_PROGRAM_DIGEST = NHIP_CH_CompressProgramDigestIndeterminate,
                          CH_STANDARD_INPUT = NHIP_CH_StandardInputIndeterminate,
                          CH_STANDARD_OUTPUT = NHIP_CH_StandardOutputIndeterminate,
                          CH_LOOKUP_TABLE_PUBLIC = NHIP_CH_LookupTablePublicIndeterminate;
static_assert(CH_LOOKUP_TABLE_PUBLIC == 54 && NHIP_CHALLENGE_SAMPLE_COUNT == 59 && NHIP_CHALLENGE_COUNT == 63,
              "triton-air ChallengeId layout");
static_assert(NHIP_CH_StandardInputTerminal == NHIP_CHALLENGE_SAMPLE_COUNT && NHIP_CH_CompressedProgramDigest == 62,
              "derived challenges follow the sampled ones");

__device__ __forceinline__ Xfe shfl_xor_xfe(Xfe v, int m) {
    return {(uint64_t)__shfl_xor((long long)v.c0, m), (uint64_t)__shfl_xor((long long)v.c1, m),
            (uint64_t)__shfl_xor((long long)v.c2, m)};
}

// EvalArg::compute_terminal(symbols[0..n), initial 1, c) on one full wave: lane j folds the chunk
// [j ch, (j + 1) ch) by Horner, scales it by c^(n - chunk end), and the wave sums the chunks plus
// c^n (the initial 1).  Same value as the sequential fold; n / 64 + ~2 log2 n products per lane.
template <class Sym>
__device__ Xfe eval_terminal_wave(uint32_t n, Xfe c, Sym sym) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t ch = (n + 63u) / 64u;
    const uint32_t lo = min(n, lane * ch), hi = min(n, lo + ch);
    Xfe h = x_zero();
    for (uint32_t i = lo; i < hi; ++i) h = x_add(x_mul(h, c), x_lift(sym(i)));
    Xfe t = hi > lo ? x_mul(h, x_pow(c, n - hi)) : x_zero();
    if (lane == 0) t = x_add(t, x_pow(c, n));
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) t = x_add(t, shfl_xor_xfe(t, m));
    return t;
}

// ------------------------------------------------------------------ OOD: AIR + quotient identity
// One workgroup per proof.  The compiled AIR program (OodIns, stark.hpp) runs step by step:
// OOD-row inputs are loaded into LDS slots, each ADD/SUB/MUL writes its value (XFE) to a reusable
// slot, and each constraint value is copied into its own slot one step after it is produced; after
// the last step the workgroup forms sum_i w_i * C_i * Z_type(i)^-1 over those slots and compares it
// with sum_k z^k * segment_k(z^4).  Also stores the OOD linear combinations used by DEEP:
// [sum w*curr row, sum w*next row, sum w*segs].
// BLOCK = 256 for batches that fill the GPU (the hashing needs the wave slots); 1,024 for small ones
// (OOD_WIDE_MAX_PROOFS), where one proof's evaluation is on the critical path and the CUs are idle.
#ifndef NHIP_OOD_WAVES
#define NHIP_OOD_WAVES 1
#endif

// GS: the program has slots past the LDS part (gslot_n > 0); without them every slot access is a
// plain LDS access (ds_read / ds_write) instead of a branch between LDS and the global area.
template <uint32_t BLOCK, bool MW, bool GS>
__global__ void __launch_bounds__(BLOCK, BLOCK == 256 ? NHIP_OOD_WAVES : 1) k_ood_air(const uint64_t* __restrict__ words, const ProofDesc* __restrict__ desc,
                                                 uint32_t n_proofs, StarkDims dims, const OodIns* __restrict__ prog,
                                                 const uint32_t* __restrict__ prog_off, uint32_t n_levels,
                                                 const Xfe* __restrict__ consts, uint4 cons_type_off,
                                                 const uint64_t* __restrict__ xs, uint64_t* __restrict__ ood_out,
                                                 uint32_t* __restrict__ fail, uint32_t lds_slots,
                                                 Xfe* __restrict__ gslots, uint32_t gslot_n) {
    latency_priority();
    // all LDS in the dynamic region (16-B aligned carve, no static __shared__ in front of it)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Xfe* red = reinterpret_cast<Xfe*>(smem);              // 16 (one per wave)
    Xfe* zinv = red + 16;                                  // 4
    Xfe* chal_derived = zinv + 4;                          // 4 (Challenges::new)
    Xfe* misc = chal_derived + 4;                          // 4 (1 used: z - w^-1)
    uint32_t& zero_flag = *reinterpret_cast<uint32_t*>(misc + 4);
    Xfe* val = reinterpret_cast<Xfe*>(smem + AIR_LDS_HEADER);
    const uint32_t p = blockIdx.x, tid = threadIdx.x;
    // slots [0, lds_slots) live in LDS, the rest (an AIR larger than the LDS budget) in this
    // proof's global slot area; the slot allocator reuses low slots first, so the hot ones stay in
    // LDS.  The barrier after each level orders the global writes for the workgroup as well.
    Xfe* gval = gslots + (uint64_t)p * gslot_n;
    auto slot_ld = [&](uint32_t s) -> Xfe { return !GS || s < lds_slots ? val[s] : gval[s - lds_slots]; };
    auto slot_st = [&](uint32_t s, const Xfe& v) {
        if (!GS || s < lds_slots) val[s] = v;
        else gval[s - lds_slots] = v;
    };
    if (p >= n_proofs || (fail[p] & FAIL_DECODE)) return;
    const ProofDesc& d = desc[p];
    const SampleLayout sl = SampleLayout::of(dims, d.R);
    const uint64_t xb = d.xs_off * 3;
    const Xfe z = ld_xfe_raw(xs, xb + 3ull * sl.z);
    if (tid == 0) zero_flag = 0;
    __syncthreads();
    // zerofier inverses (triton-vm verify: initial, consistency, transition, terminal), one
    // inversion per wave, and the derived challenges
    if (tid == 0) {
        const uint64_t w_inv = b_inv(root_of_unity(d.log2_ph));
        const Xfe except_last = x_sub(z, x_lift(w_inv));
        if (x_is_zero(except_last)) atomicOr(&zero_flag, 1u);
        misc[0] = except_last;
        zinv[3] = x_inv(except_last);
    } else if (tid == 64) {
        const Xfe zm1 = x_sub(z, x_one());
        if (x_is_zero(zm1)) atomicOr(&zero_flag, 1u);
        zinv[0] = x_inv(zm1);
    } else if (tid == 128) {
        Xfe zph = z;
        for (uint32_t q = 0; q < d.log2_ph; ++q) zph = x_mul(zph, zph);
        const Xfe cons = x_sub(zph, x_one());
        if (x_is_zero(cons)) atomicOr(&zero_flag, 1u);
        zinv[1] = x_inv(cons);
    } else if (tid >= 192 && tid < 256) {
        // Challenges::new: the 4 derived challenges in ChallengeId order, each an EvalArg terminal
        // folded from 1 with its named sampled indeterminate (wave 3, lane-parallel)
        auto chal = [&](uint32_t i) { return ld_xfe_raw(xs, xb + 3ull * (sl.chal + i)); };
        const Xfe ein = eval_terminal_wave(d.claim_in_n, chal(CH_STANDARD_INPUT),
                                           [&](uint32_t i) { return word_mont<MW>(words[d.claim_in_off + i]); });
        const Xfe eout = eval_terminal_wave(d.claim_out_n, chal(CH_STANDARD_OUTPUT),
                                            [&](uint32_t i) { return word_mont<MW>(words[d.claim_out_off + i]); });
        const Xfe lut = eval_terminal_wave(256u, chal(CH_LOOKUP_TABLE_PUBLIC), [&](uint32_t i) {
            const uint64_t y = i + 1;  // tip5::LOOKUP_TABLE[i] = (i + 1)^3 - 1 mod 257
            return to_mont((y * y % 257u * y % 257u + 256u) % 257u);
        });
        const Xfe comp = eval_terminal_wave(5u, chal(CH_COMPRESS_PROGRAM_DIGEST),
                                            [&](uint32_t i) { return word_mont<MW>(words[d.claim_digest_off + i]); });
        if (tid == 192) {
            chal_derived[0] = ein;
            chal_derived[1] = eout;
            chal_derived[2] = lut;
            chal_derived[3] = comp;
        }
    }
    __syncthreads();
    if (tid == 0) zinv[2] = x_mul(misc[0], zinv[1]);
    __syncthreads();
    const uint32_t offs[5] = {0u, cons_type_off.x, cons_type_off.y, cons_type_off.z, cons_type_off.w};
    auto fetch = [&](uint32_t ref) -> Xfe {
        const uint32_t t = ref >> 30;
        if (t == 0) return slot_ld(ref);
        if (t == 1) return consts[ref & 0x3FFFFFFFu];
        const uint32_t kind = (ref >> 27) & 7u, i = ref & 0x7FFFFFFu;
        switch (kind) {
            case IN_MAIN_CURR: return ld_xfe_w<MW>(words, d.ood_mc + 3ull * i);
            case IN_AUX_CURR: return ld_xfe_w<MW>(words, d.ood_ac + 3ull * i);
            case IN_MAIN_NEXT: return ld_xfe_w<MW>(words, d.ood_mn + 3ull * i);
            case IN_AUX_NEXT: return ld_xfe_w<MW>(words, d.ood_an + 3ull * i);
            default:
                return i < dims.num_sampled ? ld_xfe_raw(xs, xb + 3ull * (sl.chal + i)) : chal_derived[i - dims.num_sampled];
        }
    };
    // The program step by step (air_compile: a step's instructions are independent; a barrier
    // between steps).  Batching a thread's instructions of a step (all operands requested first)
    // and loading the next step's instruction words during the current one measured slower: config
    // 4 -1.3% at 4,096 proofs, -1% at 512 (profiles/r04e), so each instruction runs on its own.
    for (uint32_t lvl = 0; lvl < n_levels; ++lvl) {
        for (uint32_t q = prog_off[lvl] + tid; q < prog_off[lvl + 1]; q += blockDim.x) {
            const uint4 ins = reinterpret_cast<const uint4*>(prog)[q];  // (op, a, b, dst): one 16-B load
            if (ins.x >= OOD_LOAD) {  // an input into its slot, or a constraint into its own slot
                slot_st(ins.w, fetch(ins.y));
            } else {
                // operands are slots (air_compile copies inputs and constants into slots first)
                const Xfe x = slot_ld(ins.y), y = slot_ld(ins.z);
                slot_st(ins.w, ins.x == OOD_ADD ? x_add(x, y) : (ins.x == OOD_SUB ? x_sub(x, y) : x_mul(x, y)));
            }
        }
        __syncthreads();
    }
    // sum_c w_c * C_c * Z_type(c)^-1 over the constraint slots (the top C), every lane busy
    const uint32_t C = dims.num_constraints, cbase = lds_slots + gslot_n - C;
    Xfe acc = x_zero();
    for (uint32_t c = tid; c < C; c += blockDim.x) {
        uint32_t t = 0;
        while (t < 3 && c >= offs[t + 1]) ++t;
        const Xfe w = ld_xfe_raw(xs, xb + 3ull * (sl.quot_w + c));
        acc = x_add(acc, x_mul(w, x_mul(slot_ld(cbase + c), zinv[t])));
    }
    const Xfe ood_q = block_sum_xfe_waves(acc, red);
    // OOD linear combinations (DEEP needs them): lin weights = [main | aux | quot segs | deep]
    const uint32_t M = dims.num_main, A = dims.num_aux, Q = dims.num_quot_seg;
    Xfe lc = x_zero(), ln = x_zero();
    for (uint32_t c = tid; c < M + A; c += blockDim.x) {
        const Xfe w = ld_xfe_raw(xs, xb + 3ull * (sl.lin_w + c));
        const Xfe vc = c < M ? ld_xfe_w<MW>(words, d.ood_mc + 3ull * c) : ld_xfe_w<MW>(words, d.ood_ac + 3ull * (c - M));
        const Xfe vn = c < M ? ld_xfe_w<MW>(words, d.ood_mn + 3ull * c) : ld_xfe_w<MW>(words, d.ood_an + 3ull * (c - M));
        lc = x_add(lc, x_mul(w, vc));
        ln = x_add(ln, x_mul(w, vn));
    }
    const Xfe sum_c = block_sum_xfe_waves(lc, red);
    const Xfe sum_n = block_sum_xfe_waves(ln, red);
    if (tid == 0) {
        Xfe seg = x_zero(), zk = x_one(), qlin = x_zero();
        for (uint32_t q = 0; q < Q; ++q) {
            const Xfe sq = ld_xfe_w<MW>(words, d.ood_qs + 3ull * q);
            seg = x_add(seg, x_mul(zk, sq));
            zk = x_mul(zk, z);
            qlin = x_add(qlin, x_mul(ld_xfe_raw(xs, xb + 3ull * (sl.lin_w + M + A + q)), sq));
        }
        uint32_t f = 0;
        if (zero_flag) f |= FAIL_ZERO_INVERSE;
        if (!x_eq(seg, ood_q)) f |= FAIL_OOD;
        if (f) atomicOr(&fail[p], f);
        uint64_t* o = ood_out + (uint64_t)p * 9;
        st_xfe_raw(o, 0, sum_c);
        st_xfe_raw(o, 3, sum_n);
        st_xfe_raw(o, 6, qlin);
    }
}

// ------------------------------------------------------------------ FRI
// One workgroup per proof.  Lane j follows collinearity check j through all rounds:
// a_{r+1} = line through (x_a, a_r), (x_b, b_r) evaluated at alpha_r.  The round-r domain point of
// check j is x_r = (7 * g^i)^(2^r) and its partner is -x_r (the a/b indices differ by half the
// round-r domain), so one exponentiation and one inversion per lane serve every round:
// x_{r+1} = x_r^2, 1/x_{r+1} = (1/x_r)^2, slope = (b - a) * (-1/2) / x_r.  The lane also stores x_0
// (raw) for DEEP.  Then the last codeword: agreement at the a-indices, and Horner(last polynomial, t)
// == barycentric(last codeword, t).  The last codeword's Merkle tree is hashed with the multiproof
// levels (k_mp_hash) and its root checked in k_mp_roots.
__device__ __forceinline__ uint64_t lds_pow(const uint64_t* __restrict__ sq, uint64_t e) {
    // sq[b] = g^(2^b); e < 2^32
    uint64_t r = MONT_ONE;
    for (uint32_t b = 0; e; ++b, e >>= 1)
        if (e & 1) r = mont_mul(r, sq[b]);
    return r;
}

#ifndef NHIP_FRI_WAVES
#define NHIP_FRI_WAVES 1
#endif
// (the body, for proof p: also run by k_plan_fri_small)
template <bool MW>
__device__ __forceinline__ void fri_body(uint32_t p, const uint64_t* __restrict__ words, const ProofDesc* __restrict__ desc,
                                         uint32_t n_proofs, StarkDims dims, const uint64_t* __restrict__ xs,
                                         const uint32_t* __restrict__ idx_all, uint64_t* __restrict__ xdom,
                                         uint32_t* __restrict__ fail) {
    __shared__ Xfe red[256];
    __shared__ uint64_t gsq[33], wsq[33];
    __shared__ uint32_t lflag;
    const uint32_t tid = threadIdx.x;
    if (p >= n_proofs || (fail[p] & FAIL_DECODE)) return;
    const ProofDesc& d = desc[p];
    const SampleLayout sl = SampleLayout::of(dims, d.R);
    const uint64_t xb = d.xs_off * 3;
    const uint32_t k = dims.num_checks;
    const uint32_t* __restrict__ idx = idx_all + d.idx_off;
    const uint32_t L = d.last_cw_n;
    const uint32_t log2L = 31 - __clz(L);
    if (tid == 0) {
        lflag = 0;
        uint64_t g = root_of_unity(d.log2_N);
        for (uint32_t q = 0; q < d.log2_N; ++q, g = mont_mul(g, g)) gsq[q] = g;
    } else if (tid == 64) {
        uint64_t w = root_of_unity(log2L);
        for (uint32_t q = 0; q < log2L; ++q, w = mont_mul(w, w)) wsq[q] = w;
    }
    __syncthreads();
    uint32_t f = 0;
    if (tid < k) {
        const uint32_t i0 = idx[tid];
        Xfe a = ld_xfe_w<MW>(words, d.fri[0].leaves_off + 3ull * tid);
        uint64_t x = mont_mul(to_mont(7), lds_pow(gsq, i0));
        xdom[(uint64_t)p * k + tid] = x;
        uint64_t xinv = b_inv(x);
        const uint64_t neg_half = to_mont((GL_P - 1) / 2);  // -1/2
        for (uint32_t r = 0; r < d.R; ++r) {
            const Xfe b = ld_xfe_w<MW>(words, d.fri[1 + r].leaves_off + 3ull * tid);
            const Xfe alpha = ld_xfe_raw(xs, xb + 3ull * (sl.alpha + r));
            const Xfe slope = x_scale(x_sub(b, a), mont_mul(neg_half, xinv));
            a = x_add(a, x_mul(slope, x_sub(alpha, x_lift(x))));
            x = mont_mul(x, x);
            xinv = mont_mul(xinv, xinv);
        }
        const Xfe last = ld_xfe_w<MW>(words, d.last_cw_off + 3ull * (i0 & (L - 1)));
        if (!x_eq(last, a)) f |= FAIL_FRI_LAST_AGREE;
    }
    // barycentric evaluation of the last codeword at the indeterminate vs Horner of the polynomial
    const Xfe t = ld_xfe_raw(xs, xb + 3ull * sl.indeterminate);
    Xfe num = x_zero(), den = x_zero();
    if (tid < L) {
        uint64_t wi = lds_pow(wsq, tid);
        const uint64_t wstep = blockDim.x < L ? wsq[31 - __clz(blockDim.x)] : MONT_ONE;
        // the lane's points two at a time with one inversion (Montgomery's trick: 1/d0 = d1 / (d0 d1));
        // a zero difference (t on the domain: the proof is rejected either way) takes the one-at-a-time
        // form, so num / den are those of the reference's per-point inverses in every case
        auto term = [&](uint32_t i, uint64_t w, Xfe inv) {
            const Xfe q = x_scale(inv, w);
            num = x_add(num, x_mul(q, ld_xfe_w<MW>(words, d.last_cw_off + 3ull * i)));
            den = x_add(den, q);
        };
        uint32_t i = tid;
        for (; i + blockDim.x < L; i += 2 * blockDim.x) {
            const uint64_t w1 = mont_mul(wi, wstep);
            const Xfe d0 = x_sub(t, x_lift(wi)), d1 = x_sub(t, x_lift(w1));
            const Xfe pr = x_mul(d0, d1);
            if (x_is_zero(pr)) {
                atomicOr(&lflag, 1u);
                term(i, wi, x_inv(d0));
                term(i + blockDim.x, w1, x_inv(d1));
            } else {
                const Xfe inv = x_inv(pr);
                term(i, wi, x_mul(inv, d1));
                term(i + blockDim.x, w1, x_mul(inv, d0));
            }
            wi = mont_mul(w1, wstep);
        }
        if (i < L) {
            const Xfe diff = x_sub(t, x_lift(wi));
            if (x_is_zero(diff)) atomicOr(&lflag, 1u);
            term(i, wi, x_inv(diff));
        }
    }
    const Xfe snum = block_sum_xfe(num, red);
    const Xfe sden = block_sum_xfe(den, red);
    // the last polynomial at t, in parallel instead of a one-lane Horner chain: lane c takes
    // coef_c * t^c (t^c from the t^(2^j) table), then a block sum (field values: the order of
    // the sum does not change the result)
    __shared__ Xfe tpow[32];
    const uint32_t pbits = d.last_poly_n ? 32 - __clz(d.last_poly_n) : 0;
    if (tid == 0) {
        Xfe q = t;
        for (uint32_t j = 0; j < pbits; ++j, q = x_mul(q, q)) tpow[j] = q;
    }
    __syncthreads();
    Xfe hp = x_zero();
    for (uint32_t c = tid; c < d.last_poly_n; c += blockDim.x) {
        Xfe pw = x_one();
        for (uint32_t j = 0; (c >> j) != 0; ++j)
            if ((c >> j) & 1u) pw = x_mul(pw, tpow[j]);
        hp = x_add(hp, x_mul(pw, ld_xfe_w<MW>(words, d.last_poly_off + 3ull * c)));
    }
    const Xfe h = block_sum_xfe(hp, red);
    if (tid == 0) {
        if (lflag || x_is_zero(sden)) f |= FAIL_ZERO_INVERSE;
        else if (!x_eq(h, x_mul(snum, x_inv(sden)))) f |= FAIL_FRI_EVAL;
        if (!d.last_poly_degree_ok) f |= FAIL_FRI_DEGREE;
    }
    if (f) atomicOr(&fail[p], f);
}
template <bool MW>
__global__ void __launch_bounds__(256, NHIP_FRI_WAVES) k_fri(const uint64_t* __restrict__ words, const ProofDesc* __restrict__ desc,
                                             uint32_t n_proofs, StarkDims dims, const uint64_t* __restrict__ xs,
                                             const uint32_t* __restrict__ idx_all, uint64_t* __restrict__ xdom,
                                             uint32_t* __restrict__ fail) {
    latency_priority();
    fri_body<MW>(blockIdx.x, words, desc, n_proofs, dims, xs, idx_all, xdom, fail);
}

// One-stream small batches: the Merkle plan (workgroups [0, n * groups): proof bx % n, tree group
// bx / n) and FRI (the next n workgroups, one per proof) in ONE launch.  Both need only the sponge
// samples and decode's words, neither reads the other's output, so the batch's dependent chain is one
// packet and one phase shorter.
template <bool MW>
__global__ void __launch_bounds__(256) k_plan_fri_small(const uint64_t* __restrict__ words,
                                                        const ProofDesc* __restrict__ desc, uint32_t n_proofs,
                                                        uint32_t k, uint32_t trees_per_proof, uint32_t groups,
                                                        const uint64_t* __restrict__ dig,
                                                        const uint32_t* __restrict__ idx_all, MpPlan plan,
                                                        uint32_t* __restrict__ fail,
                                                        unsigned long long* __restrict__ perm_counter,
                                                        StarkDims dims, const uint64_t* __restrict__ xs,
                                                        uint64_t* __restrict__ xdom) {
    latency_priority();
    const uint32_t bx = blockIdx.x, np = n_proofs * groups;
    if (bx < np)
        mp_plan_body<256>(bx % n_proofs, bx / n_proofs, words, desc, n_proofs, k, trees_per_proof, dig, idx_all, plan,
                          fail, perm_counter);
    else
        fri_body<MW>(bx - np, words, desc, n_proofs, dims, xs, idx_all, xdom, fail);
}

// ------------------------------------------------------------------ DEEP
// One workgroup per proof; lane (r, q) of the 256 threads takes words q, q + 8, q + 16, ... of
// revealed row r of the current pass (32 rows per pass), so one load instruction of a wave reads
// 8 rows x 64 contiguous bytes.  Row linear combinations sum_c w_c * row_c are accumulated lazily:
// the weights are raw Montgomery (w R), split into 22 / 22 / 20-bit limbs; each proof word enters as
// its two 32-bit halves, so every partial product is < 2^54 and one 64-bit accumulator per (limb,
// half) takes a whole row share without carries (one v_mad_u64_u32 per partial product).  Each
// lane reduces its accumulators once, the 8 lanes of a row add theirs (3 xor shuffles): with
// canonical words the sum R * sum w x mod p is the raw Montgomery word of the combination; with
// Montgomery words (x R) it is R^2 * sum w x, and one from_mont makes it the same word.  An XFE
// product w * x is sum_m x_m * (w X^m) with w X = (-w2, w0 + w2, w1) and w X^2 = (-w1, w1 - w2,
// w0 + w2) (X^3 = X - 1), precomputed per aux column in LDS.  Then thread j takes row j's three DEEP
// terms (x - z, x - z w_trace, x - z^Q; x from k_fri), inverts their product once (Montgomery's
// trick), and compares the recombined value with the FRI round-0 leaf.
typedef unsigned __int128 u128_t;
static constexpr uint32_t DEEP_UNROLL = 8;

// lo + hi * 2^64 mod p for hi < 2^44
__device__ __forceinline__ uint64_t reduce_u108(u128_t y) {
    const uint64_t y0 = (uint64_t)y, y1 = (uint64_t)(y >> 64);
    const uint64_t r = reduce96(y0, (uint32_t)y1);
    return gl_sub(r, y1 >> 32);  // 2^96 == -1 (mod p)
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    return (uint64_t)__shfl_xor((long long)v, m);
}

// k_deep_rows8's accumulation: each weight (raw Montgomery, < 2^64) split into limbs of 22, 22 and
// 20 bits (held in LDS as one uint4 per XFE coefficient), each proof word into its two 32-bit halves
// (no extraction instructions); every partial product is < 2^54.  A lane takes ceil(M / 8) +
// ceil(3A / 8) words of a row (81 for triton-vm's 379 / 88 columns; < DEEP_LANE_TERMS_MAX = 258 under
// dims_from's M + 3A < DEEP_ROW_WORDS_MAX), so each 64-bit accumulator stays below 258 * 2^54 < 2^63
// (static_assert in kernels.hpp), and wl_reduce's U, W below 2^63 * (1 + 2^22 + 2^44) < 2^108 (its
// reduce_u108 needs the high word < 2^44).  6 multiply-adds per (word, coefficient).
__device__ __forceinline__ uint4 w_limbs(uint64_t w) {
    return make_uint4((uint32_t)w & 0x3FFFFFu, (uint32_t)(w >> 22) & 0x3FFFFFu, (uint32_t)(w >> 44), 0u);
}
__device__ __forceinline__ void wl_mac(uint64_t (&a)[6], uint4 wl, uint32_t x0, uint32_t x1) {
    a[0] += (uint64_t)wl.x * x0;
    a[1] += (uint64_t)wl.y * x0;
    a[2] += (uint64_t)wl.z * x0;
    a[3] += (uint64_t)wl.x * x1;
    a[4] += (uint64_t)wl.y * x1;
    a[5] += (uint64_t)wl.z * x1;
}
// (sum_{i<3, h<2} a[3h + i] * 2^(22 i + 32 h)) mod p, a < 2^63 (U, W < 2^108)
__device__ __forceinline__ uint64_t wl_reduce(const uint64_t (&a)[6]) {
    const u128_t U = (u128_t)a[0] + ((u128_t)a[1] << 22) + ((u128_t)a[2] << 44);
    const u128_t W = (u128_t)a[3] + ((u128_t)a[4] << 22) + ((u128_t)a[5] << 44);
    const uint64_t ur = reduce_u108(U), wr = reduce_u108(W);
    return gl_add(ur, reduce96(wr << 32, (uint32_t)(wr >> 32)));  // + wr * 2^32
}

// 6 waves per SIMD (80 VGPRs with a 64-byte spill; 127 VGPRs and 4 waves unconstrained): the
// kernel waits on its row loads, and more waves cover the wait: config 4 +0.9% at 4,096 proofs,
// 512 equal (profiles/r03zc; 5 waves +0.5%)
#ifndef NHIP_DEEP_WAVES
#define NHIP_DEEP_WAVES 6
#endif
template <bool MW>
__global__ void __launch_bounds__(256, NHIP_DEEP_WAVES) k_deep_rows8(const uint64_t* __restrict__ words,
                                                    const ProofDesc* __restrict__ desc, uint32_t n_proofs,
                                                    StarkDims dims, const uint64_t* __restrict__ xs,
                                                    const uint64_t* __restrict__ xdom,
                                                    const uint64_t* __restrict__ ood, uint32_t* __restrict__ fail) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t M = dims.num_main, A = dims.num_aux, Q = dims.num_quot_seg, k = dims.num_checks;
    uint4* wm = reinterpret_cast<uint4*>(smem);        // [M][3 coeff] main weights (raw), w_limbs
    uint4* wa = wm + 3 * M;                            // [A][3 m][3 coeff] aux weights w X^m (raw), w_limbs
    Xfe* rowsum = reinterpret_cast<Xfe*>(wa + 9 * A);  // [k] row linear combinations (raw)
    __shared__ Xfe s_quot[MAX_CHECKS];
    __shared__ Xfe s_at[3];
    const uint32_t p = blockIdx.x, tid = threadIdx.x;
    if (p >= n_proofs || (fail[p] & FAIL_DECODE)) return;
    const ProofDesc& d = desc[p];
    const SampleLayout sl = SampleLayout::of(dims, d.R);
    const uint64_t xb = d.xs_off * 3;
    const uint64_t* __restrict__ lw = xs + xb + 3ull * sl.lin_w;
    for (uint32_t i = tid; i < 3 * M; i += blockDim.x) wm[i] = w_limbs(lw[i]);
    for (uint32_t c = tid; c < A; c += blockDim.x) {
        const uint64_t w0 = lw[3 * (M + c)], w1 = lw[3 * (M + c) + 1], w2 = lw[3 * (M + c) + 2];
        uint4* o = wa + 9 * c;
        o[0] = w_limbs(w0), o[1] = w_limbs(w1), o[2] = w_limbs(w2);
        o[3] = w_limbs(gl_sub(0, w2)), o[4] = w_limbs(gl_add(w0, w2)), o[5] = w_limbs(w1);
        o[6] = w_limbs(gl_sub(0, w1)), o[7] = w_limbs(gl_sub(w1, w2)), o[8] = w_limbs(gl_add(w0, w2));
    }
    if (tid == blockDim.x - 1) {
        const Xfe z = ld_xfe_raw(xs, xb + 3ull * sl.z);
        s_at[0] = z;
        s_at[1] = x_scale(z, root_of_unity(d.log2_ph));
        Xfe zq = x_one();
        for (uint32_t q = 0; q < Q; ++q) zq = x_mul(zq, z);
        s_at[2] = zq;
    }
    __syncthreads();
    const uint32_t q8 = tid & 7u, rloc = tid >> 3;
    const uint32_t rows_per_pass = blockDim.x >> 3;
    for (uint32_t j0 = 0; j0 < k; j0 += rows_per_pass) {
        const uint32_t j = j0 + rloc;
        uint64_t acc[3][6];
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int q = 0; q < 6; ++q) acc[c][q] = 0;
        if (j < k) {
            const uint64_t* __restrict__ mrow = words + d.main_rows_off + (uint64_t)j * M;
            uint32_t c = q8;
            for (; c + 8 * (DEEP_UNROLL - 1) < M; c += 8 * DEEP_UNROLL) {
                uint64_t xv[DEEP_UNROLL];
#pragma unroll
                for (uint32_t u = 0; u < DEEP_UNROLL; ++u) xv[u] = mrow[c + 8 * u];
#pragma unroll
                for (uint32_t u = 0; u < DEEP_UNROLL; ++u) {
                    const uint32_t cc = c + 8 * u, x0 = (uint32_t)xv[u], x1 = (uint32_t)(xv[u] >> 32);
                    wl_mac(acc[0], wm[3 * cc], x0, x1);
                    wl_mac(acc[1], wm[3 * cc + 1], x0, x1);
                    wl_mac(acc[2], wm[3 * cc + 2], x0, x1);
                }
            }
            for (; c < M; c += 8) {
                const uint64_t xw = mrow[c];
                const uint32_t x0 = (uint32_t)xw, x1 = (uint32_t)(xw >> 32);
                wl_mac(acc[0], wm[3 * c], x0, x1);
                wl_mac(acc[1], wm[3 * c + 1], x0, x1);
                wl_mac(acc[2], wm[3 * c + 2], x0, x1);
            }
            // aux row: word w is coefficient m = w % 3 of column w / 3
            const uint64_t* __restrict__ arow = words + d.aux_rows_off + (uint64_t)j * 3 * A;
            const uint32_t WA = 3 * A;
            uint32_t w = q8;
            for (; w + 8 * (DEEP_UNROLL - 1) < WA; w += 8 * DEEP_UNROLL) {
                uint64_t xv[DEEP_UNROLL];
#pragma unroll
                for (uint32_t u = 0; u < DEEP_UNROLL; ++u) xv[u] = arow[w + 8 * u];
#pragma unroll
                for (uint32_t u = 0; u < DEEP_UNROLL; ++u) {
                    // aux word ww is coefficient m = ww % 3 of column ww / 3: weight row 3 ww of wa
                    const uint4* wt = wa + 3 * (w + 8 * u);
                    const uint32_t x0 = (uint32_t)xv[u], x1 = (uint32_t)(xv[u] >> 32);
                    wl_mac(acc[0], wt[0], x0, x1);
                    wl_mac(acc[1], wt[1], x0, x1);
                    wl_mac(acc[2], wt[2], x0, x1);
                }
            }
            for (; w < WA; w += 8) {
                const uint4* wt = wa + 3 * w;
                const uint64_t xw = arow[w];
                const uint32_t x0 = (uint32_t)xw, x1 = (uint32_t)(xw >> 32);
                wl_mac(acc[0], wt[0], x0, x1);
                wl_mac(acc[1], wt[1], x0, x1);
                wl_mac(acc[2], wt[2], x0, x1);
            }
        }
        // the row's 8 lanes: reduce, then add (every lane of the wave takes part in the shuffles)
        uint64_t v0 = wl_reduce(acc[0]), v1 = wl_reduce(acc[1]), v2 = wl_reduce(acc[2]);
#pragma unroll
        for (int m = 1; m < 8; m <<= 1) {
            v0 = gl_add(v0, shfl_xor_u64(v0, m));
            v1 = gl_add(v1, shfl_xor_u64(v1, m));
            v2 = gl_add(v2, shfl_xor_u64(v2, m));
        }
        if (j < k && q8 == 0) {
            // canonical words: R * sum w x, the raw word; Montgomery words: R^2 * sum w x, one reduction
            if constexpr (MW) rowsum[j] = {from_mont(v0), from_mont(v1), from_mont(v2)};
            else rowsum[j] = {v0, v1, v2};
        }
        if (j < k && q8 == 1) {
            // quotient segments: sum_q w_q * seg_q; Montgomery products of the raw weights with canonical
            // words are canonical values (to_mont makes them raw), with Montgomery words raw already
            Xfe qv = x_zero();
            for (uint32_t q = 0; q < Q; ++q)
                qv = x_add(qv, x_mul(ld_xfe_raw(lw, 3ull * (M + A + q)),
                                     ld_xfe_raw(words, d.quot_rows_off + (uint64_t)j * 3 * Q + 3ull * q)));
            if constexpr (MW) s_quot[j] = qv;
            else s_quot[j] = {to_mont(qv.c0), to_mont(qv.c1), to_mont(qv.c2)};
        }
    }
    __syncthreads();
    uint32_t f = 0;
    for (uint32_t j2 = tid; j2 < k; j2 += blockDim.x) {
        const Xfe row = rowsum[j2];
        const Xfe x = x_lift(xdom[(uint64_t)p * k + j2]);
        const Xfe d0 = x_sub(x, s_at[0]), d1 = x_sub(x, s_at[1]), d2 = x_sub(x, s_at[2]);
        const Xfe d01 = x_mul(d0, d1);
        const Xfe prod = x_mul(d01, d2);
        if (x_is_zero(prod)) {
            f |= FAIL_ZERO_INVERSE;
            continue;
        }
        const Xfe inv = x_inv(prod);
        const Xfe inv2 = x_mul(inv, d01);   // 1 / d2
        const Xfe inv01 = x_mul(inv, d2);   // 1 / (d0 d1)
        const Xfe inv0 = x_mul(inv01, d1);  // 1 / d0
        const Xfe inv1 = x_mul(inv01, d0);  // 1 / d1
        const uint64_t* __restrict__ oo = ood + (uint64_t)p * 9;
        const uint64_t* __restrict__ wd = lw + 3ull * (M + A + Q);
        const Xfe t0 = x_mul(x_mul(x_sub(row, ld_xfe_raw(oo, 0)), inv0), ld_xfe_raw(wd, 0));
        const Xfe t1 = x_mul(x_mul(x_sub(row, ld_xfe_raw(oo, 3)), inv1), ld_xfe_raw(wd, 3));
        const Xfe t2 = x_mul(x_mul(x_sub(s_quot[j2], ld_xfe_raw(oo, 6)), inv2), ld_xfe_raw(wd, 6));
        const Xfe deep = x_add(x_add(t0, t1), t2);
        const Xfe fri_v = ld_xfe_w<MW>(words, d.fri[0].leaves_off + 3ull * j2);
        if (!x_eq(deep, fri_v)) f |= FAIL_DEEP;
    }
    if (f) atomicOr(&fail[p], f);
}

__global__ void k_verdicts(const uint32_t* __restrict__ fail, uint32_t n, uint8_t* __restrict__ v) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = fail[i] == 0 ? 1 : 0;
    if (i == 0) atomicAdd(&g_batches_done, 1u);  // the batch's last kernel: one more finished launch
}
// Small batches (n_records + n_proofs <= ROOTS_ONE_WG): the root checks and the verdicts in one
// workgroup, one launch (one dependent packet fewer).  The fail words are read back past the L1 (a
// root check's atomicOr lands in L2) after every lane's atomics have completed (fence + barrier).
static constexpr uint32_t ROOTS_ONE_WG = 1024;
template <bool MW>
__global__ void __launch_bounds__(ROOTS_ONE_WG) k_roots_verdicts_small(
    const uint64_t* __restrict__ words, const ProofDesc* __restrict__ desc, const uint64_t* __restrict__ dig,
    MpPlan plan, uint32_t n_records, uint32_t trees_per_proof, uint32_t k, uint32_t* __restrict__ fail,
    uint32_t n_proofs, LcwTree lcw, uint8_t* __restrict__ v) {
    const uint32_t i = threadIdx.x;
    mp_roots_body<MW>(i, words, desc, dig, plan, n_records, trees_per_proof, k, fail, n_proofs, lcw);
    __threadfence();
    __syncthreads();
    if (i < n_proofs) v[i] = __hip_atomic_load(&fail[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 ? 1 : 0;
    if (i == 0) atomicAdd(&g_batches_done, 1u);  // the batch's last kernel: one more finished launch
}

// ------------------------------------------------------------------ launchers
// A launch with dispatch begin / end events when given (hipExtLaunchKernel: the launch-timing
// passes), a plain launch otherwise, so an untimed batch's launch sequence can be captured into a
// HIP graph (nhip_batch_launch).
template <typename K, typename... A>
static void launch_ev(K kernel, dim3 grid, dim3 block, size_t shm, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                      A... args) {
    if (e0 || e1) hipExtLaunchKernelGGL(kernel, grid, block, shm, s, e0, e1, 0, args...);
    else hipLaunchKernelGGL(kernel, grid, block, shm, s, args...);
}

// OOD evaluator workgroup: 1,024 threads for batches of at most OOD_WIDE_MAX_PROOFS proofs
// (NHIP_OOD_WIDE_MAX overrides, A/B runs), else 256
static bool ood_wide(uint32_t n) {
    static const uint32_t lim = [] {
        const char* v = nhip::ab_env("NHIP_OOD_WIDE_MAX");
        return v ? (uint32_t)std::strtoul(v, nullptr, 10) : OOD_WIDE_MAX_PROOFS;
    }();
    return n <= lim;
}

// Level-synchronous batches of deep trees (>= CLIMB_FROM_MIN_LEVELS hash levels: BASELINE config 5's
// height-23 proofs have 26) hand the rest of their trees to one per-tree climb launch (k_mp_climb
// from a start level) at the first level with at most climb_from_ops() hash ops: the top levels of a
// deep tree are launch-bound, not VALU-bound.  Measured (profiles/r05z/ab/climb_from_ab_r05q.txt):
// config 5's 64 proofs +3-6% at 4,096 ops; config 4's trees (<= 19 levels) are not affected (at
// 4,096 ops without the depth gate: 512 proofs -2 to -4%, 4,096 equal; 16K / 64K ops: worse).
// nhip_set_climb_from_ops sets the threshold for every depth (tests: 0 = never).
static constexpr uint32_t CLIMB_FROM_MIN_LEVELS = 24;
static constexpr uint64_t CLIMB_FROM_OPS_DEFAULT = 4096;
static std::atomic<int64_t>& climb_from_forced() {
    static std::atomic<int64_t> v(-1);
    return v;
}
int set_climb_from_ops(int64_t ops) {
    if (ops < -1) return -1;
    climb_from_forced().store(ops, std::memory_order_relaxed);
    return 0;
}
static uint64_t climb_from_ops(uint32_t hash_levels) {
    const int64_t v = climb_from_forced().load(std::memory_order_relaxed);
    if (v >= 0) return (uint64_t)v;
    return hash_levels >= CLIMB_FROM_MIN_LEVELS ? CLIMB_FROM_OPS_DEFAULT : 0ull;
}


// batches of at most this many proofs hash their revealed rows in the 16-lane form (k_hash_rows_wide)
static constexpr uint32_t ROWS_WIDE_MAX_PROOFS = 32;
static uint32_t rows_wide_max() {
    static const uint32_t v = [] {
        const char* e = nhip::ab_env("NHIP_ROWS_WIDE_MAX");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : ROWS_WIDE_MAX_PROOFS;
    }();
    return v;
}

// Fiat-Shamir replay form for an n-proof batch (see k_fs_replay_wide / k_fs_replay_quad):
// 0 = 16-lane row, 1 = two-row pair, 2 = quad.  A forced form (nhip_set_fs_form: tests and A/B
// runs; NHIP_FS_FORM=row|pair|quad sets the initial value, read once) overrides the size rule.
enum FsForm { FS_ROW = 0, FS_PAIR = 1, FS_QUAD = 2 };
// k_fs_replay_quad workgroup size (NHIP_QUAD_WG = 64..1024 overrides, A/B runs)
static uint32_t quad_wg() {
    static const uint32_t v = [] {
        const char* e = nhip::ab_env("NHIP_QUAD_WG");
        const uint32_t w = e ? (uint32_t)std::strtoul(e, nullptr, 10) : FS_QUAD_WG;
        return (w >= 64 && w <= 1024 && w % 64 == 0) ? w : FS_QUAD_WG;
    }();
    return v;
}
static std::atomic<int>& fs_form_forced() {
    static std::atomic<int> f([] {
        if (const char* v = nhip::ab_env("NHIP_FS_FORM")) {
            if (v[0] == 'q') return (int)FS_QUAD;
            if (v[0] == 'p') return (int)FS_PAIR;
            if (v[0] == 'r') return (int)FS_ROW;
        }
        return -1;
    }());
    return f;
}
int set_fs_form(int form) {
    if (form < -1 || form > (int)FS_QUAD) return -1;
    fs_form_forced().store(form, std::memory_order_relaxed);
    return 0;
}
static FsForm fs_form(uint32_t n) {
    static const uint32_t quad_min = [] {
        const char* v = nhip::ab_env("NHIP_FS_QUAD_MIN");
        return v ? (uint32_t)std::strtoul(v, nullptr, 10) : FS_QUAD_MIN_PROOFS;
    }();
    const int forced = fs_form_forced().load(std::memory_order_relaxed);
    if (forced >= 0) return (FsForm)forced;
    if (n < FS_PAIR_MAX_PROOFS) return FS_PAIR;
    return n >= quad_min ? FS_QUAD : FS_ROW;
}

#ifdef NHIP_AB_BUILD
// A/B build only: an empty kernel, NHIP_PAD_PACKETS of them after each kernel of the batch (what one
// more dependent packet in a batch's chain costs under load)
__global__ void k_pad_packet() {}
#endif

template <bool MW>
static hipError_t launch_phases(const StarkBatchDev& b, hipStream_t st, hipStream_t sa, StarkPhaseTimer* tm) {
    const uint32_t n = b.n_proofs;
    if (n == 0) return hipSuccess;
    (void)hipGetLastError();  // the launch errors below are this launch's, not an earlier call's
    const uint32_t k = b.dims.num_checks;
    const uint32_t tpp = 4 + b.max_R;
    // Events: the phase timestamps (every one, when tm->phase_marks) and the cross-stream fork / join
    // points (SYNC: recorded whenever the batch runs on two streams).  A replayed graph of a
    // one-stream batch (no phase split, nhip_batch_set_graph) records none and waits on none: each
    // record or wait is one more packet in the batch's dependent chain.
    const bool two = st != sa;
    constexpr uint32_t SYNC = (1u << 12) | (1u << 0) | (1u << 1) | (1u << 3) | (1u << 7) | (1u << 10) | (1u << 8);
    auto mark = [&](int i, hipStream_t s) {
        if (tm->phase_marks || (two && ((SYNC >> i) & 1u))) (void)hipEventRecord(tm->ev[i], s);
    };
    auto wait = [&](hipStream_t s, int i) {
        if (two) (void)hipStreamWaitEvent(s, tm->ev[i], 0);
    };
#ifdef NHIP_AB_BUILD
    static const int pad_n = [] {
        const char* e = nhip::ab_env("NHIP_PAD_PACKETS");
        return e ? std::atoi(e) : 0;
    }();
    auto pad = [&](hipStream_t s) {
        for (int i = 0; i < pad_n; ++i) hipLaunchKernelGGL(k_pad_packet, dim3(1), dim3(64), 0, s);
    };
#else
    auto pad = [](hipStream_t) {};
#endif
    // small batches: every Merkle tree climbed in one launch (k_mp_climb), and FRI on the main
    // stream (it needs only the sponge samples) concurrent with the plan and OOD on the aux stream;
    // DEEP (which needs both) waits for it.  With the climb that short, OOD -> FRI -> DEEP in a row
    // would be the critical path.
    const bool small = n <= climb_max_proofs();
    // this launch's place in the device's launch order, for the oldest-first priority: the 2 oldest
    // batches in flight one level up, for batches of at least AGE_PRIO_MIN_PROOFS (A/B knobs:
    // NHIP_AGE_PRIO=k sets k for every size, 0 = off; NHIP_AGE_PRIO_FS=1 raises the sponge too)
    static const int64_t age_env = [] {
        const char* e = nhip::ab_env("NHIP_AGE_PRIO");
        return e ? (int64_t)std::strtoul(e, nullptr, 10) : (int64_t)-1;
    }();
    const uint32_t age_k = age_env >= 0 ? (uint32_t)age_env : (n >= AGE_PRIO_MIN_PROOFS ? AGE_PRIO_OLDEST : 0u);
    static std::atomic<uint32_t> seq_ctr[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    const AgePrio age{seq_ctr[(uint32_t)dev & 63u].fetch_add(1u, std::memory_order_relaxed), age_k};
    static const bool age_fs = [] {  // NHIP_AGE_PRIO_FS=1 (A/B): the sponge replay raised as well
        const char* e = nhip::ab_env("NHIP_AGE_PRIO_FS");
        return e && e[0] == '1';
    }();
    const AgePrio age_sponge{age.seq, age_fs ? age.k : 0u};
    // fork: the aux stream starts after everything already queued on st (counter resets)
    mark(12, st);
    wait(sa, 12);
    // proof-stream decode of every proof (descriptors, Fiat-Shamir programs, fail words), on the
    // aux stream: the Fiat-Shamir replay is the next packet of that queue, so it is dispatched
    // the moment decode ends, before the row hashing (main stream, waiting on the same event) can
    // fill the CUs.  Decoding on the main stream instead let k_hash_rows take every wave slot first
    // and stretched the latency-bound sponge replay 1.6 -> 5.0 ms (config 4, one step in flight).
    hipLaunchKernelGGL(k_decode<MW>, dim3(n), dim3(64), 0, sa, b.words, b.in, n, b.D, b.fs_stride, b.xs_stride, b.desc,
                       b.ops, b.fail, b.counters);
    pad(sa);
    mark(0, sa);
    wait(st, 0);
    // ---- aux stream: latency-bound chain
    // small batches: the sponge replay is the critical path and most SIMDs are idle, so two rows
    // per proof (pair form) for a shorter permutation; large ones: one row per proof (fewer
    // lane-instructions while the other steps' hashing fills the GPU); the largest: four lanes per
    // proof (quad form, fewer lane-instructions again).  NHIP_FS_FORM forces one.
    const FsForm ff = fs_form(n);
    // one stream, pair form, 16-lane rows: the replay and the row hashing in one launch
    static const bool fuse_env = [] {  // A/B build: NHIP_FUSE_SMALL=0 launches them apart
        const char* e = nhip::ab_env("NHIP_FUSE_SMALL");
        return !(e && e[0] == '0');
    }();
    const bool fused = fuse_env && !two && ff == FS_PAIR && n <= rows_wide_max() && !tm->launch_events;
    const uint64_t rows = (uint64_t)n * k;
    if (fused) {
        const uint32_t fs_blocks = (n * 32 + 255) / 256;
        const uint32_t rows_gx = (uint32_t)((rows * 16 + 255) / 256);
        hipLaunchKernelGGL(k_fs_rows_small<MW>, dim3(fs_blocks + 3 * rows_gx), dim3(256), 0, sa, b.words, b.desc,
                           b.ops, n, b.xs, b.idx, b.fail, age_sponge, fs_blocks, rows_gx, k, b.dims, b.dig);
    } else if (ff == FS_PAIR)
        hipLaunchKernelGGL((k_fs_replay_wide<true, MW>), dim3((n * 32 + 255) / 256), dim3(256), 0, sa, b.words, b.desc,
                           b.ops, n, b.xs, b.idx, b.fail, age_sponge);
    else if (ff == FS_QUAD)
        hipLaunchKernelGGL(k_fs_replay_quad<MW>, dim3((n * 4 + quad_wg() - 1) / quad_wg()), dim3(quad_wg()), 0, sa, b.words, b.desc, b.ops, n,
                           b.xs, b.idx, b.fail, age_sponge);
    else
        hipLaunchKernelGGL((k_fs_replay_wide<false, MW>), dim3((n * 16 + 255) / 256), dim3(256), 0, sa, b.words, b.desc,
                           b.ops, n, b.xs, b.idx, b.fail, age_sponge);
    pad(sa);
    mark(1, sa);
    // one stream, small, k <= 256: the plan and FRI in one launch
    static const bool fuse2_env = [] {  // A/B build: NHIP_FUSE_PLAN_FRI=0 launches them apart
        const char* e = nhip::ab_env("NHIP_FUSE_PLAN_FRI");
        return !(e && e[0] == '0');
    }();
    const bool fused2 = fuse2_env && !two && small && k <= 256;
    if (fused2) {
        mark(13, sa);
        hipLaunchKernelGGL(k_plan_fri_small<MW>, dim3(n * (1 + b.max_R) + n), dim3(256), 0, sa, b.words, b.desc, n,
                           k, tpp, 1 + b.max_R, b.dig, b.idx, b.mp, b.fail, b.counters + CNT_MP_SKIPPED, b.dims, b.xs,
                           b.xdom);
    } else if (k <= 128)
        hipLaunchKernelGGL(k_mp_plan<128>, dim3(n, 1 + b.max_R), dim3(128), 0, sa, b.words, b.desc, n, k, tpp, b.dig,
                           b.idx, b.mp, b.fail, b.counters + CNT_MP_SKIPPED);
    else
        hipLaunchKernelGGL(k_mp_plan<256>, dim3(n, 1 + b.max_R), dim3(256), 0, sa, b.words, b.desc, n, k, tpp, b.dig,
                           b.idx, b.mp, b.fail, b.counters + CNT_MP_SKIPPED);
    pad(sa);
    mark(3, sa);
    // ---- main stream: VALU-bound hashing
    if (!fused) {
        unsigned gx = (unsigned)((rows + 255) / 256);
        if (gx > 16384) gx = 16384;
        // dispatch begin / end events (the row kernel's own duration, as the kernel trace has it)
        hipEvent_t r0 = tm->launch_events ? tm->rev[0] : nullptr, r1 = tm->launch_events ? tm->rev[1] : nullptr;
        if (n <= rows_wide_max())
            launch_ev(k_hash_rows_wide<MW>, dim3((unsigned)((rows * 16 + 255) / 256), 3), dim3(256), 0, st,
                                  r0, r1, b.words, b.desc, n, k, b.dims, b.dig, b.fail);
        else
            launch_ev(k_hash_rows<MW>, dim3(gx, 3), dim3(256), 0, st, r0, r1, b.words, b.desc, n, k,
                                  b.dims, b.dig, b.fail, age);
    }
    pad(st);
    mark(2, st);
    if (small && fused2) {
        mark(7, st);  // FRI ran with the plan
    } else if (small) {
        wait(st, 1);  // sponge replay done
        mark(13, st);
        hipLaunchKernelGGL(k_fri<MW>, dim3(n), dim3(256), 0, st, b.words, b.desc, n, b.dims, b.xs, b.idx, b.xdom, b.fail);
        pad(st);
        mark(7, st);
    }
    wait(st, 3);  // plan done
    // The OOD / FRI / DEEP chain only needs the Fiat-Shamir samples, but its kernels are latency-bound
    // and hold CU resources for long; started after the first `aux_after_level` (wide, VALU-bound)
    // hash levels it overlaps the narrow, latency-bound top levels instead.
    auto launch_aux_chain = [&]() {
        mark(10, st);
        if (!small) wait(sa, 10);  // small: OOD right after the plan
        mark(11, sa);
#define NHIP_OOD_LAUNCH(BLK, GS, THREADS)                                                                       \
    hipLaunchKernelGGL((k_ood_air<BLK, MW, GS>), dim3(n), dim3(THREADS), b.air_lds_bytes, sa, b.words, b.desc, n,    \
                       b.dims, b.air_prog, b.air_prog_off, b.air_n_levels, b.air_consts, b.air_cons_off, b.xs, b.ood, \
                       b.fail, b.air_lds_slots, b.air_gslots, b.air_gslot_n)
        const bool gs = b.air_gslot_n > 0;
        if (ood_wide(n)) {
            if (gs) NHIP_OOD_LAUNCH(1024, true, 1024);
            else NHIP_OOD_LAUNCH(1024, false, 1024);
        } else {
            if (gs) NHIP_OOD_LAUNCH(256, true, b.air_block);
            else NHIP_OOD_LAUNCH(256, false, b.air_block);
        }
#undef NHIP_OOD_LAUNCH
        pad(sa);
        mark(6, sa);
        if (small) {
            wait(sa, 7);  // FRI done (main stream)
        } else {
            hipLaunchKernelGGL(k_fri<MW>, dim3(n), dim3(256), 0, sa, b.words, b.desc, n, b.dims, b.xs, b.idx, b.xdom, b.fail);
            mark(7, sa);
        }
        hipLaunchKernelGGL(k_deep_rows8<MW>, dim3(n), dim3(256), deep_rows8_lds_bytes(b.dims), sa, b.words, b.desc, n,
                           b.dims, b.xs, b.xdom, b.ood, b.fail);
        pad(sa);
        mark(8, sa);
    };
    uint32_t launches = 0;
    bool aux_started = false;
    if (small) {  // every tree climbed by its own workgroup, one launch
        launch_aux_chain();
        aux_started = true;
        const bool timed = tm->launch_events && tm->lev[0] != nullptr;
        launch_ev(k_mp_climb<MW>, dim3(n, tpp + 1), dim3(MP_CLIMB_THREADS), 0, st,
                              timed ? tm->lev[0] : nullptr, timed ? tm->lev[1] : nullptr, b.words, b.dig, b.mp,
                              tpp, b.desc, n, (const uint32_t*)b.fail, LcwTree{b.lcw, b.max_lcw}, 0u);
        pad(st);
        launches = 1;
    }
    const LcwTree lcw{b.lcw, b.max_lcw};
    const uint32_t log2_lcw = 31 - __builtin_clz(b.max_lcw);
    const uint32_t hash_levels = b.mp.levels > log2_lcw ? b.mp.levels : log2_lcw;
    static const uint32_t mp_small_max = [] {
        const char* v = nhip::ab_env("NHIP_MP_SMALL_MAX");
        return v ? (uint32_t)std::strtoul(v, nullptr, 10) : MP_SMALL_MAX_PROOFS;
    }();
    // first level of the tail climbed in one launch (every level from it on is small)
    uint32_t tail0 = hash_levels;
    while (tail0 > 0 && hash_levels - tail0 < MP_TAIL_LEVELS_MAX) {
        const uint32_t l = tail0 - 1;
        const uint64_t ops = (l < b.mp.levels ? b.mp_cap_host[l] : 0) + (uint64_t)(b.max_lcw >> (l + 1)) * n;
        if (ops > MP_TAIL_MAX_OPS) break;
        --tail0;
    }
    if (hash_levels - tail0 < 2) tail0 = hash_levels;  // a single small level: the per-level launch
    for (uint32_t l = 0; l < hash_levels && !small; ++l) {
        if (!aux_started && (l >= tm->aux_after_level || l == tail0)) {  // the tail is one workgroup
            launch_aux_chain();
            aux_started = true;
        }
        const bool timed = tm->launch_events && launches < MAX_HASH_LAUNCHES && tm->lev[0] != nullptr;
        hipEvent_t e0 = timed ? tm->lev[2 * launches] : nullptr, e1 = timed ? tm->lev[2 * launches + 1] : nullptr;
        {
            // the rest of every tree climbed per (proof, tree group) in one launch once a level is small
            // (deep trees: climb_from_ops above)
            const uint64_t ops_l = (l < b.mp.levels ? b.mp_cap_host[l] : 0) + (uint64_t)(b.max_lcw >> (l + 1)) * n;
            const uint64_t cf = climb_from_ops(hash_levels);
            if (cf && ops_l <= cf && hash_levels - l >= 3) {
                launch_ev(k_mp_climb<MW>, dim3(n, tpp + 1), dim3(MP_CLIMB_THREADS), 0, st, e0, e1, b.words,
                                      b.dig, b.mp, tpp, b.desc, n, (const uint32_t*)b.fail, lcw, l);
                ++launches;
                break;
            }
        }
        if (l == tail0) {
            TailCaps caps{};
            for (uint32_t t = l; t < hash_levels; ++t) caps.cap[t - l] = t < b.mp.levels ? (uint32_t)b.mp_cap_host[t] : 0u;
            launch_ev(k_mp_hash_tail<MW>, dim3(1), dim3(MP_TAIL_THREADS), 0, st, e0, e1, b.words, b.dig,
                                  b.mp, l, hash_levels, caps, b.desc, n, (const uint32_t*)b.fail, lcw);
            ++launches;
            break;
        }
        const uint64_t cap = l < b.mp.levels ? b.mp_cap_host[l] : 0;
        const uint32_t mp_blocks = (uint32_t)((cap + 255) / 256);
        const uint64_t per = b.max_lcw >> (l + 1);
        const uint32_t lcw_blocks = (uint32_t)((per * n + 255) / 256);
        if (mp_blocks + lcw_blocks == 0) continue;
        const bool wide = cap + per * n <= MP_WIDE_MAX_OPS;
        // hipExtLaunchKernel's start / stop events take the dispatch's own begin / end timestamps
        // (what the rocprofv3 kernel trace reports): the launch's duration without the dispatch
        // gap before it, which a plain event pair around back-to-back launches would also hold
        if (wide)
            launch_ev(k_mp_hash_wide<MW>, dim3((unsigned)(((cap + per * n) * 16 + 255) / 256)), dim3(256), 0,
                                  st, e0, e1, b.words, b.dig, b.mp, l, cap, b.desc, n, (const uint32_t*)b.fail, lcw);
        else if (n < mp_small_max)
            launch_ev((k_mp_hash<NHIP_MP_WAVES_SMALL, MW>), dim3(mp_blocks + lcw_blocks), dim3(256), 0, st, e0,
                                  e1, b.words, b.dig, b.mp, l, mp_blocks, b.desc, n, (const uint32_t*)b.fail, lcw, age);
        else
            launch_ev((k_mp_hash<NHIP_MP_WAVES, MW>), dim3(mp_blocks + lcw_blocks), dim3(256), 0, st, e0, e1,
                                  b.words, b.dig, b.mp, l, mp_blocks, b.desc, n, (const uint32_t*)b.fail, lcw, age);
        ++launches;
    }
    if (!aux_started) launch_aux_chain();
    tm->mp_hash_launches = launches;
    mark(4, st);
    const uint32_t nrec = n * tpp;
    if (!two && nrec + n <= ROOTS_ONE_WG) {  // one stream (the aux chain is already in order): one launch
        hipLaunchKernelGGL(k_roots_verdicts_small<MW>, dim3(1), dim3(ROOTS_ONE_WG), 0, st, b.words, b.desc, b.dig,
                           b.mp, nrec, tpp, k, b.fail, n, lcw, b.verdicts);
        mark(5, st);
    } else {
        hipLaunchKernelGGL(k_mp_roots<MW>, dim3((nrec + n + 255) / 256), dim3(256), 0, st, b.words, b.desc, b.dig,
                           b.mp, nrec, tpp, k, b.fail, n, lcw);
        pad(st);
        mark(5, st);
        wait(st, 8);  // join the aux chain
        hipLaunchKernelGGL(k_verdicts, dim3((n + 255) / 256), dim3(256), 0, st, b.fail, n, b.verdicts);
    }
    mark(9, st);
    return hipGetLastError();
}

hipError_t launch_stark_phases(const StarkBatchDev& b, hipStream_t st, hipStream_t sa, StarkPhaseTimer* tm) {
    return b.D.mont_words ? launch_phases<true>(b, st, sa, tm) : launch_phases<false>(b, st, sa, tm);
}

template <bool MW>
static hipError_t set_attributes() {
    for (const void* f : {(const void*)k_ood_air<256, MW, false>, (const void*)k_ood_air<256, MW, true>,
                          (const void*)k_ood_air<1024, MW, false>, (const void*)k_ood_air<1024, MW, true>}) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, AIR_LDS_BUDGET);
        if (e != hipSuccess) return e;
    }
    return hipFuncSetAttribute((const void*)k_deep_rows8<MW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024 - 8192);
}

hipError_t stark_set_kernel_attributes() {
    const hipError_t e = set_attributes<false>();
    return e != hipSuccess ? e : set_attributes<true>();
}

}  // namespace nhip
