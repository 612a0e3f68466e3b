// Internal launch wrappers (C++ linkage) shared between kernel TUs and the C-ABI layer.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ab_env.hpp"
#include "proof_codec.hpp"
#include "stark.hpp"
#include "xfe.hpp"

namespace nhip {

hipError_t launch_permutation(uint64_t* d_states, size_t n, hipStream_t st);
hipError_t launch_hash_pair(const uint64_t* d_l, const uint64_t* d_r, uint64_t* d_out, size_t n, hipStream_t st);
hipError_t launch_hash_varlen(const uint64_t* d_data, const uint64_t* d_off, size_t n, uint64_t* d_out,
                              hipStream_t st);
hipError_t launch_mtree_level(const uint64_t* d_children, uint64_t* d_parents, size_t n_parents, hipStream_t st);
hipError_t launch_mtree_verify(const uint64_t* d_roots, int per_path_root, const uint64_t* d_indices,
                               const uint64_t* d_leaves, const uint64_t* d_paths, uint32_t depth, size_t n,
                               uint8_t* d_verdicts, hipStream_t st);

// ---- MAST / mutator-set hashing (mast_kernels.hip)
hipError_t launch_mast_roots(const uint64_t* d_leaves, uint32_t fields, uint32_t pow2, size_t n, uint64_t* d_roots,
                             hipStream_t st);
hipError_t launch_absolute_index_sets(const uint64_t* d_digests, const uint64_t* d_aocl, size_t n, uint64_t* d_min,
                                      uint32_t* d_dist, hipStream_t st);

// ---- batched STARK verifier (stark_kernels.hip)
static constexpr uint32_t AIR_LDS_HEADER = (16 + 4 + 4 + 4) * 24 + 16;  // red (per wave), zinv, derived, misc, flag
static constexpr uint32_t AIR_LDS_BUDGET = 160 * 1024 - 8192;              // k_ood_air dynamic LDS cap
static constexpr uint32_t AIR_LDS_SLOTS_MAX = (AIR_LDS_BUDGET - AIR_LDS_HEADER) / 24;

// Level-synchronous Merkle multiproof plan (see k_mp_plan in stark_kernels.hip).  Ops of level l
// live in MP_SHARDS shards (shard = proof index % MP_SHARDS) so the per-level slot reservations of
// the plan workgroups spread over MP_SHARDS counters instead of contending on one.
static constexpr uint32_t MP_SHARDS = 16;
// levels with at most this many hash ops run the 16-lane-row Tip5 (latency-bound regime)
static constexpr uint64_t MP_WIDE_MAX_OPS = 48 * 1024;
// the last levels whose ops (multiproof + last-codeword parents) all fit this many rows are climbed
// by one workgroup in one launch (k_mp_hash_tail), up to MP_TAIL_LEVELS_MAX levels
#ifndef NHIP_MP_TAIL_MAX_OPS
#define NHIP_MP_TAIL_MAX_OPS 256
#endif
static constexpr uint64_t MP_TAIL_MAX_OPS = NHIP_MP_TAIL_MAX_OPS;
static constexpr uint32_t MP_TAIL_LEVELS_MAX = 32;
// batches of at most this many proofs climb every tree in its own workgroup (k_mp_climb), one
// launch for all levels, instead of one launch per level
static constexpr uint32_t MP_CLIMB_MAX_PROOFS = 32;
inline uint32_t climb_max_proofs() {  // NHIP_CLIMB_MAX overrides (A/B runs)
    static const uint32_t v = [] {
        const char* e = nhip::ab_env("NHIP_CLIMB_MAX");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : MP_CLIMB_MAX_PROOFS;
    }();
    return v;
}
// batches below this many proofs replay Fiat-Shamir on the two-row pair Tip5 (k_fs_replay_wide):
// one-collection latency 1.89 -> 1.65 ms, while from 512 proofs on (several steps in flight) the
// one-row form is 2-3% faster (profiles/r01i/ab_pair.log)
static constexpr uint32_t FS_PAIR_MAX_PROOFS = 512;
// batches of at least this many proofs replay Fiat-Shamir on the quad Tip5 (k_fs_replay_quad);
// NHIP_FS_QUAD_MIN overrides (A/B runs).  0.61x the row form's VALU instructions (profiles/r03g
// PMC), but fewer, longer replay waves: with 256-thread workgroups (one replay wave per SIMD of the
// CUs they land on) 4,096 proofs +1.5% and 2,048 +1.6% over the row form, 1,024 -3%; 64-thread
// workgroups -7 to -9% at every size, 512 / 1,024 threads -1 to -25% (profiles/r03g, 2 repetitions)
static constexpr uint32_t FS_QUAD_MIN_PROOFS = 2048;
static constexpr uint32_t FS_QUAD_WG = 256;  // k_fs_replay_quad workgroup size
// batches below this many proofs hash their Merkle levels with the 7-wave k_mp_hash instance, larger
// ones with the 6-wave one; NHIP_MP_SMALL_MAX overrides (A/B runs).  7 waves: 2,048 proofs +1.3%,
// 1,024 +1.2%, 512 +3%; 4,096 -0.6% (profiles/r03ze, r03zf)
static constexpr uint32_t MP_SMALL_MAX_PROOFS = 4096;
static constexpr uint32_t OOD_WIDE_MAX_PROOFS = 64;  // k_ood_air<1024> up to this many proofs per batch
struct MpRoot {
    uint64_t code;  // source code of the tree's final node, ~0 = no check (skipped or already failed)
    uint64_t root_off;
    uint32_t fail_bit, pad;
};
struct MpPlan {
    uint64_t* ops;                // 2 source codes per op
    uint64_t* arena;              // parent digest of op g (Montgomery), 5 words
    const uint64_t* shard_base;   // [levels][MP_SHARDS] first op index of the shard
    const uint64_t* shard_cap;    // [levels][MP_SHARDS] op capacity of the shard
    uint32_t* counter;            // [levels][MP_SHARDS] ops appended (zeroed per run)
    MpRoot* roots;                // n_proofs x (4 + max_R)
    uint32_t* dups;               // [n_proofs][1 + max_R][k] (slot, earlier slot) pairs of equal leaf indices
    uint32_t* ndup;               // [n_proofs][1 + max_R]
    uint32_t levels;
    // per (proof, tree group) and level: the group's first op and its ops per tree (written by the
    // plan; k_mp_climb walks them), and the number of levels recorded
    uint64_t* lvl_g0;   // [n_proofs][1 + max_R][levels]
    uint32_t* lvl_cnt;  // [n_proofs][1 + max_R][levels]
    uint32_t* lvl_n;    // [n_proofs][1 + max_R]
};

// One proof of a batch as staged for k_decode: its raw words and its staged claim encoding in the
// batch word buffer, and the padded height the host sized the batch's scratch with (from the
// proof header; SHAPE_NONE = malformed header).
struct ProofIn {
    uint64_t off, len;
    uint64_t claim_off;
    uint32_t claim_in_n, claim_out_n;
    uint32_t sized_log2_ph, pad;
};

// Merkle hash launches (k_mp_hash / k_mp_hash_wide) timed per launch (start / stop event pairs)
static constexpr uint32_t MAX_HASH_LAUNCHES = 64;

// device counters of a run (zeroed per run, read back with the verdicts)
enum : uint32_t { CNT_MP_SKIPPED = 0, CNT_PERMS_STATIC = 1, CNT_PERMS_LCW = 2, CNT_N = 4 };

struct StarkBatchDev {
    uint32_t n_proofs, max_R;
    StarkDims dims;
    Dims D;
    uint32_t fs_stride, xs_stride;  // per-proof Fiat-Shamir program slots / sample areas (k_decode)
    const ProofIn* in;
    const uint64_t* words;
    ProofDesc* desc;
    FsOp* ops;
    uint64_t* xs;
    uint32_t* idx;
    uint64_t* dig;
    uint64_t* ood;
    uint64_t* xdom;        // [n_proofs][k] round-0 FRI domain point of each check (raw), k_fri -> k_deep
    uint64_t* lcw;         // [n_proofs][max_lcw][5] last-codeword Merkle tree nodes (heap order)
    uint32_t max_lcw;      // max last-codeword length (power of two)
    uint32_t* fail;                    // set by k_decode (FAIL_DECODE or 0), then ORed by every check
    uint8_t* verdicts;
    unsigned long long* counters;      // CNT_*: multiproof ops skipped (trees whose authentication
                                       // structure failed), decoded permutation counts
    MpPlan mp;
    const uint64_t* mp_cap_host;  // host: op capacity per level (launch sizes)
    const OodIns* air_prog;        // compiled AIR (OodIns per level)
    const uint32_t* air_prog_off;  // [n_levels + 1]
    uint32_t air_n_levels;
    const Xfe* air_consts;         // constant table (raw Montgomery)
    uint4 air_cons_off;            // constraint-type boundaries
    size_t air_lds_bytes;
    uint32_t air_block;  // k_ood_air workgroup size (1,024 when the slot area keeps one workgroup per CU)
    uint32_t air_lds_slots;        // slots held in LDS
    uint32_t air_gslot_n;          // slots past the LDS budget, per proof, in air_gslots
    Xfe* air_gslots;               // [n_proofs][air_gslot_n]
};

// events: 0 start (after k_decode, aux stream) | fs | rows | mp plan | mp hash levels | mp roots | ood | fri | deep | 9 verdicts
// 10: main stream at the aux-chain release point, 11: aux stream after that wait, 12: before k_decode,
// 13: before FRI on the main stream (small batches)
static constexpr int STARK_EVENTS = 14;
struct StarkPhaseTimer {
    hipEvent_t ev[STARK_EVENTS];
    hipEvent_t lev[2 * MAX_HASH_LAUNCHES];  // per hash launch: dispatch begin / end (nullptr = untimed)
    hipEvent_t rev[2] = {nullptr, nullptr};  // the row-hashing launch: dispatch begin / end (nullptr = untimed)
    bool launch_events = false;  // use lev / rev on this launch (nhip_batch_set_launch_timing)
    bool phase_marks = true;     // record the phase events (off in a captured graph: no phase split)
    uint32_t mp_hash_launches;
    uint32_t aux_after_level = 0;  // hash levels launched before the OOD/FRI/DEEP chain is released
};

// Phases on two streams: st_aux runs the latency-bound chain (Fiat-Shamir -> Merkle plan -> OOD ->
// FRI -> DEEP), st the VALU-bound hashing (rows -> per-level Merkle hashes -> roots -> verdicts).
hipError_t launch_stark_phases(const StarkBatchDev& b, hipStream_t st, hipStream_t st_aux, StarkPhaseTimer* tm);
hipError_t stark_set_kernel_attributes();
// nhip_set_fs_form: -1 = by batch size (default), 0 row, 1 pair, 2 quad; -1 return = bad form
int set_fs_form(int form);
// nhip_set_climb_from_ops: -1 = default, 0 = never, k = at k hash ops; -1 return = bad value
int set_climb_from_ops(int64_t ops);

// k_deep_rows8's carry-free accumulation (stark_kernels.hip): a row has M + 3A < DEEP_ROW_WORDS_MAX
// words (dims_from), a lane takes at most ceil(M / 8) + ceil(3A / 8) <= DEEP_LANE_TERMS_MAX of them,
// each partial product is < 2^54, and a 64-bit accumulator must not reach 2^63
static constexpr uint32_t DEEP_ROW_WORDS_MAX = 2048;
static constexpr uint64_t DEEP_LANE_TERMS_MAX = (DEEP_ROW_WORDS_MAX - 1 + 14) / 8;
static_assert(DEEP_LANE_TERMS_MAX * (1ull << 54) < (1ull << 63), "k_deep_rows8 accumulators stay below 2^63");
// k_deep_rows8: the weights (one uint4 of limbs per coefficient), then one XFE per revealed row
inline size_t deep_rows8_lds_bytes(const StarkDims& d) {
    return (size_t)(3 * d.num_main + 9 * d.num_aux) * 16 + (size_t)d.num_checks * 24;
}

}  // namespace nhip
