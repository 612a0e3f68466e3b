// MAST and mutator-set Tip5 workloads:
//
//  MastHash::merkle_tree / mast_hash (neptune-core/src/protocol/proof_abstractions/mast_hash.rs:22-39):
//    leaf i = Tip5::hash_varlen(field sequence i), padded with Digest::default() to a power of two,
//    root of the Merkle tree (parent = hash_pair(left, right)).  TransactionKernel has 8 fields
//    (transaction_kernel.rs:246-277), BlockHeader 8, BlockKernel 3, Block 2.  Field sequences are
//    hashed by k_hash_varlen; k_mast_roots climbs each object's small tree (one lane per object).
//  AbsoluteIndexSet::compute (util_types/mutator_set/removal_record/absolute_index_set.rs:86-113):
//    sponge = Tip5::init(); pad_and_absorb_all(item ++ sender_randomness ++ receiver_preimage ++
//    aocl_leaf_index.encode()); sample_indices(WINDOW_SIZE = 2^20, NUM_TRIALS = 45)
//    (util_types/mutator_set/shared.rs:12-15); minimum + batch offset, distances.  One lane per item.
#include "kernels.hpp"
#include "tip5_device.hpp"

namespace nhip {

// leaves: n_objects x fields digests (canonical, from k_hash_varlen); pow2 >= fields
__global__ void __launch_bounds__(256) k_mast_roots(const uint64_t* __restrict__ leaves, uint32_t fields, uint32_t pow2,
                                                    size_t n, uint64_t* __restrict__ roots) {
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    // iterative binary-counter climb over the pow2 leaves (missing ones = Digest::default())
    uint64_t stack[5][5];  // pow2 <= 16
    uint64_t cur[5];
    for (uint32_t j = 0; j < pow2; ++j) {
        if (j < fields) {
#pragma unroll
            for (int q = 0; q < 5; ++q) cur[q] = to_mont(leaves[((size_t)i * fields + j) * 5 + q]);
        } else {
#pragma unroll
            for (int q = 0; q < 5; ++q) cur[q] = 0;
        }
        uint32_t lvl = 0;
        for (uint32_t t = j; t & 1u; t >>= 1, ++lvl) {
            uint64_t s[16];
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                s[q] = stack[lvl][q];
                s[5 + q] = cur[q];
            }
            tip5_hash_pair_digest(s, t5.lut);  // capacity 1: FixedLength domain
#pragma unroll
            for (int q = 0; q < 5; ++q) cur[q] = s[q];
        }
#pragma unroll
        for (int q = 0; q < 5; ++q) stack[lvl][q] = cur[q];
    }
    const uint32_t top = 31 - __clz(pow2);
#pragma unroll
    for (int q = 0; q < 5; ++q) roots[i * 5 + q] = from_mont(stack[top][q]);
}

static constexpr uint32_t MS_WINDOW_SIZE = 1u << 20, MS_CHUNK_SIZE = 1u << 12, MS_BATCH_SIZE = 1u << 3,
                          MS_NUM_TRIALS = 45;

// in: n x 15 canonical words (item, sender_randomness, receiver_preimage), aocl leaf indices;
// out: minimum as u128 (2 u64, little-endian), 45 u32 distances
__global__ void __launch_bounds__(256) k_absolute_index_sets(const uint64_t* __restrict__ digests,
                                                             const uint64_t* __restrict__ aocl, size_t n,
                                                             uint64_t* __restrict__ minimum,
                                                             uint32_t* __restrict__ distances) {
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    // input = 15 digest words ++ u64 BFieldCodec (2 x u32 limbs, low limb first) = 17 words
    const uint64_t leaf = aocl[i];
    uint64_t s[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) s[q] = 0;
#pragma unroll
    for (int q = 0; q < 10; ++q) s[q] = to_mont(digests[i * 15 + q]);
    tip5_permute_raw(s, t5.lut);
#pragma unroll
    for (int q = 0; q < 5; ++q) s[q] = to_mont(digests[i * 15 + 10 + q]);
    s[5] = to_mont(leaf & 0xFFFFFFFFull);
    s[6] = to_mont(leaf >> 32);
    s[7] = MONT_ONE;  // padding: 7 of 10 rate words used
    s[8] = 0;
    s[9] = 0;
    tip5_permute_raw(s, t5.lut);
    uint32_t idx[MS_NUM_TRIALS];
    uint32_t got = 0;
    while (got < MS_NUM_TRIALS) {
        uint64_t out[TIP5_RATE];
#pragma unroll
        for (int q = 0; q < TIP5_RATE; ++q) out[q] = from_mont(s[q]);
        tip5_permute_raw(s, t5.lut);
        for (int q = 0; q < TIP5_RATE && got < MS_NUM_TRIALS; ++q)
            if (out[q] != GL_P - 1) idx[got++] = (uint32_t)(out[q] & 0xFFFFFFFFull) % MS_WINDOW_SIZE;
    }
    uint32_t mn = idx[0];
    for (uint32_t t = 1; t < MS_NUM_TRIALS; ++t) mn = idx[t] < mn ? idx[t] : mn;
    for (uint32_t t = 0; t < MS_NUM_TRIALS; ++t) distances[i * MS_NUM_TRIALS + t] = idx[t] - mn;
    // minimum = relative minimum + (aocl_leaf_index / BATCH_SIZE) * CHUNK_SIZE  (u128)
    const unsigned __int128 m = (unsigned __int128)mn + (unsigned __int128)(leaf / MS_BATCH_SIZE) * MS_CHUNK_SIZE;
    minimum[2 * i] = (uint64_t)m;
    minimum[2 * i + 1] = (uint64_t)(m >> 64);
}

hipError_t launch_mast_roots(const uint64_t* d_leaves, uint32_t fields, uint32_t pow2, size_t n, uint64_t* d_roots,
                             hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mast_roots, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_leaves, fields, pow2, n,
                       d_roots);
    return hipGetLastError();
}

hipError_t launch_absolute_index_sets(const uint64_t* d_digests, const uint64_t* d_aocl, size_t n, uint64_t* d_min,
                                      uint32_t* d_dist, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_absolute_index_sets, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_digests, d_aocl, n,
                       d_min, d_dist);
    return hipGetLastError();
}

}  // namespace nhip
