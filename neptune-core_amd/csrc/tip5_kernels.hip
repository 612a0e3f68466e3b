// Batched Tip5 / Merkle kernels for gfx950.
//
//  k_permutation   : Tip5::permutation over n independent states (canonical in/out).
//  k_hash_pair     : Tip5::hash_pair (FixedLength domain) over n digest pairs.
//  k_hash_varlen   : Tip5::hash_varlen over n ragged rows (row hashing of revealed STARK rows,
//                    MAST leaf hashing; mast_hash.rs:22-28 in the reference).
//  k_mtree_level   : one level of MTree::build_inplace (pow.rs:73-119): parent i = hash_pair(2i, 2i+1).
//  k_mtree_verify  : MTree::verify (pow.rs:162-180) for n authentication paths, one lane per path.
//
// Layout in HBM (canonical u64, BFieldElement::value()):
//   digest        = 5 consecutive u64                         (40 B)
//   path i        = depth digests, leaf-sibling first          (paths + i*depth*5)
//   states        = 16 consecutive u64 per state
// One lane owns one state; the state never leaves VGPRs between levels of a path.
#include "tip5_device.hpp"
#include "kernels.hpp"

#ifndef NHIP_MINWAVES
#define NHIP_MINWAVES 1  // min waves per SIMD requested from the register allocator
#endif
#ifndef NHIP_PAIR_WAVES
#define NHIP_PAIR_WAVES 6  // the hash_pair-only kernels (80 VGPRs with the MDS finished in pairs)
#endif

namespace nhip {

__device__ __forceinline__ void load_digest_mont(const uint64_t* __restrict__ p, uint64_t* d) {
#pragma unroll
    for (int k = 0; k < 5; ++k) d[k] = to_mont(p[k]);
}

__device__ __forceinline__ void store_digest_canon(uint64_t* __restrict__ p, const uint64_t* d) {
#pragma unroll
    for (int k = 0; k < 5; ++k) p[k] = from_mont(d[k]);
}

__global__ void __launch_bounds__(256, NHIP_MINWAVES) k_permutation(uint64_t* __restrict__ states, size_t n) {
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t s[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) s[k] = to_mont(states[i * 16 + k]);
        tip5_permute_raw(s, lds.lut);
#pragma unroll
        for (int k = 0; k < 16; ++k) states[i * 16 + k] = from_mont(s[k]);
    }
}

__global__ void __launch_bounds__(256, NHIP_PAIR_WAVES) k_hash_pair(const uint64_t* __restrict__ left, const uint64_t* __restrict__ right,
                                                   uint64_t* __restrict__ out, size_t n) {
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t s[16];
        load_digest_mont(left + 5 * i, s);
        load_digest_mont(right + 5 * i, s + 5);
        tip5_hash_pair_digest(s, lds.lut);  // capacity 1: FixedLength domain
        store_digest_canon(out + 5 * i, s);
    }
}

__global__ void __launch_bounds__(256, NHIP_MINWAVES) k_hash_varlen(const uint64_t* __restrict__ data, const uint64_t* __restrict__ offsets,
                                                     size_t n, uint64_t* __restrict__ out) {
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t beg = offsets[i], end = offsets[i + 1];
        const uint64_t len = end - beg;
        const uint64_t* __restrict__ row = data + beg;
        uint64_t s[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) s[k] = 0;
        uint64_t pos = 0;
        for (; pos + TIP5_RATE <= len; pos += TIP5_RATE) {
#pragma unroll
            for (int k = 0; k < TIP5_RATE; ++k) s[k] = to_mont(row[pos + k]);
            tip5_permute_raw(s, lds.lut);
        }
        const uint64_t rem = len - pos;
#pragma unroll
        for (int k = 0; k < TIP5_RATE; ++k) {
            const uint64_t v = (uint64_t)k < rem ? row[pos + k] : ((uint64_t)k == rem ? 1ull : 0ull);
            s[k] = to_mont(v);
        }
        tip5_permute_raw(s, lds.lut);
        store_digest_canon(out + 5 * i, s);
    }
}

__global__ void __launch_bounds__(256, NHIP_PAIR_WAVES) k_mtree_level(const uint64_t* __restrict__ children, uint64_t* __restrict__ parents,
                                                     size_t n_parents) {
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_parents;
         i += (size_t)gridDim.x * blockDim.x) {
        uint64_t s[16];
        load_digest_mont(children + 10 * i, s);
        load_digest_mont(children + 10 * i + 5, s + 5);
        tip5_hash_pair_digest(s, lds.lut);  // capacity 1: FixedLength domain
        store_digest_canon(parents + 5 * i, s);
    }
}

__global__ void __launch_bounds__(256, NHIP_PAIR_WAVES) k_mtree_verify(const uint64_t* __restrict__ roots, int per_path_root,
                                                      const uint64_t* __restrict__ indices,
                                                      const uint64_t* __restrict__ leaves,
                                                      const uint64_t* __restrict__ paths, uint32_t depth, size_t n,
                                                      uint8_t* __restrict__ verdicts) {
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t index = indices[i];
        // pow.rs:164-166: `if index > 1 << path.len() { return false; }` (release-mode shift masking)
        const uint64_t bound = 1ull << (depth & 63u);
        if (index > bound) {
            verdicts[i] = 0;
            continue;
        }
        uint64_t run[5];
        load_digest_mont(leaves + 5 * i, run);
        const uint64_t* __restrict__ path = paths + (size_t)5 * depth * i;
        uint64_t ri = index;
        for (uint32_t lvl = 0; lvl < depth; ++lvl) {
            uint64_t sib[5];
            load_digest_mont(path + 5 * (size_t)lvl, sib);
            uint64_t s[16];
            const bool odd = (ri & 1ull) != 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                s[k] = odd ? sib[k] : run[k];      // pow.rs:171-175: odd => hash_pair(sibling, running)
                s[5 + k] = odd ? run[k] : sib[k];
            }
            tip5_hash_pair_digest(s, lds.lut);  // capacity 1: FixedLength domain
#pragma unroll
            for (int k = 0; k < 5; ++k) run[k] = s[k];
            ri >>= 1;
        }
        const uint64_t* __restrict__ root = roots + (per_path_root ? 5 * i : 0);
        bool eq = true;
#pragma unroll
        for (int k = 0; k < 5; ++k) eq &= (run[k] == to_mont(root[k]));
        verdicts[i] = eq ? 1 : 0;
    }
}

static inline unsigned grid_for(size_t n, unsigned block) {
    size_t g = (n + block - 1) / block;
    const size_t cap = 256u * 64u;  // grid-stride beyond 16k workgroups
    if (g > cap) g = cap;
    if (g == 0) g = 1;
    return (unsigned)g;
}

hipError_t launch_permutation(uint64_t* d_states, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_permutation, dim3(grid_for(n, 256)), dim3(256), 0, st, d_states, n);
    return hipGetLastError();
}

hipError_t launch_hash_pair(const uint64_t* d_l, const uint64_t* d_r, uint64_t* d_out, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hash_pair, dim3(grid_for(n, 256)), dim3(256), 0, st, d_l, d_r, d_out, n);
    return hipGetLastError();
}

hipError_t launch_hash_varlen(const uint64_t* d_data, const uint64_t* d_off, size_t n, uint64_t* d_out,
                              hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hash_varlen, dim3(grid_for(n, 256)), dim3(256), 0, st, d_data, d_off, n, d_out);
    return hipGetLastError();
}

hipError_t launch_mtree_level(const uint64_t* d_children, uint64_t* d_parents, size_t n_parents, hipStream_t st) {
    if (n_parents == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mtree_level, dim3(grid_for(n_parents, 256)), dim3(256), 0, st, d_children, d_parents,
                       n_parents);
    return hipGetLastError();
}

hipError_t launch_mtree_verify(const uint64_t* d_roots, int per_path_root, const uint64_t* d_indices,
                               const uint64_t* d_leaves, const uint64_t* d_paths, uint32_t depth, size_t n,
                               uint8_t* d_verdicts, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mtree_verify, dim3(grid_for(n, 256)), dim3(256), 0, st, d_roots, per_path_root, d_indices,
                       d_leaves, d_paths, depth, n, d_verdicts);
    return hipGetLastError();
}

}  // namespace nhip
