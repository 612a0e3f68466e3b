// Proof-of-work Tip5 workloads, neptune-core/src/protocol/consensus/block/pow.rs:
//
//  guesser buffer  Pow::preprocess (:365-469) for MERKLE_TREE_HEIGHT h: 2^h buds
//                  bud(prefix, i) = hash_pair(prefix, [i, 0, 0, 0, 0]) (:321-323), NUM_BUD_LAYERS = 5
//                  sliding layers leaf[k] = hash_pair(bud[k], bud[(k + 2^i) mod 2^h]) (:427-435) so
//                  leaf k = the MTree root of buds k..k+31 (Pow::leaf, :325-331), the HardforkAlpha
//                  bit-reversal swap of the leaves (:451-458, bitreverse :349-356), then
//                  MTree::build_inplace (:66-119).  7 * 2^h permutations; h = 29 -> 3.8e9.
//  guess           Pow::guess (:471-507): indices (:333-343, NUM_INDEX_REPETITIONS = 63 chained
//                  hash_pairs), the two authentication paths (MTree::path, :151-160) read from the
//                  buffer, PowMastPaths::fast_mast_hash (:219-241) of the Pow, compared with the
//                  target.  One lane per nonce.
//  validate        Pow::validate (:509-557): index picker, both leaves rebuilt from buds (63
//                  permutations each), both MTree::verify climbs, fast_mast_hash, threshold.  One
//                  lane per block.
// Buffers hold raw Montgomery digests (5 u64); the C ABI converts at the boundary.
#include "kernels.hpp"
#include "pow.hpp"
#include "tip5_device.hpp"

namespace nhip {

__device__ __forceinline__ void hp_raw(const uint64_t* l, const uint64_t* r, uint64_t* out,
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

__device__ __forceinline__ void ld5(const uint64_t* __restrict__ p, uint64_t* d) {
#pragma unroll
    for (int q = 0; q < 5; ++q) d[q] = p[q];
}
__device__ __forceinline__ void st5(uint64_t* __restrict__ p, const uint64_t* d) {
#pragma unroll
    for (int q = 0; q < 5; ++q) p[q] = d[q];
}

__device__ __forceinline__ void bud_raw(const uint64_t* prefix, uint64_t index, uint64_t* out,
                                        const uint8_t* __restrict__ lut) {
    const uint64_t idx[5] = {to_mont(index), 0, 0, 0, 0};
    hp_raw(prefix, idx, out, lut);
}

__device__ __forceinline__ uint32_t bitreverse(uint32_t k, uint32_t log2_n) {
    return log2_n ? (__brev(k) >> (32u - log2_n)) : 0u;
}

__global__ void __launch_bounds__(256) k_pow_buds(PowPrefix prefix, uint64_t n, uint64_t* __restrict__ out) {
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t d[5];
    bud_raw(prefix.d, i, d, t5.lut);
    st5(out + 5 * i, d);
}

__global__ void __launch_bounds__(256) k_pow_layer(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                   uint64_t n, uint64_t shift) {
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint64_t a[5], b[5], d[5];
    ld5(in + 5 * k, a);
    ld5(in + 5 * ((k + shift) & (n - 1)), b);
    hp_raw(a, b, d, t5.lut);
    st5(out + 5 * k, d);
}

// leafs.swap(k, rev_k) for k < rev_k (disjoint pairs: one lane per pair owner)
__global__ void k_pow_bitrev_swap(uint64_t* __restrict__ leafs, uint64_t n, uint32_t log2_n) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint64_t r = bitreverse((uint32_t)k, log2_n);
    if (k >= r) return;
    uint64_t a[5], b[5];
    ld5(leafs + 5 * k, a);
    ld5(leafs + 5 * r, b);
    st5(leafs + 5 * k, b);
    st5(leafs + 5 * r, a);
}

// parents [p0, 2 p0) of the MTree from children (leaves: node n + k lives at leafs[k])
__global__ void __launch_bounds__(256) k_pow_tree_level(const uint64_t* __restrict__ children, uint64_t* __restrict__ nodes,
                                                        uint64_t p0) {
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p0) return;
    uint64_t a[5], b[5], d[5];
    ld5(children + 10 * i, a);
    ld5(children + 10 * i + 5, b);
    hp_raw(a, b, d, t5.lut);
    st5(nodes + 5 * (p0 + i), d);
}

// ---------------------------------------------------------------- shared per-lane helpers
// Pow::indices (:333-343): indexer = hash_pair(hash, nonce), 62 x hash_pair(indexer, default)
__device__ void pow_indices(const uint64_t* picker, const uint64_t* nonce, uint32_t h, uint64_t& ia, uint64_t& ib,
                            const uint8_t* __restrict__ lut) {
    uint64_t x[5];
    hp_raw(picker, nonce, x, lut);
    const uint64_t zero[5] = {0, 0, 0, 0, 0};
    for (int r = 1; r < POW_NUM_INDEX_REPETITIONS; ++r) hp_raw(x, zero, x, lut);
    const uint64_t mask = (h >= 64) ? ~0ull : ((1ull << h) - 1);
    ia = from_mont(x[0]) & mask;
    ib = from_mont(x[1]) & mask;
}

// Tip5::hash_varlen of `len` raw words produced by `get(i)` (VariableLength sponge)
template <class F>
__device__ void varlen_raw(F get, uint32_t len, uint64_t* out, const uint8_t* __restrict__ lut) {
    uint64_t s[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) s[q] = 0;
    uint32_t pos = 0;
    for (; pos + TIP5_RATE <= len; pos += TIP5_RATE) {
        for (int q = 0; q < TIP5_RATE; ++q) s[q] = get(pos + q);
        tip5_permute_raw(s, lut);
    }
    const uint32_t rem = len - pos;
    for (uint32_t q = 0; q < TIP5_RATE; ++q) s[q] = q < rem ? get(pos + q) : (q == rem ? MONT_ONE : 0ull);
    tip5_permute_raw(s, lut);
#pragma unroll
    for (int q = 0; q < 5; ++q) out[q] = s[q];
}

// PowMastPaths::fast_mast_hash (:219-241).  pow.encode() = nonce ++ path_b ++ path_a ++ root
// (BFieldCodec: derived struct fields in reverse order, static-size fields without prefix).
template <class PathA, class PathB>
__device__ void fast_mast_hash(const PowMast& m, const uint64_t* root, PathA pa, PathB pb, const uint64_t* nonce,
                               uint32_t h, uint64_t* out, const uint8_t* __restrict__ lut) {
    const uint32_t len = 10 * h + 10;
    auto get = [&](uint32_t i) -> uint64_t {
        if (i < 5) return nonce[i];
        i -= 5;
        if (i < 5 * h) return pb(i / 5)[i % 5];
        i -= 5 * h;
        if (i < 5 * h) return pa(i / 5)[i % 5];
        return root[i - 5 * h];
    };
    uint64_t x[5], y[5];
    varlen_raw(get, len, x, lut);
    hp_raw(x, m.pow[0], y, lut);
    hp_raw(y, m.pow[1], x, lut);
    hp_raw(m.pow[2], x, y, lut);  // header mast hash
    varlen_raw([&](uint32_t i) { return y[i]; }, 5, x, lut);
    hp_raw(x, m.header[0], y, lut);
    hp_raw(y, m.header[1], x, lut);  // kernel mast hash
    varlen_raw([&](uint32_t i) { return x[i]; }, 5, y, lut);
    hp_raw(y, m.kernel[0], out, lut);
}

// twenty-first Digest ordering (unpinned): canonical values compared from the last
// element down.  Returns a <= b.
__device__ __forceinline__ bool digest_le(const uint64_t* a_raw, const uint64_t* b_raw) {
    for (int q = 4; q >= 0; --q) {
        const uint64_t a = from_mont(a_raw[q]), b = from_mont(b_raw[q]);
        if (a != b) return a < b;
    }
    return true;
}

__global__ void __launch_bounds__(256) k_pow_guess(const uint64_t* __restrict__ leafs, const uint64_t* __restrict__ nodes,
                                                   uint32_t h, PowMast mast, PowPrefix picker,
                                                   const uint64_t* __restrict__ nonces, uint64_t n, PowPrefix target,
                                                   uint64_t* __restrict__ out_digest, uint64_t* __restrict__ out_idx,
                                                   uint8_t* __restrict__ out_ok) {
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t nonce[5];
    ld5(nonces + 5 * i, nonce);
    uint64_t ia, ib;
    pow_indices(picker.d, nonce, h, ia, ib, t5.lut);
    const uint64_t N = 1ull << h;
    // MTree::path(index)[j]: j == 0 -> leafs[index ^ 1]; else internal[((index + N) >> j) ^ 1]
    auto path_of = [&](uint64_t index) {
        return [=](uint32_t j) -> const uint64_t* {
            return j == 0 ? leafs + 5 * (index ^ 1) : nodes + 5 * (((index + N) >> j) ^ 1);
        };
    };
    uint64_t d[5];
    fast_mast_hash(mast, nodes + 5, path_of(ia), path_of(ib), nonce, h, d, t5.lut);
    st5(out_digest + 5 * i, d);
    out_idx[2 * i] = ia;
    out_idx[2 * i + 1] = ib;
    out_ok[i] = digest_le(d, target.d) ? 1 : 0;
}

// Pow::leaf (:325-331): MTree root of buds index..index+31 (mod 2^h)
__device__ void pow_leaf(const uint64_t* prefix, uint64_t index, uint32_t h, uint64_t* out,
                         const uint8_t* __restrict__ lut) {
    // iterative bottom-up merge with a stack of 5 subtree roots (binary counter)
    uint64_t stack[POW_NUM_BUD_LAYERS + 1][5];
    const uint64_t mask = (1ull << h) - 1;
    for (uint32_t j = 0; j < POW_BUDS_PER_LEAF; ++j) {
        uint64_t cur[5];
        bud_raw(prefix, (index + j) & mask, cur, lut);
        uint32_t lvl = 0;
        for (uint32_t t = j; t & 1u; t >>= 1, ++lvl) hp_raw(stack[lvl], cur, cur, lut);
        st5(stack[lvl], cur);
    }
    st5(out, stack[POW_NUM_BUD_LAYERS]);
}

__global__ void __launch_bounds__(64) k_pow_validate(const PowBlock* __restrict__ blocks, uint64_t n, uint32_t h,
                                                     uint8_t* __restrict__ verdicts) {
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PowBlock& b = blocks[i];
    uint64_t picker[5];
    hp_raw(b.root, b.commit, picker, t5.lut);  // index_picker_preimage = hash_pair(root, commit)
    uint64_t ia, ib;
    pow_indices(picker, b.nonce, h, ia, ib, t5.lut);
    const uint64_t* prefix = b.reboot ? b.commit : b.parent;
    uint64_t leaf_a[5], leaf_b[5];
    pow_leaf(prefix, b.reboot ? ia : bitreverse((uint32_t)ia, h), h, leaf_a, t5.lut);
    pow_leaf(prefix, b.reboot ? ib : bitreverse((uint32_t)ib, h), h, leaf_b, t5.lut);
    uint8_t ok = 1;
    // MTree::verify (:162-180) for both paths (index <= 2^h always holds here)
    for (int w = 0; w < 2; ++w) {
        uint64_t run[5];
        st5(run, w == 0 ? leaf_a : leaf_b);
        uint64_t ri = w == 0 ? ia : ib;
        const uint64_t* path = w == 0 ? b.path_a : b.path_b;
        for (uint32_t j = 0; j < h; ++j) {
            const uint64_t* sib = path + 5 * j;
            if (ri & 1) hp_raw(sib, run, run, t5.lut);
            else hp_raw(run, sib, run, t5.lut);
            ri >>= 1;
        }
        for (int q = 0; q < 5; ++q) ok &= run[q] == b.root[q];
    }
    uint64_t d[5];
    fast_mast_hash(b.mast, b.root, [&](uint32_t j) { return b.path_a + 5 * j; }, [&](uint32_t j) { return b.path_b + 5 * j; },
                   b.nonce, h, d, t5.lut);
    if (!digest_le(d, b.target)) ok = 0;
    verdicts[i] = ok;
}

// ---------------------------------------------------------------- launchers
static unsigned blocks_for(uint64_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_pow_preprocess(const PowPrefix& prefix, uint32_t h, bool bitrev_swap, uint64_t* d_a, uint64_t* d_b,
                                 uint64_t** leafs_out, uint64_t** nodes_out, hipStream_t st) {
    const uint64_t N = 1ull << h;
    hipLaunchKernelGGL(k_pow_buds, dim3(blocks_for(N, 256)), dim3(256), 0, st, prefix, N, d_a);
    uint64_t *in = d_a, *out = d_b;
    for (uint32_t i = 0; i < POW_NUM_BUD_LAYERS; ++i) {
        hipLaunchKernelGGL(k_pow_layer, dim3(blocks_for(N, 256)), dim3(256), 0, st, in, out, N, 1ull << i);
        uint64_t* t = in;
        in = out;
        out = t;
    }
    uint64_t* leafs = in;   // after the last layer
    uint64_t* nodes = out;  // the other buffer holds the internal nodes
    if (bitrev_swap)
        hipLaunchKernelGGL(k_pow_bitrev_swap, dim3(blocks_for(N, 256)), dim3(256), 0, st, leafs, N, h);
    for (uint64_t p0 = N >> 1; p0 >= 1; p0 >>= 1) {
        const uint64_t* children = p0 == (N >> 1) ? leafs : nodes + 5 * (2 * p0);
        hipLaunchKernelGGL(k_pow_tree_level, dim3(blocks_for(p0, 256)), dim3(256), 0, st, children, nodes, p0);
    }
    *leafs_out = leafs;
    *nodes_out = nodes;
    return hipGetLastError();
}

hipError_t launch_pow_guess(const uint64_t* leafs, const uint64_t* nodes, uint32_t h, const PowMast& mast,
                            const PowPrefix& picker, const uint64_t* d_nonces, uint64_t n, const PowPrefix& target,
                            uint64_t* d_digest, uint64_t* d_idx, uint8_t* d_ok, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pow_guess, dim3(blocks_for(n, 256)), dim3(256), 0, st, leafs, nodes, h, mast, picker, d_nonces,
                       n, target, d_digest, d_idx, d_ok);
    return hipGetLastError();
}

hipError_t launch_pow_validate(const PowBlock* d_blocks, uint64_t n, uint32_t h, uint8_t* d_verdicts, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pow_validate, dim3(blocks_for(n, 64)), dim3(64), 0, st, d_blocks, n, h, d_verdicts);
    return hipGetLastError();
}

}  // namespace nhip
