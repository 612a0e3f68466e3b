// Microbenchmark + bit-exactness check: Tip5 lane-per-state (tip5_permute_raw) vs the quad layout
// with the MDS on the f64 matrix cores (tip5_permute_quad).  n states x ITER chained permutations
// on raw Montgomery words; outputs compared word for word.
//   cd neptune-core_amd/tools && hipcc -O3 -std=c++17 --offload-arch=gfx950 -I. -I../csrc tip5_quad_bench.hip -o tip5_quad_bench
//   (-DNHIP_QUAD_NO_MFMA=1: MDS skipped, wrong results, timing of everything else)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "tip5_quad.hpp"

using namespace nhip;

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

__global__ void __launch_bounds__(256) k_ref(uint64_t* st, size_t n, int iters) {
    __shared__ Tip5Lds lds;
    tip5_lds_init(lds);
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) s[k] = st[i * 16 + k];
    for (int it = 0; it < iters; ++it) tip5_permute_raw(s, lds.lut);
#pragma unroll
    for (int k = 0; k < 16; ++k) st[i * 16 + k] = s[k];
}

__global__ void __launch_bounds__(256) k_quad(uint64_t* st, size_t n, int iters) {
    __shared__ Tip5QuadLds lds;
    tip5_quad_lds_init(lds);
    const Tip5QuadMat A = tip5_quad_mat();
    const uint32_t lane = threadIdx.x & 63, q = lane >> 4;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t idx = wave * 16 + (lane & 15);
    const bool live = idx < n;
    const size_t si = live ? idx : 0;
    uint64_t w[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) w[s] = st[si * 16 + quad_word(q, s)];
    for (int it = 0; it < iters; ++it) tip5_permute_quad(w, A, lds, q);
    if (live) {
#pragma unroll
        for (int s = 0; s < 4; ++s) st[si * 16 + quad_word(q, s)] = w[s];
    }
}

static uint64_t sm(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : (1u << 20);
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    std::vector<uint64_t> h(n * 16);
    uint64_t seed = 0xC2;
    for (auto& v : h) {
        do v = sm(seed);
        while (v >= GL_P);
    }
    uint64_t *d_ref, *d_quad;
    CK(hipMalloc(&d_ref, n * 128));
    CK(hipMalloc(&d_quad, n * 128));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // correctness: one pass of each
    CK(hipMemcpy(d_ref, h.data(), n * 128, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_quad, h.data(), n * 128, hipMemcpyHostToDevice));
    const unsigned g_ref = (unsigned)((n + 255) / 256);
    const unsigned g_quad = (unsigned)((n * 4 + 255) / 256);
    hipLaunchKernelGGL(k_ref, dim3(g_ref), dim3(256), 0, 0, d_ref, n, iters);
    hipLaunchKernelGGL(k_quad, dim3(g_quad), dim3(256), 0, 0, d_quad, n, iters);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> a(n * 16), b(n * 16);
    CK(hipMemcpy(a.data(), d_ref, n * 128, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), d_quad, n * 128, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n * 16; ++i) bad += a[i] != b[i];
    printf("{\"n\": %zu, \"iters\": %d, \"mismatched_words\": %zu", n, iters, bad);
    for (int which = 0; which < 2; ++which) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            if (which == 0) hipLaunchKernelGGL(k_ref, dim3(g_ref), dim3(256), 0, 0, d_ref, n, iters);
            else hipLaunchKernelGGL(k_quad, dim3(g_quad), dim3(256), 0, 0, d_quad, n, iters);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        printf(", \"%s_ms\": %.4f, \"%s_perms_per_s\": %.4e", which ? "quad" : "ref", best, which ? "quad" : "ref",
               (double)n * iters / (best * 1e-3));
    }
    printf("}\n");
    return bad ? 2 : 0;
}
