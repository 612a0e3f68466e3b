// Latency of one Tip5 permutation in the latency-bound row forms (one wave, a dependent chain of
// permutations), cycles per permutation: the 16-lane row form (carry-chain and carry-light
// arithmetic) and the two-row pair form.  Build + run:
//   hipcc -O3 --offload-arch=gfx950 -I neptune-core_amd/csrc neptune-core_amd/tools/tip5_row_latency.hip -o /tmp/rl && /tmp/rl
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "tip5_device.hpp"
using namespace nhip;
#define N 256
template <int FORM>
__global__ void k(uint64_t* out) {
    __shared__ Tip5Lds t5;
    tip5_lds_init(t5);
    const uint32_t lane = threadIdx.x & 63u, e = lane & 15u, h = (lane >> 4) & 1u;
    uint64_t rcs[TIP5_ROUNDS];
    for (int r = 0; r < TIP5_ROUNDS; ++r) rcs[r] = c_tip5_rc_raw[r * 16 + e];
    uint32_t cm[8];
    for (int j = 0; j < 8; ++j) cm[j] = h ? TIP5_MDS[j + 8] : TIP5_MDS[j];
    uint64_t s = e + 1;
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int i = 0; i < N; ++i) {
        if constexpr (FORM == 0) s = tip5_permute_wide<false>(s, e, rcs, t5.lut);
        else if constexpr (FORM == 1) s = tip5_permute_wide<true>(s, e, rcs, t5.lut);
        else s = tip5_permute_pair(s, e, h, rcs, cm, t5.lut);
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) out[64] = t1 - t0;
}
int main() {
    uint64_t* d;
    if (hipMalloc(&d, 65 * 8) != hipSuccess) return 1;
    uint64_t h[65];
    const char* names[] = {"row form, carry chains", "row form, carry-light", "pair form (carry-light)"};
    for (int f = 0; f < 3; ++f) {
        for (int rep = 0; rep < 3; ++rep) {
            if (f == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, d);
            if (f == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, d);
            if (f == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, d);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h, d, 65 * 8, hipMemcpyDeviceToHost);
        printf("%-28s %.0f cycles per permutation (%.0f per round)\n", names[f], (double)h[64] / N, (double)h[64] / N / 5);
    }
    return 0;
}
