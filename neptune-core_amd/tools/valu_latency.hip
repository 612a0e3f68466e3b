// Dependent-chain latency of VALU instruction kinds on one wave (gfx950): cycles per dependent step.
// Build + run: hipcc -O3 --offload-arch=gfx950 neptune-core_amd/tools/valu_latency.hip -o /tmp/lat && /tmp/lat
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N 512
__global__ void k_mad(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t x = threadIdx.x; uint32_t m = a;
  uint64_t t0 = __builtin_readcyclecounter();
#pragma unroll 64
  for (int i = 0; i < N; ++i) x = (uint64_t)m * (uint32_t)x + x;   // v_mad_u64_u32 chain
  uint64_t t1 = __builtin_readcyclecounter();
  out[threadIdx.x] = x; if (threadIdx.x == 0) out[64] = t1 - t0;
}
__global__ void k_add(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t x = threadIdx.x, y = b; unsigned c = 0;
  uint64_t t0 = __builtin_readcyclecounter();
#pragma unroll 64
  for (int i = 0; i < N; ++i) { x = __builtin_addc(x, y, c, &c); }   // v_addc chain through carry and value
  uint64_t t1 = __builtin_readcyclecounter();
  out[threadIdx.x] = x; if (threadIdx.x == 0) out[64] = t1 - t0;
}
__global__ void k_add32(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t x = threadIdx.x;
  uint64_t t0 = __builtin_readcyclecounter();
#pragma unroll 64
  for (int i = 0; i < N; ++i) { x = (x + a) ^ b; }   // v_add_u32 + v_xor chain (2 per iter)
  uint64_t t1 = __builtin_readcyclecounter();
  out[threadIdx.x] = x; if (threadIdx.x == 0) out[64] = t1 - t0;
}
__global__ void k_add64(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t x = threadIdx.x, y = ((uint64_t)a << 32) | b;
  uint64_t t0 = __builtin_readcyclecounter();
#pragma unroll 64
  for (int i = 0; i < N; ++i) { x = x + y; asm volatile("" : "+v"(x)); }   // v_lshl_add_u64 chain (not folded)
  uint64_t t1 = __builtin_readcyclecounter();
  out[threadIdx.x] = x; if (threadIdx.x == 0) out[64] = t1 - t0;
}
int main() {
  uint64_t* d; hipMalloc(&d, 65 * 8); uint64_t h[65];
  const char* names[] = {"mad_u64_u32 chain", "addc chain", "add_u32+xor chain (2 instr/iter)", "64-bit add chain"};
  void (*ks[])(uint64_t*, uint32_t, uint32_t) = {k_mad, k_add, k_add32, k_add64};
  for (int k = 0; k < 4; ++k) {
    for (int rep = 0; rep < 3; ++rep) { hipLaunchKernelGGL(ks[k], dim3(1), dim3(64), 0, 0, d, 12345u, 678u); hipDeviceSynchronize(); }
    hipMemcpy(h, d, 65 * 8, hipMemcpyDeviceToHost);
    printf("%-34s %.2f cycles per iteration\n", names[k], (double)h[64] / N);
  }
  return 0;
}
