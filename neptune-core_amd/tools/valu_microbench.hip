// Instruction-throughput microbenchmark for the Tip5 kernel's building blocks on gfx950.
// Each kernel issues ITERS x 8 independent instances of one instruction per lane (inline asm,
// nothing folded).  Reported: wave-instructions per CU per cycle at a nominal 2.4 GHz, and the
// rate relative to the first row (v_add_u32_e32).  Results: DESIGN.md §Microbenchmarks.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
#define BODY8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

#define K32(NAME, ASM)                                                                  \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                   \
        uint32_t r[8]; uint32_t a = threadIdx.x * 0x01010101u + 7u;                     \
        for (int k = 0; k < 8; ++k) r[k] = threadIdx.x + k;                             \
        for (int i = 0; i < ITERS; ++i) {                                               \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(ASM : "+v"(r[k]) : "v"(a), "v"(s)); \
        }                                                                               \
        uint32_t x = 0; for (int k = 0; k < 8; ++k) x ^= r[k];                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                 \
    }
#define K32C(NAME, ASM)                                                                 \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                   \
        uint32_t r[8]; uint32_t a = threadIdx.x * 0x01010101u + 7u;                     \
        for (int k = 0; k < 8; ++k) r[k] = threadIdx.x + k;                             \
        for (int i = 0; i < ITERS; ++i) {                                               \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) { uint64_t sd; asm volatile(ASM : "+v"(r[k]), "=s"(sd) : "v"(a), "v"(s)); } \
        }                                                                               \
        uint32_t x = 0; for (int k = 0; k < 8; ++k) x ^= r[k];                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                 \
    }
#define K64(NAME, ASM)                                                                  \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                   \
        uint64_t r[8]; uint64_t a = threadIdx.x * 3ull + ((uint64_t)s << 40);           \
        for (int k = 0; k < 8; ++k) r[k] = threadIdx.x + k;                             \
        for (int i = 0; i < ITERS; ++i) {                                               \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(ASM : "+v"(r[k]) : "v"(a), "v"(s)); \
        }                                                                               \
        uint32_t x = 0; for (int k = 0; k < 8; ++k) x ^= (uint32_t)r[k];                \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                 \
    }
#define K64C(NAME, ASM)                                                                 \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                   \
        uint64_t r[8]; uint32_t a = threadIdx.x | 1u;                                   \
        for (int k = 0; k < 8; ++k) r[k] = threadIdx.x + k;                             \
        for (int i = 0; i < ITERS; ++i) {                                               \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) { uint64_t sd; asm volatile(ASM : "+v"(r[k]), "=s"(sd) : "v"(a), "v"(s)); } \
        }                                                                               \
        uint32_t x = 0; for (int k = 0; k < 8; ++k) x ^= (uint32_t)r[k];                \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                 \
    }

#define K32S(NAME, ASM)                                                                 \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                   \
        uint32_t r[8]; uint32_t a = threadIdx.x * 0x01010101u + 7u;                     \
        uint64_t m = 0x5555555555555555ull ^ (uint64_t)s;                               \
        for (int k = 0; k < 8; ++k) r[k] = threadIdx.x + k;                             \
        for (int i = 0; i < ITERS; ++i) {                                               \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(ASM : "+v"(r[k]) : "v"(a), "s"(m)); \
        }                                                                               \
        uint32_t x = 0; for (int k = 0; k < 8; ++k) x ^= r[k];                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                 \
    }
K32S(k_cndmask_e64s, "v_cndmask_b32_e64 %0, %1, %0, %2")
K32S(k_subb_e64s, "v_subb_co_u32_e64 %0, s[40:41], %1, %0, %2")
K32(k_add_e32, "v_add_u32_e32 %0, %1, %0")
K32(k_add_e64, "v_add_u32_e64 %0, %1, %0")
K32(k_xor_e32, "v_xor_b32_e32 %0, %1, %0")
K32(k_add3, "v_add3_u32 %0, %1, %0, %2")
K32(k_lshl_e32, "v_lshlrev_b32_e32 %0, 3, %0")
K32(k_mul24_e32, "v_mul_u32_u24_e32 %0, %1, %0")
K32(k_mulhi24_e32, "v_mul_hi_u32_u24_e32 %0, %1, %0")
K32(k_mad24, "v_mad_u32_u24 %0, %1, %2, %0")
K32(k_mullo, "v_mul_lo_u32 %0, %1, %0")
K32(k_mulhi, "v_mul_hi_u32 %0, %1, %0")
K32(k_perm, "v_perm_b32 %0, %1, %0, %2")
K32(k_bfe, "v_bfe_u32 %0, %0, 8, 8")
K32(k_cndmask_e32, "v_cndmask_b32_e32 %0, %1, %0, vcc")
K32C(k_addco_e64, "v_add_co_u32_e64 %0, %1, %0, %2")
K32(k_addco_e32, "v_add_co_u32_e32 %0, vcc, %1, %0")
K32(k_addc_e32, "v_addc_co_u32_e32 %0, vcc, %1, %0, vcc")
K64C(k_mad64, "v_mad_u64_u32 %0, %1, %2, %3, %0")
K64(k_lshladd64, "v_lshl_add_u64 %0, %1, 2, %0")
K64(k_lshr64, "v_lshrrev_b64 %0, 3, %0")
K64(k_cmp64, "v_cmp_lt_u64_e32 vcc, %0, %1")
K64(k_fma64, "v_fma_f64 %0, %1, %0, %1")
// second batch: the remaining instruction classes of the Tip5 round
K32(k_mov_e32, "v_mov_b32_e32 %0, %1")
K32(k_or_e32, "v_or_b32_e32 %0, %1, %0")
K32(k_and_e32, "v_and_b32_e32 %0, %1, %0")
K32(k_sub_e32, "v_sub_u32_e32 %0, %1, %0")
K32(k_lshl_or, "v_lshl_or_b32 %0, %1, 8, %0")
K32(k_or3, "v_or3_b32 %0, %1, %0, %2")
K32(k_lshl_add32, "v_lshl_add_u32 %0, %1, 3, %0")
K32(k_alignbit, "v_alignbit_b32 %0, %1, %0, 7")
K32(k_lshr_e32, "v_lshrrev_b32_e32 %0, %1, %0")
K32(k_max_e32, "v_max_u32_e32 %0, %1, %0")
K32(k_subco_e32, "v_sub_co_u32_e32 %0, vcc, %1, %0")
K32(k_subb_e32, "v_subb_co_u32_e32 %0, vcc, %1, %0, vcc")
K32(k_subbrev_e32, "v_subbrev_co_u32_e32 %0, vcc, 0, %0, vcc")
K64(k_mov64, "v_mov_b64 %0, %1")
K64(k_lshl64, "v_lshlrev_b64 %0, 3, %0")
#define K32Q(NAME, ASM)                                                                 \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                   \
        uint32_t r[8]; uint32_t a = threadIdx.x * 0x01010101u + 7u;                     \
        for (int k = 0; k < 8; ++k) r[k] = threadIdx.x + k;                             \
        for (int i = 0; i < ITERS; ++i) {                                               \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(ASM : "+v"(r[k]) : "v"(a), "s"(s)); \
        }                                                                               \
        uint32_t x = 0; for (int k = 0; k < 8; ++k) x ^= r[k];                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                 \
    }
#define K64CS(NAME, ASM)                                                                \
    __global__ void NAME(uint32_t* out, uint32_t s) {                                   \
        uint64_t r[8]; uint32_t a = threadIdx.x | 1u; uint64_t s64 = (uint64_t)s * 0x100000001ull; \
        for (int k = 0; k < 8; ++k) r[k] = threadIdx.x + k;                             \
        for (int i = 0; i < ITERS; ++i) {                                               \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) { uint64_t sd; asm volatile(ASM : "+v"(r[k]), "=s"(sd) : "v"(a), "s"(s), "s"(s64)); } \
        }                                                                               \
        uint32_t x = 0; for (int k = 0; k < 8; ++k) x ^= (uint32_t)r[k];                \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                 \
    }
K64CS(k_mad64_smul, "v_mad_u64_u32 %0, %1, %2, %3, %0")
K64CS(k_mad64_sadd, "v_mad_u64_u32 %0, %1, %2, %2, %4")
K64CS(k_mad64_cmul, "v_mad_u64_u32 %0, %1, %2, -1, %0")
// third batch: does the operand kind (VGPR / inline constant / literal / SGPR) set the issue class?
K32(k_lshl_v, "v_lshlrev_b32_e32 %0, %1, %0")
K32(k_lshr_c, "v_lshrrev_b32_e32 %0, 3, %0")
K32(k_add_c, "v_add_u32_e32 %0, 3, %0")
K32(k_add_lit, "v_add_u32_e32 %0, 0x12345, %0")
K32(k_and_lit, "v_and_b32_e32 %0, 0xff, %0")
K32(k_and_c, "v_and_b32_e32 %0, 63, %0")
K32Q(k_add_s, "v_add_u32_e64 %0, %2, %0")
K32Q(k_xor_s, "v_xor_b32_e64 %0, %2, %0")
K32(k_sub_c, "v_sub_u32_e32 %0, 7, %0")
K32(k_mov_c, "v_mov_b32_e32 %0, 7")
K32Q(k_mov_s, "v_mov_b32_e32 %0, %2")
K32(k_lshr_v64, "v_lshrrev_b32_e64 %0, %1, %0")
K32(k_lshl_v64, "v_lshlrev_b32_e64 %0, %1, %0")
K32(k_bfe_v, "v_bfe_u32 %0, %0, %1, %1")
K32(k_cndmask_v, "v_cndmask_b32_e64 %0, %1, %0, s[40:41]")
K32(k_min_v, "v_min_u32_e32 %0, %1, %0")
K32(k_not_v, "v_not_b32_e32 %0, %0")

__global__ void k_ds_u8(uint32_t* out, uint32_t s) {
    __shared__ uint8_t lut[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    uint32_t a = threadIdx.x * 2654435761u;
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += lut[((a >> (k * 3)) + i) & 255u];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_ds_u16_128k(uint32_t* out, uint32_t s) {
    extern __shared__ uint16_t lut16[];
    for (int i = threadIdx.x; i < 65536; i += blockDim.x) lut16[i] = (uint16_t)(i * 7 + 3);
    __syncthreads();
    uint32_t a = threadIdx.x * 2654435761u;
    uint32_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += lut16[((a >> (k * 2)) + i * 40503u) & 65535u];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t* out; CHECK(hipMalloc(&out, (size_t)cus * 8 * 1024 * 4));
    struct { const char* name; kfn f; int instr_per_iter; size_t lds; } ks[] = {
        {"v_add_u32_e32", k_add_e32, 8, 0}, {"v_add_u32_e64", k_add_e64, 8, 0}, {"v_xor_b32_e32", k_xor_e32, 8, 0},
        {"v_add3_u32", k_add3, 8, 0}, {"v_lshlrev_b32_e32", k_lshl_e32, 8, 0}, {"v_mul_u32_u24_e32", k_mul24_e32, 8, 0},
        {"v_mul_hi_u32_u24_e32", k_mulhi24_e32, 8, 0}, {"v_mad_u32_u24", k_mad24, 8, 0}, {"v_mul_lo_u32", k_mullo, 8, 0},
        {"v_mul_hi_u32", k_mulhi, 8, 0}, {"v_perm_b32", k_perm, 8, 0}, {"v_bfe_u32", k_bfe, 8, 0},
        {"v_cndmask_b32_e32", k_cndmask_e32, 8, 0}, {"v_cndmask_b32_e64(sgpr)", k_cndmask_e64s, 8, 0},
        {"v_subb_co_u32_e64(sgpr cin)", k_subb_e64s, 8, 0}, {"v_add_co_u32_e64(sgpr)", k_addco_e64, 8, 0},
        {"v_add_co_u32_e32(vcc)", k_addco_e32, 8, 0}, {"v_addc_co_u32_e32 chain", k_addc_e32, 8, 0},
        {"v_mad_u64_u32", k_mad64, 8, 0}, {"v_lshl_add_u64", k_lshladd64, 8, 0}, {"v_lshrrev_b64", k_lshr64, 8, 0},
        {"v_cmp_lt_u64_e32", k_cmp64, 8, 0}, {"v_fma_f64", k_fma64, 8, 0},
        {"v_mov_b32_e32", k_mov_e32, 8, 0}, {"v_or_b32_e32", k_or_e32, 8, 0}, {"v_and_b32_e32", k_and_e32, 8, 0},
        {"v_sub_u32_e32", k_sub_e32, 8, 0}, {"v_lshl_or_b32", k_lshl_or, 8, 0}, {"v_or3_b32", k_or3, 8, 0},
        {"v_lshl_add_u32", k_lshl_add32, 8, 0}, {"v_alignbit_b32", k_alignbit, 8, 0},
        {"v_lshrrev_b32_e32(vgpr)", k_lshr_e32, 8, 0}, {"v_max_u32_e32", k_max_e32, 8, 0},
        {"v_sub_co_u32_e32(vcc)", k_subco_e32, 8, 0}, {"v_subb_co_u32_e32 chain", k_subb_e32, 8, 0},
        {"v_subbrev_co_u32_e32 chain", k_subbrev_e32, 8, 0}, {"v_mov_b64", k_mov64, 8, 0},
        {"v_mad_u64_u32(sgpr mul)", k_mad64_smul, 8, 0}, {"v_mad_u64_u32(sgpr addend)", k_mad64_sadd, 8, 0},
        {"v_mad_u64_u32(const -1 mul)", k_mad64_cmul, 8, 0},
        {"v_lshlrev_b32_e32(vgpr)", k_lshl_v, 8, 0}, {"v_lshrrev_b32_e32(const)", k_lshr_c, 8, 0},
        {"v_add_u32_e32(const)", k_add_c, 8, 0}, {"v_add_u32_e32(literal)", k_add_lit, 8, 0},
        {"v_and_b32_e32(literal 0xff)", k_and_lit, 8, 0}, {"v_and_b32_e32(const 63)", k_and_c, 8, 0},
        {"v_add_u32_e64(sgpr)", k_add_s, 8, 0}, {"v_xor_b32_e64(sgpr)", k_xor_s, 8, 0},
        {"v_sub_u32_e32(const)", k_sub_c, 8, 0}, {"v_mov_b32_e32(const)", k_mov_c, 8, 0},
        {"v_mov_b32_e32(sgpr)", k_mov_s, 8, 0}, {"v_lshrrev_b32_e64(vgpr)", k_lshr_v64, 8, 0},
        {"v_lshlrev_b32_e64(vgpr)", k_lshl_v64, 8, 0}, {"v_bfe_u32(vgpr)", k_bfe_v, 8, 0},
        {"v_cndmask_b32_e64(vgpr,s40)", k_cndmask_v, 8, 0}, {"v_min_u32_e32", k_min_v, 8, 0},
        {"v_not_b32_e32", k_not_v, 8, 0},
        {"ds_read_u8 256B (+3 valu)", k_ds_u8, 8, 0}, {"ds_read_u16 128KiB (+3 valu)", k_ds_u16_128k, 8, 131072}};
    hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    CHECK(hipFuncSetAttribute((const void*)k_ds_u16_128k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    printf("CUs=%d\n", cus);
    for (int waves_per_simd : {8, 4, 1}) {
        double base = 0;
        printf("--- %d waves/SIMD ---\n", waves_per_simd);
        for (auto& k : ks) {
            int block = 256, blocks = cus * waves_per_simd;   // 4 waves per block = 1 per SIMD
            if (k.lds) { block = 64 * 4 * (waves_per_simd > 4 ? 4 : waves_per_simd); blocks = cus; }
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(block), k.lds, 0, out, 3u);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(a));
            for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(block), k.lds, 0, out, 3u);
            CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
            float ms; CHECK(hipEventElapsedTime(&ms, a, b));
            double wi = 3.0 * blocks * (block / 64) * (double)ITERS * k.instr_per_iter;
            double per_cu_clk = wi / (ms * 1e-3) / cus / 2.4e9;
            if (base == 0) base = per_cu_clk;
            printf("%-30s %8.3f ms  %.3f wave-instr/CU-clk  rel %.3f\n", k.name, ms, per_cu_clk, per_cu_clk / base);
        }
    }
    return 0;
}
