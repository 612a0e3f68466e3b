// Proof-of-work descriptors shared by pow_kernels.hip and pow_host.cpp (raw Montgomery words).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nhip {

static constexpr int POW_NUM_BUD_LAYERS = 5;                       // pow.rs:43
static constexpr uint32_t POW_BUDS_PER_LEAF = 1u << POW_NUM_BUD_LAYERS;  // pow.rs:44
static constexpr int POW_NUM_INDEX_REPETITIONS = 63;               // pow.rs:42
static constexpr uint32_t POW_MAX_HEIGHT = 32;

struct PowPrefix {
    uint64_t d[5];
};
// PowMastPaths (pow.rs:202-207): pow [BlockHeader::MAST_HEIGHT = 3], header [BlockKernel = 2],
// kernel [Block = 1]
struct PowMast {
    uint64_t pow[3][5];
    uint64_t header[2][5];
    uint64_t kernel[1][5];
};
struct PowBlock {
    uint64_t root[5], nonce[5], commit[5], parent[5], target[5];
    uint64_t path_a[POW_MAX_HEIGHT * 5], path_b[POW_MAX_HEIGHT * 5];
    PowMast mast;
    uint32_t reboot, pad;
};

hipError_t launch_pow_preprocess(const PowPrefix& prefix, uint32_t h, bool bitrev_swap, uint64_t* d_a, uint64_t* d_b,
                                 uint64_t** leafs_out, uint64_t** nodes_out, hipStream_t st);
hipError_t launch_pow_guess(const uint64_t* leafs, const uint64_t* nodes, uint32_t h, const PowMast& mast,
                            const PowPrefix& picker, const uint64_t* d_nonces, uint64_t n, const PowPrefix& target,
                            uint64_t* d_digest, uint64_t* d_idx, uint8_t* d_ok, hipStream_t st);
hipError_t launch_pow_validate(const PowBlock* d_blocks, uint64_t n, uint32_t h, uint8_t* d_verdicts, hipStream_t st);

}  // namespace nhip
