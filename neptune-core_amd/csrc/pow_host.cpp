// C ABI of the proof-of-work Tip5 workloads (include/neptune_hip.h "proof of work"; kernels and
// reference citations in pow_kernels.hip).  Canonical u64 at the boundary, raw Montgomery inside.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/neptune_hip.h"
#include "device_scope.hpp"
#include "goldilocks.hpp"
#include "pow.hpp"

using namespace nhip;

extern "C" hipStream_t nhip_internal_stream(nhip_ctx* c);
extern "C" int nhip_internal_device(nhip_ctx* c);
extern "C" std::mutex* nhip_internal_mutex(nhip_ctx* c);

struct nhip_pow_buffer {
    uint32_t height = 0;
    int device = 0;
    uint64_t* d_a = nullptr;  // two 2^h-digest buffers (the reference's `ins` / `outs`)
    uint64_t* d_b = nullptr;
    uint64_t* leafs = nullptr;  // -> d_a or d_b
    uint64_t* nodes = nullptr;  // internal nodes, nodes[1] = root
    uint64_t prev_block_digest[5] = {};
};

namespace {

int hipfail(hipError_t e) { return e == hipSuccess ? NHIP_OK : (e == hipErrorOutOfMemory ? NHIP_ERR_OOM : NHIP_ERR_HIP); }

PowMast mast_raw(const nhip_pow_mast_paths* m) {
    PowMast r{};
    for (int q = 0; q < 5; ++q) {
        for (int i = 0; i < 3; ++i) r.pow[i][q] = to_mont(m->pow[i][q]);
        for (int i = 0; i < 2; ++i) r.header[i][q] = to_mont(m->header[i][q]);
        r.kernel[0][q] = to_mont(m->kernel[0][q]);
    }
    return r;
}

// PowMastPaths::commit (pow.rs:209-217): hash_varlen of the 6 digests, pow then header then kernel
int mast_commit(nhip_ctx* ctx, const nhip_pow_mast_paths* m, uint64_t out[5]) {
    uint64_t w[30];
    for (int q = 0; q < 5; ++q) {
        for (int i = 0; i < 3; ++i) w[5 * i + q] = m->pow[i][q];
        for (int i = 0; i < 2; ++i) w[15 + 5 * i + q] = m->header[i][q];
        w[25 + q] = m->kernel[0][q];
    }
    const uint64_t off[2] = {0, 30};
    return nhip_tip5_hash_varlen(ctx, w, off, 1, out);
}

int copy_digest_d2h(nhip_ctx* ctx, const uint64_t* d_src, uint64_t out[5]) {
    uint64_t raw[5];
    hipError_t e = hipMemcpyAsync(raw, d_src, 40, hipMemcpyDeviceToHost, nhip_internal_stream(ctx));
    if (e == hipSuccess) e = hipStreamSynchronize(nhip_internal_stream(ctx));
    if (e != hipSuccess) return hipfail(e);
    for (int q = 0; q < 5; ++q) out[q] = from_mont(raw[q]);
    return NHIP_OK;
}

}  // namespace

extern "C" {

int nhip_pow_mast_commit(nhip_ctx* ctx, const nhip_pow_mast_paths* mast, uint64_t out[5]) {
    if (!ctx || !mast || !out) return NHIP_ERR_ARG;
    return mast_commit(ctx, mast, out);
}

int nhip_pow_preprocess(nhip_ctx* ctx, uint32_t height, const nhip_pow_mast_paths* mast, int reboot_rules,
                        const uint64_t prev_block_digest[5], nhip_pow_buffer** out) {
    if (!ctx || !out || !prev_block_digest || (reboot_rules && !mast) || height < 1 || height > 31)
        return NHIP_ERR_ARG;
    *out = nullptr;
    // bud prefix: Reboot -> commitment to the proposal (mast paths); HardforkAlpha -> parent digest
    uint64_t prefix[5];
    if (reboot_rules) {
        const int rc = mast_commit(ctx, mast, prefix);
        if (rc) return rc;
    } else {
        for (int q = 0; q < 5; ++q) prefix[q] = prev_block_digest[q];
    }
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    nhip_pow_buffer* b = new (std::nothrow) nhip_pow_buffer();
    if (!b) return NHIP_ERR_OOM;
    b->height = height;
    b->device = nhip_internal_device(ctx);
    const DeviceScope device_scope(b->device);
    for (int q = 0; q < 5; ++q) b->prev_block_digest[q] = prev_block_digest[q] % GL_P;
    const size_t bytes = ((size_t)1 << height) * 40;
    hipError_t e = hipMalloc(&b->d_a, bytes);
    if (e == hipSuccess) e = hipMalloc(&b->d_b, bytes);
    if (e != hipSuccess) {
        nhip_pow_buffer_destroy(b);
        return hipfail(e);
    }
    PowPrefix p{};
    for (int q = 0; q < 5; ++q) p.d[q] = to_mont(prefix[q]);
    hipStream_t st = nhip_internal_stream(ctx);
    e = launch_pow_preprocess(p, height, !reboot_rules, b->d_a, b->d_b, &b->leafs, &b->nodes, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        nhip_pow_buffer_destroy(b);
        return hipfail(e);
    }
    *out = b;
    return NHIP_OK;
}

void nhip_pow_buffer_destroy(nhip_pow_buffer* b) {
    if (!b) return;
    const DeviceScope device_scope(b->device);
    if (b->d_a) (void)hipFree(b->d_a);
    if (b->d_b) (void)hipFree(b->d_b);
    delete b;
}

int nhip_pow_buffer_root(nhip_ctx* ctx, const nhip_pow_buffer* b, uint64_t out[5]) {
    if (!ctx || !b || !out) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    return copy_digest_d2h(ctx, b->nodes + 5, out);
}

int nhip_pow_buffer_leaf(nhip_ctx* ctx, const nhip_pow_buffer* b, uint64_t index, uint64_t out[5]) {
    if (!ctx || !b || !out || index >= (1ull << b->height)) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    return copy_digest_d2h(ctx, b->leafs + 5 * index, out);
}

// MTree::path (pow.rs:151-160): leafs[index ^ 1], then internal[((index + N) >> j) ^ 1]
int nhip_pow_buffer_path(nhip_ctx* ctx, const nhip_pow_buffer* b, uint64_t index, uint64_t* out) {
    if (!ctx || !b || !out || index >= (1ull << b->height)) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    const uint64_t N = 1ull << b->height;
    int rc = copy_digest_d2h(ctx, b->leafs + 5 * (index ^ 1), out);
    for (uint32_t j = 1; !rc && j < b->height; ++j) rc = copy_digest_d2h(ctx, b->nodes + 5 * (((index + N) >> j) ^ 1), out + 5 * j);
    return rc;
}

int nhip_pow_guess_batch(nhip_ctx* ctx, const nhip_pow_buffer* b, const nhip_pow_mast_paths* mast,
                         const uint64_t index_picker_preimage[5], const uint64_t* nonces, size_t n,
                         const uint64_t target[5], uint64_t* digests_out, uint64_t* indices_out, uint8_t* success_out) {
    if (!ctx || !b || !mast || !index_picker_preimage || !target || (n && (!nonces || !success_out))) return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    const DeviceScope device_scope(b->device);
    hipStream_t st = nhip_internal_stream(ctx);
    std::vector<uint64_t> nr(5 * n);
    for (size_t i = 0; i < 5 * n; ++i) nr[i] = to_mont(nonces[i]);
    uint64_t *d_n = nullptr, *d_d = nullptr, *d_i = nullptr;
    uint8_t* d_ok = nullptr;
    hipError_t e = hipMalloc(&d_n, 40 * n);
    if (e == hipSuccess) e = hipMalloc(&d_d, 40 * n);
    if (e == hipSuccess) e = hipMalloc(&d_i, 16 * n);
    if (e == hipSuccess) e = hipMalloc(&d_ok, n);
    if (e == hipSuccess) e = hipMemcpyAsync(d_n, nr.data(), 40 * n, hipMemcpyHostToDevice, st);
    PowPrefix picker{}, tgt{};
    for (int q = 0; q < 5; ++q) {
        picker.d[q] = to_mont(index_picker_preimage[q]);
        tgt.d[q] = to_mont(target[q]);
    }
    if (e == hipSuccess)
        e = launch_pow_guess(b->leafs, b->nodes, b->height, mast_raw(mast), picker, d_n, n, tgt, d_d, d_i, d_ok, st);
    std::vector<uint64_t> dr(5 * n);
    if (e == hipSuccess) e = hipMemcpyAsync(dr.data(), d_d, 40 * n, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && indices_out) e = hipMemcpyAsync(indices_out, d_i, 16 * n, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(success_out, d_ok, n, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(d_n);
    (void)hipFree(d_d);
    (void)hipFree(d_i);
    (void)hipFree(d_ok);
    if (e != hipSuccess) return hipfail(e);
    if (digests_out)
        for (size_t i = 0; i < 5 * n; ++i) digests_out[i] = from_mont(dr[i]);
    return NHIP_OK;
}

int nhip_pow_validate_batch(nhip_ctx* ctx, uint32_t height, const uint64_t* roots, const uint64_t* paths_a,
                            const uint64_t* paths_b, const uint64_t* nonces, const nhip_pow_mast_paths* masts,
                            const uint64_t* targets, const uint64_t* parents, const uint8_t* reboot_rules, size_t n,
                            uint8_t* verdicts) {
    if (!ctx || height < 1 || height > POW_MAX_HEIGHT ||
        (n && (!roots || !paths_a || !paths_b || !nonces || !masts || !targets || !parents || !reboot_rules ||
               !verdicts)))
        return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    // commitments first (they are Tip5 hashes themselves; computed with the batch hash entry point)
    std::vector<uint64_t> cw(30 * n), off(n + 1), commit(5 * n);
    for (size_t i = 0; i < n; ++i) {
        const nhip_pow_mast_paths& m = masts[i];
        for (int q = 0; q < 5; ++q) {
            for (int k = 0; k < 3; ++k) cw[30 * i + 5 * k + q] = m.pow[k][q];
            for (int k = 0; k < 2; ++k) cw[30 * i + 15 + 5 * k + q] = m.header[k][q];
            cw[30 * i + 25 + q] = m.kernel[0][q];
        }
        off[i] = 30 * i;
    }
    off[n] = 30 * n;
    int rc = nhip_tip5_hash_varlen(ctx, cw.data(), off.data(), n, commit.data());
    if (rc) return rc;
    std::vector<PowBlock> blk(n);
    for (size_t i = 0; i < n; ++i) {
        PowBlock& b = blk[i];
        std::memset(&b, 0, sizeof(b));
        for (int q = 0; q < 5; ++q) {
            b.root[q] = to_mont(roots[5 * i + q]);
            b.nonce[q] = to_mont(nonces[5 * i + q]);
            b.commit[q] = to_mont(commit[5 * i + q]);
            b.parent[q] = to_mont(parents[5 * i + q]);
            b.target[q] = to_mont(targets[5 * i + q]);
        }
        for (uint32_t j = 0; j < 5 * height; ++j) {
            b.path_a[j] = to_mont(paths_a[(size_t)5 * height * i + j]);
            b.path_b[j] = to_mont(paths_b[(size_t)5 * height * i + j]);
        }
        b.mast = mast_raw(&masts[i]);
        b.reboot = reboot_rules[i] ? 1u : 0u;
    }
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    const DeviceScope device_scope(nhip_internal_device(ctx));
    hipStream_t st = nhip_internal_stream(ctx);
    PowBlock* d_b = nullptr;
    uint8_t* d_v = nullptr;
    hipError_t e = hipMalloc(&d_b, sizeof(PowBlock) * n);
    if (e == hipSuccess) e = hipMalloc(&d_v, n);
    if (e == hipSuccess) e = hipMemcpyAsync(d_b, blk.data(), sizeof(PowBlock) * n, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = launch_pow_validate(d_b, n, height, d_v, st);
    if (e == hipSuccess) e = hipMemcpyAsync(verdicts, d_v, n, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(d_b);
    (void)hipFree(d_v);
    return hipfail(e);
}

}  // extern "C"
