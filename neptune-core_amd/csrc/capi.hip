// C-ABI layer of libneptune_hip.so (declarations: include/neptune_hip.h).
//
// One nhip_ctx = one GPU, one non-blocking HIP stream, a grow-only device workspace for the
// host-buffer entry points, and an optional event timer around every kernel launch.  Calls on
// one context are serialized by a mutex (the reference calls verify() concurrently from many
// tokio tasks: neptune-core/src/protocol/proof_abstractions/verifier.rs:60-63).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/neptune_hip.h"
#include "device_scope.hpp"
#include "host_numa.hpp"
#include "kernels.hpp"

struct nhip_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    void* ws = nullptr;  // workspace for host-buffer calls
    size_t ws_bytes = 0;
    void* staging = nullptr;  // pinned host staging for batch uploads (grow-only, under mu)
    size_t staging_bytes = 0;
    void* verify_scratch = nullptr;  // reusable device / stream resources of nhip_verify_batch
    void (*verify_scratch_free)(void*) = nullptr;
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;  // recorded, not yet read
    std::vector<hipEvent_t> free_events;
    double timed_ms = 0.0;
    uint64_t timed_launches = 0;
    nhip::HostTopo topo;       // the GPU's NUMA node and its CPUs (host_numa.cpp)
    unsigned host_threads = 0;  // staging copy threads per upload (0: the default)
};

namespace {

int hip_fail(hipError_t e) {
    if (e == hipSuccess) return NHIP_OK;
    if (e == hipErrorOutOfMemory) return NHIP_ERR_OOM;
    return NHIP_ERR_HIP;
}

hipEvent_t take_event(nhip_ctx* c) {
    if (!c->free_events.empty()) {
        hipEvent_t e = c->free_events.back();
        c->free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Launch helper: brackets the launch with events when timing is on.
template <class F>
int timed_launch(nhip_ctx* c, F&& f) {
    hipEvent_t a = nullptr, b = nullptr;
    if (c->timing) {
        a = take_event(c);
        b = take_event(c);
        if (a && b) (void)hipEventRecord(a, c->stream);
    }
    hipError_t e = f();
    if (c->timing && a && b) {
        (void)hipEventRecord(b, c->stream);
        c->pending.emplace_back(a, b);
    }
    return hip_fail(e);
}

int ensure_ws(nhip_ctx* c, size_t bytes) {
    if (bytes <= c->ws_bytes) return NHIP_OK;
    if (c->ws) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipFree(c->ws);
        c->ws = nullptr;
        c->ws_bytes = 0;
    }
    size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
    hipError_t e = hipMalloc(&c->ws, want);
    if (e != hipSuccess) return hip_fail(e);
    c->ws_bytes = want;
    return NHIP_OK;
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Carve a list of sizes out of the workspace.
template <size_t N>
int carve(nhip_ctx* c, const size_t (&sizes)[N], void* (&ptrs)[N]) {
    size_t total = 0;
    for (size_t i = 0; i < N; ++i) total += align_up(sizes[i] ? sizes[i] : 1);
    int rc = ensure_ws(c, total);
    if (rc) return rc;
    char* base = (char*)c->ws;
    size_t off = 0;
    for (size_t i = 0; i < N; ++i) {
        ptrs[i] = base + off;
        off += align_up(sizes[i] ? sizes[i] : 1);
    }
    return NHIP_OK;
}

// Batch verdict: any_bad |= (v[i] != 1) over n bytes; 16 B per lane per step, one atomic per wave.
__global__ void __launch_bounds__(256) k_any_bad(const uint8_t* __restrict__ v, size_t n, uint32_t* __restrict__ any_bad) {
    uint32_t bad = 0;
    const size_t n16 = (reinterpret_cast<uintptr_t>(v) & 15u) ? 0 : n / 16;  // unaligned: byte path
    const uint4* __restrict__ v16 = reinterpret_cast<const uint4*>(v);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 w = v16[i];
        bad |= (w.x ^ 0x01010101u) | (w.y ^ 0x01010101u) | (w.z ^ 0x01010101u) | (w.w ^ 0x01010101u);
    }
    for (size_t i = n16 * 16 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        bad |= (v[i] != 1) ? 1u : 0u;
    if (__any(bad != 0) && (threadIdx.x & 63) == 0) atomicOr(any_bad, 1u);
}

int build_tree_dev(nhip_ctx* c, const uint64_t* d_leafs, size_t n, uint64_t* d_nodes) {
    // level 0: leafs -> nodes[n/2 .. n)
    int rc = timed_launch(c, [&] { return nhip::launch_mtree_level(d_leafs, d_nodes + 5 * (n / 2), n / 2, c->stream); });
    if (rc) return rc;
    for (size_t parents = n / 4; parents >= 1; parents /= 2) {
        rc = timed_launch(c, [&] {
            return nhip::launch_mtree_level(d_nodes + 5 * (2 * parents), d_nodes + 5 * parents, parents, c->stream);
        });
        if (rc) return rc;
    }
    hipError_t e = hipMemsetAsync(d_nodes, 0, 5 * sizeof(uint64_t), c->stream);
    return hip_fail(e);
}

bool is_pow2(size_t n) { return n >= 2 && (n & (n - 1)) == 0; }

}  // namespace

extern "C" {

// 2000: nhip_stark_params.input_form (the struct grew), nhip_set_fs_form, the streaming group
// 2100: nhip_stats.ms_row_hash_exec (the struct grew), the NUMA entry points (nhip_host_alloc_near,
// nhip_device_numa, nhip_numa_from_sysfs, nhip_cpulist_parse, nhip_host_page_node,
// nhip_set_host_threads)
// 2200: nhip_batch_set_launch_timing (per-dispatch timestamps off by default), nhip_batch_set_streams
// 2300: nhip_air_create_ex (compiler options instead of environment variables), nhip_set_climb_from_ops,
// the per-member proof arenas (nhip_arena_*, nhip_group_stream_submit_placed), nhip_queue_latencies,
// nhip_batch_set_graph
int nhip_abi_version(void) { return 2300; }

int nhip_set_fs_form(int form) { return nhip::set_fs_form(form) == 0 ? NHIP_OK : NHIP_ERR_ARG; }
int nhip_set_climb_from_ops(int64_t ops) { return nhip::set_climb_from_ops(ops) == 0 ? NHIP_OK : NHIP_ERR_ARG; }

const char* nhip_strerror(int code) {
    switch (code) {
        case NHIP_OK: return "ok";
        case NHIP_ERR_NO_DEVICE: return "no HIP device";
        case NHIP_ERR_HIP: return "HIP runtime error";
        case NHIP_ERR_OOM: return "out of device memory";
        case NHIP_ERR_ARG: return "invalid argument";
        case NHIP_ERR_DECODE: return "malformed encoding";
        default: return "unknown error";
    }
}

int nhip_init(uint32_t device_mask, nhip_ctx** out) {
    if (!out) return NHIP_ERR_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return NHIP_ERR_NO_DEVICE;
    int dev = 0;
    if (device_mask) {
        dev = __builtin_ctz(device_mask);
        if (dev >= count) return NHIP_ERR_NO_DEVICE;
    }
    nhip_ctx* c = new (std::nothrow) nhip_ctx();
    if (!c) return NHIP_ERR_OOM;
    c->device = dev;
    // the caller's current device is left as it was (a host with its own HIP user, e.g. torch,
    // must not find another device current after creating a context)
    int prev = -1;
    (void)hipGetDevice(&prev);
    const bool ok = hipSetDevice(dev) == hipSuccess &&
                    hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess;
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    if (!ok) {
        delete c;
        return NHIP_ERR_HIP;
    }
    try {
        c->topo = nhip::device_topo(dev);
    } catch (const std::bad_alloc&) {
        c->topo = nhip::HostTopo{};
    }
    *out = c;
    return NHIP_OK;
}

void nhip_destroy(nhip_ctx* c) {
    if (!c) return;
    const DeviceScope device_scope(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto& p : c->pending) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    for (auto e : c->free_events) (void)hipEventDestroy(e);
    if (c->ws) (void)hipFree(c->ws);
    if (c->staging) (void)hipHostFree(c->staging);
    if (c->verify_scratch && c->verify_scratch_free) c->verify_scratch_free(c->verify_scratch);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

int nhip_device_ordinal(const nhip_ctx* c) { return c ? c->device : -1; }

// internal accessors for the other translation units (not in the public header)
hipStream_t nhip_internal_stream(nhip_ctx* c) { return c->stream; }
int nhip_internal_device(nhip_ctx* c) { return c->device; }
std::mutex* nhip_internal_mutex(nhip_ctx* c) { return &c->mu; }
// The context's nhip_verify_batch scratch (created by `make` on first use, freed by `freefn` in
// nhip_destroy).
void* nhip_internal_verify_scratch(nhip_ctx* c, void* (*make)(), void (*freefn)(void*)) {
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->verify_scratch) {
        c->verify_scratch = make();
        c->verify_scratch_free = freefn;
    }
    return c->verify_scratch;
}
// Pinned staging of at least `bytes` (caller holds c->mu); nullptr if it cannot be pinned.
void* nhip_internal_staging(nhip_ctx* c, size_t bytes) {
    if (bytes <= c->staging_bytes) return c->staging;
    const size_t have = c->staging_bytes;
    if (c->staging) (void)hipHostFree(c->staging);
    c->staging = nullptr;
    c->staging_bytes = 0;
    // headroom, at least doubling: hipHostFree waits for the device, so a context whose batches
    // vary in size should stop reallocating after a few calls
    const size_t want = std::max(bytes + bytes / 4, 2 * have);
    // on the GPU's NUMA node: the copy threads (bound there) write it and the DMA reads it locally
    if (nhip::host_malloc_on(&c->staging, want, c->topo.numa_node, hipHostMallocDefault) != hipSuccess) {
        c->staging = nullptr;
        return nullptr;
    }
    c->staging_bytes = want;
    return c->staging;
}

const void* nhip_internal_topo(nhip_ctx* c) { return &c->topo; }  // a const nhip::HostTopo*
unsigned nhip_internal_host_threads(nhip_ctx* c) { return c->host_threads; }

int nhip_device_numa(nhip_ctx* c, int* numa_node, int* cpus, size_t cpu_cap, size_t* n_cpus) {
    if (!c || !numa_node) return NHIP_ERR_ARG;
    *numa_node = c->topo.numa_node;
    if (n_cpus) *n_cpus = c->topo.cpus.size();
    if (cpus)
        for (size_t i = 0; i < std::min(cpu_cap, c->topo.cpus.size()); ++i) cpus[i] = c->topo.cpus[i];
    return NHIP_OK;
}

int nhip_set_host_threads(nhip_ctx* c, unsigned threads) {
    if (!c || threads > 256) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    c->host_threads = threads;
    return NHIP_OK;
}

// ------------------------------------------------------------------ device-resident form
int nhip_dev_alloc(nhip_ctx* c, size_t bytes, void** dptr) {
    if (!c || !dptr) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    return hip_fail(hipMalloc(dptr, bytes ? bytes : 1));
}

int nhip_dev_free(nhip_ctx* c, void* d) {
    if (!c) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    (void)hipStreamSynchronize(c->stream);
    return hip_fail(hipFree(d));
}

int nhip_memcpy_h2d(nhip_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

int nhip_memcpy_d2h(nhip_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

int nhip_synchronize(nhip_ctx* c) {
    if (!c) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    return hip_fail(hipStreamSynchronize(c->stream));
}

int nhip_tip5_permutation_dev(nhip_ctx* c, uint64_t* d_states, size_t n) {
    if (!c || (n && !d_states)) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    return timed_launch(c, [&] { return nhip::launch_permutation(d_states, n, c->stream); });
}

int nhip_tip5_hash_pair_dev(nhip_ctx* c, const uint64_t* l, const uint64_t* r, size_t n, uint64_t* o) {
    if (!c || (n && (!l || !r || !o))) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    return timed_launch(c, [&] { return nhip::launch_hash_pair(l, r, o, n, c->stream); });
}

int nhip_tip5_hash_varlen_dev(nhip_ctx* c, const uint64_t* d, const uint64_t* off, size_t n, uint64_t* o) {
    if (!c || (n && (!off || !o))) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    return timed_launch(c, [&] { return nhip::launch_hash_varlen(d, off, n, o, c->stream); });
}

int nhip_mtree_build_dev(nhip_ctx* c, const uint64_t* d_leafs, size_t n, uint64_t* d_nodes) {
    if (!c || !is_pow2(n) || !d_leafs || !d_nodes) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    return build_tree_dev(c, d_leafs, n, d_nodes);
}

int nhip_mtree_verify_dev(nhip_ctx* c, const uint64_t* roots, size_t n_roots, const uint64_t* idx,
                          const uint64_t* leafs, const uint64_t* paths, uint32_t depth, size_t n, uint8_t* v) {
    if (!c || (n_roots != 1 && n_roots != n)) return NHIP_ERR_ARG;
    if (n && (!roots || !idx || !leafs || !v || (depth && !paths))) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    const int per_path = (n_roots == n && n != 1) ? 1 : 0;
    return timed_launch(c, [&] {
        return nhip::launch_mtree_verify(roots, per_path, idx, leafs, paths, depth, n, v, c->stream);
    });
}

int nhip_verdicts_all_dev(nhip_ctx* c, const uint8_t* d_v, size_t n, uint8_t* all_ok) {
    if (!c || !all_ok || (n && !d_v)) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    size_t sizes[1] = {sizeof(uint32_t)};
    void* p[1];
    int rc = carve(c, sizes, p);
    if (rc) return rc;
    uint32_t* d_out = (uint32_t*)p[0];
    hipError_t e = hipMemsetAsync(d_out, 0, sizeof(uint32_t), c->stream);
    if (e != hipSuccess) return hip_fail(e);
    size_t blocks = (n / 16 + 255) / 256;
    if (blocks < 1) blocks = 1;
    if (blocks > 1024) blocks = 1024;
    rc = timed_launch(c, [&] {
        hipLaunchKernelGGL(k_any_bad, dim3((unsigned)blocks), dim3(256), 0, c->stream, d_v, n, d_out);
        return hipGetLastError();
    });
    if (rc) return rc;
    uint32_t h = 1;
    e = hipMemcpyAsync(&h, d_out, sizeof(h), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(e);
    h = h ? 0u : 1u;
    *all_ok = (uint8_t)(h ? 1 : 0);
    return NHIP_OK;
}

// ------------------------------------------------------------------ host-buffer form
int nhip_tip5_permutation(nhip_ctx* c, uint64_t* states, size_t n) {
    if (!c || (n && !states)) return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    const size_t bytes = n * 16 * sizeof(uint64_t);
    size_t sizes[1] = {bytes};
    void* p[1];
    int rc = carve(c, sizes, p);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(p[0], states, bytes, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(e);
    rc = timed_launch(c, [&] { return nhip::launch_permutation((uint64_t*)p[0], n, c->stream); });
    if (rc) return rc;
    e = hipMemcpyAsync(states, p[0], bytes, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

int nhip_tip5_hash_pair(nhip_ctx* c, const uint64_t* l, const uint64_t* r, size_t n, uint64_t* o) {
    if (!c || (n && (!l || !r || !o))) return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    const size_t db = n * 5 * sizeof(uint64_t);
    size_t sizes[3] = {db, db, db};
    void* p[3];
    int rc = carve(c, sizes, p);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(p[0], l, db, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(p[1], r, db, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(e);
    rc = timed_launch(c, [&] {
        return nhip::launch_hash_pair((const uint64_t*)p[0], (const uint64_t*)p[1], (uint64_t*)p[2], n, c->stream);
    });
    if (rc) return rc;
    e = hipMemcpyAsync(o, p[2], db, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

int nhip_tip5_hash_varlen(nhip_ctx* c, const uint64_t* data, const uint64_t* offsets, size_t n, uint64_t* o) {
    if (!c || (n && (!offsets || !o))) return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    for (size_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return NHIP_ERR_ARG;
    const size_t total = (size_t)offsets[n];
    if (total && !data) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    size_t sizes[3] = {total * sizeof(uint64_t), (n + 1) * sizeof(uint64_t), n * 5 * sizeof(uint64_t)};
    void* p[3];
    int rc = carve(c, sizes, p);
    if (rc) return rc;
    hipError_t e = hipSuccess;
    if (total) e = hipMemcpyAsync(p[0], data, sizes[0], hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(p[1], offsets, sizes[1], hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(e);
    rc = timed_launch(c, [&] {
        return nhip::launch_hash_varlen((const uint64_t*)p[0], (const uint64_t*)p[1], n, (uint64_t*)p[2], c->stream);
    });
    if (rc) return rc;
    e = hipMemcpyAsync(o, p[2], sizes[2], hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

int nhip_mtree_build(nhip_ctx* c, const uint64_t* leafs, size_t n, uint64_t* nodes_out) {
    if (!c || !is_pow2(n) || !leafs || !nodes_out) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    const size_t db = n * 5 * sizeof(uint64_t);
    size_t sizes[2] = {db, db};
    void* p[2];
    int rc = carve(c, sizes, p);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(p[0], leafs, db, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(e);
    rc = build_tree_dev(c, (const uint64_t*)p[0], n, (uint64_t*)p[1]);
    if (rc) return rc;
    e = hipMemcpyAsync(nodes_out, p[1], db, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

int nhip_mtree_verify(nhip_ctx* c, const uint64_t* roots, size_t n_roots, const uint64_t* idx,
                      const uint64_t* leafs, const uint64_t* paths, uint32_t depth, size_t n, uint8_t* v) {
    if (!c || (n_roots != 1 && n_roots != n)) return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    if (!roots || !idx || !leafs || !v || (depth && !paths)) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    size_t sizes[5] = {n_roots * 5 * sizeof(uint64_t), n * sizeof(uint64_t), n * 5 * sizeof(uint64_t),
                       n * (size_t)depth * 5 * sizeof(uint64_t), n};
    void* p[5];
    int rc = carve(c, sizes, p);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(p[0], roots, sizes[0], hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(p[1], idx, sizes[1], hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(p[2], leafs, sizes[2], hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && depth) e = hipMemcpyAsync(p[3], paths, sizes[3], hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(e);
    const int per_path = (n_roots == n && n != 1) ? 1 : 0;
    rc = timed_launch(c, [&] {
        return nhip::launch_mtree_verify((const uint64_t*)p[0], per_path, (const uint64_t*)p[1],
                                         (const uint64_t*)p[2], (const uint64_t*)p[3], depth, n, (uint8_t*)p[4],
                                         c->stream);
    });
    if (rc) return rc;
    e = hipMemcpyAsync(v, p[4], n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

// ------------------------------------------------------------------ timing
int nhip_timing_enable(nhip_ctx* c, int on) {
    if (!c) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    c->timing = on != 0;
    return NHIP_OK;
}

int nhip_timing_read(nhip_ctx* c, double* total_ms, uint64_t* launches, int reset) {
    if (!c) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(e);
    for (auto& pr : c->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) c->timed_ms += ms;
        c->timed_launches += 1;
        c->free_events.push_back(pr.first);
        c->free_events.push_back(pr.second);
    }
    c->pending.clear();
    if (total_ms) *total_ms = c->timed_ms;
    if (launches) *launches = c->timed_launches;
    if (reset) {
        c->timed_ms = 0.0;
        c->timed_launches = 0;
    }
    return NHIP_OK;
}

// MastHash::mast_hash (mast_hash.rs:22-39) for n objects of `fields` field sequences each:
// field sequence (i, f) = data[offsets[i*fields+f] .. offsets[i*fields+f+1]).
int nhip_mast_hash_batch(nhip_ctx* c, const uint64_t* data, const uint64_t* offsets, uint32_t fields, size_t n,
                         uint64_t* roots_out) {
    if (!c || fields < 1 || fields > 16 || (n && (!offsets || !roots_out))) return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    const size_t nl = n * fields;
    for (size_t i = 0; i < nl; ++i)
        if (offsets[i + 1] < offsets[i]) return NHIP_ERR_ARG;
    const size_t total = (size_t)offsets[nl];
    if (total && !data) return NHIP_ERR_ARG;
    uint32_t pow2 = 1;
    while (pow2 < fields) pow2 <<= 1;
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    size_t sizes[4] = {total * 8, (nl + 1) * 8, nl * 40, n * 40};
    void* p[4];
    int rc = carve(c, sizes, p);
    if (rc) return rc;
    hipError_t e = hipSuccess;
    if (total) e = hipMemcpyAsync(p[0], data, sizes[0], hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(p[1], offsets, sizes[1], hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(e);
    rc = timed_launch(c, [&] {
        return nhip::launch_hash_varlen((const uint64_t*)p[0], (const uint64_t*)p[1], nl, (uint64_t*)p[2], c->stream);
    });
    if (rc) return rc;
    rc = timed_launch(c, [&] {
        return nhip::launch_mast_roots((const uint64_t*)p[2], fields, pow2, n, (uint64_t*)p[3], c->stream);
    });
    if (rc) return rc;
    e = hipMemcpyAsync(roots_out, p[3], sizes[3], hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

// AbsoluteIndexSet::compute (absolute_index_set.rs:86-113) for n removal records.
int nhip_absolute_index_sets(nhip_ctx* c, const uint64_t* items, const uint64_t* sender_randomness,
                             const uint64_t* receiver_preimages, const uint64_t* aocl_leaf_indices, size_t n,
                             uint64_t* minimum_out, uint32_t* distances_out) {
    if (!c || (n && (!items || !sender_randomness || !receiver_preimages || !aocl_leaf_indices || !minimum_out ||
                     !distances_out)))
        return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    std::vector<uint64_t> in(15 * n);
    for (size_t i = 0; i < n; ++i)
        for (int q = 0; q < 5; ++q) {
            in[15 * i + q] = items[5 * i + q];
            in[15 * i + 5 + q] = sender_randomness[5 * i + q];
            in[15 * i + 10 + q] = receiver_preimages[5 * i + q];
        }
    std::lock_guard<std::mutex> g(c->mu);
    const DeviceScope device_scope(c->device);
    size_t sizes[4] = {15 * n * 8, n * 8, 2 * n * 8, 45 * n * 4};
    void* p[4];
    int rc = carve(c, sizes, p);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(p[0], in.data(), sizes[0], hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(p[1], aocl_leaf_indices, sizes[1], hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_fail(e);
    rc = timed_launch(c, [&] {
        return nhip::launch_absolute_index_sets((const uint64_t*)p[0], (const uint64_t*)p[1], n, (uint64_t*)p[2],
                                                (uint32_t*)p[3], c->stream);
    });
    if (rc) return rc;
    e = hipMemcpyAsync(minimum_out, p[2], sizes[2], hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(distances_out, p[3], sizes[3], hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return hip_fail(e);
}

}  // extern "C"
