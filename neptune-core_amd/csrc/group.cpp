// Multi-GPU verification from ONE process: a group of contexts, one per member device.
//
// neptune-core is a single process (the node), and its callers hand over whole batches:
// proof_collection.rs:342-388 (one ProofCollection), state/mod.rs:2226-2272 (bootstrap import),
// peer_loop.rs:315-323 (block batches), each of which ends in n calls of
// triton_vm::verify(Stark::default(), &claim, &proof) at verifier.rs:60-63.  Proofs are
// independent, so nhip_group_verify_batch shards a batch over the member GPUs at proof
// granularity (LPT on the proof length, the per-proof cost proxy: revealed rows, authentication
// structures and FRI responses all grow with it), runs every shard concurrently on its member's
// own streams (nhip_verify_batch per member, one host thread each) and writes the verdicts back
// in the caller's order.  The only exchange is the verdict bytes, which every member already
// copies to the host; the batch AND is taken there.  (The multi-process form - one rank per GPU,
// one RCCL all-gather of the batch and per-proof verdicts per step - is neptune_hip.shard /
// bench.py.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <new>
#include <numeric>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/neptune_hip.h"

struct nhip_group {
    std::vector<nhip_ctx*> members;
};

extern "C" {

int nhip_group_create(const int* devices, size_t n_devices, nhip_group** out) {
    if (!out || !devices || n_devices == 0) return NHIP_ERR_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return NHIP_ERR_NO_DEVICE;
    for (size_t i = 0; i < n_devices; ++i)
        if (devices[i] < 0 || devices[i] >= count || devices[i] >= 32) return NHIP_ERR_NO_DEVICE;
    nhip_group* g = new (std::nothrow) nhip_group();
    if (!g) return NHIP_ERR_OOM;
    try {
        g->members.reserve(n_devices);
    } catch (const std::bad_alloc&) {
        delete g;
        return NHIP_ERR_OOM;
    }
    for (size_t i = 0; i < n_devices; ++i) {
        nhip_ctx* c = nullptr;
        const int rc = nhip_init(1u << devices[i], &c);
        if (rc) {
            nhip_group_destroy(g);
            return rc;
        }
        g->members.push_back(c);
    }
    *out = g;
    return NHIP_OK;
}

int nhip_group_init(uint32_t device_mask, nhip_group** out) {
    if (!out) return NHIP_ERR_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return NHIP_ERR_NO_DEVICE;
    int devs[32];
    size_t n = 0;
    for (int d = 0; d < count && d < 32; ++d)
        if (device_mask == 0 || (device_mask >> d) & 1u) devs[n++] = d;
    if (n == 0) return NHIP_ERR_NO_DEVICE;
    return nhip_group_create(devs, n, out);
}

void nhip_group_destroy(nhip_group* g) {
    if (!g) return;
    for (nhip_ctx* c : g->members) nhip_destroy(c);
    delete g;
}

size_t nhip_group_size(const nhip_group* g) { return g ? g->members.size() : 0; }

nhip_ctx* nhip_group_member(nhip_group* g, size_t i) {
    return (g && i < g->members.size()) ? g->members[i] : nullptr;
}

int nhip_group_shard(const nhip_proof* proofs, size_t n, size_t n_members, uint32_t* member_of) {
    if ((n && (!proofs || !member_of)) || n_members == 0) return NHIP_ERR_ARG;
    try {
        std::vector<size_t> order(n);
        std::iota(order.begin(), order.end(), 0);
        // longest first (stable: equal lengths keep the caller's order), each to the least loaded
        std::stable_sort(order.begin(), order.end(),
                         [&](size_t a, size_t b) { return proofs[a].len > proofs[b].len; });
        std::vector<uint64_t> load(n_members, 0);
        for (size_t i : order) {
            const size_t m = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
            member_of[i] = (uint32_t)m;
            load[m] += (uint64_t)proofs[i].len + 1;
        }
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
    return NHIP_OK;
}

int nhip_group_verify_batch(nhip_group* g, nhip_air* air, const nhip_stark_params* params, const nhip_claim* claims,
                            const nhip_proof* proofs, size_t n, uint8_t* verdicts, uint8_t* all_ok) {
    if (!g || g->members.empty() || !air) return NHIP_ERR_ARG;
    if (n && (!claims || !proofs || !verdicts)) return NHIP_ERR_ARG;
    const size_t M = g->members.size();
    try {
        std::vector<uint32_t> member_of(n);
        int rc = nhip_group_shard(proofs, n, M, member_of.data());
        if (rc) return rc;
        std::vector<std::vector<size_t>> idx(M);
        for (size_t i = 0; i < n; ++i) idx[member_of[i]].push_back(i);
        std::vector<std::vector<nhip_claim>> c(M);
        std::vector<std::vector<nhip_proof>> p(M);
        std::vector<std::vector<uint8_t>> v(M);
        for (size_t m = 0; m < M; ++m) {
            c[m].reserve(idx[m].size());
            p[m].reserve(idx[m].size());
            for (size_t i : idx[m]) {
                c[m].push_back(claims[i]);
                p[m].push_back(proofs[i]);
            }
            v[m].assign(idx[m].size(), 0);
        }
        std::vector<int> rcs(M, NHIP_OK);
        auto run = [&](size_t m) {
            if (idx[m].empty()) return;
            rcs[m] = nhip_verify_batch(g->members[m], air, params, c[m].data(), p[m].data(), idx[m].size(),
                                       v[m].data(), nullptr);
        };
        // one host thread per busy member (member 0 on the calling thread); a thread that cannot be
        // started runs its shard on the calling thread afterwards
        // (both vectors are reserved up front: no allocation, hence no throw, once a thread runs)
        std::vector<std::thread> threads;
        std::vector<size_t> inline_members;
        threads.reserve(M);
        inline_members.reserve(M);
        for (size_t m = 1; m < M; ++m) {
            if (idx[m].empty()) continue;
            try {
                threads.emplace_back(run, m);
            } catch (const std::system_error&) {
                inline_members.push_back(m);
            } catch (const std::bad_alloc&) {
                inline_members.push_back(m);
            }
        }
        run(0);
        for (auto& t : threads) t.join();
        for (size_t m : inline_members) run(m);
        for (size_t m = 0; m < M; ++m)
            if (rcs[m]) return rcs[m];  // infrastructure fault: the batch verdict is unknown, never accept
        uint8_t ok = 1;
        for (size_t m = 0; m < M; ++m)
            for (size_t k = 0; k < idx[m].size(); ++k) {
                verdicts[idx[m][k]] = v[m][k];
                ok &= (uint8_t)(v[m][k] != 0);
            }
        if (all_ok) *all_ok = ok;
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
    return NHIP_OK;
}

}  // extern "C"
