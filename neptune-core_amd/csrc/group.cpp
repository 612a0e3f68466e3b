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
#include <cstring>
#include <functional>
#include <new>
#include <numeric>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/neptune_hip.h"
#include "group.hpp"
#include "host_numa.hpp"


// Each member's host work on its GPU's NUMA node: the member threads a group starts are bound to
// the node's CPUs, and the node's CPUs are divided among the members on it for their staging copy
// threads (8 GPUs on two sockets: 4 members share a socket's cores instead of 8 x 16 unbound
// threads contending for them).
static void place_members(nhip_group* g) {
    const size_t M = g->members.size();
    g->cpus.assign(M, {});
    if (!nhip::numa_enabled()) return;  // NHIP_NUMA=0: no binding and the default copy threads
    std::vector<int> node(M, -1);
    for (size_t m = 0; m < M; ++m) {
        size_t n = 0;
        int nd = -1;
        if (nhip_device_numa(g->members[m], &nd, nullptr, 0, &n) != NHIP_OK) continue;
        node[m] = nd;
        g->cpus[m].resize(n);
        size_t got = 0;
        (void)nhip_device_numa(g->members[m], &nd, g->cpus[m].data(), n, &got);
        g->cpus[m].resize(std::min(n, got));
    }
    for (size_t m = 0; m < M; ++m) {
        if (node[m] < 0 || g->cpus[m].empty()) continue;
        size_t sharing = 0;
        for (size_t q = 0; q < M; ++q) sharing += node[q] == node[m] ? 1 : 0;
        const size_t per = std::max<size_t>(1, g->cpus[m].size() / std::max<size_t>(1, sharing));
        (void)nhip_set_host_threads(g->members[m], (unsigned)std::min<size_t>(16, per));
    }
}

static void bind_member_thread(const nhip_group* g, size_t m) {
    if (m < g->cpus.size()) (void)nhip::bind_thread(g->cpus[m]);
}

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
    try {
        place_members(g);
    } catch (const std::bad_alloc&) {
        g->cpus.clear();  // unplaced: still correct
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
                threads.emplace_back([&, m] {
                    bind_member_thread(g, m);
                    run(m);
                });
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

// ---------------------------------------------------------------------- streaming group
// Per member two device batches (slot k % 2 holds batch k's share).  submit(k): every busy member,
// on its own host thread, refills slot k % 2 (host staging + upload; the member's slot (k - 1) % 2
// is still running batch k - 1 on its GPU), launches it, then waits for slot (k - 1) % 2 and
// scatters batch k - 1's verdicts.  So the upload of batch k overlaps the device run of batch k - 1
// on every member at once, as the one-context refill / launch / wait loop does (bench.py's
// pcie_inclusive), and the members stream concurrently.
namespace {

struct StreamBatch {
    uint8_t* verdicts = nullptr;
    uint8_t* all_ok = nullptr;
    size_t n = 0;
    std::vector<std::vector<size_t>> idx;  // per member: the caller's positions of its share
    bool live = false;                     // submitted, verdicts / AND not yet written
};

struct MemberSlots {
    nhip_batch* b[2] = {nullptr, nullptr};
    bool in_flight[2] = {false, false};
    std::vector<nhip_claim> claims;
    std::vector<nhip_proof> proofs;
    std::vector<uint8_t> v[2];  // per slot: sized to that slot's share when the slot is refilled
};

}  // namespace

struct nhip_group_stream {
    nhip_group* g = nullptr;
    nhip_air* air = nullptr;
    nhip_stark_params params{};
    std::vector<MemberSlots> m;
    StreamBatch sb[2];
    uint64_t next = 0;  // batches submitted
    uint64_t batches = 0, proofs = 0;

    // Run f(member) for every member in `who` concurrently (member threads; the caller's thread
    // takes the first, and any share whose thread cannot be started); returns the first error.
    int on_members(const std::vector<size_t>& who, const std::function<int(size_t)>& f) {
        std::vector<int> rcs(who.size(), NHIP_OK);
        std::vector<std::thread> th;
        std::vector<size_t> inline_k;
        th.reserve(who.size());
        inline_k.reserve(who.size());
        for (size_t k = 1; k < who.size(); ++k) {
            try {
                th.emplace_back([&, k] {
                    bind_member_thread(g, who[k]);
                    rcs[k] = f(who[k]);
                });
            } catch (const std::system_error&) {
                inline_k.push_back(k);
            }
        }
        if (!who.empty()) rcs[0] = f(who[0]);
        for (auto& t : th) t.join();
        for (size_t k : inline_k) rcs[k] = f(who[k]);
        for (int rc : rcs)
            if (rc) return rc;
        return NHIP_OK;
    }

    // member mm: wait for its share of batch sb[s] and scatter the verdicts
    int complete_member(size_t mm, int s) {
        MemberSlots& ms = m[mm];
        if (!ms.in_flight[s]) return NHIP_OK;
        ms.in_flight[s] = false;
        StreamBatch& B = sb[s];
        const size_t cnt = B.idx[mm].size();
        // sized at submit, so never short; if it were, the batch is still waited for (the slot must
        // be idle before it is refilled or destroyed) and its verdicts are not read
        const bool fits = ms.v[s].size() >= cnt;
        const int rc = nhip_batch_wait(g->members[mm], ms.b[s], fits ? ms.v[s].data() : nullptr, nullptr);
        if (rc) return rc;
        if (!fits) return NHIP_ERR_ARG;
        for (size_t q = 0; q < cnt; ++q) B.verdicts[B.idx[mm][q]] = ms.v[s][q];
        nhip_stats st{};
        nhip_batch_stats(ms.b[s], &st);
        dev_ms[mm] += st.ms_device_total;
        return NHIP_OK;
    }

    std::vector<double> stage_ms, upload_ms, dev_ms;  // per member, written by that member's thread only

    void finish_batch(int s) {
        StreamBatch& B = sb[s];
        if (!B.live) return;
        B.live = false;
        if (B.all_ok) {
            uint8_t ok = 1;
            for (size_t i = 0; i < B.n; ++i) ok &= (uint8_t)(B.verdicts[i] != 0);
            *B.all_ok = ok;
        }
    }

    // after a fault: wait for whatever is still running so every slot is idle again
    void drain() {
        for (size_t mm = 0; mm < m.size(); ++mm)
            for (int s = 0; s < 2; ++s)
                if (m[mm].in_flight[s]) {
                    (void)nhip_batch_wait(g->members[mm], m[mm].b[s], nullptr, nullptr);
                    m[mm].in_flight[s] = false;
                }
        sb[0].live = sb[1].live = false;
    }
};

extern "C" {

int nhip_group_stream_create(nhip_group* g, nhip_air* air, const nhip_stark_params* params,
                             nhip_group_stream** out) {
    if (!g || g->members.empty() || !air || !params || !out) return NHIP_ERR_ARG;
    *out = nullptr;
    nhip_group_stream* st = new (std::nothrow) nhip_group_stream();
    if (!st) return NHIP_ERR_OOM;
    try {
        st->g = g;
        st->air = air;
        st->params = *params;
        st->m.resize(g->members.size());
        st->stage_ms.assign(g->members.size(), 0.0);
        st->upload_ms.assign(g->members.size(), 0.0);
        st->dev_ms.assign(g->members.size(), 0.0);
        for (auto& b : st->sb) b.idx.resize(g->members.size());
    } catch (const std::bad_alloc&) {
        delete st;
        return NHIP_ERR_OOM;
    }
    *out = st;
    return NHIP_OK;
}

static int stream_submit(nhip_group_stream* st, const nhip_claim* claims, const nhip_proof* proofs,
                         const uint32_t* placed, size_t n, uint8_t* verdicts, uint8_t* all_ok) {
    if (!st) return NHIP_ERR_ARG;
    if (n && (!claims || !proofs || !verdicts)) return NHIP_ERR_ARG;
    const size_t M = st->m.size();
    if (placed)
        for (size_t i = 0; i < n; ++i)
            if (placed[i] >= M) return NHIP_ERR_ARG;
    const int s = (int)(st->next & 1u), sp = s ^ 1;
    try {
        StreamBatch& B = st->sb[s];
        B.verdicts = verdicts;
        B.all_ok = all_ok;
        B.n = n;
        std::vector<uint32_t> member_of(n);
        int rc = NHIP_OK;
        if (placed) std::copy(placed, placed + n, member_of.begin());  // the caller's placement (arenas)
        else rc = nhip_group_shard(proofs, n, M, member_of.data());
        if (rc) return rc;
        for (auto& v : B.idx) v.clear();
        for (size_t i = 0; i < n; ++i) B.idx[member_of[i]].push_back(i);
        std::vector<size_t> who;  // members with a share of this batch or a previous share to complete
        for (size_t mm = 0; mm < M; ++mm) {
            MemberSlots& ms = st->m[mm];
            ms.claims.clear();
            ms.proofs.clear();
            for (size_t i : B.idx[mm]) {
                ms.claims.push_back(claims[i]);
                ms.proofs.push_back(proofs[i]);
            }
            // slot s is idle (its batch k - 2 was completed by the previous submit): size its verdict
            // buffer to THIS share, the one complete_member(mm, s) will read back (here, on the
            // calling thread, so an allocation failure is a return code, not a throw in a member thread)
            ms.v[s].resize(std::max<size_t>(1, B.idx[mm].size()));
            if (!B.idx[mm].empty() || ms.in_flight[sp]) who.push_back(mm);
        }
        B.live = true;  // an empty batch too: its AND (1) is written with the others'
        rc = st->on_members(who, [&](size_t mm) -> int {
            MemberSlots& ms = st->m[mm];
            nhip_ctx* c = st->g->members[mm];
            const size_t cnt = B.idx[mm].size();
            if (cnt) {
                // slot s is idle: its batch (k - 2) was completed by the previous submit
                int r = ms.b[s] ? nhip_batch_refill(c, ms.b[s], st->air, &st->params, ms.claims.data(),
                                                    ms.proofs.data(), cnt)
                                : nhip_batch_prepare(c, st->air, &st->params, ms.claims.data(), ms.proofs.data(),
                                                     cnt, &ms.b[s]);
                if (!r) {
                    nhip_stats bs{};
                    nhip_batch_stats(ms.b[s], &bs);
                    st->stage_ms[mm] += bs.ms_decode;
                    st->upload_ms[mm] += bs.ms_upload;
                    r = nhip_batch_launch(c, ms.b[s]);
                }
                if (r) return r;
                ms.in_flight[s] = true;
            }
            return st->complete_member(mm, sp);
        });
        if (rc) {
            st->drain();
            ++st->next;
            return rc;
        }
        st->finish_batch(sp);
        st->batches += n ? 1 : 0;
        st->proofs += n;
        ++st->next;
    } catch (const std::bad_alloc&) {
        st->drain();
        ++st->next;
        return NHIP_ERR_OOM;
    }
    return NHIP_OK;
}

int nhip_group_stream_submit(nhip_group_stream* st, const nhip_claim* claims, const nhip_proof* proofs, size_t n,
                             uint8_t* verdicts, uint8_t* all_ok) {
    return stream_submit(st, claims, proofs, nullptr, n, verdicts, all_ok);
}

int nhip_group_stream_submit_placed(nhip_group_stream* st, const nhip_claim* claims, const nhip_proof* proofs,
                                    const uint32_t* member_of, size_t n, uint8_t* verdicts, uint8_t* all_ok) {
    if (n && !member_of) return NHIP_ERR_ARG;
    return stream_submit(st, claims, proofs, member_of, n, verdicts, all_ok);
}

int nhip_group_stream_finish(nhip_group_stream* st) {
    if (!st) return NHIP_ERR_ARG;
    const int sp = (int)((st->next & 1u) ^ 1u);  // the last submitted batch's slot
    std::vector<size_t> who;
    for (size_t mm = 0; mm < st->m.size(); ++mm)
        if (st->m[mm].in_flight[sp]) who.push_back(mm);
    int rc;
    try {
        rc = st->on_members(who, [&](size_t mm) { return st->complete_member(mm, sp); });
    } catch (const std::bad_alloc&) {
        rc = NHIP_ERR_OOM;
    }
    if (rc) {
        st->drain();
        return rc;
    }
    st->finish_batch(sp);
    return NHIP_OK;
}

int nhip_group_stream_stats(const nhip_group_stream* st, uint64_t* batches, uint64_t* proofs, double* ms_stage,
                            double* ms_upload, double* ms_device) {
    if (!st) return NHIP_ERR_ARG;
    double a = 0, b = 0, c = 0;
    for (size_t mm = 0; mm < st->m.size(); ++mm) {
        a += st->stage_ms[mm];
        b += st->upload_ms[mm];
        c += st->dev_ms[mm];
    }
    if (batches) *batches = st->batches;
    if (proofs) *proofs = st->proofs;
    if (ms_stage) *ms_stage = a;
    if (ms_upload) *ms_upload = b;
    if (ms_device) *ms_device = c;
    return NHIP_OK;
}

void nhip_group_stream_destroy(nhip_group_stream* st) {
    if (!st) return;
    st->drain();
    for (size_t mm = 0; mm < st->m.size(); ++mm)
        for (nhip_batch* b : st->m[mm].b)
            if (b) nhip_batch_destroy(b);
    delete st;
}

}  // extern "C"
