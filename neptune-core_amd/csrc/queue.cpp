// Coalescing verification queue (include/neptune_hip.h, nhip_queue_*).
//
// The reference verifies one proof per call: `verify(claim, proof, network)` hops onto tokio's
// blocking pool and runs `triton_vm::verify` there (neptune-core/src/protocol/proof_abstractions/
// verifier.rs:60-63), called concurrently from many tasks, e.g. one per peer transaction
// (application/loops/peer_loop.rs:1342 -> Transaction::is_valid).  One GPU verify of a single
// proof is latency-bound (~1.7 ms, almost all of it the sequential Fiat-Shamir sponge), so
// serializing such calls would cap a context at ~500 proofs/s.  The queue gathers concurrent
// callers' proofs into one batch instead ("the internal queue may coalesce small
// calls into batches"): a worker thread takes every pending request (up to max_batch proofs, after
// at most max_wait_us from the oldest arrival), stages them into one of two nhip_batch slots, and
// launches it; while that batch runs on the device the next one is collected, so the device sees
// back-to-back batches whose size follows the load.  Each caller blocks until its own verdicts are
// written, with nhip_verify_batch semantics (0 = reject; a non-zero return is an infrastructure
// fault, never "accept").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/neptune_hip.h"
#include "ab_env.hpp"
#include "pinned_ring.hpp"

// stark_host.cpp: true once every phase of a launched batch has completed (a stream query, no wait)
extern "C" bool nhip_internal_batch_done(nhip_batch* b);

namespace {

using Clock = std::chrono::steady_clock;
// how often the in-flight batch is polled while a coalescing window is open
constexpr std::chrono::microseconds POLL_SLICE{25};

struct Req {
    const nhip_claim* claims;
    const nhip_proof* proofs;
    size_t n;
    uint8_t* verdicts;
    Clock::time_point arrived;
    int rc = NHIP_OK;
    bool done = false;
    uint64_t arena_at = ~0ull;  // its proofs' range in the pinned arena (~0: its own memory)
};

// Arena size: at most 256 MB (about two full batches of config-4-sized proofs from concurrent
// callers), at most 2 MB per proof of two max_batch batches (a Stark::default() proof of padded
// height 2^23 is ~1.4 MB), at least 16 MB.  NHIP_QUEUE_ARENA_MB overrides it (read at create; 0 =
// no arena: every request goes through the context's staging).  A node with one queue per GPU
// pins this much host memory per queue.
constexpr uint64_t ARENA_MAX_BYTES = 256ull << 20, ARENA_MIN_BYTES = 16ull << 20;
static uint64_t arena_bytes(uint32_t max_batch) {
    if (const char* e = std::getenv("NHIP_QUEUE_ARENA_MB")) return (uint64_t)std::strtoull(e, nullptr, 10) << 20;
    const uint64_t by_batch = (uint64_t)max_batch * 2 * (2ull << 20);
    return std::max(ARENA_MIN_BYTES, std::min(ARENA_MAX_BYTES, by_batch));
}

}  // namespace

struct nhip_queue {
    nhip_ctx* ctx = nullptr;
    nhip_air* air = nullptr;
    nhip_stark_params params{};
    size_t max_batch = 0;
    std::chrono::microseconds max_wait{0};
    std::mutex mu;
    std::condition_variable cv_in, cv_out;
    std::deque<Req*> pending;
    size_t pending_proofs = 0;
    bool stop = false;
    std::thread worker;
    // batch slots: up to slots_used batches on the device while the next is collected and staged (a
    // batch is launched when its window closes and a slot is free; the worker polls the batches on the
    // device instead of blocking on the oldest, so a request arriving meanwhile opens its window at
    // once).  Two slots measured best (profiles/r06/ab_queue_slots.txt): three or four split the same
    // load into smaller batches of nearly the same device time each, and the tail grows.
    static constexpr int QUEUE_SLOTS = 4;
    int slots_used = 2;  // A/B build: NHIP_QUEUE_SLOTS (1-4)
    nhip_batch* slot[QUEUE_SLOTS] = {};
    std::vector<Req*> in_slot[QUEUE_SLOTS];
    bool in_flight[QUEUE_SLOTS] = {};
    std::vector<nhip_claim> claims;
    std::vector<nhip_proof> proofs;
    std::vector<uint8_t> verdicts;
    std::atomic<uint64_t> n_batches{0}, n_proofs{0};
    nhip::PinnedRing ring;  // guarded by mu
    // nhip_queue_profile: written by the worker under prof_mu, read by nhip_queue_profile_read
    mutable std::mutex prof_mu;
    nhip_queue_profile prof{};
    Clock::time_point oldest[QUEUE_SLOTS];  // per slot: the earliest arrival among its requests

    static double ms_since(Clock::time_point t0, Clock::time_point t1) {
        return std::chrono::duration<double, std::milli>(t1 - t0).count();
    }

    // per-request latency (arrival in nhip_queue_verify -> verdicts delivered), microseconds, the
    // last LAT_CAP requests (nhip_queue_latencies); guarded by prof_mu
    static constexpr size_t LAT_CAP = 1u << 16;
    std::vector<float> lat_us;
    uint64_t lat_n = 0;

    void deliver(std::vector<Req*>& reqs, int rc, const uint8_t* v) {
        const Clock::time_point now = Clock::now();
        {
            std::lock_guard<std::mutex> g(prof_mu);
            for (Req* r : reqs) {
                if (lat_us.size() < LAT_CAP) lat_us.push_back(0.f);
                lat_us[lat_n++ % LAT_CAP] = (float)(ms_since(r->arrived, now) * 1e3);
            }
        }
        std::lock_guard<std::mutex> g(mu);
        size_t off = 0;
        for (Req* r : reqs) {
            r->rc = rc;
            if (!rc && r->n) std::memcpy(r->verdicts, v + off, r->n);
            off += r->n;
            r->done = true;
        }
        reqs.clear();
        cv_out.notify_all();
    }

    void finish(int s) {
        if (!in_flight[s]) return;
        in_flight[s] = false;
        size_t n = 0;
        for (Req* r : in_slot[s]) n += r->n;
        int rc = NHIP_OK;
        try {
            verdicts.assign(n ? n : 1, 0);
        } catch (const std::bad_alloc&) {
            rc = NHIP_ERR_OOM;  // still wait: the slot must be idle before it is refilled
        }
        const Clock::time_point t0 = Clock::now();
        const int wrc = nhip_batch_wait(ctx, slot[s], rc ? nullptr : verdicts.data(), nullptr);
        const Clock::time_point t1 = Clock::now();
        nhip_stats st{};
        if (!wrc) nhip_batch_stats(slot[s], &st);
        deliver(in_slot[s], rc ? rc : wrc, rc ? nullptr : verdicts.data());
        std::lock_guard<std::mutex> g(prof_mu);
        prof.ms_wait += ms_since(t0, t1);
        prof.ms_device += st.ms_device_total;
        prof.ms_turnaround += ms_since(oldest[s], Clock::now());
    }

    // stage + launch the requests in in_slot[s]
    void launch(int s) {
        claims.clear();
        proofs.clear();
        oldest[s] = Clock::now();
        for (Req* r : in_slot[s]) {
            oldest[s] = std::min(oldest[s], r->arrived);
            for (size_t i = 0; i < r->n; ++i) {
                claims.push_back(r->claims[i]);
                proofs.push_back(r->proofs[i]);
            }
        }
        const Clock::time_point t0 = Clock::now();
        int rc = slot[s] ? nhip_batch_refill(ctx, slot[s], air, &params, claims.data(), proofs.data(), claims.size())
                         : nhip_batch_prepare(ctx, air, &params, claims.data(), proofs.data(), claims.size(), &slot[s]);
        const Clock::time_point t1 = Clock::now();
        {  // uploaded (or failed): the requests' arena ranges can take new proofs
            std::lock_guard<std::mutex> g(mu);
            for (Req* r : in_slot[s])
                if (r->arena_at != ~0ull) ring.release(r->arena_at);
        }
        if (!rc) rc = nhip_batch_launch(ctx, slot[s]);
        const Clock::time_point t2 = Clock::now();
        if (rc) {
            deliver(in_slot[s], rc, nullptr);
            return;
        }
        in_flight[s] = true;
        ++n_batches;
        n_proofs += claims.size();
        nhip_stats st{};
        nhip_batch_stats(slot[s], &st);
        std::lock_guard<std::mutex> g(prof_mu);
        const size_t n = claims.size();
        prof.batches += 1;
        prof.proofs += n;
        prof.size_hist[std::min<size_t>(7, n <= 1 ? 0 : (size_t)(63 - __builtin_clzll((unsigned long long)n)))] += 1;
        prof.ms_window += ms_since(oldest[s], t0);
        for (Req* r : in_slot[s]) prof.pinned_proofs += r->arena_at != ~0ull ? r->n : 0;
        prof.ms_stage += st.ms_decode;
        prof.ms_upload += st.ms_upload;
        prof.ms_launch += ms_since(t1, t2);
    }

    void run() {
        std::deque<int> flying;  // slots with a batch on the device, oldest first (worker-only state)
        auto complete = [&](std::unique_lock<std::mutex>& lk, int f) {
            lk.unlock();
            finish(f);
            lk.lock();
        };
        // answer every batch on the device that has completed, in any order
        auto answer_done = [&](std::unique_lock<std::mutex>& lk) {
            for (size_t i = 0; i < flying.size();) {
                const int f = flying[i];
                if (nhip_internal_batch_done(slot[f])) {
                    flying.erase(flying.begin() + (ptrdiff_t)i);
                    complete(lk, f);
                } else {
                    ++i;
                }
            }
        };
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            if (pending.empty()) {
                if (stop) break;  // drained; the batches still on the device are answered below
                if (flying.empty()) {
                    cv_in.wait(lk, [&] { return stop || !pending.empty(); });
                } else {  // nothing new: poll the batches on the device, take a request as it comes
                    cv_in.wait_until(lk, Clock::now() + POLL_SLICE, [&] { return stop || !pending.empty(); });
                    answer_done(lk);
                }
                continue;
            }
            // coalescing window from the oldest request's arrival, ended early by a full batch.  The
            // batches on the device are answered as soon as each completes: while the window is open
            // their streams are polled in short slices.
            const Clock::time_point deadline = pending.front()->arrived + max_wait;
            for (;;) {
                answer_done(lk);
                if (stop || pending_proofs >= max_batch || Clock::now() >= deadline) break;
                const Clock::time_point until =
                    !flying.empty() ? std::min(deadline, Clock::now() + POLL_SLICE) : deadline;
                cv_in.wait_until(lk, until, [&] { return stop || pending_proofs >= max_batch; });
            }
            // a free slot; with every slot busy, the oldest batch completes first
            int s = -1;
            for (int q = 0; q < slots_used && s < 0; ++q)
                if (!in_flight[q]) s = q;
            if (s < 0) {
                s = flying.front();
                flying.pop_front();
                complete(lk, s);
            }
            size_t taken = 0;
            while (!pending.empty() && (taken == 0 || taken + pending.front()->n <= max_batch) &&
                   in_slot[s].size() < in_slot[s].capacity()) {
                Req* r = pending.front();
                pending.pop_front();
                pending_proofs -= r->n;
                taken += r->n;
                in_slot[s].push_back(r);
            }
            lk.unlock();
            try {
                launch(s);
            } catch (const std::bad_alloc&) {
                deliver(in_slot[s], NHIP_ERR_OOM, nullptr);
            }
            lk.lock();
            if (in_flight[s]) flying.push_back(s);
        }
        lk.unlock();
        for (int f : flying) finish(f);
    }
};

extern "C" {

int nhip_queue_create(nhip_ctx* ctx, nhip_air* air, const nhip_stark_params* params, uint32_t max_batch,
                      uint32_t max_wait_us, nhip_queue** out) {
    if (!ctx || !air || !params || !out) return NHIP_ERR_ARG;
    *out = nullptr;
    nhip_queue* q = new (std::nothrow) nhip_queue();
    if (!q) return NHIP_ERR_OOM;
    q->ctx = ctx;
    q->air = air;
    q->params = *params;
    q->max_batch = max_batch ? max_batch : 4096;
    q->max_wait = std::chrono::microseconds(max_wait_us);
    {
        void* a = nullptr;
        const uint64_t ab = arena_bytes(q->max_batch);
        if (ab && nhip_host_alloc(ab, &a) == NHIP_OK) {  // without it every request is staged
            q->ring.base = (uint8_t*)a;
            q->ring.cap = ab;
        }
    }
    try {
        // a slot holds at most max_batch requests (each of >= 1 proof): the worker's push_back
        // under its lock never allocates
        for (auto& v : q->in_slot) v.reserve(std::min<size_t>(q->max_batch, 1u << 16) + 1);
        if (const char* e = nhip::ab_env("NHIP_QUEUE_SLOTS"))
            q->slots_used = std::max(1, std::min(nhip_queue::QUEUE_SLOTS, std::atoi(e)));
        q->worker = std::thread([q] { q->run(); });
    } catch (const std::system_error&) {
        if (q->ring.base) nhip_host_free(q->ring.base);
        delete q;
        return NHIP_ERR_HIP;
    } catch (const std::bad_alloc&) {
        if (q->ring.base) nhip_host_free(q->ring.base);
        delete q;
        return NHIP_ERR_OOM;
    }
    *out = q;
    return NHIP_OK;
}

int nhip_queue_verify(nhip_queue* q, const nhip_claim* claims, const nhip_proof* proofs, size_t n,
                      uint8_t* verdicts) {
    if (!q || (n && (!claims || !proofs || !verdicts))) return NHIP_ERR_ARG;
    if (n == 0) return NHIP_OK;
    // argument errors stay this caller's: checked here, before the proofs join a shared batch
    for (size_t i = 0; i < n; ++i)
        if ((proofs[i].len && !proofs[i].words) || (claims[i].input_len && !claims[i].input) ||
            (claims[i].output_len && !claims[i].output) || claims[i].input_len > 0xFFFFFFFFull ||
            claims[i].output_len > 0xFFFFFFFFull)
            return NHIP_ERR_ARG;
    // this caller's proofs into the pinned arena, copied on this thread while the other callers copy
    // theirs: the worker then DMAs them without a staging copy (adjacent requests as one copy)
    uint64_t bytes = 0;
    for (size_t i = 0; i < n; ++i) bytes += proofs[i].len * 8;
    std::vector<nhip_proof> mine;
    uint64_t at = ~0ull;
    {
        std::lock_guard<std::mutex> g(q->mu);
        if (q->stop) return NHIP_ERR_ARG;
        at = q->ring.take(bytes);
    }
    if (at != ~0ull) {
        try {
            mine.resize(n);
        } catch (const std::bad_alloc&) {
            std::lock_guard<std::mutex> g(q->mu);
            q->ring.release(at);
            return NHIP_ERR_OOM;
        }
        uint8_t* dst = q->ring.ptr(at);
        for (size_t i = 0; i < n; ++i) {
            if (proofs[i].len) std::memcpy(dst, proofs[i].words, proofs[i].len * 8);
            mine[i].words = proofs[i].len ? (const uint64_t*)dst : nullptr;
            mine[i].len = proofs[i].len;
            dst += proofs[i].len * 8;
        }
    }
    Req r{claims, at != ~0ull ? mine.data() : proofs, n, verdicts, Clock::now()};
    r.arena_at = at;
    std::unique_lock<std::mutex> lk(q->mu);
    if (q->stop) {
        if (at != ~0ull) q->ring.release(at);
        return NHIP_ERR_ARG;
    }
    try {
        q->pending.push_back(&r);
    } catch (const std::bad_alloc&) {
        if (at != ~0ull) q->ring.release(at);
        return NHIP_ERR_OOM;
    }
    q->pending_proofs += n;
    q->cv_in.notify_one();
    q->cv_out.wait(lk, [&] { return r.done; });
    return r.rc;
}

int nhip_queue_stats(const nhip_queue* q, uint64_t* batches, uint64_t* proofs) {
    if (!q) return NHIP_ERR_ARG;
    if (batches) *batches = q->n_batches.load();
    if (proofs) *proofs = q->n_proofs.load();
    return NHIP_OK;
}

int nhip_queue_profile_read(const nhip_queue* q, nhip_queue_profile* out, int reset) {
    if (!q || !out) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(q->prof_mu);
    *out = q->prof;
    if (reset) const_cast<nhip_queue*>(q)->prof = nhip_queue_profile{};
    return NHIP_OK;
}

int nhip_queue_latencies(const nhip_queue* q, float* us_out, size_t cap, size_t* n, int reset) {
    if (!q || (cap && !us_out)) return NHIP_ERR_ARG;
    auto* m = const_cast<nhip_queue*>(q);
    std::lock_guard<std::mutex> g(m->prof_mu);
    const size_t have = m->lat_us.size();
    if (n) *n = have;
    // oldest first: the ring's next write position is the oldest entry once it has wrapped
    const size_t start = m->lat_n > have ? (size_t)(m->lat_n % have) : 0;
    for (size_t i = 0; i < std::min(cap, have); ++i) us_out[i] = m->lat_us[(start + i) % have];
    if (reset) {
        m->lat_us.clear();
        m->lat_n = 0;
    }
    return NHIP_OK;
}

void nhip_queue_destroy(nhip_queue* q) {
    if (!q) return;
    {
        std::lock_guard<std::mutex> g(q->mu);
        q->stop = true;
    }
    q->cv_in.notify_all();
    q->worker.join();
    for (nhip_batch* b : q->slot)
        if (b) nhip_batch_destroy(b);
    if (q->ring.base) nhip_host_free(q->ring.base);
    delete q;
}

}  // extern "C"
