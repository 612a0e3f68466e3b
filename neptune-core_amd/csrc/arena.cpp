// Per-member proof arenas: wire bytes decoded straight into pinned memory on each GPU's NUMA node
// (the receive side of the feed path).
//
// A node receives proofs as bytes: blk files of the bootstrap import
// (state/archival_state/import_blocks_from_files.rs:100-115, then state/mod.rs:2226-2272) and peer
// messages (protocol/peer/transfer_transaction.rs:31-47, peer_loop.rs:315-323).  The reference
// deserializes each proof into a Vec<BFieldElement> and hands it to triton_vm::verify one at a time
// (verifier.rs:60-63).  Here one arena set per group holds, for every member GPU, pinned host memory
// on that GPU's NUMA node (nhip_host_alloc_near); the ingest functions scan the bincode bytes, give
// each proof to the least-loaded member with room (list scheduling by words, the streaming form of
// nhip_group_shard's LPT) and decode its words - 8-byte little-endian, BFieldElement::new - into that
// member's arena with streaming stores, on copy threads bound to that member's node.  The proofs are
// then submitted with nhip_group_stream_submit_placed: each member's share is already adjacent in
// its pinned arena, so it is DMA'd as it lies (one host pass over the proof bytes between the receive
// buffer and the GPU; the pageable path's staging copy is this same pass, done by the library).
#include <algorithm>
#include <atomic>
#include <memory>
#include <cstring>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/neptune_hip.h"
#include "group.hpp"
#include "host_copy.hpp"
#include "host_numa.hpp"

extern "C" unsigned nhip_internal_host_threads(nhip_ctx* c);

namespace nhip {

unsigned member_copy_threads(const nhip_group* g, size_t member) {
    if (const unsigned e = host_threads_env()) return std::min(e, 256u);
    if (member < g->members.size())
        if (const unsigned set = nhip_internal_host_threads(g->members[member])) return set;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    return std::max(1u, std::min(16u, hw / (unsigned)std::max<size_t>(1, g->members.size())));
}

}  // namespace nhip

struct nhip_arena {
    nhip_group* g = nullptr;
    struct Part {
        uint64_t* base = nullptr;
        uint64_t cap = 0;   // words
        uint64_t used = 0;  // words placed since the last reset
    };
    std::vector<Part> parts;
};

namespace {

struct Job {
    const uint8_t* src;
    uint64_t* dst;
    uint64_t words;
};

// the least-loaded member with room for `words` (ties: the lowest index); -1 when none has room
int place(const nhip_arena* a, uint64_t words) {
    int best = -1;
    for (size_t m = 0; m < a->parts.size(); ++m) {
        const auto& p = a->parts[m];
        if (p.cap - p.used < words) continue;
        if (best < 0 || p.used < a->parts[(size_t)best].used) best = (int)m;
    }
    return best;
}

// Decode every job, the jobs of member m on member_copy_threads(m) threads bound to m's CPUs, all
// members at once.  Jobs are cut into 1 MB pieces so the threads of a member share its work evenly.
int copy_all(const nhip_arena* a, const std::vector<std::vector<Job>>& per_member) {
    constexpr uint64_t PIECE = 1ull << 17;  // words
    const size_t M = per_member.size();
    std::vector<std::vector<Job>> pieces(M);
    for (size_t m = 0; m < M; ++m)
        for (const Job& j : per_member[m])
            for (uint64_t o = 0; o < j.words; o += PIECE)
                pieces[m].push_back(Job{j.src + 8 * o, j.dst + o, std::min(PIECE, j.words - o)});
    std::unique_ptr<std::atomic<size_t>[]> next(new std::atomic<size_t>[M]);
    for (size_t m = 0; m < M; ++m) next[m].store(0);
    auto work = [&](size_t m) {
        for (size_t q; (q = next[m].fetch_add(1)) < pieces[m].size();) {
            const Job& j = pieces[m][q];
            nhip::copy_le_words_nt(j.dst, j.src, j.words);
        }
        _mm_sfence();  // the streaming stores are visible before the DMA reads the arena
    };
    std::vector<std::thread> th;
    std::vector<size_t> inline_m;
    for (size_t m = 0; m < M; ++m) {
        if (pieces[m].empty()) continue;
        const unsigned t = std::min<unsigned>(nhip::member_copy_threads(a->g, m), (unsigned)pieces[m].size());
        for (unsigned k = 0; k < t; ++k) {
            try {
                th.emplace_back([&, m] {
                    (void)nhip::bind_thread(a->g->cpus.size() > m ? a->g->cpus[m] : std::vector<int>{});
                    work(m);
                });
            } catch (const std::system_error&) {
                inline_m.push_back(m);  // fewer threads: the calling thread takes the rest below
                break;
            }
        }
    }
    for (size_t m : inline_m) work(m);
    for (auto& t : th) t.join();
    return NHIP_OK;
}

// Place proofs given as (byte offset, words) spans of `bytes`; false when a member's arena cannot
// take one (nothing of that proof is placed; the ones before it are).
bool place_spans(nhip_arena* a, const uint8_t* bytes, const uint64_t* spans, size_t n, nhip_proof* proofs,
                 uint32_t* member_of, std::vector<std::vector<Job>>& jobs, size_t& placed) {
    for (size_t i = 0; i < n; ++i) {
        const uint64_t off = spans[2 * i], w = spans[2 * i + 1];
        const int m = place(a, w);
        if (m < 0) return false;
        auto& p = a->parts[(size_t)m];
        uint64_t* dst = p.base + p.used;
        p.used += w;
        jobs[(size_t)m].push_back(Job{bytes + off, dst, w});
        proofs[placed] = nhip_proof{dst, (size_t)w};
        if (member_of) member_of[placed] = (uint32_t)m;
        ++placed;
    }
    return true;
}

}  // namespace

namespace nhip {
// bincode.cpp: the proof spans (byte offset from `bytes`, words) of the TransferTransaction at the
// start of bytes[0, n), appended to `spans`, and its size; false when malformed
bool tx_proof_spans(const uint8_t* bytes, size_t n, std::vector<uint64_t>& spans, uint64_t& size);
}  // namespace nhip

extern "C" {

int nhip_arena_create(nhip_group* g, size_t bytes_per_member, nhip_arena** out) {
    if (!g || g->members.empty() || !out || bytes_per_member < 8) return NHIP_ERR_ARG;
    *out = nullptr;
    nhip_arena* a = new (std::nothrow) nhip_arena();
    if (!a) return NHIP_ERR_OOM;
    try {
        a->g = g;
        a->parts.resize(g->members.size());
    } catch (const std::bad_alloc&) {
        delete a;
        return NHIP_ERR_OOM;
    }
    for (size_t m = 0; m < g->members.size(); ++m) {
        void* p = nullptr;
        const int rc = nhip_host_alloc_near(g->members[m], bytes_per_member, &p);
        if (rc) {
            nhip_arena_destroy(a);
            return rc;
        }
        a->parts[m].base = (uint64_t*)p;
        a->parts[m].cap = bytes_per_member / 8;
    }
    *out = a;
    return NHIP_OK;
}

void nhip_arena_destroy(nhip_arena* a) {
    if (!a) return;
    for (auto& p : a->parts)
        if (p.base) (void)nhip_host_free(p.base);
    delete a;
}

int nhip_arena_reset(nhip_arena* a) {
    if (!a) return NHIP_ERR_ARG;
    for (auto& p : a->parts) p.used = 0;
    return NHIP_OK;
}

int nhip_arena_member_info(const nhip_arena* a, size_t member, uint64_t* used_words, uint64_t* cap_words,
                           int* page_node) {
    if (!a || member >= a->parts.size()) return NHIP_ERR_ARG;
    const auto& p = a->parts[member];
    if (used_words) *used_words = p.used;
    if (cap_words) *cap_words = p.cap;
    if (page_node) *page_node = nhip_host_page_node(p.base);
    return NHIP_OK;
}

int nhip_arena_ingest_spans(nhip_arena* a, const uint8_t* bytes, size_t n_bytes, const uint64_t* spans, size_t n,
                            nhip_proof* proofs, uint32_t* member_of) {
    if (!a || (n && (!bytes || !spans || !proofs))) return NHIP_ERR_ARG;
    for (size_t i = 0; i < n; ++i)
        if (spans[2 * i] > n_bytes || spans[2 * i + 1] > (n_bytes - spans[2 * i]) / 8) return NHIP_ERR_ARG;
    try {
        std::vector<std::vector<Job>> jobs(a->parts.size());
        size_t placed = 0;
        const bool all = place_spans(a, bytes, spans, n, proofs, member_of, jobs, placed);
        const int rc = copy_all(a, jobs);
        if (rc) return rc;
        return all ? NHIP_OK : NHIP_ERR_OOM;
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
}

int nhip_arena_ingest_txs(nhip_arena* a, const uint8_t* bytes, size_t n_bytes, size_t max_txs, nhip_proof* proofs,
                          uint32_t* member_of, size_t proof_cap, size_t* n_txs, size_t* n_proofs, size_t* consumed) {
    if (n_txs) *n_txs = 0;
    if (n_proofs) *n_proofs = 0;
    if (consumed) *consumed = 0;
    if (!a || (n_bytes && !bytes) || (proof_cap && !proofs)) return NHIP_ERR_ARG;
    try {
        std::vector<std::vector<Job>> jobs(a->parts.size());
        std::vector<uint64_t> spans;
        size_t pos = 0, txs = 0, placed = 0;
        int rc = NHIP_OK;
        while (pos < n_bytes && txs < max_txs) {
            spans.clear();
            uint64_t size = 0;
            if (!nhip::tx_proof_spans(bytes + pos, n_bytes - pos, spans, size)) {
                rc = NHIP_ERR_DECODE;  // the transactions before it stay placed and decoded
                break;
            }
            const size_t np = spans.size() / 2;
            if (placed + np > proof_cap) break;  // the caller's proof array is full: stop before this tx
            uint64_t need = 0;
            for (size_t i = 0; i < np; ++i) {
                spans[2 * i] += pos;
                need += spans[2 * i + 1];
            }
            // every proof of the tx must fit somewhere (checked before any is placed): total room
            uint64_t room = 0;
            for (const auto& p : a->parts) room += p.cap - p.used;
            if (need > room) break;
            const auto saved = a->parts;
            const size_t saved_placed = placed;
            std::vector<size_t> njobs(jobs.size());
            for (size_t m = 0; m < jobs.size(); ++m) njobs[m] = jobs[m].size();
            if (!place_spans(a, bytes, spans.data(), np, proofs, member_of, jobs, placed)) {
                // fragmented: undo this tx and stop before it
                a->parts = saved;
                placed = saved_placed;
                for (size_t m = 0; m < jobs.size(); ++m) jobs[m].resize(njobs[m]);
                break;
            }
            pos += size;
            ++txs;
        }
        const int crc = copy_all(a, jobs);
        if (n_txs) *n_txs = txs;
        if (n_proofs) *n_proofs = placed;
        if (consumed) *consumed = pos;
        return crc ? crc : rc;
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
}

int nhip_arena_ingest_blocks(nhip_arena* a, const uint8_t* bytes, size_t n_bytes, uint32_t pow_tree_height,
                             nhip_proof* proofs, uint32_t* member_of, uint64_t* block_of, size_t proof_cap,
                             size_t* n_proofs, size_t* n_blocks) {
    if (n_proofs) *n_proofs = 0;
    if (n_blocks) *n_blocks = 0;
    if (!a || (n_bytes && !bytes) || (proof_cap && !proofs)) return NHIP_ERR_ARG;
    try {
        size_t nb = 0;
        int rc = nhip_blk_scan(bytes, n_bytes, pow_tree_height, nullptr, 0, &nb);
        if (rc) {
            if (n_blocks) *n_blocks = nb;
            return rc;  // a malformed block fails the whole file (import_blocks_from_files.rs:100-115)
        }
        std::vector<nhip_blk_block> blocks(std::max<size_t>(nb, 1));
        rc = nhip_blk_scan(bytes, n_bytes, pow_tree_height, blocks.data(), nb, &nb);
        if (rc) return rc;
        std::vector<uint64_t> spans;
        std::vector<uint64_t> which;
        for (size_t b = 0; b < nb; ++b)
            if (blocks[b].proof_kind == NHIP_BLOCK_PROOF_SINGLE) {
                spans.push_back(blocks[b].proof_offset);
                spans.push_back(blocks[b].proof_len);
                which.push_back(b);
            }
        if (which.size() > proof_cap) return NHIP_ERR_ARG;
        std::vector<std::vector<Job>> jobs(a->parts.size());
        size_t placed = 0;
        const bool all = place_spans(a, bytes, spans.data(), which.size(), proofs, member_of, jobs, placed);
        rc = copy_all(a, jobs);
        if (block_of)
            for (size_t i = 0; i < placed; ++i) block_of[i] = which[i];
        if (n_proofs) *n_proofs = placed;
        if (n_blocks) *n_blocks = nb;
        if (rc) return rc;
        return all ? NHIP_OK : NHIP_ERR_OOM;
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
}

}  // extern "C"
