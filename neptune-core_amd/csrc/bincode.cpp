// Block files and peer transactions: bincode decoding straight into the
// verifier's inputs.
//
//  * Block files: `blocks_from_file_without_record`
//    (neptune-core/src/state/archival_state/import_blocks_from_files.rs:100-115) deserializes
//    `Block`s back to back with bincode 1.x legacy options (fixed little-endian integers, u64
//    sequence lengths, u32 enum variants, u8 Option tags and bools, trailing bytes allowed) and
//    advances by each block's serialized size.  nhip_blk_scan walks a whole buffer (an mmap'd
//    blk file) once and reports, per block, what `Block::validate` rules 1.a-1.d and the
//    BlockProgram claim need: the proof's word span, the appendix claims and the BFieldCodec MAST
//    sequences of the transaction kernel and the body.
//  * Peer transactions: `TransferTransaction { kernel, proof }` (protocol/peer/
//    transfer_transaction.rs:31-47) with `TransferTransactionProof::{ProofCollection(Box<..>),
//    SingleProof(Proof)}`; nhip_tx_scan / nhip_tx_parts give the member proofs' word spans in
//    ProofCollection field order, its digests and the kernel's MAST sequences.
//
// Field lists (serde declaration order): block/mod.rs:114-119,175-187; block_kernel.rs:26-31;
// block_header.rs:39-57 with BlockPow = Pow<POW_MEMORY_TREE_HEIGHT> (pow.rs:33-37,187-199);
// block_body.rs:69-99; block_appendix.rs:31-33; transaction_kernel.rs:30-50;
// removal_record.rs:40-43; absolute_index_set.rs:32-39; chunk_dictionary.rs:27-33; chunk.rs:40-42;
// addition_record.rs:26-28; announcement.rs:34-36; mutator_set_accumulator.rs:32-36;
// active_window.rs:18-21; native_currency_amount.rs:50 (i128); difficulty_control.rs:43,238;
// guesser_receiver_data.rs:15-18; proof_collection.rs:36-49; neptune_proof.rs:42-44,193.
// crates.io types ([EXT], not vendored, unpinned): BFieldElement = its canonical u64 (reduced mod p
// on the way in, as BFieldElement::new), Digest = 5 of them, Claim = {program_digest, version: u32,
// input, output}, Proof = Vec<BFieldElement>, MmrAccumulator = {leaf_count: u64, peaks: Vec<Digest>},
// MmrMembershipProof = {authentication_path: Vec<Digest>}.
//
// BFieldCodec (the MAST sequences; transaction_kernel.rs:246-277, block_body.rs:175-182): struct
// fields last-first (pow.rs:196-197), dynamically sized fields length-prefixed, Vec = [len] + items
// (each prefixed when dynamic), tuples in order with the same rule, Option = [0] | [1] + value,
// u64 / u128 as u32 limbs low first [EXT, unpinned].  The test restatement is
// oracle/bincode_ref.py.
//
// Everything is host code: parsing is byte-serial and a few hundred MB/s per thread is far above
// what a verifier batch consumes.
#include <cstring>
#include <new>
#include <vector>

#include "../../include/neptune_hip.h"

namespace {
constexpr uint64_t P = 0xFFFFFFFF00000001ull;
constexpr uint32_t NUM_TRIALS = 45;  // util_types/mutator_set/shared.rs:15

struct Rd {
    const uint8_t* b;
    size_t n, o;
    bool ok = true;
    bool need(size_t k) {
        if (!ok || k > n - o) {
            ok = false;
            return false;
        }
        return true;
    }
    uint64_t le(int k) {
        if (!need((size_t)k)) return 0;
        uint64_t v = 0;
        for (int i = k - 1; i >= 0; --i) v = (v << 8) | b[o + i];
        o += (size_t)k;
        return v;
    }
    uint8_t u8() { return (uint8_t)le(1); }
    uint32_t u32() { return (uint32_t)le(4); }
    uint64_t u64() { return le(8); }
    uint64_t bfe() {
        const uint64_t v = u64();
        return v >= P ? v - P : v;
    }
    void u128(uint64_t& lo, uint64_t& hi) {
        lo = u64();
        hi = u64();
    }
    bool boolean() {
        const uint8_t v = u8();
        if (v > 1) ok = false;
        return v == 1;
    }
    // sequence length: every element takes at least `min_elem` bytes, so a length the rest of the
    // input cannot hold is rejected before anything is allocated or walked
    uint64_t len(size_t min_elem) {
        const uint64_t v = u64();
        if (ok && min_elem && v > (n - o) / min_elem) ok = false;
        return ok ? v : 0;
    }
    uint32_t variant(uint32_t count) {
        const uint32_t v = u32();
        if (v >= count) ok = false;
        return v;
    }
    void skip(size_t k) {
        if (need(k)) o += k;
    }
    void digest(uint64_t d[5]) {
        for (int i = 0; i < 5; ++i) d[i] = bfe();
    }
};

// BFieldCodec emitter; `mark` / `close` make a length prefix
struct Em {
    std::vector<uint64_t> w;
    size_t mark() {
        w.push_back(0);
        return w.size();
    }
    void close(size_t m) { w[m - 1] = w.size() - m; }
    void put(uint64_t v) { w.push_back(v); }
    void u64(uint64_t v) {
        w.push_back(v & 0xFFFFFFFFull);
        w.push_back(v >> 32);
    }
    void u128(uint64_t lo, uint64_t hi) {
        u64(lo);
        u64(hi);
    }
};

// ---- serde walkers; each also emits the field's BFieldCodec encoding when `e` is non-null
void vec_digests(Rd& r, Em* e) {  // Vec<Digest> (static items): [len] + digests
    const uint64_t n = r.len(40);
    if (e) e->put(n);
    for (uint64_t i = 0; i < n && r.ok; ++i)
        for (int q = 0; q < 5; ++q) {
            const uint64_t v = r.bfe();
            if (e) e->put(v);
        }
}

void vec_u32(Rd& r, Em* e) {
    const uint64_t n = r.len(4);
    if (e) e->put(n);
    for (uint64_t i = 0; i < n && r.ok; ++i) {
        const uint32_t v = r.u32();
        if (e) e->put(v);
    }
}

void vec_bfe(Rd& r, Em* e) {
    const uint64_t n = r.len(8);
    if (e) e->put(n);
    for (uint64_t i = 0; i < n && r.ok; ++i) {
        const uint64_t v = r.bfe();
        if (e) e->put(v);
    }
}

// MmrAccumulator {leaf_count, peaks}: BFieldCodec peaks (dynamic, prefixed) then leaf_count
void mmr_accumulator(Rd& r, Em* e) {
    const uint64_t leaf_count = r.u64();
    size_t m = e ? e->mark() : 0;
    vec_digests(r, e);
    if (e) {
        e->close(m);
        e->u64(leaf_count);
    }
}

// RemovalRecord {absolute_indices: {minimum: u128, distances: [u32; 45]}, target_chunks}
void removal_record(Rd& r, Em* e) {
    uint64_t lo, hi;
    r.u128(lo, hi);
    uint32_t dist[NUM_TRIALS];
    for (uint32_t i = 0; i < NUM_TRIALS; ++i) dist[i] = r.u32();
    // target_chunks (dynamic) first: [len(ChunkDictionary)] + [len(dictionary)] + Vec of tuples
    const size_t m_cd = e ? e->mark() : 0;
    const size_t m_dict = e ? e->mark() : 0;
    const uint64_t n = r.len(8 + 8 + 8);
    if (e) e->put(n);
    for (uint64_t i = 0; i < n && r.ok; ++i) {
        const size_t m_item = e ? e->mark() : 0;  // dynamic tuple item
        const uint64_t idx = r.u64();
        if (e) e->u64(idx);
        const size_t m_pair = e ? e->mark() : 0;   // (MmrMembershipProof, Chunk), dynamic
        const size_t m_mmp = e ? e->mark() : 0;    // MmrMembershipProof in the tuple
        const size_t m_path = e ? e->mark() : 0;   // its authentication_path field
        vec_digests(r, e);
        if (e) {
            e->close(m_path);
            e->close(m_mmp);
        }
        const size_t m_chunk = e ? e->mark() : 0;  // Chunk in the tuple
        const size_t m_rel = e ? e->mark() : 0;    // its relative_indices field
        vec_u32(r, e);
        if (e) {
            e->close(m_rel);
            e->close(m_chunk);
            e->close(m_pair);
            e->close(m_item);
        }
    }
    if (e) {
        e->close(m_dict);
        e->close(m_cd);
        for (uint32_t i = 0; i < NUM_TRIALS; ++i) e->put(dist[i]);  // absolute_indices, static
        e->u128(lo, hi);
    }
}

// TransactionKernel: emits its 8 MAST sequences, `ends[i]` = end of sequence i in e->w
void tx_kernel(Rd& r, Em* e, size_t ends[8]) {
    auto end = [&](int i) {
        if (e) ends[i] = e->w.size();
    };
    uint64_t n = r.len(16 + 4 * NUM_TRIALS + 8);  // inputs: Vec<RemovalRecord> (dynamic items)
    if (e) e->put(n);
    for (uint64_t i = 0; i < n && r.ok; ++i) {
        const size_t m = e ? e->mark() : 0;
        removal_record(r, e);
        if (e) e->close(m);
    }
    end(0);
    vec_digests(r, e);  // outputs: Vec<AdditionRecord{canonical_commitment}>
    end(1);
    n = r.len(8);  // announcements: Vec<Announcement{message}>
    if (e) e->put(n);
    for (uint64_t i = 0; i < n && r.ok; ++i) {
        const size_t m_item = e ? e->mark() : 0;
        const size_t m_msg = e ? e->mark() : 0;
        vec_bfe(r, e);
        if (e) {
            e->close(m_msg);
            e->close(m_item);
        }
    }
    end(2);
    uint64_t lo, hi;
    r.u128(lo, hi);  // fee: NativeCurrencyAmount(i128)
    if (e) e->u128(lo, hi);
    end(3);
    const uint8_t tag = r.u8();  // coinbase: Option<NativeCurrencyAmount>
    if (tag > 1) r.ok = false;
    if (e) e->put(tag);
    if (tag == 1) {
        r.u128(lo, hi);
        if (e) e->u128(lo, hi);
    }
    end(4);
    const uint64_t ts = r.bfe();  // timestamp
    if (e) e->put(ts);
    end(5);
    uint64_t d[5];
    r.digest(d);  // mutator_set_hash
    if (e)
        for (int q = 0; q < 5; ++q) e->put(d[q]);
    end(6);
    const bool mb = r.boolean();  // merge_bit
    if (e) e->put(mb ? 1 : 0);
    end(7);
}

void claim_skip(Rd& r) {
    r.skip(40 + 4);
    r.skip(8 * r.len(8));
    r.skip(8 * r.len(8));
}

// Walk one block at r.o.  With `e`, emit the kernel's 8 and the body's 3 tail sequences.
bool parse_block(Rd& r, uint32_t tree_height, nhip_blk_block& b, Em* e, size_t ends[11]) {
    std::memset(&b, 0, sizeof(b));
    b.offset = r.o;
    r.bfe();  // version
    b.height = r.bfe();
    r.digest(b.prev_block_digest);
    b.timestamp = r.bfe();
    // pow: root, path_a, path_b, nonce; cumulative_proof_of_work [u32; 6]; difficulty [u32; 5];
    // guesser_receiver_data: 2 digests
    r.skip(40ull * (2ull * tree_height + 2) + 4 * 6 + 4 * 5 + 80);
    b.kernel_offset = r.o;
    size_t k_ends[8] = {};
    tx_kernel(r, e, k_ends);
    if (e)
        for (int i = 0; i < 8; ++i) ends[i] = k_ends[i];
    // body: mutator_set_accumulator {aocl, swbf_inactive, swbf_active{sbf: Vec<u32>}} -- BFieldCodec
    // fields last-first, so the three parts are emitted into scratch and concatenated reversed
    {
        Em parts[3];
        mmr_accumulator(r, e ? &parts[0] : nullptr);
        mmr_accumulator(r, e ? &parts[1] : nullptr);
        {
            Em* pe = e ? &parts[2] : nullptr;
            const size_t m = pe ? pe->mark() : 0;
            vec_u32(r, pe);
            if (pe) pe->close(m);
        }
        if (e) {
            for (int i = 2; i >= 0; --i) {
                e->put(parts[i].w.size());
                e->w.insert(e->w.end(), parts[i].w.begin(), parts[i].w.end());
            }
            ends[8] = e->w.size();
        }
    }
    mmr_accumulator(r, e);  // lock_free_mmr_accumulator
    if (e) ends[9] = e->w.size();
    mmr_accumulator(r, e);  // block_mmr_accumulator
    if (e) ends[10] = e->w.size();
    // appendix
    b.appendix_offset = r.o;
    const uint64_t nc = r.len(40 + 4 + 16);
    uint64_t claim_words = 0;
    for (uint64_t i = 0; i < nc && r.ok; ++i) {
        const size_t o0 = r.o;
        claim_skip(r);
        claim_words += (r.o - o0 - 44 - 16) / 8;
    }
    b.n_claims = (uint32_t)nc;
    b.claim_words = claim_words;
    if (nc > 0xFFFFFFFFull) r.ok = false;
    // proof
    b.proof_kind = r.variant(3);
    if (r.ok && b.proof_kind == NHIP_BLOCK_PROOF_SINGLE) {
        b.proof_len = r.len(8);
        b.proof_offset = r.o;
        r.skip(8 * b.proof_len);
    }
    b.size = r.o - b.offset;
    return r.ok;
}

uint64_t rd_word(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);  // little-endian host (x86-64 / the MI355X hosts)
    return v >= P ? v - P : v;
}
}  // namespace

extern "C" {

int nhip_blk_scan(const uint8_t* bytes, size_t n_bytes, uint32_t pow_tree_height, nhip_blk_block* blocks,
                  size_t cap, size_t* n_blocks) {
    if (!n_blocks || (n_bytes && !bytes) || pow_tree_height > 64) return NHIP_ERR_ARG;
    *n_blocks = 0;
    try {
        Rd r{bytes, n_bytes, 0};
        Em e;
        size_t ends[11];
        size_t count = 0;
        while (r.o < n_bytes) {
            nhip_blk_block b;
            e.w.clear();
            if (!parse_block(r, pow_tree_height, b, blocks ? &e : nullptr, ends)) {
                *n_blocks = count;  // blocks before the malformed one
                return NHIP_ERR_DECODE;
            }
            b.seq_words = blocks ? e.w.size() : 0;
            if (blocks) {
                if (count >= cap) return NHIP_ERR_ARG;
                blocks[count] = b;
            }
            ++count;
        }
        *n_blocks = count;
        return NHIP_OK;
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
}

int nhip_blk_sequences(const uint8_t* bytes, size_t n_bytes, uint32_t pow_tree_height, const nhip_blk_block* block,
                       uint64_t* words, size_t cap, uint64_t offsets[12]) {
    if (!bytes || !block || !offsets || block->offset > n_bytes || pow_tree_height > 64) return NHIP_ERR_ARG;
    try {
        Rd r{bytes, n_bytes, (size_t)block->offset};
        Em e;
        size_t ends[11];
        nhip_blk_block b;
        if (!parse_block(r, pow_tree_height, b, &e, ends)) return NHIP_ERR_DECODE;
        offsets[0] = 0;
        for (int i = 0; i < 11; ++i) offsets[i + 1] = ends[i];
        if (!words) return NHIP_OK;  // size query: offsets[11]
        if (cap < e.w.size()) return NHIP_ERR_ARG;
        std::memcpy(words, e.w.data(), e.w.size() * 8);
        return NHIP_OK;
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
}

int nhip_blk_claims(const uint8_t* bytes, size_t n_bytes, const nhip_blk_block* block, uint64_t* words,
                    nhip_claim* claims) {
    if (!bytes || !block || block->appendix_offset > n_bytes || (block->claim_words && !words) ||
        (block->n_claims && !claims))
        return NHIP_ERR_ARG;
    Rd r{bytes, n_bytes, (size_t)block->appendix_offset};
    const uint64_t nc = r.len(40 + 4 + 16);
    if (!r.ok || nc != block->n_claims) return NHIP_ERR_DECODE;
    uint64_t used = 0;
    for (uint64_t i = 0; i < nc; ++i) {
        nhip_claim& c = claims[i];
        r.digest(c.program_digest);
        c.version = r.u32();
        for (int side = 0; side < 2; ++side) {
            const uint64_t n = r.len(8);
            if (!r.ok || used + n > block->claim_words) return NHIP_ERR_DECODE;
            uint64_t* dst = words + used;
            for (uint64_t k = 0; k < n; ++k) dst[k] = r.bfe();
            (side == 0 ? c.input : c.output) = dst;
            (side == 0 ? c.input_len : c.output_len) = (size_t)n;
            used += n;
        }
        if (!r.ok) return NHIP_ERR_DECODE;
    }
    return NHIP_OK;
}

int nhip_le_words(const uint8_t* bytes, size_t n_bytes, uint64_t offset, size_t n, uint64_t* out) {
    if ((n && (!bytes || !out)) || offset > n_bytes || n > (n_bytes - offset) / 8) return NHIP_ERR_ARG;
    for (size_t i = 0; i < n; ++i) out[i] = rd_word(bytes + offset + 8 * i);
    return NHIP_OK;
}

// ---- TransferTransaction
static bool parse_tx(Rd& r, nhip_tx* t, Em* e, size_t ends[8], uint64_t* spans, uint64_t* digests) {
    std::memset(t, 0, sizeof(*t));
    tx_kernel(r, e, ends);
    t->kind = r.variant(2);
    if (!r.ok) return false;
    if (t->kind == NHIP_TX_SINGLE_PROOF) {
        const uint64_t n = r.len(8);
        if (spans) {
            spans[0] = r.o;
            spans[1] = n;
        }
        r.skip(8 * n);
        t->n_proofs = 1;
    } else {
        // removal_records_integrity, collect_lock_scripts, lock_scripts_halt, kernel_to_outputs,
        // collect_type_scripts, type_scripts_halt (proof_collection.rs:36-49 field order)
        uint32_t np = 0;
        auto proof = [&]() {
            const uint64_t n = r.len(8);
            if (spans) {
                spans[2 * np] = r.o;
                spans[2 * np + 1] = n;
            }
            r.skip(8 * n);
            ++np;
        };
        proof();
        proof();
        uint64_t nl = r.len(8);
        for (uint64_t i = 0; i < nl && r.ok; ++i) proof();
        proof();
        proof();
        uint64_t nt = r.len(8);
        for (uint64_t i = 0; i < nt && r.ok; ++i) proof();
        t->n_lock_scripts = (uint32_t)nl;
        t->n_type_scripts = (uint32_t)nt;
        t->n_proofs = np;
        uint64_t nd = 0;
        auto digs = [&](uint64_t cnt) {
            for (uint64_t i = 0; i < cnt && r.ok; ++i) {
                uint64_t d[5];
                r.digest(d);
                if (digests) std::memcpy(digests + 5 * nd, d, 40);
                ++nd;
            }
        };
        t->n_lock_hashes = (uint32_t)r.len(40);
        digs(t->n_lock_hashes);
        t->n_type_hashes = (uint32_t)r.len(40);
        digs(t->n_type_hashes);
        digs(3);  // kernel_mast_hash, salted_inputs_hash, salted_outputs_hash
        t->n_merge_path = (uint32_t)r.len(40);
        digs(t->n_merge_path);
        t->n_digests = nd;
    }
    t->size = r.o;
    if (e) t->seq_words = e->w.size();
    return r.ok;
}

int nhip_tx_scan(const uint8_t* bytes, size_t n_bytes, nhip_tx* tx) {
    if (!tx || (n_bytes && !bytes)) return NHIP_ERR_ARG;
    try {
        Rd r{bytes, n_bytes, 0};
        Em e;
        size_t ends[8];
        return parse_tx(r, tx, &e, ends, nullptr, nullptr) ? NHIP_OK : NHIP_ERR_DECODE;
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
}

int nhip_tx_parts(const uint8_t* bytes, size_t n_bytes, const nhip_tx* tx, uint64_t* seq_words,
                  uint64_t seq_offsets[9], uint64_t* proof_spans, uint64_t* digests) {
    if (!tx || !bytes || !seq_words || !seq_offsets || !proof_spans || (tx->n_digests && !digests))
        return NHIP_ERR_ARG;
    try {
        Rd r{bytes, n_bytes, 0};
        Em e;
        size_t ends[8];
        nhip_tx t;
        // the caller's buffers are sized from tx (a scan of the same bytes); re-check before copying
        std::vector<uint64_t> spans(2ull * tx->n_proofs + 2), dig(5ull * tx->n_digests + 5);
        Rd probe{bytes, n_bytes, 0};
        if (!parse_tx(probe, &t, nullptr, ends, nullptr, nullptr)) return NHIP_ERR_DECODE;
        if (t.n_proofs != tx->n_proofs || t.n_digests != tx->n_digests) return NHIP_ERR_ARG;
        if (!parse_tx(r, &t, &e, ends, spans.data(), dig.data())) return NHIP_ERR_DECODE;
        if (t.seq_words != tx->seq_words) return NHIP_ERR_ARG;
        seq_offsets[0] = 0;
        for (int i = 0; i < 8; ++i) seq_offsets[i + 1] = ends[i];
        std::memcpy(seq_words, e.w.data(), e.w.size() * 8);
        std::memcpy(proof_spans, spans.data(), 16ull * t.n_proofs);
        if (t.n_digests) std::memcpy(digests, dig.data(), 40ull * t.n_digests);
        return NHIP_OK;
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
}

}  // extern "C"

namespace nhip {
// The proof spans of the TransferTransaction at the start of bytes[0, n) (arena.cpp): (byte offset
// from `bytes`, words) per proof in ProofCollection field order, appended to `spans`, and its size.
bool tx_proof_spans(const uint8_t* bytes, size_t n, std::vector<uint64_t>& spans, uint64_t& size) {
    size_t ends[8];
    nhip_tx t;
    Rd probe{bytes, n, 0};
    if (!parse_tx(probe, &t, nullptr, ends, nullptr, nullptr)) return false;  // sizes first
    const size_t base = spans.size();
    spans.resize(base + 2ull * t.n_proofs);
    Rd r{bytes, n, 0};
    if (!parse_tx(r, &t, nullptr, ends, spans.data() + base, nullptr)) return false;
    size = t.size;
    return true;
}
}  // namespace nhip
