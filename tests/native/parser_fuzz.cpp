// ASan / UBSan harness for the host code that parses untrusted bytes ("host
// ASan/UBSan"): the proof-stream walk (neptune-core_amd/csrc/proof_codec.hpp, the same code
// k_decode runs on the device and nhip_proof_decodes on the host), the bincode block-file and
// TransferTransaction decoders (csrc/bincode.cpp; import_blocks_from_files.rs:100-115,
// transfer_transaction.rs:31-47) and the proof-file reader (csrc/ingest.cpp; program.rs:374-390).
// Built by tests/native/Makefile with -fsanitize=address,undefined (host only, no GPU) and driven
// by tests/test_sanitizers.py: each input file is parsed as given, at many truncations, and after
// thousands of seeded mutations (byte flips, 8-byte words replaced by boundary values).  Any
// sanitizer report aborts the process (-fno-sanitize-recover).
//
// usage: parser_fuzz <mutations per input> {proof-tiny|proof-full|blk10|tx|be}:<path> ...
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/neptune_hip.h"
#include "../../neptune-core_amd/csrc/host_copy.hpp"
#include "../../neptune-core_amd/csrc/proof_codec.hpp"

namespace nhip {
bool tx_proof_spans(const uint8_t* bytes, size_t n, std::vector<uint64_t>& spans, uint64_t& size);
}
using namespace nhip;

// ingest.cpp's nhip_claim_hash calls the GPU hash; the parsers under test never reach it
extern "C" int nhip_tip5_hash_varlen(nhip_ctx*, const uint64_t*, const uint64_t*, size_t, uint64_t*) {
    return NHIP_ERR_NO_DEVICE;
}

namespace {

uint64_t g_state = 0x5EEDF00Dull;
uint64_t next_u64() {
    g_state += 0x9E3779B97F4A7C15ull;
    uint64_t z = g_state;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

const uint64_t INTERESTING[] = {0, 1, 2, 3, 5, 7, 8, 11, 12, 80, 255, 256, 0xFFFF, 0x7FFFFFFF, 0xFFFFFFFF,
                                0x100000000ull, GL_P - 1, GL_P, GL_P + 1, 0x7FFFFFFFFFFFFFFFull, ~0ull};

Dims dims_of(uint32_t checks, uint32_t main, uint32_t aux) {
    Dims D{};
    D.d.num_main = main;
    D.d.num_aux = aux;
    D.d.num_quot_seg = 4;
    D.d.num_checks = checks;
    D.d.num_deep = 3;
    D.d.log2_expansion = 2;
    D.d.num_trace_randomizers = checks + 6;
    D.d.num_sampled = 59;
    D.d.num_constraints = 505;
    D.expansion = 4;
    return D;
}

uint64_t g_ok = 0, g_runs = 0, g_mismatch = 0;

// the walk reads exactly words[0, n): parse from a heap copy of that size so ASan sees any overrun.
// Both input forms (canonical values, Montgomery words): the same bytes, different structural values.
template <bool MW>
void run_proof_form(const uint64_t* words, size_t n, const Dims& D) {
    ProofDesc pd;
    FsOp ops[fs_ops_for(MAX_FRI_ROUNDS)];
    uint64_t perms, plcw;
    const ClaimLoc cl{0, 3, 1};
    const uint32_t f = decode_stream<MW>(words, 0, n, cl, D, pd, ops, perms, plcw);
    if (!f) {
        const int64_t deg = last_poly_degree_host(words, pd);
        last_poly_finish(pd, deg, D);
        ++g_ok;
    }
    uint64_t lph;
    (void)header_log2_ph<MW>(words, n, lph);
}

void run_proof(const std::vector<uint8_t>& bytes, const Dims& D) {
    const size_t n = bytes.size() / 8;
    std::vector<uint64_t> w(n);
    if (n) std::memcpy(w.data(), bytes.data(), n * 8);
    const uint64_t* words = n ? w.data() : nullptr;
    run_proof_form<false>(words, n, D);
    run_proof_form<true>(words, n, D);
    ++g_runs;
}

void run_blk(const std::vector<uint8_t>& b, uint32_t height) {
    size_t nb = 0;
    const int rc = nhip_blk_scan(b.data(), b.size(), height, nullptr, 0, &nb);
    ++g_runs;
    if (rc && nb == 0) return;
    std::vector<nhip_blk_block> blocks(nb ? nb : 1);
    size_t got = 0;
    nhip_blk_scan(b.data(), b.size(), height, blocks.data(), blocks.size(), &got);
    for (size_t i = 0; i < got; ++i) {
        uint64_t offs[12];
        if (nhip_blk_sequences(b.data(), b.size(), height, &blocks[i], nullptr, 0, offs) == NHIP_OK) {
            std::vector<uint64_t> seq(offs[11] + 1);
            nhip_blk_sequences(b.data(), b.size(), height, &blocks[i], seq.data(), seq.size(), offs);
        }
        std::vector<uint64_t> cw(blocks[i].claim_words + 1);
        std::vector<nhip_claim> claims(blocks[i].n_claims + 1);
        nhip_blk_claims(b.data(), b.size(), &blocks[i], cw.data(), claims.data());
        if (blocks[i].proof_kind == NHIP_BLOCK_PROOF_SINGLE && blocks[i].proof_len < (1u << 24)) {
            std::vector<uint64_t> pw(blocks[i].proof_len + 1);
            nhip_le_words(b.data(), b.size(), blocks[i].proof_offset, blocks[i].proof_len, pw.data());
        }
        ++g_ok;
    }
}

void run_tx(const std::vector<uint8_t>& b) {
    nhip_tx tx{};
    ++g_runs;
    // the arena ingest's scanner (nhip::tx_proof_spans, csrc/bincode.cpp) on an exact-size heap copy:
    // it must agree with the scan below on validity and, when valid, on every proof span
    std::vector<uint64_t> arena_spans;
    uint64_t arena_size = 0;
    const bool arena_ok = nhip::tx_proof_spans(b.data(), b.size(), arena_spans, arena_size);
    if (nhip_tx_scan(b.data(), b.size(), &tx) != NHIP_OK) {
        if (arena_ok) g_mismatch++;
        return;
    }
    if (!arena_ok || arena_size != tx.size || arena_spans.size() != 2ull * tx.n_proofs) g_mismatch++;
    if (tx.seq_words > (1u << 24) || tx.n_proofs > (1u << 16) || tx.n_digests > (1u << 16)) return;
    std::vector<uint64_t> seq(tx.seq_words + 1), spans(2ull * tx.n_proofs + 2), dig(5ull * tx.n_digests + 5);
    uint64_t offs[9];
    if (nhip_tx_parts(b.data(), b.size(), &tx, seq.data(), offs, spans.data(), dig.data()) == NHIP_OK) {
        for (uint32_t p = 0; p < tx.n_proofs; ++p) {
            if (arena_ok && (arena_spans[2 * p] != spans[2 * p] || arena_spans[2 * p + 1] != spans[2 * p + 1]))
                g_mismatch++;
            if (spans[2 * p + 1] > (1u << 24)) continue;
            std::vector<uint64_t> pw(spans[2 * p + 1] + 1), aw(spans[2 * p + 1] + 2);
            nhip_le_words(b.data(), b.size(), spans[2 * p], spans[2 * p + 1], pw.data());
            // the arena's streaming decode of the same span (into an odd-aligned destination)
            nhip::copy_le_words_nt(aw.data() + 1, b.data() + spans[2 * p], spans[2 * p + 1]);
            _mm_sfence();
            if (std::memcmp(aw.data() + 1, pw.data(), spans[2 * p + 1] * 8) != 0) g_mismatch++;
        }
        ++g_ok;
    }
}

void run_be(const std::vector<uint8_t>& b) {
    size_t nw = 0;
    ++g_runs;
    if (nhip_proof_from_be_bytes(b.data(), b.size(), nullptr, 0, &nw) != NHIP_OK) return;
    std::vector<uint64_t> w(nw + 1);
    if (nhip_proof_from_be_bytes(b.data(), b.size(), w.data(), w.size(), &nw) == NHIP_OK) ++g_ok;
}

template <class F>
void fuzz(const std::vector<uint8_t>& in, size_t mutations, size_t word, F&& run) {
    run(in);
    // truncations: every length for small inputs, ~400 spread lengths otherwise
    const size_t step = in.size() <= 2048 ? 1 : in.size() / 400;
    for (size_t len = 0; len < in.size(); len += step) run(std::vector<uint8_t>(in.begin(), in.begin() + len));
    for (size_t m = 0; m < mutations && !in.empty(); ++m) {
        std::vector<uint8_t> x(in);
        const uint64_t r = next_u64();
        const size_t k = 1 + (r & 3);  // 1..4 edits
        for (size_t e = 0; e < k; ++e) {
            const uint64_t q = next_u64();
            if ((q & 1) || x.size() < word) {
                x[(q >> 8) % x.size()] ^= (uint8_t)(1u << ((q >> 4) & 7));
            } else {
                const size_t pos = ((q >> 8) % (x.size() / word)) * word;
                uint64_t v = (q & 2) ? INTERESTING[(q >> 40) % (sizeof(INTERESTING) / 8)] : next_u64();
                if (word == 8) std::memcpy(&x[pos], &v, 8);
                else std::memcpy(&x[pos], &v, 4);
            }
        }
        if ((r >> 8) % 16 == 0) x.resize((r >> 16) % (x.size() + 1));  // also truncate some
        run(x);
    }
}

std::vector<uint8_t> read_file(const char* path) {
    std::vector<uint8_t> b;
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        std::fprintf(stderr, "cannot open %s\n", path);
        std::exit(2);
    }
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) b.insert(b.end(), buf, buf + n);
    std::fclose(f);
    return b;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <mutations> kind:path ...\n", argv[0]);
        return 2;
    }
    const size_t mutations = std::strtoull(argv[1], nullptr, 10);
    const Dims tiny = dims_of(8, 24, 9), full = dims_of(80, 379, 88);
    for (int a = 2; a < argc; ++a) {
        const std::string arg = argv[a];
        const size_t colon = arg.find(':');
        if (colon == std::string::npos) return 2;
        const std::string kind = arg.substr(0, colon);
        const std::vector<uint8_t> in = read_file(arg.c_str() + colon + 1);
        if (kind == "proof-tiny") fuzz(in, mutations, 8, [&](const std::vector<uint8_t>& x) { run_proof(x, tiny); });
        else if (kind == "proof-full") fuzz(in, mutations, 8, [&](const std::vector<uint8_t>& x) { run_proof(x, full); });
        else if (kind == "blk10") fuzz(in, mutations, 4, [&](const std::vector<uint8_t>& x) { run_blk(x, 10); });
        else if (kind == "tx") fuzz(in, mutations, 4, [&](const std::vector<uint8_t>& x) { run_tx(x); });
        else if (kind == "be") fuzz(in, mutations, 8, [&](const std::vector<uint8_t>& x) { run_be(x); });
        else return 2;
    }
    std::printf("runs %llu ok %llu mismatch %llu\n", (unsigned long long)g_runs, (unsigned long long)g_ok,
                (unsigned long long)g_mismatch);
    return g_mismatch ? 1 : 0;
}
