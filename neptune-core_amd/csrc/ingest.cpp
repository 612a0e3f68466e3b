// Proof ingestion formats: the reference's proof files and claim hashing.
//
//  * Proof files: neptune-core/src/protocol/proof_abstractions/tasm/program.rs:374-390 reads a
//    proof as consecutive 8-byte big-endian u64 chunks, each through BFieldElement::new (reduced
//    mod p); a trailing chunk shorter than 8 bytes makes the load fail (`None`).  The writer
//    (program.rs:565-572) emits value().to_be_bytes() per element.
//  * File name: program.rs:355-358, `Tip5::hash(claim).to_hex() + ".proof"`, i.e. hash_varlen of
//    the claim's BFieldCodec encoding (the staged layout of stark_host.cpp) — computed on the GPU.
#include <cstring>
#include <vector>

#include "../../include/neptune_hip.h"

namespace {
constexpr uint64_t P = 0xFFFFFFFF00000001ull;
inline uint64_t be64(const uint8_t* b) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | b[i];
    return v;
}
}  // namespace

extern "C" {

int nhip_proof_from_be_bytes(const uint8_t* bytes, size_t n_bytes, uint64_t* words, size_t cap, size_t* n_words) {
    if (n_words) *n_words = 0;
    if (n_bytes && !bytes) return NHIP_ERR_ARG;
    if (n_bytes % 8) return NHIP_ERR_ARG;  // program.rs:383-386: chunk not 8 bytes -> None
    const size_t n = n_bytes / 8;
    if (n_words) *n_words = n;
    if (!words) return NHIP_OK;  // size query
    if (cap < n) return NHIP_ERR_ARG;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t v = be64(bytes + 8 * i);
        words[i] = v >= P ? v - P : v;  // BFieldElement::new
    }
    return NHIP_OK;
}

int nhip_proof_to_be_bytes(const uint64_t* words, size_t n, uint8_t* out) {
    if (n && (!words || !out)) return NHIP_ERR_ARG;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t v = words[i] % P;  // value()
        for (int k = 0; k < 8; ++k) out[8 * i + k] = (uint8_t)(v >> (56 - 8 * k));
    }
    return NHIP_OK;
}

int nhip_claim_hash(nhip_ctx* ctx, const nhip_claim* claim, uint64_t digest_out[5]) {
    if (!ctx || !claim || !digest_out || (claim->input_len && !claim->input) || (claim->output_len && !claim->output))
        return NHIP_ERR_ARG;
    // Claim encoding (fields reversed, new_claim.rs:38-100):
    // [len(out)+1, len(out), out.., len(in)+1, len(in), in.., version, digest(5)]
    std::vector<uint64_t> enc;
    enc.reserve(claim->input_len + claim->output_len + 10);
    enc.push_back(claim->output_len + 1);
    enc.push_back(claim->output_len);
    for (size_t i = 0; i < claim->output_len; ++i) enc.push_back(claim->output[i] % P);
    enc.push_back(claim->input_len + 1);
    enc.push_back(claim->input_len);
    for (size_t i = 0; i < claim->input_len; ++i) enc.push_back(claim->input[i] % P);
    enc.push_back(claim->version);
    for (int i = 0; i < 5; ++i) enc.push_back(claim->program_digest[i] % P);
    const uint64_t off[2] = {0, (uint64_t)enc.size()};
    return nhip_tip5_hash_varlen(ctx, enc.data(), off, 1, digest_out);
}

}  // extern "C"
