// Proof-stream codec of the batched STARK verifier, shared by the device decoder (k_decode in
// stark_kernels.hip: every batch run decodes its proofs on the GPU from the raw words in HBM) and
// the host-only structural check (nhip_proof_decodes, the CPU tests and the sanitizer build).  One
// source, so the two can never disagree.
//
// Restates triton-vm 1.0's `ProofStream::try_from(&Proof)` (BFieldCodec of Vec<ProofItem>) and
// the dequeue order of `Stark::verify` / `Fri::verify` (parity unpinned beyond the
// Claim layout, pinned by neptune-core/src/protocol/consensus/transaction/validity/tasm/claims/
// new_claim.rs:38-100).  Any structural error gives FAIL_DECODE, i.e. verdict 0: triton_vm::verify
// returns false on every Err (reject tests verifier.rs:95-118, neptune_proof.rs:118-133).
//
// Streaming walk: the first item fixes the padded height and with it the FRI round count R, the
// exact item count (19 + 2R) and the kind of every later item, so the items are checked as they
// are read and no item list is kept.  A proof whose item count differs, or whose items do not
// decode or come in another order, is rejected: the same verdicts as decoding every item first
// and then dequeuing (and no allocation driven by the untrusted item count).
//
// Words may be any u64, in either input form (nhip_stark_params.input_form): canonical values
// (MW = false, BFieldElement::new semantics) or twenty-first's in-memory Montgomery words (MW = true,
// x * 2^64 mod p).  Structural words (lengths, counts, discriminants, the padded height) are read
// through word_value<MW> (the element's canonical value); the arithmetic kernels load through
// word_mont<MW> (the canonical raw Montgomery word) or reduce mod p as they accumulate, so no
// separate conversion pass over the proof is needed in either form.
#pragma once
#include <stdint.h>

#include "goldilocks.hpp"
#include "stark.hpp"

namespace nhip {

enum ItemKind : uint32_t {
    MERKLE_ROOT = 0, OOD_MAIN_ROW, OOD_AUX_ROW, OOD_QUOT_SEGMENTS, AUTH_STRUCTURE, MAIN_ROWS, AUX_ROWS,
    LOG2_PADDED_HEIGHT, QUOT_SEGMENTS_ELEMENTS, FRI_CODEWORD, FRI_POLYNOMIAL, FRI_RESPONSE, N_KINDS
};

struct Dims {
    StarkDims d;
    uint32_t expansion;
    uint32_t mont_words;  // input form: 0 canonical values, 1 Montgomery words (NHIP_INPUT_*)
};

// Proof geometry implied by the padded height (the first item).
struct ProofShape {
    uint32_t log2_ph, log2_T, log2_N, R;
};

// Where the staged claim encoding of a proof lives in the batch word buffer (encode_claim layout:
// [out_n + 1, out_n, out.., in_n + 1, in_n, in.., version, digest(5)]).
struct ClaimLoc {
    uint64_t off;
    uint32_t in_n, out_n;
};

static constexpr uint32_t SHAPE_NONE = 0xFFFFFFFFu;  // header malformed: the proof is rejected

__host__ __device__ __forceinline__ uint64_t canon(uint64_t v) { return v >= GL_P ? v - GL_P : v; }
// A batch word as the element's canonical value (structural words) ...
template <bool MW>
__host__ __device__ __forceinline__ uint64_t word_value(uint64_t w) {
    if constexpr (MW) return from_mont(w);  // montyred(w, 0): any u64 -> w * 2^-64 mod p, in [0, p)
    else return canon(w);
}
// ... and as the canonical raw Montgomery word the arithmetic works on (Tip5 reads its bytes)
template <bool MW>
__host__ __device__ __forceinline__ uint64_t word_mont(uint64_t w) {
    if constexpr (MW) return canon(w);
    else return to_mont(w);
}
__host__ __device__ __forceinline__ uint32_t log2_u64(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }

// Fri::num_rounds for a FRI domain of fri_len: rounds until the code dimension reaches
// 2 * num_collinearity_checks.
__host__ __device__ __forceinline__ uint32_t fri_num_rounds(const Dims& D, uint64_t fri_len) {
    const uint64_t dim = fri_len / D.expansion;
    const uint32_t max_rounds = dim > 1 ? 64u - (uint32_t)__builtin_clzll(dim - 1) : 0u;
    const uint32_t all = log2_u64(D.d.num_checks);
    return max_rounds > all + 1 ? max_rounds - (all + 1) : 0u;
}

// Stark::verify's derived sizes: randomized trace length T = next_pow2(padded height + trace
// randomizers), FRI domain N = T * expansion.  false when out of range (rejected): padded height
// > 2^LOG2_PH_MAX, a FRI domain above 2^31 (sample_indices takes a u32 upper bound), or more FRI
// rounds than the descriptors hold.
__host__ __device__ __forceinline__ bool shape_of(const Dims& D, uint64_t log2_ph, ProofShape& s) {
    if (log2_ph > LOG2_PH_MAX) return false;
    const uint64_t need = (1ull << log2_ph) + D.d.num_trace_randomizers;
    uint64_t T = 1;
    while (T < need) T <<= 1;
    s.log2_ph = (uint32_t)log2_ph;
    s.log2_T = log2_u64(T);
    s.log2_N = s.log2_T + D.d.log2_expansion;
    if (s.log2_N > 31) return false;
    s.R = fri_num_rounds(D, 1ull << s.log2_N);
    return s.R <= (uint32_t)MAX_FRI_ROUNDS;
}

// Items of Stark::verify's dequeue sequence for R FRI rounds and the kind of item t.
__host__ __device__ __forceinline__ uint64_t expected_items(uint32_t R) { return 19ull + 2ull * R; }
__host__ __device__ __forceinline__ uint32_t expected_kind(uint64_t t, uint32_t R) {
    if (t == 0) return LOG2_PADDED_HEIGHT;
    if (t <= 3) return MERKLE_ROOT;                       // main, aux, quotient roots
    if (t <= 8) return t == 8 ? OOD_QUOT_SEGMENTS : ((t & 1) ? OOD_AUX_ROW : OOD_MAIN_ROW);  // 4..8
    if (t <= 9ull + R) return MERKLE_ROOT;                // FRI round roots 0..R
    if (t == 10ull + R) return FRI_CODEWORD;
    if (t == 11ull + R) return FRI_POLYNOMIAL;
    if (t <= 12ull + 2 * R) return FRI_RESPONSE;          // round-0 a-values, rounds 0..R-1 b-values
    const uint64_t q = t - (13ull + 2 * R);  // rows / authentication structure pairs
    if (q & 1) return AUTH_STRUCTURE;
    return q == 0 ? MAIN_ROWS : (q == 2 ? AUX_ROWS : QUOT_SEGMENTS_ELEMENTS);
}

// The padded height the proof declares, if its header is well formed: [len - 1, n_items,
// 2, LOG2_PADDED_HEIGHT, log2_ph, ...].  Host sizing of a batch peeks at it; k_decode re-reads it.
template <bool MW>
__host__ __device__ __forceinline__ bool header_log2_ph(const uint64_t* w, uint64_t len, uint64_t& log2_ph) {
    if (len < 5 || word_value<MW>(w[0]) != len - 1 || word_value<MW>(w[2]) != 2 ||
        word_value<MW>(w[3]) != LOG2_PADDED_HEIGHT)
        return false;
    log2_ph = word_value<MW>(w[4]);
    return log2_ph < (1ull << 32);
}

struct Item {
    uint32_t kind;
    uint64_t lo, hi;      // item words [lo, hi) starting at the discriminant (absolute)
    uint64_t payload;     // first payload element (after counts)
    uint64_t n;           // element count (dynamic kinds) / value (Log2PaddedHeight)
    uint64_t leaves_off, leaves_n, auth_off, auth_n;  // FRI response only
};

// Decode one ProofItem occupying words[lo, hi).  false on any malformation.
template <bool MW>
__host__ __device__ inline bool decode_item(const uint64_t* w, uint64_t lo, uint64_t hi, const Dims& D, Item& it) {
    if (lo >= hi) return false;
    it = Item{};
    const uint64_t disc = word_value<MW>(w[lo]);
    it.kind = (uint32_t)(disc < N_KINDS ? disc : N_KINDS);
    it.lo = lo;
    it.hi = hi;
    const uint64_t len = hi - lo;
    const StarkDims& d = D.d;
    switch (it.kind) {
        case MERKLE_ROOT: it.payload = lo + 1; return len == 1 + 5;
        case OOD_MAIN_ROW: it.payload = lo + 1; return len == 1 + 3ull * d.num_main;
        case OOD_AUX_ROW: it.payload = lo + 1; return len == 1 + 3ull * d.num_aux;
        case OOD_QUOT_SEGMENTS: it.payload = lo + 1; return len == 1 + 3ull * d.num_quot_seg;
        case LOG2_PADDED_HEIGHT:
            if (len != 2) return false;
            it.n = word_value<MW>(w[lo + 1]);
            return it.n < (1ull << 32);
        case N_KINDS: return false;
        default: break;
    }
    // dynamically sized payload: [kind, blen, body(blen)]
    if (len < 2) return false;
    const uint64_t blen = word_value<MW>(w[lo + 1]);
    if (blen != len - 2) return false;
    const uint64_t b0 = lo + 2;
    if (it.kind == FRI_RESPONSE) {
        // FriResponse { auth_structure, revealed_leaves } encoded fields-reversed:
        // [len(rl), n_leaves, leaves.., len(au), n_auth, digests..]
        if (blen < 1) return false;
        const uint64_t lrl = word_value<MW>(w[b0]);
        if (lrl < 1 || lrl >= blen) return false;
        const uint64_t nl = word_value<MW>(w[b0 + 1]);
        if (nl > (lrl - 1) / 3 || 3 * nl != lrl - 1) return false;
        it.leaves_off = b0 + 2;
        it.leaves_n = nl;
        const uint64_t pa = b0 + 1 + lrl;
        if (pa >= b0 + blen) return false;
        const uint64_t lau = word_value<MW>(w[pa]);
        if (lau < 1 || 1 + lrl + 1 + lau != blen) return false;
        const uint64_t na = word_value<MW>(w[pa + 1]);
        if (na > (lau - 1) / 5 || 5 * na != lau - 1) return false;
        it.auth_off = pa + 2;
        it.auth_n = na;
        return true;
    }
    uint64_t width = 0;
    switch (it.kind) {
        case AUTH_STRUCTURE: width = 5; break;
        case MAIN_ROWS: width = d.num_main; break;
        case AUX_ROWS: width = 3ull * d.num_aux; break;
        case QUOT_SEGMENTS_ELEMENTS: width = 3ull * d.num_quot_seg; break;
        case FRI_CODEWORD: width = 3; break;
        case FRI_POLYNOMIAL: width = 3; break;
        default: return false;
    }
    if (blen < 1) return false;
    const uint64_t n = word_value<MW>(w[b0]);
    if (width == 0 || n > (blen - 1) / width || n * width != blen - 1) return false;
    it.n = n;
    it.payload = b0 + 1;
    return true;
}

__host__ __device__ __forceinline__ uint64_t absorb_perms(uint64_t len) { return len / 10 + 1; }

// Fiat-Shamir program length for R FRI rounds (claim, 3 roots with their squeezes, 5 OOD items +
// the linear-combination squeeze, R + 1 FRI roots with R folding-challenge squeezes, the FRI
// indices, the last-round indeterminate).
__host__ __device__ constexpr uint32_t fs_ops_for(uint32_t R) { return 16u + 2u * R; }

// Decode the proof at words[base, base + len) with its staged claim at `cl` into `pd` and its
// Fiat-Shamir program `ops` (fs_ops_for(R) entries; absolute word offsets).  Returns 0 or
// FAIL_DECODE; on failure pd holds only the claim offsets.  perms / perms_lcw: Tip5 permutations of
// the sponge replay + row hashing, and of the last-codeword tree.  pd.last_poly_degree_ok is left
// to last_poly_finish (the degree scan is lane-parallel on the device).  xs_off / idx_off /
// fs_op_off / n_xs are the caller's (batch layout).
__host__ __device__ __forceinline__ void claim_offsets(ProofDesc& pd, const ClaimLoc& cl) {
    const uint64_t clen = (uint64_t)cl.out_n + cl.in_n + 10;
    pd.claim_out_off = cl.off + 2;
    pd.claim_out_n = cl.out_n;
    pd.claim_in_off = cl.off + 2 + cl.out_n + 2;
    pd.claim_in_n = cl.in_n;
    pd.claim_digest_off = cl.off + clen - 5;
}

template <bool MW>
__host__ __device__ inline uint32_t decode_stream_walk(const uint64_t* w, uint64_t base, uint64_t len,
                                                       const ClaimLoc& cl, const Dims& D, ProofDesc& pd, FsOp* ops,
                                                       uint64_t& perms, uint64_t& perms_lcw) {
    const StarkDims& d = D.d;
    const uint64_t clen = (uint64_t)cl.out_n + cl.in_n + 10;
    const uint64_t end = base + len;
    if (len < 2 || word_value<MW>(w[base]) != len - 1) return FAIL_DECODE;
    const uint64_t n_items = word_value<MW>(w[base + 1]);
    uint64_t pos = base + 2;
    ProofShape sh{};
    uint64_t t = 0;
    uint32_t n_ops = 0;
    uint64_t p = 0;
    auto absorb = [&](uint64_t off, uint64_t n) {
        ops[n_ops++] = FsOp{FS_ABSORB, (uint32_t)n, off};
        p += absorb_perms(n);
    };
    auto squeeze = [&](uint32_t n) {
        ops[n_ops++] = FsOp{FS_SQUEEZE_X, n, 0};
        p += (3ull * n + 9) / 10;
    };
    absorb(cl.off, clen);
    uint32_t R = 0;
    Item it;
    for (;; ++t) {
        if (t > 0 && t == expected_items(R)) break;
        if (t >= n_items || pos >= end) return FAIL_DECODE;
        const uint64_t ln = word_value<MW>(w[pos++]);
        if (ln > end - pos) return FAIL_DECODE;
        if (!decode_item<MW>(w, pos, pos + ln, D, it)) return FAIL_DECODE;
        pos += ln;
        if (it.kind != expected_kind(t, R)) return FAIL_DECODE;
        const uint32_t k = d.num_checks;
        const uint64_t item_lo = it.lo, item_n = it.hi - it.lo;
        if (t == 0) {
            if (!shape_of(D, it.n, sh)) return FAIL_DECODE;
            R = sh.R;
            if (n_items != expected_items(R)) return FAIL_DECODE;
            continue;
        }
        if (t <= 3) {  // roots: main (then the challenges), aux (then the quotient weights), quotient (then z)
            absorb(item_lo, item_n);
            if (t == 1) pd.main_root = it.payload, squeeze(d.num_sampled);
            if (t == 2) pd.aux_root = it.payload, squeeze(d.num_constraints);
            if (t == 3) pd.quot_root = it.payload, squeeze(1);
        } else if (t <= 8) {
            absorb(item_lo, item_n);
            if (t == 4) pd.ood_mc = it.payload;
            if (t == 5) pd.ood_ac = it.payload;
            if (t == 6) pd.ood_mn = it.payload;
            if (t == 7) pd.ood_an = it.payload;
            if (t == 8) pd.ood_qs = it.payload;
            if (t == 8) squeeze(d.num_main + d.num_aux + d.num_quot_seg + d.num_deep);
        } else if (t <= 9ull + R) {  // FRI roots, each followed by its folding challenge but the last
            const uint32_t r = (uint32_t)(t - 9);
            absorb(item_lo, item_n);
            pd.fri_root[r] = it.payload;
            if (r < R) squeeze(1);
        } else if (t == 10ull + R) {
            if (it.n != (1ull << (sh.log2_N - R))) return FAIL_DECODE;
            pd.last_cw_off = it.payload;
            pd.last_cw_n = (uint32_t)it.n;
        } else if (t == 11ull + R) {
            pd.last_poly_off = it.payload;
            pd.last_poly_n = (uint32_t)(it.n < 0xFFFFFFFFull ? it.n : 0xFFFFFFFFull);
        } else if (t <= 12ull + 2 * R) {
            const uint32_t r = (uint32_t)(t - (12 + R));
            if (it.leaves_n != k) return FAIL_DECODE;
            pd.fri[r].auth_off = it.auth_off;
            pd.fri[r].auth_n = (uint32_t)it.auth_n;
            pd.fri[r].leaves_off = it.leaves_off;
            pd.fri[r].leaves_n = (uint32_t)it.leaves_n;
        } else {
            const uint64_t q = t - (13 + 2ull * R);
            if ((q == 0 || q == 2 || q == 4) && it.n != k) return FAIL_DECODE;  // revealed rows
            if (q == 0) pd.main_rows_off = it.payload;
            if (q == 1) pd.main_auth_off = it.payload, pd.main_auth_n = (uint32_t)it.n;
            if (q == 2) pd.aux_rows_off = it.payload;
            if (q == 3) pd.aux_auth_off = it.payload, pd.aux_auth_n = (uint32_t)it.n;
            if (q == 4) pd.quot_rows_off = it.payload;
            if (q == 5) pd.quot_auth_off = it.payload, pd.quot_auth_n = (uint32_t)it.n;
        }
    }
    if (pos != end) return FAIL_DECODE;  // trailing words after the last item
    pd.log2_ph = sh.log2_ph;
    pd.log2_T = sh.log2_T;
    pd.log2_N = sh.log2_N;
    pd.R = R;
    pd.rows_n = d.num_checks;
    ops[n_ops++] = FsOp{FS_SAMPLE_IDX, d.num_checks, 1ull << sh.log2_N};
    p += (d.num_checks + 9) / 10;
    squeeze(1);  // last-round indeterminate
    pd.fs_op_n = n_ops;
    p += (uint64_t)d.num_checks * (absorb_perms(d.num_main) + absorb_perms(3ull * d.num_aux) +
                                   absorb_perms(3ull * d.num_quot_seg));
    perms = p;
    perms_lcw = pd.last_cw_n - 1;
    return 0;
}

template <bool MW>
__host__ __device__ inline uint32_t decode_stream(const uint64_t* w, uint64_t base, uint64_t len, const ClaimLoc& cl,
                                                  const Dims& D, ProofDesc& pd, FsOp* ops, uint64_t& perms,
                                                  uint64_t& perms_lcw) {
    pd = ProofDesc{};
    perms = perms_lcw = 0;
    const uint32_t f = decode_stream_walk<MW>(w, base, len, cl, D, pd, ops, perms, perms_lcw);
    if (f) {
        pd = ProofDesc{};
        perms = perms_lcw = 0;
    }
    claim_offsets(pd, cl);
    return f;
}

// FRI's last-polynomial check: degree (highest non-zero coefficient, -1 for none) <= the last
// round's maximal degree.  The polynomial is trimmed to degree + 1 coefficients for the evaluation
// (trailing zeros add nothing to Horner); a polynomial above the bound is not evaluated at all
// (the proof is rejected by FAIL_FRI_DEGREE), so a prover-padded polynomial costs no work.
__host__ __device__ __forceinline__ void last_poly_finish(ProofDesc& pd, int64_t degree, const Dims& D) {
    const uint64_t first_max = (1ull << pd.log2_N) / D.expansion - 1;
    const uint64_t last_max = first_max >> pd.R;
    pd.last_poly_degree_ok = degree <= (int64_t)last_max ? 1u : 0u;
    pd.last_poly_n = pd.last_poly_degree_ok ? (uint32_t)(degree + 1) : 0u;
}

// Sequential degree scan (host).
inline int64_t last_poly_degree_host(const uint64_t* w, const ProofDesc& pd) {
    int64_t deg = -1;
    for (uint64_t c = 0; c < pd.last_poly_n; ++c) {
        const uint64_t* x = w + pd.last_poly_off + 3 * c;
        if (canon(x[0]) | canon(x[1]) | canon(x[2])) deg = (int64_t)c;
    }
    return deg;
}

}  // namespace nhip
