/*
 * C restatement of the STARK verifier — TEST ORACLE AND CPU BASELINE ONLY.
 *
 * Test infrastructure: only tests/ and bench.py's cpu_baseline leg load it (through
 * oracle/coracle.py), as the checker or as the timed CPU baseline.  The shipped library
 * (neptune-core_amd/) never links or calls it.
 *
 * What it restates: `triton_vm::verify(Stark::default(), &claim, &proof) -> bool`, the single
 * production call at neptune-core/src/protocol/proof_abstractions/verifier.rs:60-63.  triton-vm
 * 1.0.0 / twenty-first 1.0.0 (Cargo.lock:4260, 4297) are not vendored, so this file follows the
 * Python restatement oracle/stark_ref.py step by step (function names match: decode_proof,
 * ProofStream, merkle_multiproof_root, zerofier_inverses, fri_verify, _verify); every point that
 * file marks "unpinned" is unpinned here too.  Pinned: Tip5 (tip5_oracle.c, KAT-V/KAT-F) and the
 * Claim encoding (neptune-core/.../tasm/claims/new_claim.rs:38-100).
 *
 * It is written as a native CPU verifier would be (u128 Goldilocks products, one proof per
 * thread, Tip5 with the reference's split-lo/hi MDS), so the CPU baseline of bench.py measures
 * a compiled verifier rather than Python.  Field elements are canonical u64 here (the GPU works
 * in Montgomery form), Tip5 states raw Montgomery.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* the ChallengeId table, shared with the kernels (stark_ref.CHALLENGE_IDS is the independent copy) */
#include "../include/nhip_challenge_id.h"

#define P 0xFFFFFFFF00000001ull
#define EPS 0xFFFFFFFFull
typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ Tip5 (raw Montgomery) */
extern void oracle_tip5_permutation_raw_fast(uint64_t s[16]);
extern uint64_t oracle_to_mont(uint64_t x);
extern uint64_t oracle_from_mont(uint64_t r);

/* ------------------------------------------------------------------ base field (canonical) */
static inline uint64_t fadd(uint64_t a, uint64_t b) {
    uint64_t s = a + b;
    uint64_t c = s < a;
    s += c * EPS;  /* 2^64 == 2^32 - 1 */
    return s >= P ? s - P : s;
}
static inline uint64_t fsub(uint64_t a, uint64_t b) { return a >= b ? a - b : a + (P - b); }
static inline uint64_t fred(u128 x) {
    /* x = lo + hi*2^64, hi = h0 + h1*2^32: 2^64 == 2^32 - 1, 2^96 == -1 */
    uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
    uint64_t h0 = hi & 0xFFFFFFFFull, h1 = hi >> 32;
    uint64_t t = fsub(lo >= P ? lo - P : lo, h1);
    return fadd(t, (h0 << 32) - h0);
}
static inline uint64_t fmul(uint64_t a, uint64_t b) { return fred((u128)a * b); }
static uint64_t fpow(uint64_t a, uint64_t e) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = fmul(r, a);
        a = fmul(a, a);
        e >>= 1;
    }
    return r;
}
static inline uint64_t finv(uint64_t a) { return fpow(a, P - 2); }
static uint64_t root_of_unity(uint32_t log2n) { return fpow(7, (P - 1) >> log2n); }

/* ------------------------------------------------------------------ XFE = F_p[x]/(x^3 - x + 1) */
typedef struct { uint64_t c[3]; } xfe;
static const xfe X0 = {{0, 0, 0}}, X1 = {{1, 0, 0}};
static inline xfe xadd(xfe a, xfe b) { return (xfe){{fadd(a.c[0], b.c[0]), fadd(a.c[1], b.c[1]), fadd(a.c[2], b.c[2])}}; }
static inline xfe xsub(xfe a, xfe b) { return (xfe){{fsub(a.c[0], b.c[0]), fsub(a.c[1], b.c[1]), fsub(a.c[2], b.c[2])}}; }
static inline xfe xscale(xfe a, uint64_t s) { return (xfe){{fmul(a.c[0], s), fmul(a.c[1], s), fmul(a.c[2], s)}}; }
static inline xfe xlift(uint64_t b) { return (xfe){{b, 0, 0}}; }
static inline int xeq(xfe a, xfe b) { return a.c[0] == b.c[0] && a.c[1] == b.c[1] && a.c[2] == b.c[2]; }
static inline int xzero(xfe a) { return (a.c[0] | a.c[1] | a.c[2]) == 0; }
static xfe xmul(xfe a, xfe b) {
    /* x^3 = x - 1, x^4 = x^2 - x (field_ref.xmul) */
    uint64_t c0 = fmul(a.c[0], b.c[0]);
    uint64_t c1 = fadd(fmul(a.c[0], b.c[1]), fmul(a.c[1], b.c[0]));
    uint64_t c2 = fadd(fadd(fmul(a.c[0], b.c[2]), fmul(a.c[1], b.c[1])), fmul(a.c[2], b.c[0]));
    uint64_t c3 = fadd(fmul(a.c[1], b.c[2]), fmul(a.c[2], b.c[1]));
    uint64_t c4 = fmul(a.c[2], b.c[2]);
    return (xfe){{fsub(c0, c3), fsub(fadd(c1, c3), c4), fadd(c2, c4)}};
}
/* a^-1 = adj(M_a) e_0 / det(M_a), M_a the matrix of multiplication by a (columns a, a x, a x^2) */
static xfe xinv(xfe a, int* zero) {
    if (xzero(a)) {
        *zero = 1;
        return X0;
    }
    const uint64_t a0 = a.c[0], a1 = a.c[1], a2 = a.c[2];
    /* a*x = (-a2, a0 + a2, a1);  a*x^2 = (-a1, a1 - a2, a0 + a2) */
    const uint64_t m[3][3] = {{a0, fsub(0, a2), fsub(0, a1)},
                              {a1, fadd(a0, a2), fsub(a1, a2)},
                              {a2, a1, fadd(a0, a2)}};
    /* solve M y = e0 by Cramer: y_i = det(M with column i := e0) / det(M) */
    const uint64_t det = fsub(fadd(fmul(m[0][0], fsub(fmul(m[1][1], m[2][2]), fmul(m[1][2], m[2][1]))),
                                   fmul(m[0][2], fsub(fmul(m[1][0], m[2][1]), fmul(m[1][1], m[2][0])))),
                              fmul(m[0][1], fsub(fmul(m[1][0], m[2][2]), fmul(m[1][2], m[2][0]))));
    const uint64_t di = finv(det);
    const uint64_t y0 = fsub(fmul(m[1][1], m[2][2]), fmul(m[1][2], m[2][1]));
    const uint64_t y1 = fsub(fmul(m[1][2], m[2][0]), fmul(m[1][0], m[2][2]));
    const uint64_t y2 = fsub(fmul(m[1][0], m[2][1]), fmul(m[1][1], m[2][0]));
    return (xfe){{fmul(y0, di), fmul(y1, di), fmul(y2, di)}};
}
static inline xfe xld(const uint64_t* w) { return (xfe){{w[0], w[1], w[2]}}; }

/* ------------------------------------------------------------------ sponge (VariableLength) */
typedef struct { uint64_t s[16]; } sponge;
static void sp_absorb_all(sponge* sp, const uint64_t* data, size_t len) {  /* pad_and_absorb_all */
    size_t k = 0;
    for (; k + 10 <= len; k += 10) {
        for (int i = 0; i < 10; ++i) sp->s[i] = oracle_to_mont(data[k + i]);
        oracle_tip5_permutation_raw_fast(sp->s);
    }
    const size_t rem = len - k;
    for (size_t i = 0; i < 10; ++i) sp->s[i] = oracle_to_mont(i < rem ? data[k + i] : (i == rem ? 1 : 0));
    oracle_tip5_permutation_raw_fast(sp->s);
}
static void sp_squeeze(sponge* sp, uint64_t out[10]) {
    for (int i = 0; i < 10; ++i) out[i] = oracle_from_mont(sp->s[i]);
    oracle_tip5_permutation_raw_fast(sp->s);
}
static void sp_sample_scalars(sponge* sp, size_t n, xfe* out) {
    uint64_t buf[10];
    size_t got = 0;  /* flat words */
    const size_t need = 3 * n, n_sq = (need + 9) / 10;
    for (size_t q = 0; q < n_sq; ++q) {
        sp_squeeze(sp, buf);
        for (int i = 0; i < 10 && got < need; ++i, ++got) out[got / 3].c[got % 3] = buf[i];
    }
}
static void sp_sample_indices(sponge* sp, uint64_t bound, size_t n, uint32_t* out) {
    uint64_t buf[10];
    size_t got = 0;
    while (got < n) {
        sp_squeeze(sp, buf);
        for (int i = 0; i < 10 && got < n; ++i)
            if (buf[i] != P - 1) out[got++] = (uint32_t)((buf[i] & 0xFFFFFFFFull) % bound);
    }
}
static void hash_varlen(const uint64_t* data, size_t len, uint64_t out[5]) {
    sponge sp;
    memset(&sp, 0, sizeof(sp));
    sp_absorb_all(&sp, data, len);
    for (int i = 0; i < 5; ++i) out[i] = oracle_from_mont(sp.s[i]);
}
static void hash_pair(const uint64_t l[5], const uint64_t r[5], uint64_t out[5]) {
    uint64_t s[16];
    for (int i = 0; i < 5; ++i) {
        s[i] = oracle_to_mont(l[i]);
        s[5 + i] = oracle_to_mont(r[i]);
    }
    for (int i = 10; i < 16; ++i) s[i] = oracle_to_mont(1);
    oracle_tip5_permutation_raw_fast(s);
    for (int i = 0; i < 5; ++i) out[i] = oracle_from_mont(s[i]);
}

/* ------------------------------------------------------------------ parameters */
typedef struct {
    uint32_t log2_expansion, num_checks, num_main, num_aux, num_quot;
} params_t;

enum { MERKLE_ROOT = 0, OOD_MAIN_ROW, OOD_AUX_ROW, OOD_QUOT_SEGMENTS, AUTH_STRUCTURE, MAIN_ROWS, AUX_ROWS,
       LOG2_PADDED_HEIGHT, QUOT_SEGMENTS_ELEMENTS, FRI_CODEWORD, FRI_POLYNOMIAL, FRI_RESPONSE };

/* one decoded item: words [lo, hi) of the item encoding (discriminant first); payload views */
typedef struct {
    uint32_t kind;
    uint64_t lo, hi;
    const uint64_t* pay;  /* first payload element (after counts) */
    uint64_t n;           /* element count / value */
    const uint64_t *leaves, *auth;  /* FRI response */
    uint64_t n_leaves, n_auth;
} item_t;

#define MAX_ITEMS 128

/* decode_item / decode_proof (stark_ref.py): any malformation -> 0 */
static int decode_item(const uint64_t* w, uint64_t lo, uint64_t hi, const params_t* pp, item_t* it) {
    if (lo >= hi) return 0;
    memset(it, 0, sizeof(*it));
    it->kind = (uint32_t)w[lo];
    it->lo = lo;
    it->hi = hi;
    const uint64_t len = hi - lo;
    if (w[lo] >= 12) return 0;
    switch (it->kind) {
        case MERKLE_ROOT: it->pay = w + lo + 1; return len == 6;
        case OOD_MAIN_ROW: it->pay = w + lo + 1; return len == 1 + 3ull * pp->num_main;
        case OOD_AUX_ROW: it->pay = w + lo + 1; return len == 1 + 3ull * pp->num_aux;
        case OOD_QUOT_SEGMENTS: it->pay = w + lo + 1; return len == 1 + 3ull * pp->num_quot;
        case LOG2_PADDED_HEIGHT:
            it->n = len == 2 ? w[lo + 1] : 0;
            return len == 2 && it->n < (1ull << 32);
        default: break;
    }
    if (len < 2) return 0;
    const uint64_t blen = w[lo + 1];
    if (blen != len - 2) return 0;
    const uint64_t b = lo + 2;
    if (it->kind == FRI_RESPONSE) {
        if (blen < 1) return 0;
        const uint64_t lrl = w[b];
        if (lrl < 1 || 1 + lrl > blen) return 0;
        const uint64_t nl = w[b + 1];
        if (3 * (u128)nl != lrl - 1) return 0;
        it->leaves = w + b + 2;
        it->n_leaves = nl;
        const uint64_t pa = b + 1 + lrl;
        if (pa >= b + blen) return 0;
        const uint64_t lau = w[pa];
        if (lau < 1 || 1 + lrl + 1 + lau != blen) return 0;
        const uint64_t na = w[pa + 1];
        if (5 * (u128)na != lau - 1) return 0;
        it->auth = w + pa + 2;
        it->n_auth = na;
        return 1;
    }
    uint64_t width;
    switch (it->kind) {
        case AUTH_STRUCTURE: width = 5; break;
        case MAIN_ROWS: width = pp->num_main; break;
        case AUX_ROWS: width = 3ull * pp->num_aux; break;
        case QUOT_SEGMENTS_ELEMENTS: width = 3ull * pp->num_quot; break;
        default: width = 3; break;  /* FRI_CODEWORD, FRI_POLYNOMIAL */
    }
    if (blen < 1) return 0;
    const uint64_t n = w[b];
    if ((u128)n * width != blen - 1) return 0;
    it->n = n;
    it->pay = w + b + 1;
    return 1;
}

typedef struct {
    const uint64_t* w;
    item_t items[MAX_ITEMS];
    size_t n_items, next;
    sponge sp;
} stream_t;

static int decode_proof(stream_t* ps, const uint64_t* w, size_t len, const params_t* pp) {
    ps->w = w;
    ps->n_items = ps->next = 0;
    if (len < 2 || w[0] != len - 1) return 0;
    const uint64_t n = w[1];
    if (n > MAX_ITEMS) return 0;
    uint64_t pos = 2;
    for (uint64_t i = 0; i < n; ++i) {
        if (pos >= len) return 0;
        const uint64_t ln = w[pos++];
        if (ln > len - pos) return 0;
        if (!decode_item(w, pos, pos + ln, pp, &ps->items[ps->n_items++])) return 0;
        pos += ln;
    }
    return pos == len;
}

/* ProofStream::dequeue: Merkle roots and OOD items are absorbed (INCLUDED_IN_FIAT_SHAMIR) */
static const item_t* dequeue(stream_t* ps, uint32_t kind) {
    if (ps->next >= ps->n_items || ps->items[ps->next].kind != kind) return NULL;
    const item_t* it = &ps->items[ps->next++];
    if (kind <= OOD_QUOT_SEGMENTS) sp_absorb_all(&ps->sp, ps->w + it->lo, it->hi - it->lo);
    return it;
}

/* ------------------------------------------------------------------ Merkle multiproof */
typedef struct { uint64_t node; uint64_t d[5]; } mnode;
static int cmp_desc(const void* a, const void* b) {
    const uint64_t x = ((const mnode*)a)->node, y = ((const mnode*)b)->node;
    return x < y ? 1 : (x > y ? -1 : 0);
}
/* merkle_multiproof_root: leaves (index, digest), authentication structure = missing siblings in
 * descending node-index order (twenty-first MerkleTreeInclusionProof); 1 iff it climbs to root */
static int merkle_verify(const uint64_t root[5], uint32_t h, const uint32_t* idx, const uint64_t* leaf_digests,
                         size_t n, const uint64_t* auth, uint64_t n_auth) {
    if (n == 0 || n > 4096) return 0;
    mnode cur[4096], nxt[4096];
    const uint64_t nl = 1ull << h;
    for (size_t i = 0; i < n; ++i) {
        if (idx[i] >= nl) return 0;
        cur[i].node = idx[i] + nl;
        memcpy(cur[i].d, leaf_digests + 5 * i, 40);
    }
    qsort(cur, n, sizeof(mnode), cmp_desc);
    size_t m = 0;
    for (size_t i = 0; i < n; ++i) {  /* duplicate leaves must carry equal digests */
        if (m && cur[m - 1].node == cur[i].node) {
            if (memcmp(cur[m - 1].d, cur[i].d, 40)) return 0;
            continue;
        }
        cur[m++] = cur[i];
    }
    uint64_t ap = 0;
    while (!(m == 1 && cur[0].node == 1)) {
        size_t k = 0;
        for (size_t i = 0; i < m;) {
            const uint64_t v = cur[i].node;
            const uint64_t *l, *r;
            if (i + 1 < m && cur[i + 1].node == (v ^ 1)) {  /* descending: v = 2q + 1, then 2q */
                l = cur[i + 1].d;
                r = cur[i].d;
                i += 2;
            } else {
                if (ap >= n_auth) return 0;
                const uint64_t* sib = auth + 5 * ap++;
                l = (v & 1) ? sib : cur[i].d;
                r = (v & 1) ? cur[i].d : sib;
                i += 1;
            }
            nxt[k].node = v >> 1;
            hash_pair(l, r, nxt[k].d);
            ++k;
        }
        memcpy(cur, nxt, k * sizeof(mnode));
        m = k;
        if (cur[0].node == 0) return 0;
    }
    return ap == n_auth && memcmp(cur[0].d, root, 40) == 0;
}

/* ------------------------------------------------------------------ AIR as data */
typedef struct {
    uint64_t num_main, num_aux, num_sampled, n_nodes, counts[4];
    const uint64_t* nodes;  /* n_nodes x (op, a, b, c) */
    const uint64_t* cons;
    uint64_t n_cons;
} air_t;

static int air_parse(const uint64_t* w, size_t n, air_t* a) {
    if (n < 9 || w[0] != 0x41495231ull) return 0;
    a->num_main = w[1], a->num_aux = w[2], a->num_sampled = w[3], a->n_nodes = w[4];
    a->n_cons = 0;
    for (int t = 0; t < 4; ++t) a->n_cons += (a->counts[t] = w[5 + t]);
    if (n != 9 + 4 * a->n_nodes + a->n_cons) return 0;
    a->nodes = w + 9;
    a->cons = w + 9 + 4 * a->n_nodes;
    return 1;
}

/* ------------------------------------------------------------------ verifier */
typedef struct {
    const uint64_t* digest;
    uint32_t version;
    const uint64_t *input, *output;
    size_t input_len, output_len;
} claim_t;

static uint32_t log2u(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }

static int verify_one(const params_t* pp, const air_t* air, const claim_t* cl, const uint64_t* raw, size_t len) {
    int ok = 0, zero = 0;
    const size_t M = pp->num_main, A = pp->num_aux, Q = pp->num_quot, k = pp->num_checks;
    uint64_t* w = malloc((len ? len : 1) * 8);
    stream_t* ps = calloc(1, sizeof(stream_t));
    xfe* vals = malloc(air->n_nodes * sizeof(xfe) + 8);
    xfe* smp = malloc((air->num_sampled + 4 + air->n_cons + M + A + Q + 3 + 64) * sizeof(xfe));
    uint64_t* dig = malloc(k * 5 * 8 + 8);
    uint64_t* cw_dig = NULL;
    if (!w || !ps || !vals || !smp || !dig) goto out;
    for (size_t i = 0; i < len; ++i) w[i] = raw[i] >= P ? raw[i] - P : raw[i];
    if (!decode_proof(ps, w, len, pp)) goto out;
    {   /* claim (pinned layout) */
        uint64_t enc[4096];
        size_t e = 0;
        if (cl->input_len + cl->output_len + 10 > 4096) goto out;
        enc[e++] = cl->output_len + 1;
        enc[e++] = cl->output_len;
        for (size_t i = 0; i < cl->output_len; ++i) enc[e++] = cl->output[i] % P;
        enc[e++] = cl->input_len + 1;
        enc[e++] = cl->input_len;
        for (size_t i = 0; i < cl->input_len; ++i) enc[e++] = cl->input[i] % P;
        enc[e++] = cl->version;
        for (int i = 0; i < 5; ++i) enc[e++] = cl->digest[i] % P;
        sp_absorb_all(&ps->sp, enc, e);
    }
    const item_t* lph = dequeue(ps, LOG2_PADDED_HEIGHT);
    if (!lph || lph->n > 28) goto out;
    const uint32_t log2_ph = (uint32_t)lph->n;
    uint64_t T = 1;
    while (T < (1ull << log2_ph) + k + 6) T <<= 1;  /* randomized_trace_len: trace randomizers k + 2*3 */
    const uint32_t log2_N = log2u(T) + pp->log2_expansion;
    const uint64_t N = 1ull << log2_N;
    uint32_t R;
    {
        const uint64_t dim = N >> pp->log2_expansion;
        const uint32_t max_rounds = dim > 1 ? 64u - (uint32_t)__builtin_clzll(dim - 1) : 0u;
        const uint32_t all = log2u(k);
        R = max_rounds > all + 1 ? max_rounds - (all + 1) : 0u;
    }
    if (R > 26 || log2_N > 31) goto out;  /* descriptor bound; sample_indices' u32 upper bound */
    const item_t* main_root = dequeue(ps, MERKLE_ROOT);
    if (!main_root) goto out;
    xfe* chal = smp;
    sp_sample_scalars(&ps->sp, air->num_sampled, chal);
    if (air->num_sampled != NHIP_CHALLENGE_SAMPLE_COUNT) goto out;
    {   /* Challenges::new (stark_ref.derive_challenges): EvalArg terminals folded from 1 with the
           named indeterminates (ChallengeId table: include/nhip_challenge_id.h), appended in
           ChallengeId order: input, output, lookup-table public (over tip5::LOOKUP_TABLE),
           compressed program digest */
        const xfe c_in = chal[NHIP_CH_StandardInputIndeterminate], c_out = chal[NHIP_CH_StandardOutputIndeterminate];
        const xfe c_lut = chal[NHIP_CH_LookupTablePublicIndeterminate];
        const xfe c_dig = chal[NHIP_CH_CompressProgramDigestIndeterminate];
        xfe ein = X1, eout = X1, lut = X1, comp = X1;
        for (size_t i = 0; i < cl->input_len; ++i) ein = xadd(xmul(ein, c_in), xlift(cl->input[i] % P));
        for (size_t i = 0; i < cl->output_len; ++i) eout = xadd(xmul(eout, c_out), xlift(cl->output[i] % P));
        for (uint64_t x = 0; x < 256; ++x) {
            const uint64_t y = x + 1;
            lut = xadd(xmul(lut, c_lut), xlift((y * y % 257u * y % 257u + 256u) % 257u));
        }
        for (int i = 0; i < 5; ++i) comp = xadd(xmul(comp, c_dig), xlift(cl->digest[i] % P));
        chal[air->num_sampled] = ein;
        chal[air->num_sampled + 1] = eout;
        chal[air->num_sampled + 2] = lut;
        chal[air->num_sampled + 3] = comp;
    }
    const item_t* aux_root = dequeue(ps, MERKLE_ROOT);
    if (!aux_root) goto out;
    xfe* quot_w = chal + air->num_sampled + 4;
    sp_sample_scalars(&ps->sp, air->n_cons, quot_w);
    const item_t* quot_root = dequeue(ps, MERKLE_ROOT);
    if (!quot_root) goto out;
    xfe z;
    sp_sample_scalars(&ps->sp, 1, &z);
    const uint64_t w_tr = root_of_unity(log2_ph);
    const xfe z_next = xscale(z, w_tr);
    xfe z_pow = X1;
    for (size_t q = 0; q < Q; ++q) z_pow = xmul(z_pow, z);
    const item_t* mc = dequeue(ps, OOD_MAIN_ROW);
    const item_t* ac = dequeue(ps, OOD_AUX_ROW);
    const item_t* mn = dequeue(ps, OOD_MAIN_ROW);
    const item_t* an = dequeue(ps, OOD_AUX_ROW);
    const item_t* qs = dequeue(ps, OOD_QUOT_SEGMENTS);
    if (!mc || !ac || !mn || !an || !qs) goto out;
    xfe zinv[4];
    {   /* zerofier_inverses */
        const uint64_t w_inv = finv(w_tr);
        zinv[0] = xinv(xsub(z, X1), &zero);
        xfe zph = z;
        for (uint32_t q = 0; q < log2_ph; ++q) zph = xmul(zph, zph);
        zinv[1] = xinv(xsub(zph, X1), &zero);
        const xfe except_last = xsub(z, xlift(w_inv));
        zinv[2] = xmul(except_last, zinv[1]);
        zinv[3] = xinv(except_last, &zero);
        if (zero) goto out;
    }
    /* AIR evaluation at the OOD rows */
    for (uint64_t i = 0; i < air->n_nodes; ++i) {
        const uint64_t* nd = air->nodes + 4 * i;
        xfe v;
        switch (nd[0]) {
            case 0: {
                const uint64_t kind = nd[1], x = nd[2];
                if (kind == 0 && x < M) v = xld(mc->pay + 3 * x);
                else if (kind == 1 && x < A) v = xld(ac->pay + 3 * x);
                else if (kind == 2 && x < M) v = xld(mn->pay + 3 * x);
                else if (kind == 3 && x < A) v = xld(an->pay + 3 * x);
                else if (kind == 4 && x < air->num_sampled + 4) v = chal[x];
                else goto out;
                break;
            }
            case 1: v = (xfe){{nd[1], nd[2], nd[3]}}; break;
            case 2: if (nd[1] >= i || nd[2] >= i) goto out; v = xadd(vals[nd[1]], vals[nd[2]]); break;
            case 3: if (nd[1] >= i || nd[2] >= i) goto out; v = xsub(vals[nd[1]], vals[nd[2]]); break;
            case 4: if (nd[1] >= i || nd[2] >= i) goto out; v = xmul(vals[nd[1]], vals[nd[2]]); break;
            default: goto out;
        }
        vals[i] = v;
    }
    {
        xfe ood_q = X0;
        uint64_t c = 0;
        for (int t = 0; t < 4; ++t)
            for (uint64_t j = 0; j < air->counts[t]; ++j, ++c) {
                if (air->cons[c] >= air->n_nodes) goto out;
                ood_q = xadd(ood_q, xmul(quot_w[c], xmul(vals[air->cons[c]], zinv[t])));
            }
        xfe seg = X0, zk = X1;
        for (size_t q = 0; q < Q; ++q) {
            seg = xadd(seg, xmul(zk, xld(qs->pay + 3 * q)));
            zk = xmul(zk, z);
        }
        if (!xeq(seg, ood_q)) goto out;
    }
    xfe* lw = quot_w + air->n_cons;
    sp_sample_scalars(&ps->sp, M + A + Q + 3, lw);
    xfe ood_cur = X0, ood_nxt = X0, ood_q_lin = X0;
    for (size_t c = 0; c < M; ++c) {
        ood_cur = xadd(ood_cur, xmul(lw[c], xld(mc->pay + 3 * c)));
        ood_nxt = xadd(ood_nxt, xmul(lw[c], xld(mn->pay + 3 * c)));
    }
    for (size_t c = 0; c < A; ++c) {
        ood_cur = xadd(ood_cur, xmul(lw[M + c], xld(ac->pay + 3 * c)));
        ood_nxt = xadd(ood_nxt, xmul(lw[M + c], xld(an->pay + 3 * c)));
    }
    for (size_t q = 0; q < Q; ++q) ood_q_lin = xadd(ood_q_lin, xmul(lw[M + A + q], xld(qs->pay + 3 * q)));
    /* ---- fri_verify */
    const item_t* fr_root[41];
    xfe alpha[41];
    for (uint32_t r = 0; r <= R; ++r) {
        if (!(fr_root[r] = dequeue(ps, MERKLE_ROOT))) goto out;
        if (r < R) sp_sample_scalars(&ps->sp, 1, &alpha[r]);
    }
    const item_t* last_cw = dequeue(ps, FRI_CODEWORD);
    const item_t* last_poly = dequeue(ps, FRI_POLYNOMIAL);
    if (!last_cw || !last_poly) goto out;
    uint32_t* idx = malloc(k * 4 * 3 + 16);
    xfe* a = malloc(k * sizeof(xfe) + 8);
    if (!idx || !a) { free(idx); free(a); goto out; }
    uint32_t* ai = idx + k;
    uint32_t* bi = idx + 2 * k;
    sp_sample_indices(&ps->sp, N, k, idx);
    int fri_ok = 1;
    const uint64_t* leaves0 = NULL;
    const uint64_t g0 = root_of_unity(log2_N);
    for (uint32_t r = 0; fri_ok && r <= R; ++r) {
        const item_t* resp = dequeue(ps, FRI_RESPONSE);
        if (!resp || resp->n_leaves != k) { fri_ok = 0; break; }
        const uint64_t n_r = N >> (r == 0 ? 0 : r - 1);
        const uint32_t h = log2_N - (r == 0 ? 0 : r - 1);
        uint64_t* ld = malloc(k * 40);
        if (!ld) { fri_ok = 0; break; }
        for (size_t j = 0; j < k; ++j) {
            ai[j] = (uint32_t)(idx[j] % n_r);
            bi[j] = (uint32_t)((idx[j] + n_r / 2) % n_r);
            ld[5 * j] = resp->leaves[3 * j], ld[5 * j + 1] = resp->leaves[3 * j + 1];
            ld[5 * j + 2] = resp->leaves[3 * j + 2], ld[5 * j + 3] = 0, ld[5 * j + 4] = 0;
        }
        /* round 0: a-values of round 0; response r >= 1: b-values of round r - 1 */
        const uint64_t* root = fr_root[r == 0 ? 0 : r - 1]->pay;
        fri_ok = merkle_verify(root, h, r == 0 ? ai : bi, ld, k, resp->auth, resp->n_auth);
        free(ld);
        if (!fri_ok) break;
        if (r == 0) {
            leaves0 = resp->leaves;
            for (size_t j = 0; j < k; ++j) a[j] = xld(resp->leaves + 3 * j);
        } else {
            /* fold round r - 1: colinear_y((x_a, a), (x_b, b), alpha) */
            const uint32_t rr = r - 1;
            const uint64_t off = fpow(7, 1ull << rr), gen = fpow(g0, 1ull << rr);
            for (size_t j = 0; j < k; ++j) {
                const uint64_t xa = fmul(off, fpow(gen, ai[j])), xb = fmul(off, fpow(gen, bi[j]));
                const xfe b = xld(resp->leaves + 3 * j);
                const xfe slope = xscale(xsub(b, a[j]), finv(fsub(xb, xa)));
                a[j] = xadd(a[j], xmul(slope, xsub(alpha[rr], xlift(xa))));
            }
        }
    }
    if (fri_ok) {
        /* last codeword: Merkle root, agreement, degree, barycentric == Horner at a fresh point */
        const uint64_t L = last_cw->n;
        if (L != (N >> R)) fri_ok = 0;
        cw_dig = fri_ok ? malloc(2 * L * 40) : NULL;
        if (fri_ok && !cw_dig) fri_ok = 0;
        if (fri_ok) {
            uint64_t* nodes = cw_dig;  /* heap order, leaves at L..2L-1 */
            for (uint64_t i = 0; i < L; ++i) {
                uint64_t* d = nodes + 5 * (L + i);
                d[0] = last_cw->pay[3 * i], d[1] = last_cw->pay[3 * i + 1], d[2] = last_cw->pay[3 * i + 2];
                d[3] = 0, d[4] = 0;
            }
            for (uint64_t v = L - 1; v >= 1; --v) hash_pair(nodes + 5 * (2 * v), nodes + 5 * (2 * v + 1), nodes + 5 * v);
            if (memcmp(nodes + 5 * (L > 1 ? 1 : L), fr_root[R]->pay, 40)) fri_ok = 0;
        }
        for (size_t j = 0; fri_ok && j < k; ++j)
            if (!xeq(xld(last_cw->pay + 3 * (idx[j] % (N >> R))), a[j])) fri_ok = 0;
        if (fri_ok) {
            int64_t deg = -1;
            for (uint64_t c = 0; c < last_poly->n; ++c)
                if (last_poly->pay[3 * c] | last_poly->pay[3 * c + 1] | last_poly->pay[3 * c + 2]) deg = (int64_t)c;
            const uint64_t last_max = ((N >> pp->log2_expansion) - 1) >> R;
            if (deg > (int64_t)last_max) fri_ok = 0;
        }
        if (fri_ok) {
            xfe t;
            sp_sample_scalars(&ps->sp, 1, &t);
            xfe h = X0;
            for (uint64_t c = last_poly->n; c-- > 0;) h = xadd(xmul(h, t), xld(last_poly->pay + 3 * c));
            const uint64_t wL = root_of_unity(log2u(L));
            xfe num = X0, den = X0;
            uint64_t wi = 1;
            for (uint64_t i = 0; i < L; ++i, wi = fmul(wi, wL)) {
                const xfe q = xscale(xinv(xsub(t, xlift(wi)), &zero), wi);
                num = xadd(num, xmul(q, xld(last_cw->pay + 3 * i)));
                den = xadd(den, q);
            }
            if (zero || xzero(den)) fri_ok = 0;
            else if (!xeq(h, xmul(num, xinv(den, &zero)))) fri_ok = 0;
        }
    }
    if (!fri_ok) { free(idx); free(a); goto out; }
    /* ---- revealed rows: hash, authenticate, DEEP */
    const item_t *mrows = dequeue(ps, MAIN_ROWS), *mauth = dequeue(ps, AUTH_STRUCTURE);
    const item_t *arows = dequeue(ps, AUX_ROWS), *aauth = dequeue(ps, AUTH_STRUCTURE);
    const item_t *qrows = dequeue(ps, QUOT_SEGMENTS_ELEMENTS), *qauth = dequeue(ps, AUTH_STRUCTURE);
    int rows_ok = mrows && mauth && arows && aauth && qrows && qauth && mrows->n == k && arows->n == k && qrows->n == k;
    const item_t* rr[3] = {mrows, arows, qrows};
    const item_t* au[3] = {mauth, aauth, qauth};
    const item_t* roots[3] = {main_root, aux_root, quot_root};
    const size_t width[3] = {M, 3 * A, 3 * Q};
    for (int t = 0; rows_ok && t < 3; ++t) {
        for (size_t j = 0; j < k; ++j) hash_varlen(rr[t]->pay + width[t] * j, width[t], dig + 5 * j);
        rows_ok = merkle_verify(roots[t]->pay, log2_N, idx, dig, k, au[t]->pay, au[t]->n);
    }
    for (size_t j = 0; rows_ok && j < k; ++j) {
        const uint64_t x = fmul(7, fpow(g0, idx[j]));
        xfe mav = X0, qv = X0;
        const uint64_t* mr = mrows->pay + M * j;
        const uint64_t* ar = arows->pay + 3 * A * j;
        for (size_t c = 0; c < M; ++c) mav = xadd(mav, xscale(lw[c], mr[c]));
        for (size_t c = 0; c < A; ++c) mav = xadd(mav, xmul(lw[M + c], xld(ar + 3 * c)));
        for (size_t q = 0; q < Q; ++q) qv = xadd(qv, xmul(lw[M + A + q], xld(qrows->pay + 3 * Q * j + 3 * q)));
        const xfe t0 = xmul(xsub(mav, ood_cur), xinv(xsub(xlift(x), z), &zero));
        const xfe t1 = xmul(xsub(mav, ood_nxt), xinv(xsub(xlift(x), z_next), &zero));
        const xfe t2 = xmul(xsub(qv, ood_q_lin), xinv(xsub(xlift(x), z_pow), &zero));
        const xfe deep = xadd(xadd(xmul(t0, lw[M + A + Q]), xmul(t1, lw[M + A + Q + 1])), xmul(t2, lw[M + A + Q + 2]));
        if (zero || !xeq(deep, xld(leaves0 + 3 * j))) rows_ok = 0;  /* == the FRI round-0 leaf */
    }
    free(idx);
    free(a);
    if (!rows_ok) goto out;
    ok = ps->next == ps->n_items;  /* no items left */
out:
    free(w);
    free(ps);
    free(vals);
    free(smp);
    free(dig);
    free(cw_dig);
    return ok;
}

/* ------------------------------------------------------------------ batch driver */
typedef struct {
    const params_t* pp;
    const air_t* air;
    const claim_t* claims;
    const uint64_t* const* proofs;
    const size_t* lens;
    size_t n;
    uint8_t* verdicts;
    size_t next;
    pthread_mutex_t mu;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const size_t i = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (i >= j->n) return NULL;
        j->verdicts[i] = (uint8_t)verify_one(j->pp, j->air, &j->claims[i], j->proofs[i], j->lens[i]);
    }
}

/* Verify n proofs on `threads` host threads.  params: [log2_expansion, num_checks, num_main, num_aux,
 * num_quot]; claims: digests[n][5], versions[n], inputs / outputs as flat arrays with offsets[n+1].
 * Returns 0, or -1 for a malformed AIR. */
int oracle_stark_verify_batch(const uint64_t* air_words, size_t n_air, const uint32_t* params,
                              const uint64_t* digests, const uint32_t* versions, const uint64_t* in_data,
                              const uint64_t* in_off, const uint64_t* out_data, const uint64_t* out_off,
                              const uint64_t* proof_data, const uint64_t* proof_off, size_t n, uint8_t* verdicts,
                              int threads) {
    air_t air;
    if (!air_parse(air_words, n_air, &air)) return -1;
    params_t pp = {params[0], params[1], params[2], params[3], params[4]};
    if (air.num_main != pp.num_main || air.num_aux != pp.num_aux || pp.num_checks < 1 || pp.num_checks > 4096) return -1;
    claim_t* cl = calloc(n ? n : 1, sizeof(claim_t));
    const uint64_t** pr = calloc(n ? n : 1, sizeof(uint64_t*));
    size_t* ln = calloc(n ? n : 1, sizeof(size_t));
    if (!cl || !pr || !ln) return -1;
    for (size_t i = 0; i < n; ++i) {
        cl[i].digest = digests + 5 * i;
        cl[i].version = versions[i];
        cl[i].input = in_data + in_off[i];
        cl[i].input_len = in_off[i + 1] - in_off[i];
        cl[i].output = out_data + out_off[i];
        cl[i].output_len = out_off[i + 1] - out_off[i];
        pr[i] = proof_data + proof_off[i];
        ln[i] = proof_off[i + 1] - proof_off[i];
    }
    job_t j = {&pp, &air, cl, pr, ln, n, verdicts, 0, PTHREAD_MUTEX_INITIALIZER};
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &j);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(cl);
    free(pr);
    free(ln);
    return 0;
}
