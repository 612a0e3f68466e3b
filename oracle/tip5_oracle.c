/*
 * C restatement of Tip5 / Goldilocks / MTree — TEST ORACLE AND CPU BASELINE ONLY.
 *
 * Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle_tip5.so, and only as the checker or as
 * the timed CPU baseline.  The shipped library (neptune-core_amd/) never
 * links or calls it.
 *
 * Restates (crates not vendored in /root/reference; versions from Cargo.lock):
 *   - twenty-first 1.0.0 (Cargo.lock:4297) BFieldElement in Montgomery form
 *     (R = 2^64, `montyred`), Tip5 permutation (split-and-lookup on the raw
 *     Montgomery bytes of state[0..4], x^7 on state[4..16], circulant MDS
 *     out[i] = sum_j c[(i-j)&15]*in[j], round constants), Tip5 sponge
 *     (FixedLength domain: capacity = 1; VariableLength: zeros, pad [1,0,..]).
 *   - neptune-core MTree::verify, neptune-core/src/protocol/consensus/block/pow.rs:162-180
 *     and MTree::build_inplace, pow.rs:73-119 (node i -> children 2i, 2i+1).
 * Pinned by KAT-V (state/wallet/mod.rs:1379-1383) and KAT-F
 * (test_data/precalculated_pow_solution.json); see tests/test_oracle_kat.py.
 *
 * This file deliberately mirrors the Montgomery-form arithmetic of the
 * reference (the Python oracle works in canonical form), so the two oracles
 * cross-check each other.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#define P 0xFFFFFFFF00000001ull
typedef unsigned __int128 u128;

/* raw Montgomery values of the 80 round constants (filled by oracle_init) */
static uint64_t RC_RAW[80];
static const uint8_t *LUT;
static uint8_t LUT_STORE[256];
static const uint64_t MDS[16] = {61402, 1108, 28750, 33823, 7454, 43244, 53865, 12034,
                                 56951, 27521, 41351, 40901, 12021, 59689, 26798, 17845};
static int initialised = 0;
/* MDS_COL[j][i] = MDS[(i - j) & 15]: column j of the circulant (the AVX2 accumulation below) */
static uint64_t MDS_COL[16][16];
static int have_avx2 = 0;

/* twenty-first montyred: x (< p * 2^64) -> x * 2^-64 mod p, result in [0, p) */
static inline uint64_t montyred(u128 x) {
    uint64_t xl = (uint64_t)x, xh = (uint64_t)(x >> 64);
    uint64_t a = xl + (xl << 32);
    uint64_t e = a < xl;
    uint64_t b = a - (a >> 32) - e;
    uint64_t r = xh - b;
    uint64_t c = xh < b;
    return r - ((uint64_t)(uint32_t)(0u - (uint32_t)c));
}
static inline uint64_t mmul(uint64_t a, uint64_t b) { return montyred((u128)a * b); }
static inline uint64_t madd(uint64_t a, uint64_t b) {
    uint64_t x1 = a - (P - b);
    return (a < (P - b)) ? x1 + P : x1;
}
static const uint64_t R2 = 0xFFFFFFFE00000001ull; /* 2^128 mod p */
static inline uint64_t to_mont(uint64_t x) { return mmul(x, R2); }
static inline uint64_t from_mont(uint64_t r) { return montyred((u128)r); }

/* Round constants are supplied by the caller (derived in Python via BLAKE3 and
 * checked against the KATs) as raw Montgomery values. */
void oracle_init(const uint64_t rc_raw[80]) {
    for (int x = 0; x < 256; ++x) {
        unsigned y = (unsigned)x + 1u;
        LUT_STORE[x] = (uint8_t)(((y * y % 257u) * y % 257u + 256u) % 257u);
    }
    LUT = LUT_STORE;
    memcpy(RC_RAW, rc_raw, sizeof(RC_RAW));
    for (int j = 0; j < 16; ++j)
        for (int i = 0; i < 16; ++i) MDS_COL[j][i] = MDS[(i - j) & 15];
#if defined(__x86_64__)
    __builtin_cpu_init();
    have_avx2 = __builtin_cpu_supports("avx2");
#endif
    initialised = 1;
}

/* permutation on raw Montgomery state */
static void perm_raw(uint64_t s[16]) {
    for (int r = 0; r < 5; ++r) {
        for (int i = 0; i < 4; ++i) {
            uint64_t v = s[i], o = 0;
            for (int k = 0; k < 8; ++k) o |= (uint64_t)LUT[(v >> (8 * k)) & 0xFF] << (8 * k);
            s[i] = o;
        }
        for (int i = 4; i < 16; ++i) {
            uint64_t x = s[i], x2 = mmul(x, x), x4 = mmul(x2, x2);
            s[i] = mmul(mmul(x, x2), x4);
        }
        uint64_t t[16];
        for (int i = 0; i < 16; ++i) {
            u128 acc = 0;
            for (int j = 0; j < 16; ++j) acc += (u128)MDS[(i - j) & 15] * s[j];
            t[i] = (uint64_t)(acc % P);
        }
        for (int i = 0; i < 16; ++i) s[i] = madd(t[i], RC_RAW[r * 16 + i]);
    }
}

/* MDS accumulators of twenty-first's split form: al[i] = sum_j c[(i-j)&15] * lo32(s[j]),
 * ah[i] = the same over hi32(s[j]); each < 2^53, so plain 64-bit sums are exact. */
static inline void mds_acc_scalar(const uint64_t s[16], uint64_t al[16], uint64_t ah[16]) {
    for (int i = 0; i < 16; ++i) {
        uint64_t a = 0, h = 0;
        for (int j = 0; j < 16; ++j) {
            a += MDS[(i - j) & 15] * (s[j] & 0xFFFFFFFFull);
            h += MDS[(i - j) & 15] * (s[j] >> 32);
        }
        al[i] = a;
        ah[i] = h;
    }
}

#if defined(__x86_64__)
/* The same sums with AVX2: column j of the circulant times the broadcast 32-bit half of s[j]
 * (vpmuludq: 32 x 32 -> 64 per lane), 16 outputs in four 4-lane accumulators per half.  Selected
 * at run time (oracle_init) when the host has AVX2; tests/test_stark_oracle_c.py checks the fast
 * permutation against perm_raw either way. */
__attribute__((target("avx2"))) static inline void mds_acc_avx2(const uint64_t s[16], uint64_t al[16], uint64_t ah[16]) {
    __m256i a0 = _mm256_setzero_si256(), a1 = a0, a2 = a0, a3 = a0, h0 = a0, h1 = a0, h2 = a0, h3 = a0;
    for (int j = 0; j < 16; ++j) {
        const __m256i lo = _mm256_set1_epi64x((long long)(s[j] & 0xFFFFFFFFull));
        const __m256i hi = _mm256_set1_epi64x((long long)(s[j] >> 32));
        const __m256i m0 = _mm256_loadu_si256((const __m256i *)&MDS_COL[j][0]);
        const __m256i m1 = _mm256_loadu_si256((const __m256i *)&MDS_COL[j][4]);
        const __m256i m2 = _mm256_loadu_si256((const __m256i *)&MDS_COL[j][8]);
        const __m256i m3 = _mm256_loadu_si256((const __m256i *)&MDS_COL[j][12]);
        a0 = _mm256_add_epi64(a0, _mm256_mul_epu32(m0, lo));
        h0 = _mm256_add_epi64(h0, _mm256_mul_epu32(m0, hi));
        a1 = _mm256_add_epi64(a1, _mm256_mul_epu32(m1, lo));
        h1 = _mm256_add_epi64(h1, _mm256_mul_epu32(m1, hi));
        a2 = _mm256_add_epi64(a2, _mm256_mul_epu32(m2, lo));
        h2 = _mm256_add_epi64(h2, _mm256_mul_epu32(m2, hi));
        a3 = _mm256_add_epi64(a3, _mm256_mul_epu32(m3, lo));
        h3 = _mm256_add_epi64(h3, _mm256_mul_epu32(m3, hi));
    }
    _mm256_storeu_si256((__m256i *)&al[0], a0);
    _mm256_storeu_si256((__m256i *)&al[4], a1);
    _mm256_storeu_si256((__m256i *)&al[8], a2);
    _mm256_storeu_si256((__m256i *)&al[12], a3);
    _mm256_storeu_si256((__m256i *)&ah[0], h0);
    _mm256_storeu_si256((__m256i *)&ah[4], h1);
    _mm256_storeu_si256((__m256i *)&ah[8], h2);
    _mm256_storeu_si256((__m256i *)&ah[12], h3);
}
#endif

/* The same permutation with twenty-first's MDS arithmetic (split into 32-bit halves, 64-bit
 * accumulation, s = lo + hi * 2^32 reduced as s_lo + s_hi * (2^32 - 1) with the overflow fix, then
 * BFieldElement addition of the round constant), used by the STARK oracle (stark_oracle.c) where
 * speed matters (the CPU baseline); tests/test_stark_oracle_c.py checks it against perm_raw.
 * The 12 x^7 chains are written stage by stage so the independent products overlap.  One body,
 * compiled twice (MDS sums scalar, or AVX2 for hosts that have it; chosen per call). */
#define TIP5_FAST_BODY(MDS_ACC)                                                          \
    for (int r = 0; r < 5; ++r) {                                                        \
        for (int i = 0; i < 4; ++i) {                                                    \
            uint64_t v = s[i], o = 0;                                                    \
            for (int k = 0; k < 8; ++k) o |= (uint64_t)LUT[(v >> (8 * k)) & 0xFF] << (8 * k); \
            s[i] = o;                                                                    \
        }                                                                                \
        uint64_t x2[12], x3[12], x4[12];                                                 \
        for (int i = 0; i < 12; ++i) x2[i] = mmul(s[4 + i], s[4 + i]);                   \
        for (int i = 0; i < 12; ++i) {                                                   \
            x4[i] = mmul(x2[i], x2[i]);                                                  \
            x3[i] = mmul(x2[i], s[4 + i]);                                               \
        }                                                                                \
        for (int i = 0; i < 12; ++i) s[4 + i] = mmul(x3[i], x4[i]);                      \
        uint64_t al[16], ah[16];                                                         \
        MDS_ACC(s, al, ah);                                                              \
        for (int i = 0; i < 16; ++i) {                                                   \
            const u128 sum = (u128)al[i] + ((u128)ah[i] << 32);                          \
            const uint64_t s_lo = (uint64_t)sum, s_hi = (uint64_t)(sum >> 64);           \
            uint64_t res = s_lo + s_hi * 0xFFFFFFFFull;                                  \
            if (res < s_lo) res += 0xFFFFFFFFull;                                        \
            const uint64_t q = P - RC_RAW[r * 16 + i];                                   \
            uint64_t x1 = res - q;                                                       \
            if (res < q) x1 -= 0xFFFFFFFFull; /* BFieldElement add: borrow -> + p */     \
            s[i] = x1;                                                                   \
        }                                                                                \
    }

static void perm_fast_scalar(uint64_t s[16]) { TIP5_FAST_BODY(mds_acc_scalar) }
#if defined(__x86_64__)
__attribute__((target("avx2"))) static void perm_fast_avx2(uint64_t s[16]) { TIP5_FAST_BODY(mds_acc_avx2) }
#endif

/* Select the MDS form of the fast permutation (tests: both forms against perm_raw); AVX2 only where
 * the host has it.  Returns the form in use afterwards (1 = AVX2). */
int oracle_set_mds_avx2(int on) {
#if defined(__x86_64__)
    __builtin_cpu_init();
    have_avx2 = on && __builtin_cpu_supports("avx2");
#else
    (void)on;
#endif
    return have_avx2;
}

void oracle_tip5_permutation_raw_fast(uint64_t s[16]) {
#if defined(__x86_64__)
    if (have_avx2) {
        perm_fast_avx2(s);
        return;
    }
#endif
    perm_fast_scalar(s);
}
/* Any u64 (read mod p) -> raw Montgomery word x * 2^64 mod p without a division: with x = h*2^32 + l
 * and 2^64 == 2^32 - 1, x * 2^64 == l*2^32 - h - l, an integer in (-2^33, p - 1], so one conditional
 * + p makes it canonical (the same word as to_mont(x % P); tests/test_stark_oracle_c.py). */
uint64_t oracle_to_mont(uint64_t x) {
    const uint64_t l = x & 0xFFFFFFFFull, h = x >> 32;
    const uint64_t sum = h + l, t = l << 32, v = t - sum;
    return t < sum ? v + P : v;
}
uint64_t oracle_from_mont(uint64_t r) { return from_mont(r); }
void oracle_tip5_permutation_raw(uint64_t s[16]) { perm_raw(s); }

/* canonical in / canonical out */
void oracle_tip5_permutation(uint64_t s[16]) {
    for (int i = 0; i < 16; ++i) s[i] = to_mont(s[i] % P);
    perm_raw(s);
    for (int i = 0; i < 16; ++i) s[i] = from_mont(s[i]);
}

void oracle_hash_pair(const uint64_t l[5], const uint64_t r[5], uint64_t out[5]) {
    uint64_t s[16];
    for (int i = 0; i < 5; ++i) { s[i] = l[i]; s[5 + i] = r[i]; }
    for (int i = 10; i < 16; ++i) s[i] = 1;
    oracle_tip5_permutation(s);
    memcpy(out, s, 5 * sizeof(uint64_t));
}

void oracle_hash_varlen(const uint64_t *data, size_t len, uint64_t out[5]) {
    uint64_t s[16] = {0};
    size_t k = 0;
    for (; k + 10 <= len; k += 10) {
        for (int i = 0; i < 10; ++i) s[i] = to_mont(data[k + i] % P);
        perm_raw(s);
    }
    size_t rem = len - k;
    for (size_t i = 0; i < 10; ++i) {
        uint64_t v = i < rem ? data[k + i] % P : (i == rem ? 1 : 0);
        s[i] = to_mont(v);
    }
    perm_raw(s);
    for (int i = 0; i < 5; ++i) out[i] = from_mont(s[i]);
}

/* The same sponge split in two (test-data generators: rows that share a long constant prefix).
 * oracle_sponge_absorb_chunks: the raw Montgomery state of the VariableLength sponge after absorbing
 * nchunks full rate chunks of data; oracle_hash_varlen_resume: hash_varlen of (those chunks ++ tail)
 * continued from that state (tail absorbed and padded as oracle_hash_varlen does).  Both use the
 * split-form permutation (bit-exact with perm_raw, tests/test_stark_oracle_c.py). */
void oracle_sponge_absorb_chunks(const uint64_t *data, size_t nchunks, uint64_t s_raw[16]) {
    memset(s_raw, 0, 16 * sizeof(uint64_t));
    for (size_t c = 0; c < nchunks; ++c) {
        for (int i = 0; i < 10; ++i) s_raw[i] = to_mont(data[10 * c + i] % P);
        oracle_tip5_permutation_raw_fast(s_raw);
    }
}
void oracle_hash_varlen_resume(const uint64_t s_raw[16], const uint64_t *tail, size_t len, uint64_t out[5]) {
    uint64_t s[16];
    memcpy(s, s_raw, sizeof(s));
    size_t k = 0;
    for (; k + 10 <= len; k += 10) {
        for (int i = 0; i < 10; ++i) s[i] = to_mont(tail[k + i] % P);
        oracle_tip5_permutation_raw_fast(s);
    }
    const size_t rem = len - k;
    for (size_t i = 0; i < 10; ++i) s[i] = to_mont(i < rem ? tail[k + i] % P : (i == rem ? 1 : 0));
    oracle_tip5_permutation_raw_fast(s);
    for (int i = 0; i < 5; ++i) out[i] = from_mont(s[i]);
}
/* hash_pair with the split-form permutation */
void oracle_hash_pair_fast(const uint64_t l[5], const uint64_t r[5], uint64_t out[5]) {
    uint64_t s[16];
    for (int i = 0; i < 5; ++i) { s[i] = to_mont(l[i] % P); s[5 + i] = to_mont(r[i] % P); }
    for (int i = 10; i < 16; ++i) s[i] = to_mont(1);
    oracle_tip5_permutation_raw_fast(s);
    for (int i = 0; i < 5; ++i) out[i] = from_mont(s[i]);
}

void oracle_hash_varlen_batch(const uint64_t *data, const uint64_t *offsets, size_t n, uint64_t *out) {
    for (size_t i = 0; i < n; ++i)
        oracle_hash_varlen(data + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), out + 5 * i);
}

/* pow.rs:162-180 */
int oracle_mtree_verify(const uint64_t root[5], uint64_t index, const uint64_t *path, uint32_t depth,
                        const uint64_t leaf[5]) {
    uint64_t bound = 1ull << (depth & 63);
    if (index > bound) return 0;
    uint64_t run[5], tmp[5];
    memcpy(run, leaf, sizeof(run));
    uint64_t ri = index;
    for (uint32_t k = 0; k < depth; ++k) {
        const uint64_t *sib = path + 5 * (size_t)k;
        if (ri & 1) oracle_hash_pair(sib, run, tmp);
        else oracle_hash_pair(run, sib, tmp);
        memcpy(run, tmp, sizeof(run));
        ri >>= 1;
    }
    for (int i = 0; i < 5; ++i)
        if (run[i] != root[i] % P) return 0;
    return 1;
}

typedef struct {
    const uint64_t *roots; size_t n_roots; const uint64_t *indices; const uint64_t *leaves;
    const uint64_t *paths; uint32_t depth; size_t begin, end; uint8_t *verdicts;
} mt_job;

static void *mt_worker(void *arg) {
    mt_job *j = (mt_job *)arg;
    for (size_t i = j->begin; i < j->end; ++i) {
        const uint64_t *root = j->roots + 5 * (j->n_roots == 1 ? 0 : i);
        j->verdicts[i] = (uint8_t)oracle_mtree_verify(root, j->indices[i], j->paths + 5 * (size_t)j->depth * i,
                                                      j->depth, j->leaves + 5 * i);
    }
    return NULL;
}

/* Batched MTree::verify with nthreads POSIX threads (CPU baseline). */
void oracle_mtree_verify_batch(const uint64_t *roots, size_t n_roots, const uint64_t *indices,
                               const uint64_t *leaves, const uint64_t *paths, uint32_t depth, size_t n,
                               uint8_t *verdicts, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256];
    mt_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    int used = 0;
    for (int t = 0; t < nthreads; ++t) {
        size_t b = (size_t)t * per, e = b + per > n ? n : b + per;
        if (b >= e) break;
        jobs[t] = (mt_job){roots, n_roots, indices, leaves, paths, depth, b, e, verdicts};
        pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
        ++used;
    }
    for (int t = 0; t < used; ++t) pthread_join(th[t], NULL);
}

/* pow.rs MTree::build_inplace: nodes[1] = root, node i = hash_pair(node 2i, node 2i+1),
 * leaves are virtual nodes n..2n-1.  nodes has n*5 words ([0..5) unused). */
void oracle_mtree_build(const uint64_t *leaves, size_t n, uint64_t *nodes) {
    memset(nodes, 0, 5 * sizeof(uint64_t));
    for (size_t i = n / 2; i < n; ++i)
        oracle_hash_pair(leaves + 5 * (2 * i - n), leaves + 5 * (2 * i - n + 1), nodes + 5 * i);
    for (size_t i = n / 2; i-- > 1;) oracle_hash_pair(nodes + 5 * (2 * i), nodes + 5 * (2 * i + 1), nodes + 5 * i);
}

int oracle_is_initialised(void) { return initialised; }
