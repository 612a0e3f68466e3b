/*
 * Vectorised Goldilocks helpers for the oracle's fast synthetic prover — TEST DATA GENERATOR ONLY.
 *
 * Canonical u64 arithmetic mod p = 2^64 - 2^32 + 1 over arrays, multi-threaded with POSIX threads.
 * Used by oracle/stark_prover_fast.py to build large synthetic proofs (BASELINE configs 3-5); the
 * verifier oracle and the product never call this file.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define P 0xFFFFFFFF00000001ull
typedef unsigned __int128 u128;

static inline uint64_t red128(u128 x) {
    uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
    uint64_t hl = hi & 0xFFFFFFFFull, hh = hi >> 32;
    /* x = lo + hl*2^64 + hh*2^96 == lo + hl*(2^32-1) - hh */
    uint64_t t = lo - hh;
    if (lo < hh) t += P; /* borrow: add p (mod 2^64 this is - (2^32 - 1)) */
    uint64_t u = (hl << 32) - hl;
    uint64_t s = t + u;
    if (s < t) s += 0xFFFFFFFFull;
    if (s >= P) s -= P;
    return s;
}
static inline uint64_t mulm(uint64_t a, uint64_t b) { return red128((u128)a * b); }
static inline uint64_t addm(uint64_t a, uint64_t b) {
    uint64_t s = a + b;
    if (s < a) s += 0xFFFFFFFFull;
    if (s >= P) s -= P;
    return s;
}
static inline uint64_t subm(uint64_t a, uint64_t b) { return a >= b ? a - b : a + P - b; }

typedef void (*range_fn)(void *ctx, size_t lo, size_t hi);
typedef struct { range_fn f; void *ctx; size_t lo, hi; } job_t;
static void *runner(void *a) {
    job_t *j = (job_t *)a;
    j->f(j->ctx, j->lo, j->hi);
    return NULL;
}
static void parallel_for(size_t n, int threads, range_fn f, void *ctx) {
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if ((size_t)threads > n / 4096 + 1) threads = (int)(n / 4096 + 1);
    pthread_t th[64];
    job_t jb[64];
    jb[0] = (job_t){f, ctx, 0, 0};
    size_t per = (n + (size_t)threads - 1) / (size_t)threads;
    int used = 0;
    for (int t = 0; t < threads; ++t) {
        size_t lo = (size_t)t * per, hi = lo + per > n ? n : lo + per;
        if (lo >= hi) break;
        jb[t] = (job_t){f, ctx, lo, hi};
        if (t == 0) continue;
        pthread_create(&th[t], NULL, runner, &jb[t]);
        ++used;
    }
    if (n) f(ctx, jb[0].lo, jb[0].hi);
    for (int t = 1; t <= used; ++t) pthread_join(th[t], NULL);
}

/* ---- elementwise */
typedef struct { const uint64_t *a, *b; uint64_t *o; uint64_t c; int op; } ew_t;
static void ew_range(void *v, size_t lo, size_t hi) {
    ew_t *e = (ew_t *)v;
    for (size_t i = lo; i < hi; ++i) {
        switch (e->op) {
            case 0: e->o[i] = mulm(e->a[i], e->b[i]); break;
            case 1: e->o[i] = addm(e->a[i], e->b[i]); break;
            case 2: e->o[i] = subm(e->a[i], e->b[i]); break;
            case 3: e->o[i] = mulm(e->a[i], e->c); break;
            case 4: e->o[i] = addm(e->o[i], mulm(e->a[i], e->c)); break; /* axpy */
        }
    }
}
void vec_mul(const uint64_t *a, const uint64_t *b, uint64_t *o, size_t n, int th) {
    ew_t e = {a, b, o, 0, 0};
    parallel_for(n, th, ew_range, &e);
}
void vec_add(const uint64_t *a, const uint64_t *b, uint64_t *o, size_t n, int th) {
    ew_t e = {a, b, o, 0, 1};
    parallel_for(n, th, ew_range, &e);
}
void vec_sub(const uint64_t *a, const uint64_t *b, uint64_t *o, size_t n, int th) {
    ew_t e = {a, b, o, 0, 2};
    parallel_for(n, th, ew_range, &e);
}
void vec_scale(const uint64_t *a, uint64_t c, uint64_t *o, size_t n, int th) {
    ew_t e = {a, NULL, o, c % P, 3};
    parallel_for(n, th, ew_range, &e);
}
void vec_axpy(const uint64_t *a, uint64_t c, uint64_t *o, size_t n, int th) {
    ew_t e = {a, NULL, o, c % P, 4};
    parallel_for(n, th, ew_range, &e);
}

/* ---- o[i] = start * ratio^i */
void vec_geom(uint64_t start, uint64_t ratio, uint64_t *o, size_t n) {
    uint64_t x = start % P;
    for (size_t i = 0; i < n; ++i) {
        o[i] = x;
        x = mulm(x, ratio);
    }
}

/* ---- Horner: o[i] = sum_k coeffs[k] * xs[i]^k */
typedef struct { const uint64_t *c; size_t nc; const uint64_t *x; uint64_t *o; } hr_t;
static void hr_range(void *v, size_t lo, size_t hi) {
    hr_t *h = (hr_t *)v;
    for (size_t i = lo; i < hi; ++i) {
        uint64_t acc = 0;
        for (size_t k = h->nc; k-- > 0;) acc = addm(mulm(acc, h->x[i]), h->c[k]);
        h->o[i] = acc;
    }
}
void vec_horner(const uint64_t *coeffs, size_t nc, const uint64_t *xs, uint64_t *o, size_t n, int th) {
    hr_t h = {coeffs, nc, xs, o};
    parallel_for(n, th, hr_range, &h);
}

/* ---- batch inverse (single-threaded prefix products; zero not allowed) */
static uint64_t powm(uint64_t a, uint64_t e) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = mulm(r, a);
        a = mulm(a, a);
        e >>= 1;
    }
    return r;
}
void vec_batch_inv(const uint64_t *a, uint64_t *o, size_t n) {
    if (!n) return;
    uint64_t *pre = (uint64_t *)malloc(n * sizeof(uint64_t));
    uint64_t acc = 1;
    for (size_t i = 0; i < n; ++i) {
        pre[i] = acc;
        acc = mulm(acc, a[i]);
    }
    uint64_t inv = powm(acc, P - 2);
    for (size_t i = n; i-- > 0;) {
        o[i] = mulm(inv, pre[i]);
        inv = mulm(inv, a[i]);
    }
    free(pre);
}

/* ---- XFE linear combination: out[c][i] += sum_j w[j] * col_j[i] with BFE columns (stride n) */
typedef struct { const uint64_t *cols; size_t ncols; const uint64_t *w; uint64_t *o0, *o1, *o2; size_t n; int xcols; } lc_t;
static void lc_range(void *v, size_t lo, size_t hi) {
    lc_t *l = (lc_t *)v;
    for (size_t i = lo; i < hi; ++i) {
        uint64_t a0 = l->o0[i], a1 = l->o1[i], a2 = l->o2[i];
        for (size_t j = 0; j < l->ncols; ++j) {
            const uint64_t w0 = l->w[3 * j], w1 = l->w[3 * j + 1], w2 = l->w[3 * j + 2];
            if (!l->xcols) {
                const uint64_t b = l->cols[j * l->n + i];
                a0 = addm(a0, mulm(w0, b));
                a1 = addm(a1, mulm(w1, b));
                a2 = addm(a2, mulm(w2, b));
            } else {
                /* column j is XFE: planes at cols[(3j+k)*n] */
                const uint64_t b0 = l->cols[(3 * j) * l->n + i], b1 = l->cols[(3 * j + 1) * l->n + i],
                               b2 = l->cols[(3 * j + 2) * l->n + i];
                const u128 c0 = (u128)w0 * b0, c1a = (u128)w0 * b1, c1b = (u128)w1 * b0;
                const uint64_t r0 = red128(c0), r1 = addm(red128(c1a), red128(c1b));
                const uint64_t r2 = addm(addm(mulm(w0, b2), mulm(w1, b1)), mulm(w2, b0));
                const uint64_t r3 = addm(mulm(w1, b2), mulm(w2, b1));
                const uint64_t r4 = mulm(w2, b2);
                a0 = addm(a0, subm(r0, r3));
                a1 = addm(a1, subm(addm(r1, r3), r4));
                a2 = addm(a2, addm(r2, r4));
            }
        }
        l->o0[i] = a0;
        l->o1[i] = a1;
        l->o2[i] = a2;
    }
}
/* cols: ncols BFE columns (xcols=0, layout [j][n]) or ncols XFE columns (xcols=1, layout [3j+k][n]);
 * w: ncols XFE weights (3 words each); o0..o2 accumulate (must be initialised). */
void vec_xlincomb(const uint64_t *cols, size_t ncols, int xcols, const uint64_t *w, uint64_t *o0, uint64_t *o1,
                  uint64_t *o2, size_t n, int th) {
    lc_t l = {cols, ncols, w, o0, o1, o2, n, xcols};
    parallel_for(n, th, lc_range, &l);
}

/* ---- row hashing from column-major planes: row i = [plane_0[i], plane_1[i], ...] */
extern void oracle_hash_varlen(const uint64_t *data, size_t len, uint64_t out[5]);
typedef struct { const uint64_t *planes; size_t nplanes, n; uint64_t *out; } rh_t;
static void rh_range(void *v, size_t lo, size_t hi) {
    rh_t *r = (rh_t *)v;
    uint64_t *row = (uint64_t *)malloc(r->nplanes * sizeof(uint64_t) + 8);
    for (size_t i = lo; i < hi; ++i) {
        for (size_t j = 0; j < r->nplanes; ++j) row[j] = r->planes[j * r->n + i];
        oracle_hash_varlen(row, r->nplanes, r->out + 5 * i);
    }
    free(row);
}
void hash_rows_planes(const uint64_t *planes, size_t nplanes, size_t n, uint64_t *out, int th) {
    rh_t r = {planes, nplanes, n, out};
    parallel_for(n, th, rh_range, &r);
}

/* ---- row hashing when every row shares its first full rate chunks: s0 = the sponge state after
 * them (oracle_sponge_absorb_chunks), row i's remaining words = [tail_plane_0[i], ...] */
extern void oracle_hash_varlen_resume(const uint64_t s_raw[16], const uint64_t *tail, size_t len, uint64_t out[5]);
typedef struct { const uint64_t *s0, *planes; size_t ntail, n; uint64_t *out; } rt_t;
static void rt_range(void *v, size_t lo, size_t hi) {
    rt_t *r = (rt_t *)v;
    uint64_t tail[64];
    for (size_t i = lo; i < hi; ++i) {
        for (size_t j = 0; j < r->ntail; ++j) tail[j] = r->planes[j * r->n + i];
        oracle_hash_varlen_resume(r->s0, tail, r->ntail, r->out + 5 * i);
    }
}
int hash_rows_tail(const uint64_t s0[16], const uint64_t *tail_planes, size_t ntail, size_t n, uint64_t *out, int th) {
    if (ntail > 64) return -1;
    rt_t r = {s0, tail_planes, ntail, n, out};
    parallel_for(n, th, rt_range, &r);
    return 0;
}

/* ---- Merkle tree (pow.rs / twenty-first layout), level-parallel */
extern void oracle_hash_pair_fast(const uint64_t l[5], const uint64_t r[5], uint64_t out[5]);
#define oracle_hash_pair oracle_hash_pair_fast
typedef struct { const uint64_t *src; uint64_t *dst; } lv_t;
static void lv_range(void *v, size_t lo, size_t hi) {
    lv_t *l = (lv_t *)v;
    for (size_t i = lo; i < hi; ++i) oracle_hash_pair(l->src + 10 * i, l->src + 10 * i + 5, l->dst + 5 * i);
}
void mtree_build_mt(const uint64_t *leaves, size_t n, uint64_t *nodes, int th) {
    memset(nodes, 0, 5 * sizeof(uint64_t));
    lv_t l0 = {leaves, nodes + 5 * (n / 2)};
    parallel_for(n / 2, th, lv_range, &l0);
    for (size_t parents = n / 4; parents >= 1; parents /= 2) {
        lv_t l = {nodes + 5 * (2 * parents), nodes + 5 * parents};
        parallel_for(parents, th, lv_range, &l);
    }
}
