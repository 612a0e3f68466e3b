/* C consumer of the C ABI (include/neptune_hip.h), built as C99 with -pedantic -Werror: proves the
 * header is plain C (no C++ or torch types) and that a non-Python host can drive the verifier the
 * way the Rust binding of INTEGRATION.md would.
 *
 *   abi_c_check host         host-only entry points (no GPU needed): stark params default, proof
 *                            file bytes round trip, group shard; prints the nhip_init return code
 *   abi_c_check verify FILE  verify the batch in FILE on one context and on a group of every
 *                            visible GPU; prints "ctx <verdicts>" and "group <verdicts> <all_ok>"
 *   abi_c_check marshal N W  host only: time handing N proofs of W words each to the library in
 *                            both input forms, as the Rust drop-in would.  The proofs sit in memory
 *                            as twenty-first keeps Vec<BFieldElement> (Montgomery words).
 *                            canonical: a new buffer per proof, every word reduced (BFieldElement::
 *                            value(), montyred) - round 3's marshal; montgomery: the nhip_proof
 *                            array points at the words as they lie (NHIP_INPUT_MONTGOMERY).
 *                            Prints "marshal canonical_ms montgomery_ms bytes checksum".
 *
 * FILE (little-endian u64 stream, written by tests/test_capi_c.py):
 *   n_air, air[n_air], security_level, log2_fri_expansion, num_collinearity_checks, num_main,
 *   num_aux, num_quotient_segments, n, then per proof: digest[5], version, in_len, in[],
 *   out_len, out[], proof_len, proof[]
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "neptune_hip.h"

static int fail(const char *what, int rc) {
    fprintf(stderr, "%s: %d (%s)\n", what, rc, nhip_strerror(rc));
    return 1;
}

static int host_checks(void) {
    nhip_stark_params sp;
    uint64_t words[5] = {0, 1, 0xFFFFFFFF00000000ull, 0x0123456789ABCDEFull, 0xFFFFFFFFFFFFFFFFull};
    uint8_t bytes[40];
    uint64_t back[5];
    size_t n_back = 0;
    nhip_proof proofs[3];
    uint32_t member[3];
    nhip_ctx *ctx = NULL;
    int rc, i;

    nhip_stark_params_default(&sp);
    if (sp.security_level != 160 || sp.log2_fri_expansion != 2 || sp.num_collinearity_checks != 80 ||
        sp.input_form != NHIP_INPUT_CANONICAL)
        return fail("nhip_stark_params_default", -1);
    /* program.rs:374-390 / 565-572: big-endian 8-byte chunks, BFieldElement::new on the way in */
    if ((rc = nhip_proof_to_be_bytes(words, 4, bytes)) != NHIP_OK) return fail("nhip_proof_to_be_bytes", rc);
    if ((rc = nhip_proof_from_be_bytes(bytes, 32, back, 5, &n_back)) != NHIP_OK || n_back != 4)
        return fail("nhip_proof_from_be_bytes", rc);
    for (i = 0; i < 4; ++i)
        if (back[i] != words[i]) return fail("be bytes round trip", -1);
    if (nhip_proof_from_be_bytes(bytes, 31, back, 5, &n_back) != NHIP_ERR_ARG) return fail("odd length", -1);
    proofs[0].words = words;
    proofs[0].len = 5;
    proofs[1].words = words;
    proofs[1].len = 1;
    proofs[2].words = words;
    proofs[2].len = 3;
    if ((rc = nhip_group_shard(proofs, 3, 2, member)) != NHIP_OK) return fail("nhip_group_shard", rc);
    if (member[0] != 0 || member[2] != 1 || member[1] != 1) return fail("LPT split", -1);
    rc = nhip_init(0, &ctx);
    printf("init %d\n", rc);
    if (rc == NHIP_OK) nhip_destroy(ctx);
    printf("host ok\n");
    return 0;
}

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec * 1e3 + (double)t.tv_nsec * 1e-6;
}

/* twenty-first's montyred(x, 0): a Montgomery word's canonical value (BFieldElement::value()) */
static uint64_t value_of(uint64_t xl) {
    const uint64_t P_EPS = 0xFFFFFFFFull;
    uint64_t a = xl + (xl << 32);
    uint64_t e = a < xl ? 1u : 0u;
    uint64_t b = a - (a >> 32) - e;
    uint64_t r = 0 - b;
    return b > 0 ? r - P_EPS : r;
}

static int marshal_timing(size_t n, size_t w) {
    uint64_t **mem = (uint64_t **)calloc(n, sizeof(uint64_t *));
    uint64_t **canon = (uint64_t **)calloc(n, sizeof(uint64_t *));
    nhip_proof *pc = (nhip_proof *)calloc(n, sizeof(nhip_proof));
    nhip_proof *pm = (nhip_proof *)calloc(n, sizeof(nhip_proof));
    uint64_t x = 0x9E3779B97F4A7C15ull, sum = 0;
    double t0, t1, t2;
    size_t i, k;
    if (!mem || !canon || !pc || !pm) return fail("allocation", -1);
    for (i = 0; i < n; ++i) {  /* the node's proofs: Montgomery words, one allocation per proof */
        mem[i] = (uint64_t *)malloc(w * 8);
        if (!mem[i]) return fail("allocation", -1);
        for (k = 0; k < w; ++k) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            mem[i][k] = x % 0xFFFFFFFF00000001ull;
        }
    }
    t0 = now_ms();
    for (i = 0; i < n; ++i) {  /* canonical: words(&p.0) = a new Vec<u64> of value()s */
        canon[i] = (uint64_t *)malloc(w * 8);
        if (!canon[i]) return fail("allocation", -1);
        for (k = 0; k < w; ++k) canon[i][k] = value_of(mem[i][k]);
        pc[i].words = canon[i];
        pc[i].len = w;
    }
    t1 = now_ms();
    for (i = 0; i < n; ++i) {  /* montgomery: the words as they lie */
        pm[i].words = mem[i];
        pm[i].len = w;
    }
    t2 = now_ms();
    for (i = 0; i < n; ++i) sum += pc[i].words[w - 1] ^ pm[i].words[0];
    printf("marshal %.3f %.6f %llu %llu\n", t1 - t0, t2 - t1, (unsigned long long)(n * w * 8), (unsigned long long)sum);
    for (i = 0; i < n; ++i) {
        free(mem[i]);
        free(canon[i]);
    }
    free(mem);
    free(canon);
    free(pc);
    free(pm);
    return 0;
}

static uint64_t *read_all(const char *path, size_t *n_words) {
    FILE *f = fopen(path, "rb");
    long sz;
    uint64_t *buf;
    if (!f) return NULL;
    if (fseek(f, 0, SEEK_END) != 0 || (sz = ftell(f)) < 0 || fseek(f, 0, SEEK_SET) != 0) {
        fclose(f);
        return NULL;
    }
    buf = (uint64_t *)malloc((size_t)sz + 8);
    if (buf && fread(buf, 1, (size_t)sz, f) != (size_t)sz) {
        free(buf);
        buf = NULL;
    }
    fclose(f);
    *n_words = (size_t)sz / 8;
    return buf;
}

static int verify_file(const char *path) {
    size_t nw = 0, pos = 0, n, i, k;
    uint64_t *w = read_all(path, &nw);
    nhip_stark_params sp;
    nhip_air *air = NULL;
    nhip_claim *claims;
    nhip_proof *proofs;
    uint8_t *v;
    uint8_t all_ok = 0;
    nhip_ctx *ctx = NULL;
    nhip_group *group = NULL;
    int rc;
#define TAKE(dst) do { if (pos >= nw) return fail("truncated batch file", -1); (dst) = w[pos++]; } while (0)
    if (!w) return fail("read batch file", -1);
    {
        uint64_t n_air;
        TAKE(n_air);
        if (pos + n_air > nw) return fail("truncated air", -1);
        if ((rc = nhip_air_create(w + pos, (size_t)n_air, &air)) != NHIP_OK) return fail("nhip_air_create", rc);
        pos += (size_t)n_air;
    }
    nhip_stark_params_default(&sp); /* input_form: canonical */
    {
        uint64_t t[6];
        for (i = 0; i < 6; ++i) TAKE(t[i]);
        sp.security_level = (uint32_t)t[0];
        sp.log2_fri_expansion = (uint32_t)t[1];
        sp.num_collinearity_checks = (uint32_t)t[2];
        sp.num_main = (uint32_t)t[3];
        sp.num_aux = (uint32_t)t[4];
        sp.num_quotient_segments = (uint32_t)t[5];
    }
    {
        uint64_t nn;
        TAKE(nn);
        n = (size_t)nn;
    }
    claims = (nhip_claim *)calloc(n ? n : 1, sizeof(nhip_claim));
    proofs = (nhip_proof *)calloc(n ? n : 1, sizeof(nhip_proof));
    v = (uint8_t *)calloc(n ? n : 1, 1);
    if (!claims || !proofs || !v) return fail("allocation", -1);
    for (i = 0; i < n; ++i) {
        uint64_t ver, len;
        for (k = 0; k < 5; ++k) TAKE(claims[i].program_digest[k]);
        TAKE(ver);
        claims[i].version = (uint32_t)ver;
        TAKE(len);
        claims[i].input = w + pos;
        claims[i].input_len = (size_t)len;
        pos += (size_t)len;
        TAKE(len);
        claims[i].output = w + pos;
        claims[i].output_len = (size_t)len;
        pos += (size_t)len;
        TAKE(len);
        proofs[i].words = w + pos;
        proofs[i].len = (size_t)len;
        pos += (size_t)len;
        if (pos > nw) return fail("truncated proof", -1);
    }
#undef TAKE
    if ((rc = nhip_init(1u, &ctx)) != NHIP_OK) return fail("nhip_init", rc);
    if ((rc = nhip_verify_batch(ctx, air, &sp, claims, proofs, n, v, NULL)) != NHIP_OK)
        return fail("nhip_verify_batch", rc);
    printf("ctx ");
    for (i = 0; i < n; ++i) putchar(v[i] ? '1' : '0');
    putchar('\n');
    memset(v, 7, n ? n : 1);
    if ((rc = nhip_group_init(0u, &group)) != NHIP_OK) return fail("nhip_group_init", rc);
    if ((rc = nhip_group_verify_batch(group, air, &sp, claims, proofs, n, v, &all_ok)) != NHIP_OK)
        return fail("nhip_group_verify_batch", rc);
    printf("group ");
    for (i = 0; i < n; ++i) putchar(v[i] == 1 ? '1' : (v[i] == 0 ? '0' : '?'));
    printf(" %u %u\n", (unsigned)all_ok, (unsigned)nhip_group_size(group));
    nhip_group_destroy(group);
    nhip_destroy(ctx);
    nhip_air_destroy(air);
    free(claims);
    free(proofs);
    free(v);
    free(w);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 2 && strcmp(argv[1], "host") == 0) return host_checks();
    if (argc >= 3 && strcmp(argv[1], "verify") == 0) return verify_file(argv[2]);
    if (argc >= 4 && strcmp(argv[1], "marshal") == 0)
        return marshal_timing((size_t)strtoull(argv[2], NULL, 10), (size_t)strtoull(argv[3], NULL, 10));
    fprintf(stderr, "usage: %s host | verify FILE | marshal N_PROOFS WORDS\n", argv[0]);
    return 2;
}
