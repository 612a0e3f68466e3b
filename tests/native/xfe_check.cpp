// Host-side check of xfe.hpp / goldilocks.hpp against 128-bit integer arithmetic mod p: the lazily
// reduced x_mul (nine 128-bit products, three reductions) equals the Montgomery-domain product
// c_k = (sum of +-a_i b_j) * 2^-64 mod p, and gl_add equals (a + b) mod p, on edge words (0, 1,
// p - 1, 2^32 +- 1, words with all-ones limbs) and random canonical words, and with the second
// operand any u64 (p, p + 1, 2^64 - 1, random full-range words), as DEEP passes raw proof words
// (run by tests/test_goldilocks_host.py).
#include "xfe.hpp"
#include <cstdio>
#include <random>
using namespace nhip;
typedef unsigned __int128 u128;

static uint64_t mulmod(uint64_t a, uint64_t b) { return (uint64_t)((u128)a * b % GL_P); }
static uint64_t addmod(uint64_t a, uint64_t b) { return (uint64_t)(((u128)a + b) % GL_P); }
static uint64_t submod(uint64_t a, uint64_t b) { return addmod(a, GL_P - b); }
static uint64_t powmod(uint64_t a, uint64_t e) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = mulmod(r, a);
        a = mulmod(a, a);
        e >>= 1;
    }
    return r;
}

int main() {
    const uint64_t rinv = powmod((uint64_t)(((u128)1 << 64) % GL_P), GL_P - 2);
    auto ref = [&](Xfe a, Xfe b) {
        const uint64_t A[3] = {a.c0, a.c1, a.c2}, B[3] = {b.c0, b.c1, b.c2};
        uint64_t p[3][3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) p[i][j] = mulmod(A[i], B[j]);
        const uint64_t n = addmod(p[1][2], p[2][1]);
        const uint64_t c0 = submod(p[0][0], n);
        const uint64_t c1 = submod(addmod(addmod(p[0][1], p[1][0]), n), p[2][2]);
        const uint64_t c2 = addmod(addmod(addmod(p[0][2], p[1][1]), p[2][0]), p[2][2]);
        return Xfe{mulmod(c0, rinv), mulmod(c1, rinv), mulmod(c2, rinv)};
    };
    const uint64_t edge[] = {0, 1, 2, GL_P - 1, GL_P - 2, GL_EPS, GL_EPS + 1, 0x100000000ull, 0x8000000000000000ull,
                             0xFFFFFFFE00000000ull, 0xFFFFFFFF00000000ull, 0x7FFFFFFFFFFFFFFFull};
    const int NE = sizeof(edge) / sizeof(edge[0]);
    std::mt19937_64 g(11);
    uint64_t bad = 0, n = 0;
    auto chk = [&](Xfe a, Xfe b) {
        ++n;
        const Xfe r = x_mul(a, b), w = ref(a, b);
        if (!x_eq(r, w)) {
            if (bad < 5) printf("x_mul a=(%llx %llx %llx) b=(%llx %llx %llx)\n", (unsigned long long)a.c0,
                                (unsigned long long)a.c1, (unsigned long long)a.c2, (unsigned long long)b.c0,
                                (unsigned long long)b.c1, (unsigned long long)b.c2);
            ++bad;
        }
        if (b.c0 >= GL_P) return;  // gl_add takes canonical operands only
        const uint64_t s = gl_add(a.c0, b.c0);
        if (s != addmod(a.c0, b.c0)) {
            if (bad < 5) printf("gl_add %llx %llx\n", (unsigned long long)a.c0, (unsigned long long)b.c0);
            ++bad;
        }
    };
    // every edge word in every coefficient position of both operands against all-edge partners
    for (int i = 0; i < NE; ++i)
        for (int j = 0; j < NE; ++j)
            for (int k = 0; k < NE; ++k) {
                chk(Xfe{edge[i], edge[j], edge[k]}, Xfe{edge[k], edge[i], edge[j]});
                chk(Xfe{edge[i], edge[j], edge[k]}, Xfe{edge[i], edge[j], edge[k]});
                chk(Xfe{GL_P - 1, GL_P - 1, GL_P - 1}, Xfe{edge[i], edge[j], edge[k]});
            }
    auto word = [&]() -> uint64_t { return (g() & 7) == 0 ? edge[g() % NE] : g() % GL_P; };
    for (int i = 0; i < 3000000; ++i) chk(Xfe{word(), word(), word()}, Xfe{word(), word(), word()});
    // the second operand as k_deep_rows8 passes it (ld_xfe_raw of proof words): any u64, words at or
    // above p included, against a canonical first operand (the raw Montgomery weight)
    const uint64_t raw_edge[] = {GL_P, GL_P + 1, GL_P + GL_EPS, 0xFFFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFEull,
                                 0xFFFFFFFF80000000ull, 0xFFFFFFFF00000001ull, 0, 1, GL_P - 1};
    const int NR = sizeof(raw_edge) / sizeof(raw_edge[0]);
    for (int i = 0; i < NE; ++i)
        for (int j = 0; j < NR; ++j)
            for (int k = 0; k < NR; ++k) {
                chk(Xfe{edge[i], edge[(i + 3) % NE], edge[(i + 7) % NE]}, Xfe{raw_edge[j], raw_edge[k], raw_edge[(j + k) % NR]});
                chk(Xfe{GL_P - 1, GL_P - 1, GL_P - 1}, Xfe{raw_edge[j], raw_edge[k], raw_edge[j]});
            }
    auto any = [&]() -> uint64_t { return (g() & 7) == 0 ? raw_edge[g() % NR] : g(); };
    for (int i = 0; i < 2000000; ++i) chk(Xfe{word(), word(), word()}, Xfe{any(), any(), any()});
    printf("checked %llu, bad %llu\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
