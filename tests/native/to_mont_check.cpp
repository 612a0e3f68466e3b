// Host-side check of goldilocks.hpp: to_mont (closed form) == mont_mul(x, 2^128 mod p) on edge and
// random words, and the carry-light mont_mul_lat == mont_mul (twenty-first's montyred) on edge pairs
// and random canonical / non-canonical pairs (run by tests/test_goldilocks_host.py).
#include "goldilocks.hpp"
#include <cstdio>
#include <random>
using namespace nhip;
int main() {
    std::mt19937_64 g(7);
    uint64_t bad = 0, n = 0;
    auto chk = [&](uint64_t x) { ++n; if (to_mont(x) != to_mont_mul(x)) { if (bad < 5) printf("x=%llx %llx %llx\n", (unsigned long long)x, (unsigned long long)to_mont(x), (unsigned long long)to_mont_mul(x)); ++bad; } };
    for (uint64_t h = 0; h < 64; ++h) for (uint64_t l = 0; l < 64; ++l) {
        uint64_t hs[4] = {h, 0xFFFFFFFFull - h, 0x80000000ull + h, 0x7FFFFFFFull - h};
        uint64_t ls[4] = {l, 0xFFFFFFFFull - l, 0x80000000ull + l, 0x7FFFFFFFull - l};
        for (auto a : hs) for (auto b : ls) chk((a << 32) | b);
    }
    for (int i = 0; i < 2000000; ++i) chk(g());
    for (uint64_t d = 0; d < 1000; ++d) { chk(GL_P + d); chk(GL_P - d); chk(~0ull - d); }
    auto chk2 = [&](uint64_t a, uint64_t b) { ++n; if (mont_mul_lat(a, b) != mont_mul(a, b)) { if (bad < 5) printf("a=%llx b=%llx\n", (unsigned long long)a, (unsigned long long)b); ++bad; } };
    const uint64_t edge[] = {0, 1, 2, GL_P - 1, GL_P - 2, GL_P, GL_P + 1, 0xFFFFFFFFull, 0x100000000ull,
                             0xFFFFFFFF00000000ull, ~0ull, ~0ull - 1, 0x8000000000000000ull, 0x7FFFFFFFFFFFFFFFull};
    for (auto a : edge) for (auto b : edge) chk2(a, b);
    for (int i = 0; i < 4000000; ++i) {
        const uint64_t a = g(), b = g();
        chk2(a % GL_P, b % GL_P);
        chk2(a, b);
    }
    printf("checked %llu, bad %llu\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
