// Host-side check of goldilocks.hpp: to_mont (closed form) == mont_mul(x, 2^128 mod p) on edge and
// random words (run by tests/test_goldilocks_host.py).
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
    printf("checked %llu, bad %llu\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
