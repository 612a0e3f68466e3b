// Host check of the folded MDS reduction + round-constant add of mds_ark (tip5_device.hpp) against
// twenty-first's step-by-step form (reduce, then the field add of the round constant), for every
// Tip5 round constant and 3 x 10^6 other constants below 2^64 - 2^52 - (2^32 - 1) (run by
// tests/test_goldilocks_host.py).
#include "goldilocks.hpp"
#include "tip5_constants.h"
#include <cstdio>
#include <random>
#include <vector>
using namespace nhip;
typedef unsigned __int128 u128;
// step-by-step reduction + ARK of mds_ark (twenty-first): s = al + ah*2^32; res = s_lo + s_hi*EPS
// (overflowing add), y = res + over*EPS; x1 = y - (p - rc), + p on borrow
static uint64_t ref(uint64_t al, uint64_t ah, uint64_t rc) {
    u128 s = (u128)al + ((u128)ah << 32);
    uint64_t slo = (uint64_t)s, shi = (uint64_t)(s >> 64);
    uint64_t t = shi * GL_EPS;
    uint64_t res = slo + t; bool over = res < slo;
    uint64_t y = res + (over ? GL_EPS : 0);
    uint64_t q = GL_P - rc;
    uint64_t x1 = y - q;
    if (y < q) x1 += GL_P;
    return x1;
}
static uint64_t fold(uint64_t al, uint64_t ah, uint64_t rc) {
    const uint64_t K = rc + GL_EPS;  // the whole constant starts the low accumulator (no overflow:
    al += K;                          // al < 2^52 and K < 2^64 - 2^52, checked below)
    uint32_t al_hi = al >> 32, ah_lo = (uint32_t)ah;
    uint64_t m1s = (uint64_t)al_hi + ah_lo;
    uint32_t m1 = (uint32_t)m1s, k = m1s >> 32;
    uint32_t sh = (uint32_t)((ah >> 32) + k);
    u128 W = (u128)sh * 0xFFFFFFFFull + (((uint64_t)m1 << 32) | (uint32_t)al);
    uint64_t w = (uint64_t)W; bool G = (W >> 64) != 0;
    uint32_t e = G ? 0u : 0xFFFFFFFFu;
    return w - e;
}
int main() {
    std::mt19937_64 g(11);
    uint64_t bad = 0, n = 0;
    const uint64_t AMAX = (1ull << 52) - 1;
    for (int i = 0; i < 80; ++i) if (!(TIP5_RC_RAW[i] < GL_P - (1ull << 32) + 2)) { printf("rc %d out of the bound\n", i); bad++; }
    for (int i = 0; i < 80; ++i) if (!(TIP5_RC_RAW[i] + GL_EPS < (0ull - (1ull << 52)))) { printf("rc %d: K overflows the accumulator\n", i); bad++; }
    auto chk = [&](uint64_t al, uint64_t ah, uint64_t rc) { ++n; uint64_t a = ref(al, ah, rc), b = fold(al, ah, rc); if (a != b) { if (bad < 10) printf("al=%llx ah=%llx rc=%llx ref=%llx fold=%llx\n", (unsigned long long)al, (unsigned long long)ah, (unsigned long long)rc, (unsigned long long)a, (unsigned long long)b); ++bad; } };
    std::vector<uint64_t> edge;
    for (uint64_t d = 0; d < 40; ++d) { edge.push_back(d); edge.push_back(AMAX - d); edge.push_back((1ull << 32) + d - 20); edge.push_back((1ull << 32) * 0xFFFFF + d); }
    for (int i = 0; i < 80; ++i) {
        uint64_t rc = TIP5_RC_RAW[i];
        for (auto a : edge) for (auto b : edge) chk(a, b, rc);
        for (int j = 0; j < 300000; ++j) chk(g() & AMAX, g() & AMAX, rc);
    }
    // the bound and the identity for arbitrary constants in range (not only Tip5's)
    for (int j = 0; j < 3000000; ++j) { uint64_t rc = g() % ((0ull - (1ull << 52)) - GL_EPS); chk(g() & AMAX, g() & AMAX, rc); }
    printf("checked %llu, bad %llu\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
