// Host check of the staging copy's streaming-store word copy (neptune-core_amd/csrc/host_copy.hpp)
// against memcpy: every destination / source alignment (8-byte steps inside 64 bytes), lengths 0-300
// words and a few large ones, guard words around the destination untouched (run under ASan +
// UBSan by tests/test_goldilocks_host.py).
#include <emmintrin.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "host_copy.hpp"

int main() {
    std::mt19937_64 g(7);
    std::vector<uint64_t> src(1 << 18), dst(1 << 18);
    for (auto& w : src) w = g();
    unsigned long long bad = 0, n = 0;
    auto one = [&](size_t doff, size_t soff, size_t len) {
        ++n;
        const uint64_t GUARD = 0xA5A5A5A5DEADBEEFull;
        std::fill(dst.begin(), dst.begin() + doff + len + 16, GUARD);
        nhip::copy_words_nt(dst.data() + 8 + doff, src.data() + soff, len);
        _mm_sfence();
        if (std::memcmp(dst.data() + 8 + doff, src.data() + soff, len * 8) != 0) ++bad;
        for (size_t i = 0; i < 8 + doff; ++i) bad += dst[i] != GUARD;
        for (size_t i = 8 + doff + len; i < doff + len + 16; ++i) bad += dst[i] != GUARD;
    };
    for (size_t doff = 0; doff < 8; ++doff)
        for (size_t soff = 0; soff < 8; ++soff)
            for (size_t len = 0; len <= 300; ++len) one(doff, soff, len);
    for (size_t len : {4095u, 4096u, 4097u, 100003u})
        for (size_t doff = 0; doff < 2; ++doff) one(doff, 3, len);
    printf("checked %llu, bad %llu\n", n, bad);
    return bad != 0;
}
