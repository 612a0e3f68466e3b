// The coalescing queue's pinned receive arena (neptune-core_amd/csrc/pinned_ring.hpp) under ASan /
// UBSan: random requests take ranges, fill them with a pattern, and are released in random order
// (the queue's two slots release out of arrival order); every live range must keep its pattern (no
// two live ranges overlap), no range may cross the buffer's end, and once everything is released
// the whole ring is free again.  Built by tests/native/Makefile, driven by tests/test_sanitizers.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../neptune-core_amd/csrc/pinned_ring.hpp"

namespace {
uint64_t g = 0x12345678ull;
uint64_t rnd() {
    g ^= g << 13, g ^= g >> 7, g ^= g << 17;
    return g;
}
struct Live {
    uint64_t at, n;
    uint8_t tag;
};
int fail(const char* what, unsigned long long a, unsigned long long b) {
    std::fprintf(stderr, "ring_check: %s (%llu, %llu)\n", what, a, b);
    return 1;
}
}  // namespace

int main(int argc, char** argv) {
    const uint64_t cap = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4096;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 200000;
    std::vector<uint8_t> buf(cap);  // exactly cap bytes: ASan reports any write past the end
    nhip::PinnedRing r;
    r.base = buf.data();
    r.cap = cap;
    std::vector<Live> live;
    uint64_t taken = 0, refused = 0;
    for (int it = 0; it < iters; ++it) {
        const bool take = live.empty() || rnd() % 100 < 55;
        if (take) {
            const uint64_t n = 1 + rnd() % (cap / (rnd() % 4 == 0 ? 2 : 8));
            const uint64_t at = r.take(n);
            if (at == nhip::PinnedRing::NONE) {
                ++refused;
                continue;
            }
            if (at % cap + n > cap) return fail("range crosses the buffer end", at, n);
            const uint8_t tag = (uint8_t)(1 + rnd() % 255);
            std::memset(r.ptr(at), tag, n);
            live.push_back({at, n, tag});
            ++taken;
        } else {
            const size_t k = rnd() % live.size();
            const Live l = live[k];
            const uint8_t* p = r.ptr(l.at);
            for (uint64_t i = 0; i < l.n; ++i)
                if (p[i] != l.tag) return fail("live range overwritten", l.at, i);
            r.release(l.at);
            live[k] = live.back();
            live.pop_back();
        }
    }
    for (const Live& l : live) r.release(l.at);
    if (!r.live.empty() || r.tail != r.head) return fail("ranges left after releasing all", r.tail, r.head);
    if (r.take(cap) == nhip::PinnedRing::NONE) return fail("full ring not free again", cap, 0);
    if (taken < (uint64_t)iters / 4) return fail("too few takes", taken, refused);
    std::printf("ring ok: %llu taken, %llu refused\n", (unsigned long long)taken, (unsigned long long)refused);
    return 0;
}
