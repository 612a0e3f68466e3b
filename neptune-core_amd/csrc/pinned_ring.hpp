// The coalescing queue's pinned receive arena (queue.cpp): a ring of monotonically growing byte
// offsets over one pinned buffer.  Host-only; tested under ASan / UBSan by tests/native/ring_check.cpp.
#pragma once
#include <stdint.h>

#include <map>
#include <utility>

namespace nhip {

// Pinned receive arena of a queue: a ring of monotonically growing offsets.  A caller takes a
// contiguous range for its proofs (under the queue lock), copies them in on its own thread (no
// lock held), and the worker releases the range once the batch holding them has been uploaded
// (nhip_batch_refill waits for its uploads).  Ranges are taken in arrival order but may be
// released out of order (two slots); the ring's tail advances over released ranges only.
struct PinnedRing {
    static constexpr uint64_t NONE = ~0ull;  // take(): no room
    uint8_t* base = nullptr;
    uint64_t cap = 0, head = 0, tail = 0;
    std::map<uint64_t, std::pair<uint64_t, bool>> live;  // start -> (bytes, released)

    uint64_t take(uint64_t n) {
        if (!base || n == 0 || n > cap) return NONE;
        if (live.empty()) head = tail = 0;  // nothing held: the whole ring from its start
        uint64_t at = head;
        if (at % cap + n > cap) at += cap - at % cap;  // would wrap: start at the ring's beginning
        if (at + n - tail > cap) return NONE;            // full
        live.emplace(at, std::make_pair(n, false));
        head = at + n;
        return at;
    }
    void release(uint64_t at) {
        auto it = live.find(at);
        if (it == live.end()) return;
        it->second.second = true;
        while (!live.empty() && live.begin()->second.second) {
            tail = live.begin()->first + live.begin()->second.first;
            live.erase(live.begin());
        }
        if (live.empty()) tail = head;
    }
    uint8_t* ptr(uint64_t at) const { return base + at % cap; }
};


}  // namespace nhip
