// The staging copy's streaming-store word copy (stark_host.cpp; tests/native/copy_check.cpp checks it
// against memcpy at every alignment and length).  Destination lines are written with non-temporal
// 16-byte stores (no read-for-ownership: the staging is only ever read by the DMA engine); the caller
// issues _mm_sfence() before the copied words are handed to the DMA.
#pragma once
#include <emmintrin.h>

#include <cstddef>
#include <cstdint>

namespace nhip {

inline void copy_words_nt(uint64_t* dst, const uint64_t* src, size_t words) {
    if (((uintptr_t)dst & 15u) && words) {  // 8-byte head to 16-byte alignment
        *dst++ = *src++;
        --words;
    }
    __m128i* d = (__m128i*)dst;
    const __m128i* sv = (const __m128i*)src;
    for (size_t blocks = words / 8; blocks; --blocks, d += 4, sv += 4) {  // 64-byte blocks
        const __m128i a = _mm_loadu_si128(sv), b = _mm_loadu_si128(sv + 1), c = _mm_loadu_si128(sv + 2),
                      e = _mm_loadu_si128(sv + 3);
        _mm_stream_si128(d, a);
        _mm_stream_si128(d + 1, b);
        _mm_stream_si128(d + 2, c);
        _mm_stream_si128(d + 3, e);
    }
    for (size_t i = words / 8 * 8; i < words; ++i) dst[i] = src[i];  // tail
}

}  // namespace nhip
