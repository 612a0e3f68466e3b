// The staging copy's streaming-store word copy (stark_host.cpp; tests/native/copy_check.cpp checks it
// against memcpy at every alignment and length).  Destination lines are written with non-temporal
// 16-byte stores (no read-for-ownership: the staging is only ever read by the DMA engine); the caller
// issues _mm_sfence() before the copied words are handed to the DMA.
#pragma once
#include <emmintrin.h>
#include <immintrin.h>

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

// Wire bytes -> field words: `words` little-endian u64 at any byte alignment (bincode's
// Vec<BFieldElement>), each reduced mod p = 2^64 - 2^32 + 1 (BFieldElement::new, nhip_le_words), written
// with streaming stores (the arena is read only by the DMA engine).  v >= p iff its high half is
// 0xFFFFFFFF and its low half is not 0, and then v - p = v + (2^32 - 1) mod 2^64: SSE2 only.
inline void copy_le_words_nt(uint64_t* dst, const uint8_t* src, size_t words) {
    constexpr uint64_t P = 0xFFFFFFFF00000001ull;
    auto one = [](const uint8_t* b) {
        uint64_t v;
        __builtin_memcpy(&v, b, 8);
        return v >= P ? v - P : v;
    };
    if (((uintptr_t)dst & 15u) && words) {  // 8-byte head to 16-byte alignment
        *dst++ = one(src);
        src += 8;
        --words;
    }
    const __m128i ones = _mm_set1_epi32(-1), zero = _mm_setzero_si128();
    const __m128i lo_mask = _mm_set_epi32(0, -1, 0, -1);
    auto reduce = [&](__m128i v) {
        const __m128i hi_all = _mm_shuffle_epi32(_mm_cmpeq_epi32(v, ones), _MM_SHUFFLE(3, 3, 1, 1));
        const __m128i ge = _mm_andnot_si128(_mm_cmpeq_epi32(v, zero), hi_all);  // dword 2i: lane i >= p
        return _mm_add_epi64(v, _mm_and_si128(ge, lo_mask));
    };
    __m128i* d = (__m128i*)dst;
    for (size_t blocks = words / 8; blocks; --blocks, d += 4, src += 64) {  // 64-byte blocks
        const __m128i a = _mm_loadu_si128((const __m128i*)src), b = _mm_loadu_si128((const __m128i*)(src + 16)),
                      c = _mm_loadu_si128((const __m128i*)(src + 32)), e = _mm_loadu_si128((const __m128i*)(src + 48));
        _mm_stream_si128(d, reduce(a));
        _mm_stream_si128(d + 1, reduce(b));
        _mm_stream_si128(d + 2, reduce(c));
        _mm_stream_si128(d + 3, reduce(e));
    }
    uint64_t* t = (uint64_t*)d;
    for (size_t i = 0; i < words % 8; ++i) t[i] = one(src + 8 * i);  // tail
}

}  // namespace nhip
