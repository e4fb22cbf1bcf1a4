// Host side of the query read input: ASCII reads -> the device nt4 format
// (include/mm2g.h, "nt4 read batch"; SURVEY.md §8a row a1 / BASELINE north_star
// "per-read windowed minimizer hashing over 2-bit-packed bases").
//
// nt4 (src/nt4.rs:2-10) maps A/a->0, C/c->1, G/g->2, T/t->3 and every other
// byte to 4.  Reads cross PCIe and sit in HBM as 2 bits per base; the few reads
// that hold an ambiguous base (code 4) also carry a 1-bit-per-base bitmap.
// Packing runs on host threads, 32 bases per step with AVX2 where the CPU has it.
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "mm2g_reads.h"

namespace mm2g {

// ---- 32 bases -> one word of 2-bit codes (base j at bits 2j) + ambiguity bits
static inline uint8_t nt4_byte(uint8_t b) {
    switch (b | 0x20) { case 'a': return 0; case 'c': return 1; case 'g': return 2; case 't': return 3; default: return 4; }
}
static void pack_scalar(const uint8_t* s, uint64_t n, uint64_t* words, uint32_t* amb_or, std::vector<uint64_t>* amb) {
    // n bases -> ceil(n/32) words; amb (if non-null) receives ceil(n/64) bitmap words
    uint32_t any = 0;
    for (uint64_t w0 = 0; w0 < n; w0 += 32) {
        uint64_t v = 0;
        const uint64_t e = std::min<uint64_t>(n - w0, 32);
        for (uint64_t j = 0; j < e; ++j) {
            const uint8_t c = nt4_byte(s[w0 + j]);
            if (c < 4) v |= (uint64_t)c << (2 * j);
            else {
                any = 1;
                if (amb) (*amb)[(w0 + j) >> 6] |= 1ULL << ((w0 + j) & 63);
            }
        }
        words[w0 >> 5] = v;
    }
    *amb_or |= any;
}

__attribute__((target("avx2"))) static void pack_avx2(const uint8_t* s, uint64_t n, uint64_t* words, uint32_t* amb_or,
                                                            std::vector<uint64_t>* amb) {
    const __m256i lc = _mm256_set1_epi8(0x20);
    const __m256i ca = _mm256_set1_epi8('a'), cc = _mm256_set1_epi8('c'), cg = _mm256_set1_epi8('g'), ct = _mm256_set1_epi8('t');
    const __m256i one = _mm256_set1_epi8(1), two = _mm256_set1_epi8(2);
    const __m256i w14 = _mm256_set1_epi16(0x0401), w116 = _mm256_set1_epi32(0x00100001);
    const __m256i pick = _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                          0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    uint32_t any = 0;
    uint64_t w0 = 0;
    for (; w0 + 32 <= n; w0 += 32) {
        const __m256i v = _mm256_or_si256(_mm256_loadu_si256((const __m256i*)(s + w0)), lc);
        const __m256i ia = _mm256_cmpeq_epi8(v, ca), ic = _mm256_cmpeq_epi8(v, cc), ig = _mm256_cmpeq_epi8(v, cg),
                      it = _mm256_cmpeq_epi8(v, ct);
        // code = C:1, G:2, T:3 (A and ambiguous: 0)
        const __m256i code = _mm256_or_si256(_mm256_and_si256(_mm256_or_si256(ic, it), one), _mm256_and_si256(_mm256_or_si256(ig, it), two));
        const uint32_t valid = (uint32_t)_mm256_movemask_epi8(_mm256_or_si256(_mm256_or_si256(ia, ic), _mm256_or_si256(ig, it)));
        // 32 one-byte codes -> 64 bits: pairs (c0 + 4 c1), quads (+ 16 (c2 + 4 c3)),
        // then byte 0 of every 32-bit lane
        const __m256i p2 = _mm256_maddubs_epi16(code, w14);
        const __m256i p4 = _mm256_madd_epi16(p2, w116);
        const __m256i b4 = _mm256_shuffle_epi8(p4, pick);
        words[w0 >> 5] = (uint64_t)(uint32_t)_mm256_extract_epi32(b4, 0) | ((uint64_t)(uint32_t)_mm256_extract_epi32(b4, 4) << 32);
        if (valid != 0xffffffffu) {
            any = 1;
            if (amb) (*amb)[w0 >> 6] |= (uint64_t)(~valid) << (w0 & 63);
        }
    }
    if (w0 < n) {
        uint32_t a2 = 0;
        std::vector<uint64_t> tail;
        std::vector<uint64_t>* tp = nullptr;
        if (amb) { tail.assign(1, 0); tp = &tail; }
        pack_scalar(s + w0, n - w0, words + (w0 >> 5), &a2, tp);
        if (a2) {
            any = 1;
            if (amb) (*amb)[w0 >> 6] |= tail[0] << (w0 & 63);   // w0 is a multiple of 32: the tail fits the same or next word half
        }
    }
    *amb_or |= any;
}

static bool have_avx2() {
    static const bool v = __builtin_cpu_supports("avx2");
    return v;
}

static void pack_read(const uint8_t* s, uint64_t n, uint64_t* words, uint32_t* amb_or, std::vector<uint64_t>* amb) {
    if (have_avx2()) pack_avx2(s, n, words, amb_or, amb);
    else pack_scalar(s, n, words, amb_or, amb);
}

// Run fn(t) for t in [0, nt) on nt threads (the calling thread takes t = 0).
template <typename F>
static void par_run(int nt, F fn) {
    if (nt <= 1) { fn(0); return; }
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int t = 1; t < nt; ++t) th.emplace_back(fn, t);
    fn(0);
    for (auto& x : th) x.join();
}

uint64_t nt4_words_for(const uint64_t* lens, uint32_t n, uint64_t* pk_off) {
    uint64_t w = 0;
    for (uint32_t r = 0; r < n; ++r) { if (pk_off) pk_off[r] = w; w += (lens[r] + 31) / 32; }
    return w;
}

int64_t nt4_pack(const uint8_t* seq, const uint64_t* offs, uint32_t n, uint64_t* pk_off, uint64_t* amb_off, uint64_t* words,
                 uint64_t cap_words, int n_threads) {
    std::vector<uint64_t> lens(n);
    for (uint32_t r = 0; r < n; ++r) lens[r] = offs[r + 1] - offs[r];
    const uint64_t nw = nt4_words_for(lens.data(), n, pk_off);
    if (nw > cap_words) return -1;
    // 1. 2-bit codes of every read, in parallel (reads handed out in blocks);
    //    which reads hold an ambiguous base
    std::vector<uint8_t> has(n, 0);
    const int nt = std::max(1, std::min<int>(n_threads, (int)std::max<uint64_t>(1, (offs[n] - offs[0]) >> 20)));
    std::atomic<uint32_t> next{0};
    constexpr uint32_t BLK = 16;
    par_run(nt, [&](int) {
        for (;;) {
            const uint32_t r0 = next.fetch_add(BLK);
            if (r0 >= n) break;
            for (uint32_t r = r0; r < std::min(n, r0 + BLK); ++r) {
                uint32_t a = 0;
                pack_read(seq + offs[r], lens[r], words + pk_off[r], &a, nullptr);
                has[r] = (uint8_t)a;
            }
        }
    });
    // 2. bitmaps for those reads (rare), after all code words
    uint64_t w = nw;
    for (uint32_t r = 0; r < n; ++r) {
        if (has[r]) { amb_off[r] = w; w += (lens[r] + 63) / 64; }
        else amb_off[r] = ~0ULL;
    }
    if (w > cap_words) return -(int64_t)w;
    for (uint32_t r = 0; r < n; ++r) {
        if (!has[r]) continue;
        const uint64_t nb = (lens[r] + 63) / 64;
        std::vector<uint64_t> bm(nb, 0);
        std::vector<uint64_t> tmp((lens[r] + 31) / 32);
        uint32_t a = 0;
        pack_scalar(seq + offs[r], lens[r], tmp.data(), &a, &bm);
        memcpy(words + amb_off[r], bm.data(), nb * 8);
    }
    return (int64_t)w;
}

// Upper bound of the words nt4_pack needs (every read with a bitmap).
uint64_t nt4_words_bound(const uint64_t* offs, uint32_t n) {
    uint64_t w = 0;
    for (uint32_t r = 0; r < n; ++r) { const uint64_t L = offs[r + 1] - offs[r]; w += (L + 31) / 32 + (L + 63) / 64; }
    return w;
}

}  // namespace mm2g
