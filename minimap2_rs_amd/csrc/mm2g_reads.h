// Query reads -> the device nt4 format (mm2g_reads.cpp; include/mm2g.h "nt4 read batch").
#pragma once
#include <stdint.h>

namespace mm2g {
// Word offsets of each read's 2-bit codes (ceil(L/32) words per read); returns the total.
uint64_t nt4_words_for(const uint64_t* lens, uint32_t n, uint64_t* pk_off);
// Upper bound of the words nt4_pack writes (codes + a bitmap for every read).
uint64_t nt4_words_bound(const uint64_t* offs, uint32_t n);
// Pack n ASCII reads (seq[offs[r] .. offs[r+1])) on n_threads host threads.
// Returns the words written, or a negative value when cap_words is too small.
int64_t nt4_pack(const uint8_t* seq, const uint64_t* offs, uint32_t n, uint64_t* pk_off, uint64_t* amb_off, uint64_t* words,
                 uint64_t cap_words, int n_threads);
}  // namespace mm2g
