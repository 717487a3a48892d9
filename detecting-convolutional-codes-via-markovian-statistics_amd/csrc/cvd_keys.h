// Row-key definitions shared by the host table build (cvd_host.cpp), the
// compiled kernels (cvd_kernels.hip) and the kernels hipRTC specialises at run
// time (cvd_device.h): self-contained, no standard-library includes.
#pragma once

#ifndef CVD_HD
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define CVD_HD __host__ __device__ __forceinline__
#else
#define CVD_HD inline
#endif
#endif

namespace cvd {

// row record: 2^n doubles + 2^n int32 successor slots, padded to a power of
// two (64 B at n = 2: one record never straddles a cache line)
constexpr int row_words_c(int R) { return 3 * R <= 4 ? 4 : 2 * row_words_c((R + 1) / 2); }

// Device key layout (hash keys, row cursor) for 2^m >= 8: inside each 32-bit
// word, state 8w + s sits in nibble bitrev3(s) -- the order in which a lane's
// packed (D(2j), D(2j+1)) pairs collapse into nibbles with one v_perm and one
// shift-add.  key_swap converts either way (an involution: nibbles 1 <-> 4, 3 <-> 6).
CVD_HD unsigned key_swap(unsigned w) {
  const unsigned t = (w ^ (w >> 12)) & 0x0000F0F0u;
  return w ^ t ^ (t << 12);
}
constexpr CVD_HD int key_nibble(int M, int s) {   // nibble index of state s within its word
  const int b = s & 7;
  return M >= 8 ? (((b & 1) << 2) | (b & 2) | ((b >> 2) & 1)) : b;
}

CVD_HD unsigned rotl32(unsigned x, int r) { return (x << r) | (x >> (32 - r)); }
CVD_HD unsigned long long mul_wide(unsigned a, unsigned b) { return (unsigned long long)a * b; }

// Hash of a nibble-packed key (host and device must agree): a multiply-
// accumulate fold, one v_mad_u64_u32 per key word with a distinct odd
// multiplier, then one finalising 32x32->64 product p = x * C of the folded
// word.  The home slot is ph & hmask, the filter block (pl >> 3) & bmask and the
// filter pattern pair (ph >> 3) & (kFilterPatterns - 1) (the device takes both as
// byte offsets, pl & (bmask << 3) and ph & ((kFilterPatterns - 1) << 3): one AND
// each).  Quality only affects speed (probe lengths, filter false positives),
// never results.
CVD_HD void key_hash(const unsigned* w, int nw, unsigned& ph, unsigned& pl) {
  unsigned long long acc = 0x9E3779B97F4A7C15ull ^ (unsigned)nw;
  for (int i = 0; i < nw; ++i) acc += mul_wide(w[i], 0x85EBCA77u + 0x6A09E668u * (unsigned)i);
  const unsigned x = (unsigned)acc ^ (unsigned)(acc >> 32);
  const unsigned long long p = mul_wide(x, 0x85EBCA6Bu);
  ph = (unsigned)(p >> 32);
  pl = (unsigned)p;
}

// key_hash of the key whose every nibble is c less than w's (c = 0..3): the fold
// is linear in the words, and w_i - c * 0x11111111 never borrows (every nibble
// of w is >= c), so the accumulator is the plain fold of w minus c * K_nw,
// K_nw = sum_i 0x11111111 * multiplier_i (mod 2^64) -- a select of the start
// value instead of a subtraction per key word.
CVD_HD unsigned long long key_fold_offset(int nw) {
  unsigned long long k = 0;
  for (int i = 0; i < nw; ++i) k += mul_wide(0x11111111u, 0x85EBCA77u + 0x6A09E668u * (unsigned)i);
  return k;
}
CVD_HD unsigned long long key_fold_start(int nw, unsigned c) {
  return (0x9E3779B97F4A7C15ull ^ (unsigned)nw) - (unsigned long long)c * key_fold_offset(nw);
}
// kLo: the offset is kLo or kLo + 1 (two constants, one select)
template <int kLo>
CVD_HD void key_hash_less(const unsigned* w, int nw, unsigned c, unsigned& ph, unsigned& pl) {
  unsigned long long acc = c == (unsigned)kLo + 1u ? key_fold_start(nw, kLo + 1) : key_fold_start(nw, kLo);
  for (int i = 0; i < nw; ++i) acc += mul_wide(w[i], 0x85EBCA77u + 0x6A09E668u * (unsigned)i);
  const unsigned x = (unsigned)acc ^ (unsigned)(acc >> 32);
  const unsigned long long p = mul_wide(x, 0x85EBCA6Bu);
  ph = (unsigned)(p >> 32);
  pl = (unsigned)p;
}

// Blocked Bloom filter over the row keys (explicit path): one 64-bit block (two
// 32-bit words) per key, a pattern of three bits in each word.  A lookup of a
// state that is not a row (most lookups at p >= 0.05 and for every H2 sequence)
// ends on this one L2-resident 8-byte load.  The pattern pair comes from a table
// of kFilterPatterns entries indexed by bits 3..12 of ph (the device keeps it in
// LDS as 64-bit entries: one AND gives the byte offset, one LDS read the pair,
// instead of the shifts and ors of six bit positions).  Two words with three
// bits each pass a non-row ~10x less often than one word at the same filter size
// (p = 0.2, ~1.9 rows per 32-bit word: ~0.4% -> ~0.04%), and every false
// positive is a directory line read.  4,096 pattern pairs (32 KiB of LDS).  The kernel
// variant with the filter itself in LDS (walking models) builds a second copy of the
// filter with 1,024 pattern pairs (8 KiB, CVD_FILTER_PAT_BITS=10 in that kernel) to make
// room; 1,024 for every filter measured +1.6% / +2.5% per launch at p = 0.1 / 0.2, where
// a two-word block holds 3-4 keys (profiles/r03z/ab_pat.jsonl).
#ifndef CVD_FILTER_PAT_BITS
#define CVD_FILTER_PAT_BITS 12
#endif
constexpr int kFilterPatBits = CVD_FILTER_PAT_BITS, kFilterPatterns = 1 << kFilterPatBits;
constexpr int kFilterPatBitsLds = 10;
// The bit-sliced kernel's LDS pre-filter (cvd_k1s.h, CVD_K1S_PF): one bit per row at index
// pl >> (32 - kBsPfLog2Bits) of its key hash, 2^20 bits = 128 KiB, one copy per 1,024-thread
// block (one block per CU, beside the 1,024-pair pattern table); a lane whose bit is clear
// skips its L2 filter read (built by cvd_host.cpp build_hash)
// (CVD_K1S_PF_LOG2=19: 64 KiB in 512-thread blocks, two per CU; timing studies)
#ifndef CVD_K1S_PF_LOG2
#define CVD_K1S_PF_LOG2 20
#endif
constexpr int kBsPfLog2Bits = CVD_K1S_PF_LOG2;
CVD_HD unsigned filter_pattern(unsigned i) {
  unsigned x = (i + 1u) * 0x9E3779B1u;
  x ^= x >> 15;
  x *= 0x85EBCA77u;
  x ^= x >> 13;
  const unsigned b0 = x & 31u;
  unsigned b1 = (x >> 5) & 31u, b2 = (x >> 10) & 31u;
  if (b1 == b0) b1 = (b1 + 1u) & 31u;
  while (b2 == b0 || b2 == b1) b2 = (b2 + 1u) & 31u;
  return (1u << b0) | (1u << b1) | (1u << b2);
}
// pattern pair i: low word filter_pattern(i), high word filter_pattern(i + kFilterPatterns)
// (npat: the table size, kFilterPatterns unless a timing study overrides it on both sides)
CVD_HD unsigned filter_pattern_hi(unsigned i, unsigned npat = kFilterPatterns) { return filter_pattern(i + npat); }
CVD_HD unsigned filter_pattern_index(unsigned ph, unsigned npat = kFilterPatterns) { return (ph >> 3) & (npat - 1u); }
// block index (words 2b, 2b + 1); bmask = blocks - 1 (the device takes the
// block's byte offset as pl & (bmask << 3))
CVD_HD unsigned filter_block_index(unsigned pl, unsigned bmask) { return (pl >> 3) & bmask; }

// empty hash slot: key word 0 (a nibble-packed metric vector never has 15 in
// every nibble, metrics stay <= (ceil(m/k)+1) n - 1 <= 14)
constexpr unsigned kEmptyKey = 0xFFFFFFFFu;

}  // namespace cvd
