// Shared host/device definitions: the trial-stream randomness spec (Philox4x32-10)
// and the convolutional-code description in the reference's convention.
//
// The randomness spec is the build's own (the reference never seeds its trial
// simulations and its simulator is missing — SURVEY.md §0.1, §8 row A5); it is
// restated independently in oracle/philox.py and oracle/cvd_oracle.c and the
// three are checked against each other by the tests.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define CVD_HD __host__ __device__ __forceinline__
#else
#define CVD_HD inline
#endif

namespace cvd {

constexpr uint32_t kPhiloxM0 = 0xD2511F53u;
constexpr uint32_t kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u;
constexpr uint32_t kPhiloxW1 = 0xBB67AE85u;
constexpr uint32_t kKindNoise = 0;
constexpr uint32_t kKindInput = 1;
constexpr uint32_t kLearnTag = 0xC0DE1EA7u;

struct U4 { uint32_t x, y, z, w; };

// Philox4x32-10 (Salmon et al., SC'11); Random123 known-answer vectors in tests.
CVD_HD U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 multiply per product (v_mad_u64_u32 on gfx950)
    const uint64_t p0 = (uint64_t)kPhiloxM0 * c0, p1 = (uint64_t)kPhiloxM1 * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#if defined(__HIP_DEVICE_COMPILE__)
    // one v_bitop3_b32 (xor3, truth table 0x96) per output word; LLVM otherwise emits two v_xor_b32
    uint32_t n0, n2;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(hi1), "v"(c1), "s"(k0));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(hi0), "v"(c3), "s"(k1));
#else
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
#endif
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += kPhiloxW0; k1 += kPhiloxW1;
  }
  return U4{c0, c1, c2, c3};
}

// One Philox round of B independent blocks under the round key (k0, k1): the
// caller advances the key (k += W) between rounds, 10 rounds in all
template <int B>
CVD_HD void philox_round(uint32_t (&c)[B][4], uint32_t k0, uint32_t k1) {
  uint64_t p0[B], p1[B];
#pragma unroll
  for (int b = 0; b < B; ++b) {
    p0[b] = (uint64_t)kPhiloxM0 * c[b][0];
    p1[b] = (uint64_t)kPhiloxM1 * c[b][2];
  }
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const uint32_t hi0 = (uint32_t)(p0[b] >> 32), lo0 = (uint32_t)p0[b];
    const uint32_t hi1 = (uint32_t)(p1[b] >> 32), lo1 = (uint32_t)p1[b];
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t n0, n2;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(hi1), "v"(c[b][1]), "s"(k0));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(hi0), "v"(c[b][3]), "s"(k1));
#else
    const uint32_t n0 = hi1 ^ c[b][1] ^ k0, n2 = hi0 ^ c[b][3] ^ k1;
#endif
    c[b][0] = n0; c[b][1] = lo1; c[b][2] = n2; c[b][3] = lo0;
  }
}

// B independent Philox4x32-10 blocks under one key, advanced round by round
// over all blocks, so that neighbouring instructions belong to different
// blocks: each block's xor3 -> multiply dependency (a wait state on gfx950)
// is covered by the other blocks' work instead of an s_nop.
template <int B>
CVD_HD void philox_blocks(uint32_t (&c)[B][4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0[B], p1[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      p0[b] = (uint64_t)kPhiloxM0 * c[b][0];
      p1[b] = (uint64_t)kPhiloxM1 * c[b][2];
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const uint32_t hi0 = (uint32_t)(p0[b] >> 32), lo0 = (uint32_t)p0[b];
      const uint32_t hi1 = (uint32_t)(p1[b] >> 32), lo1 = (uint32_t)p1[b];
#if defined(__HIP_DEVICE_COMPILE__)
      uint32_t n0, n2;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(hi1), "v"(c[b][1]), "s"(k0));
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(hi0), "v"(c[b][3]), "s"(k1));
#else
      const uint32_t n0 = hi1 ^ c[b][1] ^ k0, n2 = hi0 ^ c[b][3] ^ k1;
#endif
      c[b][0] = n0; c[b][1] = lo1; c[b][2] = n2; c[b][3] = lo0;
    }
    k0 += kPhiloxW0; k1 += kPhiloxW1;
  }
}

// The ten round keys (k0 + r W0, k1 + r W1) of a Philox key held in VGPRs: a v_bitop3 with a
// scalar source issues at ~4.3 cycles per wave64 instruction on gfx950, with vector sources at
// ~2.8 (profiles/r05an), and the compiler re-copies a uniform key into a VGPR at every use
// rather than hoist it -- so a caller that runs many blocks under one key precomputes them
#ifndef CVD_PHILOX_VMUL
#define CVD_PHILOX_VMUL 0
#endif
struct PhiloxKeysV {
  uint32_t k[20];
  uint32_t m0 = kPhiloxM0, m1 = kPhiloxM1;   // (CVD_PHILOX_VMUL: the multipliers in VGPRs too)
  CVD_HD void init(uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (CVD_PHILOX_VMUL) asm volatile("" : "+v"(m0), "+v"(m1));
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      k[2 * r] = k0 + (uint32_t)r * kPhiloxW0;
      k[2 * r + 1] = k1 + (uint32_t)r * kPhiloxW1;
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < 20; ++i) asm volatile("" : "+v"(k[i]));
#endif
  }
};
template <int B>
CVD_HD void philox_blocks(uint32_t (&c)[B][4], const PhiloxKeysV& kv) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0[B], p1[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      p0[b] = (uint64_t)(CVD_PHILOX_VMUL ? kv.m0 : kPhiloxM0) * c[b][0];
      p1[b] = (uint64_t)(CVD_PHILOX_VMUL ? kv.m1 : kPhiloxM1) * c[b][2];
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const uint32_t hi0 = (uint32_t)(p0[b] >> 32), lo0 = (uint32_t)p0[b];
      const uint32_t hi1 = (uint32_t)(p1[b] >> 32), lo1 = (uint32_t)p1[b];
#if defined(__HIP_DEVICE_COMPILE__)
      uint32_t n0, n2;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(hi1), "v"(c[b][1]), "v"(kv.k[2 * r]));
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(hi0), "v"(c[b][3]), "v"(kv.k[2 * r + 1]));
#else
      const uint32_t n0 = hi1 ^ c[b][1] ^ kv.k[2 * r], n2 = hi0 ^ c[b][3] ^ kv.k[2 * r + 1];
#endif
      c[b][0] = n0; c[b][1] = lo1; c[b][2] = n2; c[b][3] = lo0;
    }
  }
}
// one round of B blocks under round r of VGPR round keys (the fused kernel's pipelined rounds)
template <int B>
CVD_HD void philox_round(uint32_t (&c)[B][4], const PhiloxKeysV& kv, int r) {
  uint64_t p0[B], p1[B];
#pragma unroll
  for (int b = 0; b < B; ++b) {
    p0[b] = (uint64_t)kPhiloxM0 * c[b][0];
    p1[b] = (uint64_t)kPhiloxM1 * c[b][2];
  }
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const uint32_t hi0 = (uint32_t)(p0[b] >> 32), lo0 = (uint32_t)p0[b];
    const uint32_t hi1 = (uint32_t)(p1[b] >> 32), lo1 = (uint32_t)p1[b];
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t n0, n2;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(hi1), "v"(c[b][1]), "v"(kv.k[2 * r]));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(hi0), "v"(c[b][3]), "v"(kv.k[2 * r + 1]));
#else
    const uint32_t n0 = hi1 ^ c[b][1] ^ kv.k[2 * r], n2 = hi0 ^ c[b][3] ^ kv.k[2 * r + 1];
#endif
    c[b][0] = n0; c[b][1] = lo1; c[b][2] = n2; c[b][3] = lo0;
  }
}

// the launch's key pair (SGPRs; the round keys by scalar adds per call)
struct PhiloxKeysS {
  uint32_t k0, k1;
};
template <int B>
CVD_HD void philox_blocks(uint32_t (&c)[B][4], const PhiloxKeysS& ks) {
  philox_blocks<B>(c, ks.k0, ks.k1);
}

CVD_HD uint32_t u4_get(const U4& v, uint32_t i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

// Identity of one simulated sequence.
struct StreamKey {
  uint32_t k0, k1;      // seed lo / hi
  uint32_t tag;         // grid_tag(N, p) or kLearnTag
};

CVD_HD uint32_t ctr_hi(uint64_t seq_id, uint32_t kind) {
  return (uint32_t)((seq_id >> 32) & 0xFFFFu) | (kind << 16);
}

// thr(p) = floor(p * 2^32), p in [0, 1]; flip iff uniform < thr.
inline uint64_t noise_threshold(double p) { return (uint64_t)(p * 4294967296.0); }

// BSC flips of one received word, bit-sliced (spec: oracle/philox.py).  The
// 32-bit uniform of word bit b is u_b = sum_i bit_b(P_i) 2^(31 - i) over the
// word's 32 bit-planes P_i = word (i % 4) of
// philox(ctr=(8 w + i / 4, seq_lo, ctr_hi(seq, kKindNoise), tag)), and bit b
// flips iff u_b < thr.  The planes are compared with thr most significant first
// for every bit at once: a bit is decided at the first plane where its uniform
// bit differs from thr's (a 1 in thr over a 0 in u: flip), so the planes after
// the last undecided bit are never drawn -- about 7 planes per word on one lane
// instead of one uniform per code bit.  thr = 0 draws nothing (no flips),
// thr = 2^32 flips every bit.
constexpr int kNoisePlanes = 32, kNoiseBlocksPerWord = 8;

// one plane: undecided bits U, flips F; thr bit tb of the plane
CVD_HD void noise_plane(uint32_t r, uint32_t tb, uint32_t& U, uint32_t& F) {
  if (tb) { F |= U & ~r; U &= r; }
  else U &= ~r;
}

CVD_HD uint32_t noise_word(const StreamKey& key, uint64_t seq_id, uint64_t w, uint64_t thr, uint32_t valid) {
  if (thr >= 4294967296ull) return valid;
  uint32_t U = thr ? valid : 0u, F = 0u;
  const uint32_t t = (uint32_t)thr, slo = (uint32_t)seq_id, nhi = ctr_hi(seq_id, kKindNoise);
  for (int j = 0; j < kNoiseBlocksPerWord && U; ++j) {
    const U4 x = philox((uint32_t)(w * kNoiseBlocksPerWord + (uint64_t)j), slo, nhi, key.tag, key.k0, key.k1);
    noise_plane(x.x, (t >> (31 - 4 * j)) & 1u, U, F);
    noise_plane(x.y, (t >> (30 - 4 * j)) & 1u, U, F);
    noise_plane(x.z, (t >> (29 - 4 * j)) & 1u, U, F);
    noise_plane(x.w, (t >> (28 - 4 * j)) & 1u, U, F);
  }
  return F;
}

// 32-bit tag of an (N, p) grid point (splitmix64 fold, top bit clear).
inline uint32_t grid_tag(int64_t N, double p) {
  uint64_t bits;
  __builtin_memcpy(&bits, &p, 8);
  uint64_t x = (uint64_t)N * 0x9E3779B97F4A7C15ull + bits;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)((x ^ (x >> 32)) & 0x7FFFFFFFu);
}

// Encoder description derived from generator taps (reference convention,
// viterbi_markov.py:82-106): gmask[j*k + i] bit d = taps[j][i][d] (d <= m);
// x_i = u_i | (state << 1); out_j = XOR_i parity(gmask[j][i] & x_i);
// next = (U | state << k) & (2^m - 1).
constexpr int kMaxK = 4, kMaxN = 8, kMaxM = 8;
struct CodeDesc {
  int32_t k, n, m;
  uint32_t gmask[kMaxN * kMaxK];
};

CVD_HD uint32_t parity32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popc(x) & 1u;
#else
  return (uint32_t)__builtin_popcount(x) & 1u;
#endif
}

CVD_HD uint32_t enc_out(const CodeDesc& c, uint32_t s, uint32_t U) {
  uint32_t o = 0;
  for (int j = 0; j < c.n; ++j) {
    uint32_t b = 0;
    for (int i = 0; i < c.k; ++i) b ^= parity32(c.gmask[j * c.k + i] & (((U >> i) & 1u) | (s << 1)));
    o |= b << j;
  }
  return o;
}

CVD_HD uint32_t enc_next(const CodeDesc& c, uint32_t s, uint32_t U) {
  return (U | (s << c.k)) & ((1u << c.m) - 1u);
}

// Received-word packing in HBM: each 32-bit word holds spw = floor(32 / n)
// consecutive steps, step i of the word in bits [n*i, n*i + n).  Words are
// interleaved across sequences: word w of sequence q lives at r[w * pitch + q]
// (pitch >= number of sequences), so a wave's 64 lanes read 256 contiguous bytes.
CVD_HD int steps_per_word(int n) { return 32 / n; }

}  // namespace cvd
