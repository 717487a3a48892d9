// HIP kernels for gfx950 (MI355X): the Monte-Carlo hot path of the reference
// (Pd_plotter.py:198-233 with the missing simulator of Pd_plotter.py:149/212/219,
// the Eq. 4-5 recursion of viterbi_markov.py:139-159 and the likelihood
// accumulation of Pd_plotter.py:106-116).
//
//   gen_kernel               encoder + BSC(p) -> bit-packed received words in HBM
//                            (one sequence per lane, words interleaved across lanes)
//   detect_table_kernel      enumerated-state automaton: per step one (next, c)
//                            record + one log P̂1 row entry; tables in LDS when they fit
//   detect_explicit_kernel   explicit 2^m relative-metric vector per lane (nibble
//                            packed), Eq. 4-5 for ALL 2^n received words with packed
//                            16-bit VALU ops (two received words per instruction), T_ref
//                            count by exact comparison, P̂1 row from a hashed table
//
// All sums are sequential fp64 additions in t order (no FMA, no reassociation),
// so every per-sequence sum and decision is bit-identical to the reference's
// `logp += math.log(pij)` loop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <string>

#include "../../include/cvd.h"
#include "cvd_common.h"
#include "cvd_internal.h"
#include "cvd_device.h"

using namespace cvd;

#define HIP_CHECK(x)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      set_error(std::string("HIP error '") + hipGetErrorString(e_) + "' at " #x);          \
      return CVD_E_HIP;                                                                   \
    }                                                                                     \
  } while (0)

using namespace cvd_dev;

namespace {

// ───────────────────────────── generator ────────────────────────────────────

// k = 2, n = 3 encoder form of ChunkEncoder (1: stride-3 window, 0: per-phase windows)
#ifndef CVD_GEN_K2_STRIDE3
#define CVD_GEN_K2_STRIDE3 1
#endif
// noise straggler exchange: one block per slot lane, a pair's two blocks on two lanes
// (1), or both blocks of a pair on one slot lane (0)
// gen_fast_kernel: the noise Philox keys' round keys precomputed in VGPRs (PhiloxKeysV)
#ifndef CVD_GEN_VKEYS
#define CVD_GEN_VKEYS 1
#endif
// mc_table16_kernel (the fused C1 path): the same, off by default (its 70 VGPRs hold 7 waves per
// SIMD; the round keys cost 20)
#ifndef CVD_FUSED_VKEYS
#define CVD_FUSED_VKEYS 0
#endif
#ifndef CVD_GEN_XCHG_SPLIT
#define CVD_GEN_XCHG_SPLIT 1
#endif
#ifndef CVD_GEN_SEQ_LDS       // slot lanes read the sequence ids from LDS (1) or compute them (0)
#define CVD_GEN_SEQ_LDS 0
#endif
#ifndef CVD_FUSED_XCHG_SPLIT   // the same in the fused trial kernel (ChunkEncoder::finish)
#define CVD_FUSED_XCHG_SPLIT 0
#endif
constexpr int kTapSlots = 10;     // longest unrolled tap list per output (m <= 8, k = 1: 9 taps)

struct GenArgs {
  CodeDesc enc;
  uint32_t k0, k1, tag, thr_lo;
  int32_t thr_all, random_input;
  int32_t hs;                     // gen_fast_kernel: history steps ceil(m / k)
  uint32_t slots;                 // gen_fast_kernel: noise exchange slots per round (64; tests: fewer)
  uint32_t taps[kMaxN][2];        // gen_fast_kernel: shift set of output j on input phase r
  // the same taps as window shifts (v_alignbit amounts), per output j, every unused slot
  // a shift that moves only empty lanes of the window onto lane j (ChunkEncoder kT > 0):
  // slot i in bits 5 (i % 6) of word i / 6 (v_alignbit reads the low 5 bits of its shift
  // operand, so one s_lshr extracts a slot); ntap = the longest list (0: the form has no
  // shift list, k = 2 per-phase windows)
  uint32_t tpk[kMaxN][2];
  int32_t ntap;
  int64_t N, seq_base, seq_stride, pitch, q0, count;
  uint32_t* r;
};

// Encoder output for compile-time (k, n): gm[j*k + i] are the tap masks.
template <int k, int n>
__device__ __forceinline__ uint32_t enc_out_t(const uint32_t (&gm)[n * k], uint32_t s, uint32_t U) {
  uint32_t o = 0;
#pragma unroll
  for (int j = 0; j < n; ++j) {
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < k; ++i) b ^= parity32(gm[j * k + i] & (((U >> i) & 1u) | (s << 1)));
    o |= b << j;
  }
  return o;
}

// k, n > 0: compile-time shape (only n*k tap masks live); 0, 0: runtime shape.
template <int kT, int nT>
__global__ __launch_bounds__(kBlock) void gen_kernel(GenArgs a) {
  const int64_t li = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (li >= a.count) return;
  const int64_t q = a.q0 + li;
  const uint64_t sid = (uint64_t)(a.seq_base + li * a.seq_stride);
  const uint32_t slo = (uint32_t)sid, nhi = ctr_hi(sid, kKindNoise), ihi = ctr_hi(sid, kKindInput);
  const int n = nT ? nT : a.enc.n, k = kT ? kT : a.enc.k, spw = 32 / n;
  constexpr int NK = (kT && nT) ? kT * nT : 1;
  uint32_t gm[NK];
#pragma unroll
  for (int i = 0; i < NK; ++i) gm[i] = a.enc.gmask[i];
  const uint32_t kmask = (1u << k) - 1u;
  const int64_t nwords = (a.N + spw - 1) / spw;
  uint32_t s = 0;
  int64_t cblk = -1;
  U4 cval{0, 0, 0, 0};
  uint32_t out4[4] = {0u, 0u, 0u, 0u};
  const int64_t nw4 = (nwords + 3) & ~(int64_t)3;
  for (int64_t w = 0; w < nw4; ++w) {
    if (w >= nwords) {               // zero padding of the last 16-byte chunk
      out4[w & 3] = 0u;
      if ((w & 3) == 3)
        *reinterpret_cast<uint4*>(a.r + chunk_index(w >> 2, a.pitch, q)) = make_uint4(out4[0], out4[1], out4[2], out4[3]);
      continue;
    }
    const int64_t t0 = w * spw;
    const int ns = (int)min((int64_t)spw, a.N - t0);
    // BSC flips of the word's n*ns code bits (bit-sliced noise, noise_word)
    const uint32_t valid = n * ns >= 32 ? ~0u : (1u << (uint32_t)(n * ns)) - 1u;
    const StreamKey key{a.k0, a.k1, a.tag};
    const uint32_t nmask = noise_word(key, sid, (uint64_t)w, a.thr_all ? 4294967296ull : (uint64_t)a.thr_lo, valid);
    (void)nhi;
    // encoder input bits [t0*k, (t0+ns)*k) of the input stream
    uint32_t ib = 0;
    if (a.random_input) {
      const int64_t b0 = t0 * k;
      const int64_t W = b0 >> 5;
      const uint32_t off = (uint32_t)(b0 & 31);
      uint32_t wv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t Wh = W + h;
        if (h == 1 && off + (uint32_t)(ns * k) <= 32u) { wv[1] = 0; break; }
        if ((Wh >> 2) != cblk) {
          cblk = Wh >> 2;
          uint32_t k0 = a.k0, k1 = a.k1;
          asm volatile("" : "+s"(k0), "+s"(k1));
          cval = philox((uint32_t)cblk, slo, ihi, a.tag, k0, k1);
        }
        wv[h] = u4_get(cval, (uint32_t)(Wh & 3));
      }
      ib = off ? ((wv[0] >> off) | (wv[1] << (32u - off))) : wv[0];
    }
    uint32_t word = 0;
    for (int i = 0; i < ns; ++i) {
      const uint32_t U = (ib >> (uint32_t)(i * k)) & kmask;
      uint32_t o;
      if constexpr (kT && nT) o = enc_out_t<kT, nT>(gm, s, U);
      else o = enc_out(a.enc, s, U);
      word |= o << (uint32_t)(n * i);
      s = (U | (s << k)) & ((1u << a.enc.m) - 1u);
    }
    out4[w & 3] = word ^ nmask;
    if ((w & 3) == 3)
      *reinterpret_cast<uint4*>(a.r + chunk_index(w >> 2, a.pitch, q)) = make_uint4(out4[0], out4[1], out4[2], out4[3]);
  }
}

// Bit-parallel generator for compile-time (k, n) with k <= 2 (every config
// code): the same stream spec as gen_kernel, one SPW = 32/n step word at a time.
//  * Encoder: out_j(t) = XOR_i g_{j,i}[0] u_i(t) ^ XOR_b c_j[b] s_b(t)
//    (viterbi_markov.py:82-106 with x_i = u_i | s << 1), where s bit b is
//    u_{b % k}(t - 1 - b / k) and c_j[b] = XOR_i g_{j,i}[1 + b].  Per input phase
//    r the window W_r holds hs = ceil(m/k) history steps below the word's SPW
//    input bits, so every term is one shift of a window: output stream j is the
//    XOR of W_r >> sh over the host-built tap set taps[j][r] (bit sh), and the
//    n streams are bit-interleaved into the word (step i in bits n*i .. n*i+n-1).
//  * Noise: bit-sliced (noise_word, cvd_common.h): the word's bit-planes are
//    compared with thr for all of its code bits at once, most significant first,
//    four words at a time with the undecided (lane, word) pairs compacted across
//    the wave (noise_chunk_wave): ~2.5 Philox blocks per word, against NBITS / 4 =
//    8 blocks of one uniform per code bit.
template <int n>
__device__ __forceinline__ uint32_t spread_n(uint32_t x) {   // bit i -> bit n*i
  if constexpr (n == 1) {
    return x;
  } else if constexpr (n == 2) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    return (x | (x << 1)) & 0x55555555u;
  } else {
    static_assert(n == 3, "spread_n: n in 1..3");
    x &= 0x3FFu;
    x = (x | (x << 16)) & 0xFF0000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    return (x | (x << 2)) & 0x09249249u;
  }
}

// Rate 2/3 (k = 2, n = 3): the flat input bits of a word (bit 2t + r = u_r(t), t < 10)
// moved to the received word's stride (bit 3t + r): pairs t move up by t, one stage per
// bit of t (8, 4, 2, 1), three VALU each.  Lane 2 of every step stays 0.
__device__ __forceinline__ uint32_t spread23(uint32_t x) {
  x &= 0xFFFFFu;
  x = (x & 0x0000FFFFu) | ((x << 8) & 0x0F000000u);   // t = 8, 9: bits 16..19 -> 24..27
  x = (x & 0x0F0000FFu) | ((x << 4) & 0x000FF000u);   // t = 4..7: 8..15 -> 12..19
  x = (x & 0x0F00F00Fu) | ((x << 2) & 0x003C03C0u);   // t & 2: +2
  return (x & 0x030C30C3u) | ((x << 1) & 0x18618618u);   // t & 1: +1 -> bit 3t + r
}

__device__ __forceinline__ uint32_t even_bits(uint32_t x) {   // bit 2i -> bit i
  x &= 0x55555555u;
  x = (x | (x >> 1)) & 0x33333333u;
  x = (x | (x >> 2)) & 0x0F0F0F0Fu;
  x = (x | (x >> 4)) & 0x00FF00FFu;
  return (x | (x >> 8)) & 0x0000FFFFu;
}

// Four bit-planes r0..r3 (most significant first) against thr's matching 4-bit
// group `nib` (wave-uniform): the planes' value R of each code bit is below
// thr's bits (flip), equal (still undecided) or above (no flip).  R < T is a
// bit-sliced borrow chain over the planes least significant first, borrow' =
// MAJ(~r, t, borrow): one v_bitop3 per plane with t (0 or ~0) in an SGPR;
// equality e' = e & ~(r ^ t) is the other.  Two VALU per plane and no branches.
// (Tried: a 16-way switch over compile-time nibbles needs fewer VALU per case but
// compiles to a branch tree whose cases copy operands around; per-plane uniform
// branches were if-converted into selects; the direct MSB-first form with masks
// costs three VALU per plane.  Measured in profiles/r02z_gen.)
// kLaneNib: `nib` differs between lanes (t in a VGPR; the split exchange below).
template <bool kLaneNib = false>
__device__ __forceinline__ void noise_planes4(uint32_t nib, uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3,
                                              uint32_t& U, uint32_t& F) {
  const uint32_t r[4] = {r0, r1, r2, r3};
  const uint32_t b = kLaneNib ? nib : __builtin_amdgcn_readfirstlane(nib);
  uint32_t lt = 0u, eq = U;
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    const uint32_t ti = 0u - ((b >> (3 - i)) & 1u);
    // lt = MAJ(~r, t, lt) (truth table 0x8E), eq &= ~(r ^ t) (0x90)
    if constexpr (kLaneNib) {
      asm("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x8e" : "+v"(lt) : "v"(r[i]), "v"(ti));
      asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x90" : "+v"(eq) : "v"(r[i]), "v"(ti));
    } else {
      asm("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x8e" : "+v"(lt) : "v"(r[i]), "s"(ti));
      asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x90" : "+v"(eq) : "v"(r[i]), "s"(ti));
    }
  }
  F |= U & lt;
  U = eq;
}

// Per-wave LDS of the straggler exchange: slot records, and every lane's
// sequence counter words (a slot computes blocks of another lane's sequence)
struct NoiseLds {
  uint32_t u[64], m[64], slo[64], nhi[64];
};
__device__ __forceinline__ void wave_lds_sync() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); __builtin_amdgcn_wave_barrier(); }

// Flip masks F[g] of the words w4 + g (g < 4) of every lane's sequence, noise_word's
// spec (cvd_common.h) for the wave; live[g] = word exists for this lane.
//  * Planes 1-8 (Philox blocks 0 and 1) of all four words run unconditionally.  A code
//    bit is then still undecided with probability 2^-8, so ~12% of the wave's 256
//    (lane, word) pairs hold one (~30).
//  * Those pairs are compacted into consecutive lanes through LDS (su, sm: 64 words
//    each per wave): slot i computes the next two blocks (8 planes) of the i-th pair
//    and the result goes back to the owner.  After 16 planes ~0.1 undecided bits are
//    left per wave and chunk; a further pass runs only while the ballot finds one.
//  * seq(l): the (counter word 1, counter word 2) = (seq_lo, ctr_hi(seq, noise)) of
//    lane l's sequence, for the slot lanes (LDS copies in gen_fast_kernel, computed
//    from the lane index in the fused kernel).
// One word at a time (3 blocks for every lane, then single blocks while any lane is
// undecided) costs ~3.4 blocks per word; this ~2.5.
// (CVD_GEN_VTHR, timing study, off: the head's eight plane masks of the threshold, 0 or ~0,
// in VGPRs as well as the round keys -- 8 more VGPRs)
#ifndef CVD_GEN_VTHR
#define CVD_GEN_VTHR 0
#endif
struct NoiseKeysV : PhiloxKeysV {
  uint32_t tm[8];
  __device__ void init_thr(uint32_t t) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      tm[i] = 0u - ((t >> (31 - i)) & 1u);
      asm volatile("" : "+v"(tm[i]));
    }
  }
};
// four planes against VGPR plane masks m[0..3] (most significant first; noise_planes4's chains)
__device__ __forceinline__ void noise_planes4_m(const uint32_t* m, uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3,
                                                uint32_t& U, uint32_t& F) {
  const uint32_t r[4] = {r0, r1, r2, r3};
  uint32_t lt = 0u, eq = U;
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    asm("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x8e" : "+v"(lt) : "v"(r[i]), "v"(m[i]));
    asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x90" : "+v"(eq) : "v"(r[i]), "v"(m[i]));
  }
  F |= U & lt;
  U = eq;
}

// noise_head's plane tests on its two Philox blocks (already computed)
__device__ __forceinline__ void noise_head_planes(const GenArgs& a, const uint32_t (&xv)[2][4], bool live,
                                                  uint32_t valid, uint32_t& U, uint32_t& F) {
  const uint32_t t = a.thr_lo;
  U = live ? valid : 0u;
  F = 0u;
  noise_planes4(t >> 28, xv[0][0], xv[0][1], xv[0][2], xv[0][3], U, F);
  noise_planes4(t >> 24, xv[1][0], xv[1][1], xv[1][2], xv[1][3], U, F);
}

// Planes 1-8 (Philox blocks 0 and 1, unconditional) of word w of the sequence whose
// counter words are `own`: U = still undecided bits, F = flips so far (straight-line
// VALU, so a caller can interleave it with other work)
template <class KS>
__device__ __forceinline__ void noise_head(const GenArgs& a, uint2 own, uint32_t w, bool live, uint32_t valid,
                                           uint32_t& U, uint32_t& F, const KS& ks) {
  const uint32_t t = a.thr_lo;
  U = live ? valid : 0u;
  F = 0u;
  uint32_t xv[2][4];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    xv[b][0] = w * kNoiseBlocksPerWord + (uint32_t)b;
    xv[b][1] = own.x; xv[b][2] = own.y; xv[b][3] = a.tag;
  }
  philox_blocks<2>(xv, ks);
  if constexpr (std::is_same<KS, NoiseKeysV>::value) {
    noise_planes4_m(ks.tm, xv[0][0], xv[0][1], xv[0][2], xv[0][3], U, F);
    noise_planes4_m(ks.tm + 4, xv[1][0], xv[1][1], xv[1][2], xv[1][3], U, F);
  } else {
    noise_planes4(t >> 28, xv[0][0], xv[0][1], xv[0][2], xv[0][3], U, F);
    noise_planes4(t >> 24, xv[1][0], xv[1][1], xv[1][2], xv[1][3], U, F);
  }
}

// The straggler exchange after the heads of words w4 .. w4 + 3 (wave-collective):
// the (lane, word) pairs with an undecided bit are compacted into consecutive lanes
// through LDS (su, sm: 64 words each per wave); slot i computes the next two blocks
// (8 planes) of the i-th pair and the result goes back to the owner.  seq(l): the
// (counter word 1, counter word 2) = (seq_lo, ctr_hi(seq, noise)) of lane l's sequence,
// for the slot lanes.
template <typename Seq, class KS>
__device__ __forceinline__ void noise_exchange_pair(const GenArgs& a, uint32_t* su, uint32_t* sm, Seq seq,
                                                    uint32_t w4, uint32_t (&U)[4], uint32_t (&F)[4], const KS& ks) {
  const uint32_t t = a.thr_lo, lane = lane_id();
  const uint32_t nslots = a.slots - 1u < 64u ? a.slots : 64u;   // 1..64: every round makes progress
#pragma nounroll
  for (uint32_t j = 2; j < (uint32_t)kNoiseBlocksPerWord; j += 2) {
    uint32_t slot[4], tot = 0u;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint64_t b = __ballot(U[g] != 0u);
      slot[g] = tot + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
      tot += (uint32_t)__builtin_popcountll(b);
    }
    if (tot == 0u) break;   // every bit of every pair decided
#pragma nounroll
    for (uint32_t s0 = 0; s0 < tot; s0 += nslots) {   // rounds of 64 slots (nearly always one)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        if (U[g] != 0u && slot[g] - s0 < nslots) { su[slot[g] - s0] = U[g]; sm[slot[g] - s0] = lane | (uint32_t)g << 6; }
      wave_lds_sync();
      const bool busy = lane < nslots && s0 + lane < tot;
      if (busy) {
        uint32_t Un = su[lane], Fn = 0u;
        const uint32_t mm = sm[lane], src = mm & 63u, w = w4 + (mm >> 6);
        const uint2 sq = seq(src);
        uint32_t xv[2][4];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          xv[b][0] = w * kNoiseBlocksPerWord + j + (uint32_t)b;
          xv[b][1] = sq.x; xv[b][2] = sq.y; xv[b][3] = a.tag;
        }
        philox_blocks<2>(xv, ks);
        noise_planes4(t >> (28u - 4u * j), xv[0][0], xv[0][1], xv[0][2], xv[0][3], Un, Fn);
        noise_planes4(t >> (24u - 4u * j), xv[1][0], xv[1][1], xv[1][2], xv[1][3], Un, Fn);
        su[lane] = Un; sm[lane] = Fn;
      }
      wave_lds_sync();
#pragma unroll
      for (int g = 0; g < 4; ++g)   // owners (U still holds the value they sent)
        if (U[g] != 0u && slot[g] - s0 < nslots) { U[g] = su[slot[g] - s0]; F[g] |= sm[slot[g] - s0]; }
      wave_lds_sync();
    }
  }
}

// Split form: the two blocks (8 planes) of a pair go to two slot lanes, which compute
// one block each at the same time; a slot compares its planes for every bit (U = ~0)
// and returns (below, equal) masks, which the owner applies in plane order.  A round
// takes one block's time for up to 32 pairs instead of two blocks' for 64 (the ~28
// pairs left after planes 1-8 of four words nearly always fit one round).  Measured:
// the generator alone 1% faster, the fused kernel (4 more VGPRs) slower
// (profiles/r04n); so the generator uses it and the fused kernel does not.
template <typename Seq, class KS>
__device__ __forceinline__ void noise_exchange_split(const GenArgs& a, uint32_t* su, uint32_t* sm, Seq seq,
                                                     uint32_t w4, uint32_t (&U)[4], uint32_t (&F)[4], const KS& ks) {
  const uint32_t t = a.thr_lo, lane = lane_id();
  const uint32_t nslots = a.slots - 1u < 64u ? a.slots : 64u;
  const uint32_t npr = nslots > 1u ? nslots >> 1 : 1u;   // pairs per round
#pragma nounroll
  for (uint32_t j = 2; j < (uint32_t)kNoiseBlocksPerWord; j += 2) {
    uint32_t slot[4], tot = 0u;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint64_t b = __ballot(U[g] != 0u);
      slot[g] = tot + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
      tot += (uint32_t)__builtin_popcountll(b);
    }
    if (tot == 0u) break;   // every bit of every pair decided
#pragma nounroll
    for (uint32_t s0 = 0; s0 < tot; s0 += npr) {   // rounds of 32 pairs (nearly always one)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        if (U[g] != 0u && slot[g] - s0 < npr) sm[slot[g] - s0] = lane | (uint32_t)g << 6;
      wave_lds_sync();
      const uint32_t pi = lane >> 1;
      if (pi < npr && s0 + pi < tot) {
        // (the read of sm[pi] returns before this lane's writes below: they depend on it)
        const uint32_t mm = sm[pi], src = mm & 63u, w = w4 + (mm >> 6), blk = j + (lane & 1u);
        const uint2 sq = seq(src);
        uint32_t xv[1][4] = {{w * kNoiseBlocksPerWord + blk, sq.x, sq.y, a.tag}};
        philox_blocks<1>(xv, ks);
        uint32_t eq = ~0u, lt = 0u;
        noise_planes4<true>(t >> (28u - 4u * blk), xv[0][0], xv[0][1], xv[0][2], xv[0][3], eq, lt);
        su[lane] = lt; sm[lane] = eq;
      }
      wave_lds_sync();
#pragma unroll
      for (int g = 0; g < 4; ++g)   // owners: planes 4j+1.. then 4j+5.., most significant first
        if (U[g] != 0u && slot[g] - s0 < npr) {
          const uint32_t s = 2u * (slot[g] - s0);
          F[g] |= U[g] & su[s];
          U[g] &= sm[s];
          F[g] |= U[g] & su[s + 1];
          U[g] &= sm[s + 1];
        }
      wave_lds_sync();
    }
  }
}

template <bool kSplit, typename Seq, class KS>
__device__ __forceinline__ void noise_exchange(const GenArgs& a, uint32_t* su, uint32_t* sm, Seq seq, uint32_t w4,
                                               uint32_t (&U)[4], uint32_t (&F)[4], const KS& ks) {
  if constexpr (kSplit) noise_exchange_split(a, su, sm, seq, w4, U, F, ks);
  else noise_exchange_pair(a, su, sm, seq, w4, U, F, ks);
}

// Flip masks F[g] of the words w4 + g (g < 4) of every lane's sequence, noise_word's
// spec (cvd_common.h) for the wave; live[g] = word exists for this lane.
//  * Planes 1-8 (Philox blocks 0 and 1) of all four words run unconditionally.  A code
//    bit is then still undecided with probability 2^-8, so ~12% of the wave's 256
//    (lane, word) pairs hold one (~30).
//  * Those pairs are compacted into consecutive lanes (noise_exchange); after 16 planes
//    ~0.1 undecided bits are left per wave and chunk; a further pass runs only while the
//    ballot finds one.
// One word at a time (3 blocks for every lane, then single blocks while any lane is
// undecided) costs ~3.4 blocks per word; this ~2.5.
template <typename Seq, class KS>
__device__ __forceinline__ void noise_chunk_wave(const GenArgs& a, uint32_t* su, uint32_t* sm, Seq seq, uint32_t w4,
                                                 const bool (&live)[4], uint32_t valid, uint32_t (&F)[4], const KS& ks) {
  uint32_t U[4];
  const uint2 own = seq(lane_id());
#pragma unroll
  for (int g = 0; g < 4; ++g) noise_head(a, own, w4 + g, live[g], valid, U[g], F[g], ks);
  noise_exchange<CVD_GEN_XCHG_SPLIT>(a, su, sm, seq, w4, U, F, ks);
}

// Encoder of one sequence, one received word at a time (bit-parallel, see above):
// the input stream's Philox block cache and the window history carried from word
// to word.  encode(w, nm) returns word w with the flip mask nm applied.
// kVK: the noise keys' ten round keys in VGPRs (PhiloxKeysV; gen_fast_kernel, CVD_GEN_VKEYS)
template <int k, int n, int kT = 0, bool kVK = false>
struct ChunkEncoder {
  static constexpr int SPW = 32 / n, NBITS = SPW * n;
  static constexpr uint32_t kValid = NBITS == 32 ? ~0u : (1u << (NBITS % 32)) - 1u;
  // k = 1 (spread-first): the input bits are Morton-spread once per word (bit i ->
  // bit n*i), and the window W = U << hs | (history) is kept in that spread form as
  // 64 bits (lo, hi): every tap W >> sh is then one v_alignbit by n*sh of (hi, lo),
  // already at the output's bit positions, so the n outputs need no spread of their
  // own (m2 generator 12.1 -> 11.6 ms, m = 6 8.6 -> 8.3 ms alone).  sprev: the
  // previous word's spread inputs (the history is its top hs steps).
  // k = 2 keeps plain windows and one spread per output: spread-first made the
  // rate-2/3 generator faster alone (16.1 -> 15.8 ms) but the overlapped C3 step
  // 1.7% slower (profiles/r02z_gen/ab_enc_*.json).
  static constexpr bool kSpreadFirst = k == 1;
  // k = 2, n = 3 (C3): the flat input bits go to the word's stride in one spread
  // (spread23: bit 2t + r -> 3t + r) and the window X = (this word << 30 | the previous
  // word) is 60 bits, so every tap u_r(t - d) of output j is one v_alignbit by
  // 30 - 3 d + r - j of X, landing on lane j of the word; the other phase's bits land on
  // lanes j +- 1 and lane 2 of X is empty, so one AND per output keeps lane j.  No
  // even/odd split of the inputs and no spread per output: 173 -> ~130 VALU per stream
  // word (profiles/pmc_markov_r23_m4.json).  CVD_GEN_K2_STRIDE3=0 restores the per-phase
  // windows (same streams).
  static constexpr bool kStride3 = CVD_GEN_K2_STRIDE3 && k == 2 && n == 3;
  // kT > 0 (spread-first and stride-3 forms): the taps of output j as a fixed list of kT
  // window shifts (GenArgs::tsh, SGPRs), fully unrolled -- one v_alignbit per slot, the
  // XORs as v_xor3, and no scalar loop (the loop over the set bits of the tap mask issues
  // 7 SALU per tap: s_ff1, the mask update, the shift arithmetic, compare and branch).
  // Padding slots move only empty lanes of the window onto lane j and the lane mask
  // after the XOR removes what they move elsewhere.
  static_assert(kT == 0 || kSpreadFirst || kStride3, "ChunkEncoder: tap lists need the spread window");
  static_assert(kT <= kTapSlots, "ChunkEncoder: tap list");
  const GenArgs* a;
  uint32_t slo, ihi;
  int64_t iblk;
  U4 iv;
  uint32_t sprev[k], hist[k];
  struct NoKeys {};
  typename std::conditional<kVK, typename std::conditional<CVD_GEN_VTHR != 0, NoiseKeysV, PhiloxKeysV>::type,
                            NoKeys>::type kv;
  // the noise blocks' key: the launch's pair (SGPRs), or the VGPR round keys
  __device__ __forceinline__ auto keys() const {
    if constexpr (kVK) return kv;
    else return PhiloxKeysS{a->k0, a->k1};
  }
  __device__ void init(const GenArgs* a_, uint64_t sid) {
    a = a_;
    if constexpr (kVK) {
      kv.init(a->k0, a->k1);
      if constexpr (CVD_GEN_VTHR != 0) kv.init_thr(a->thr_lo);
    }
    slo = (uint32_t)sid; ihi = ctr_hi(sid, kKindInput);
    iblk = -1; iv = U4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < k; ++r) sprev[r] = hist[r] = 0u;   // encoder starts in state 0
  }
  __device__ uint32_t input_word(int64_t W) {   // 32-bit word W of the input stream
    if ((W >> 2) != iblk) {
      iblk = W >> 2;
      if constexpr (kVK) {
        uint32_t c[1][4] = {{(uint32_t)iblk, slo, ihi, a->tag}};
        philox_blocks<1>(c, kv);
        iv = U4{c[0][0], c[0][1], c[0][2], c[0][3]};
      } else {
        uint32_t k0 = a->k0, k1 = a->k1;
        asm volatile("" : "+s"(k0), "+s"(k1));
        iv = philox((uint32_t)iblk, slo, ihi, a->tag, k0, k1);
      }
    }
    return u4_get(iv, (uint32_t)(W & 3));
  }
  // input bits [w*SPW*k, (w+1)*SPW*k) of the flat input stream (bit SPW*k.. unmasked)
  __device__ uint32_t flat_inputs(int64_t w) {
    uint32_t Fw = 0u;
    if (a->random_input) {
      const int64_t b0 = w * SPW * k;
      const uint32_t off = (uint32_t)(b0 & 31);
      const uint32_t lo = input_word(b0 >> 5);
      const uint32_t hi = (off + SPW * k > 32u) ? input_word((b0 >> 5) + 1) : 0u;
      Fw = off ? __builtin_amdgcn_alignbit(hi, lo, off) : lo;
    }
    return Fw;
  }
  // the same split by phase
  __device__ void word_inputs(int64_t w, uint32_t (&U)[k]) {
    const uint32_t Fw = flat_inputs(w);
    if constexpr (k == 1) U[0] = Fw;
    else { U[0] = even_bits(Fw); U[1] = even_bits(Fw >> 1); }
#pragma unroll
    for (int r = 0; r < k; ++r)
      if constexpr (SPW < 32) U[r] &= (1u << SPW) - 1u;
  }
  // history of a segment starting at word w0 > 0: the hs input steps before it
  __device__ void seek(int64_t w0) {
    if constexpr (kStride3) {
      sprev[0] = spread23(flat_inputs(w0 - 1));
      return;
    }
    uint32_t Up[k];
    word_inputs(w0 - 1, Up);
#pragma unroll
    for (int r = 0; r < k; ++r) {
      if constexpr (kSpreadFirst) sprev[r] = spread_n<n>(Up[r]);
      else hist[r] = (Up[r] >> (SPW - a->hs)) & ((1u << a->hs) - 1u);
    }
  }
  // output j's packed tap list (kT > 0), re-read per word: the asm keeps the compiler from
  // hoisting the n kT extracted shifts out of the chunk loop into SGPRs (18 for rate 2/3:
  // SGPR spills to VGPR lanes); per word the words and one s_lshr per slot
  __device__ __forceinline__ void tap_words(int j, uint32_t& p0, uint32_t& p1) const {
    p0 = __builtin_amdgcn_readfirstlane(a->tpk[j][0]);
    asm volatile("" : "+s"(p0));
    p1 = 0u;
    if constexpr (kT > 6) {
      p1 = __builtin_amdgcn_readfirstlane(a->tpk[j][1]);
      asm volatile("" : "+s"(p1));
    }
  }
  static __device__ __forceinline__ uint32_t tap_slot(int i, uint32_t p0, uint32_t p1) {
    const uint32_t p = i < 6 ? p0 : p1;
    return (i % 6) ? p >> (5 * (i % 6)) : p;   // v_alignbit uses the low 5 bits
  }
  __device__ uint32_t encode(int64_t w, uint32_t nm) {
    const int hs = a->hs;
    if constexpr (kStride3) {
      const uint32_t sc = spread23(flat_inputs(w));
      const uint32_t xlo = (sc << 30) | sprev[0], xhi = sc >> 2;   // X = sc * 2^30 + previous word
      sprev[0] = sc;
      uint32_t word = 0u;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        uint32_t o = 0u;
        if constexpr (kT > 0) {
          uint32_t p0, p1;
          tap_words(j, p0, p1);
#pragma unroll
          for (int i = 0; i < kT; ++i) o ^= __builtin_amdgcn_alignbit(xhi, xlo, tap_slot(i, p0, p1));
          word |= o & (0x09249249u << j);
          continue;
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          // window tap sh of phase r is u_r(t - (hs - sh)): X bit 30 + 3 (t - hs + sh) + r,
          // moved to bit 3t + j (the scalar loop over the set taps, as below)
          uint32_t tm = __builtin_amdgcn_readfirstlane(a->taps[j][r]);
          asm volatile("" : "+s"(tm));
#pragma nounroll
          while (tm) {
            const uint32_t sh = (uint32_t)__builtin_ctz(tm);
            tm &= tm - 1u;
            o ^= __builtin_amdgcn_alignbit(xhi, xlo, 30u - 3u * (uint32_t)hs + 3u * sh + (uint32_t)r - (uint32_t)j);
          }
        }
        word |= o & (0x09249249u << j);   // lane j of the 10 steps
      }
      word ^= nm;
      const int64_t ns = a->N - w * SPW;         // steps in this word (last word: < SPW)
      if (ns < SPW) word &= (1u << (n * ns)) - 1u;
      return word;
    }
    const uint32_t nhs = (uint32_t)(n * hs), nrest = (uint32_t)(n * (SPW - hs));   // 0 < nhs < 32, nrest < 32
    uint32_t U[k];
    word_inputs(w, U);
    uint32_t lo[k], hi[k];   // spread-first windows, or the plain windows in lo
#pragma unroll
    for (int r = 0; r < k; ++r) {
      if constexpr (kSpreadFirst) {
        const uint32_t su = spread_n<n>(U[r]);
        lo[r] = (su << nhs) | (sprev[r] >> nrest);
        hi[r] = su >> (32u - nhs);
        sprev[r] = su;
      } else {
        lo[r] = (U[r] << hs) | hist[r];
        hi[r] = 0u;
        hist[r] = (lo[r] >> SPW) & ((1u << hs) - 1u);
      }
    }
    uint32_t word = 0u;
#pragma unroll
    for (int j = 0; j < n; ++j) {
      uint32_t o = 0u;
      if constexpr (kT > 0) {   // spread-first (k = 1): lane 0 of the window, stride n
        static_assert(n == 2 || n == 3, "ChunkEncoder: spread-first tap lists for n = 2, 3");
        constexpr uint32_t kLane0 = n == 2 ? 0x55555555u : 0x09249249u;   // bits n i, i < SPW
        uint32_t p0, p1;
        tap_words(j, p0, p1);
#pragma unroll
        for (int i = 0; i < kT; ++i) o ^= __builtin_amdgcn_alignbit(hi[0], lo[0], tap_slot(i, p0, p1));
        word |= (o & kLane0) << j;
        continue;
      }
#pragma unroll
      for (int r = 0; r < k; ++r) {
        // the set taps only, as a scalar loop over the uniform mask (s_ff1):
        // two VALU per tap.  The mask is re-read per word -- hoisted out of
        // the chunk loop, per-shift conditions filled the SGPRs (spills) and
        // unrolled they became selects for every possible shift
        uint32_t tm = __builtin_amdgcn_readfirstlane(a->taps[j][r]);
        asm volatile("" : "+s"(tm));
#pragma nounroll
        while (tm) {
          const uint32_t sh = (uint32_t)__builtin_ctz(tm);
          tm &= tm - 1u;
          if constexpr (kSpreadFirst) o ^= __builtin_amdgcn_alignbit(hi[r], lo[r], (uint32_t)n * sh);
          else o ^= lo[r] >> sh;
        }
      }
      if constexpr (kSpreadFirst) {
        word |= o << j;
      } else {
        if constexpr (SPW < 32) o &= (1u << SPW) - 1u;
        word |= spread_n<n>(o) << j;
      }
    }
    if constexpr (kSpreadFirst && NBITS < 32) word &= kValid;   // n = 3: step SPW's bits at 30, 31
    word ^= nm;
    const int64_t ns = a->N - w * SPW;           // steps in this word (last word: < SPW)
    if (ns < SPW) word &= (1u << (n * ns)) - 1u;
    return word;
  }
  // flip masks and words w4 .. w4 + 3 (wave-collective: every lane of the wave calls
  // it for the same w4; live[g] = word w4 + g exists for this lane)
  template <typename Seq>
  __device__ void chunk(uint32_t* su, uint32_t* sm, Seq seq, int64_t w4, const bool (&live)[4], int64_t nwords,
                        uint32_t (&out4)[4]) {
    uint32_t nm4[4] = {0u, 0u, 0u, 0u};
    if (a->thr_all) {
#pragma unroll
      for (int g = 0; g < 4; ++g) nm4[g] = kValid;
    } else if (a->thr_lo) {
      noise_chunk_wave(*a, su, sm, seq, (uint32_t)w4, live, kValid, nm4, keys());
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) out4[g] = w4 + g < nwords ? encode(w4 + g, nm4[g]) : 0u;
  }
  // the same in two parts, so that a caller can interleave the unconditional noise
  // blocks with other work: head(g) for g = 0..3, then finish (wave-collective)
  __device__ void head(uint2 own, int64_t w, bool live, uint32_t& U, uint32_t& F) const {
    noise_head(*a, own, (uint32_t)w, live, kValid, U, F, keys());
  }
  template <typename Seq>
  __device__ void finish(uint32_t* su, uint32_t* sm, Seq seq, int64_t w4, uint32_t (&U)[4], uint32_t (&F)[4],
                         int64_t nwords, uint32_t (&out4)[4]) {
    if (a->thr_all) {
#pragma unroll
      for (int g = 0; g < 4; ++g) F[g] = kValid;
    } else if (a->thr_lo) {
      noise_exchange<CVD_FUSED_XCHG_SPLIT>(*a, su, sm, seq, (uint32_t)w4, U, F, keys());
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) F[g] = 0u;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) out4[g] = w4 + g < nwords ? encode(w4 + g, F[g]) : 0u;
  }
};

template <int k, int n, int kT>
__global__ __launch_bounds__(kBlock) void gen_fast_kernel(GenArgs a) {
  constexpr int SPW = 32 / n;
  static_assert(k >= 1 && k <= 2 && SPW * k <= 32, "gen_fast_kernel: shape");
  const int64_t li = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  // lanes past the end stay in the wave (U = 0, no stores): the noise exchange
  // uses every lane of the wave as a slot
  const bool lane_ok = li < a.count;
  const int64_t q = a.q0 + li;
  const uint64_t sid = (uint64_t)(a.seq_base + li * a.seq_stride);
#if CVD_GEN_SEQ_LDS
  __shared__ NoiseLds noise_lds[kBlock / 64];
  NoiseLds& nl = noise_lds[threadIdx.x / 64];
  nl.slo[lane_id()] = (uint32_t)sid;
  nl.nhi[lane_id()] = ctr_hi(sid, kKindNoise);
  wave_lds_sync();
  auto seq = [&](uint32_t l) { return make_uint2(nl.slo[l], nl.nhi[l]); };
  uint32_t* const su = nl.u;
  uint32_t* const sm = nl.m;
#else
  // the slot lanes' sequence ids from the lane index (one 64-bit multiply-add), so
  // that a block holds 2 KB of LDS: five generator blocks fit beside a rate-2/3
  // detector block (141 KB of a CU's 160 KB) instead of four
  __shared__ uint32_t xchg[kBlock / 64][128];
  uint32_t* const su = xchg[threadIdx.x / 64];
  uint32_t* const sm = su + 64;
  // (wave-uniform: the wave's first lane's sequence id s0 and the stride in SGPRs)
  const int64_t li0 = (int64_t)blockIdx.x * kBlock + (int64_t)__builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
  const uint64_t s0 = (uint64_t)(a.seq_base + li0 * a.seq_stride), sstr = (uint64_t)a.seq_stride;
  auto seq = [&](uint32_t l) {
    const uint64_t s = s0 + (uint64_t)l * sstr;
    return make_uint2((uint32_t)s, ctr_hi(s, kKindNoise));
  };
#endif
  const int64_t nwords = (a.N + SPW - 1) / SPW;
  const int64_t nw4 = (nwords + 3) & ~(int64_t)3;
  ChunkEncoder<k, n, kT, CVD_GEN_VKEYS != 0> enc;
  enc.init(&a, sid);
  // segment blockIdx.y of the sequence's 16-byte chunks: every word depends only
  // on its own inputs and the hs input steps before it, so segments are
  // independent (more waves in flight than one lane per sequence gives)
  const int64_t nchunks = nw4 >> 2, seg = gridDim.y;
  const int64_t c0 = nchunks * blockIdx.y / seg, c1 = nchunks * (blockIdx.y + 1) / seg;
  if (c0 > 0 && 4 * c0 <= nwords) enc.seek(4 * c0);
  for (int64_t w4 = 4 * c0; w4 < 4 * c1; w4 += 4) {
    bool live[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) live[g] = lane_ok && w4 + g < nwords;
    uint32_t out4[4];
    enc.chunk(su, sm, seq, w4, live, nwords, out4);
    if (lane_ok)
      *reinterpret_cast<uint4*>(a.r + chunk_index(w4 >> 2, a.pitch, q)) = make_uint4(out4[0], out4[1], out4[2], out4[3]);
  }
}

// ─────────────────────────── table automaton ────────────────────────────────

struct TabArgs {
  const uint32_t* rec;    // [S][R]: next << 4 | c
  const double* logp1;    // [S][R]
  const double* ltref;    // [R + 1]
  int32_t n;
  int64_t S, N, nseq, n_h1;
  const uint32_t* r;
  double* sums;
  int64_t* counts;
  int32_t early;            // early decision (counts only; sums == nullptr), see early_decide
  double lt_min, lp_min;
};

template <bool kLds>
__global__ __launch_bounds__(kBlock) void detect_table_kernel(TabArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int R = 1 << a.n;
  const int64_t SR = a.S * R;
  const uint32_t* rec = a.rec;
  const double* lp1 = a.logp1;
  const double* ltr = a.ltref;
  if (kLds) {
    double* s_lp = reinterpret_cast<double*>(smem);
    double* s_lt = s_lp + SR;
    uint32_t* s_rec = reinterpret_cast<uint32_t*>(s_lt + R + 1);
    for (int64_t i = threadIdx.x; i < SR; i += kBlock) { s_lp[i] = a.logp1[i]; s_rec[i] = a.rec[i]; }
    for (int i = threadIdx.x; i <= R; i += kBlock) s_lt[i] = a.ltref[i];
    __syncthreads();
    rec = s_rec; lp1 = s_lp; ltr = s_lt;
  }
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = q < a.nseq;
  double lp = 0.0, lr = 0.0;
  if (valid) {
    const int spw = 32 / a.n;
    const uint32_t rmask = (uint32_t)R - 1u;
    const int64_t nwords = (a.N + spw - 1) / spw;
    uint32_t st = 0;                     // index of D_0 = 0 (first BFS state)
    uint4 cache;
    int dec = 0;                         // early decision (0 = open)
    for (int64_t w = 0; w < nwords; ++w) {
      if (a.early && w > 0 && (w & 7) == 0) {   // every 8 words
        if (!dec) dec = early_decide(lp, lr, a.N - w * spw, a.lt_min, a.lp_min);
        if (__ballot(dec == 0) == 0) break;
      }
      uint32_t word = next_word(a.r, a.nseq, q, w, cache);
      const int ns = (int)min((int64_t)spw, a.N - w * spw);
      for (int i = 0; i < ns; ++i) {
        const uint32_t idx = st * (uint32_t)R + (word & rmask);
        word >>= a.n;
        const uint32_t e = rec[idx];
        lp += lp1[idx];                  // log P̂1[i, j]   (Pd_plotter.py:213)
        lr += ltr[e & 15u];              // log T_ref[i, j] = log(c / 2^n) (Pd_plotter.py:214)
        st = e >> 4;
      }
    }
    if (a.sums) { a.sums[2 * q] = lp; a.sums[2 * q + 1] = lr; }
    early_final(dec, lp, lr);
  }
  count_decisions(valid, q < a.n_h1, lp, lr, a.counts);
}

// Enumerated automaton with the whole model LDS-resident (S < 4096 and its image
// within the 160 KiB of a CU).  Two images (LdsModel):
//  * kLr = false (any table that fits): log P̂1 as f64 [S 2^n], log T_ref(c) f64
//    [2^n + 1], records 16-bit next << 4 | c [S 2^n] -- 10 B per entry.  Per step one
//    u16 and two f64 gathers, and the index math of next * 2^n + r, c * 8 and the
//    shifts (~40 issue cycles of VALU per step, measured by the ISA: the walk is
//    VALU-bound, not LDS-bound).
//  * kLr = true (small tables, S 2^n 18 B <= 32 KiB: m2, m3): log P̂1 and log T_ref(i,
//    r) = ltref[c] as two f64 arrays [S 2^n] and 16-bit next * 2^n, the next state's
//    entry base -- 18 B per entry, built from the same device arrays at kernel start.
//    Per step one bit-field extract, one add, two address shift-adds, one add and the
//    two f64 adds (~27 issue cycles), the same three gathers.
// The only dependent chain is the u16 record (next state).  The received words are
// read in 16-byte chunks one chunk ahead (64 or 40 steps of lead), and full chunks run
// fully unrolled.
//  * kCp > 1 (kLr only; timing studies, CVD_C1_COPIES): kCp interleaved copies of the
//    kLr image, entry i of copy c at element i kCp + c, lane l reading copy l mod kCp, so
//    lanes of one LDS lane group that gather different entries fall on different banks
//    more often; records hold next * 2^n * kCp.
//  * kLpG (kLr = false only; timing studies, CVD_T16_LPG=1): the 16-bit records and log
//    T_ref(c) in LDS, log P̂1 gathered from global memory (L1/L2) -- 2 B per entry of LDS
//    instead of 10.
typedef const __attribute__((address_space(1))) double gdouble;
template <int n, bool kLr, int kCp = 1, bool kLpG = false>
struct LdsModel {
  static_assert(kCp == 1 || kLr, "copies of the kLr image only");
  static_assert(!(kLpG && kLr), "log P̂1 from global memory with the 10-B image only");
  static constexpr uint32_t R = 1u << n;
  const double* lp;      // [SR] log P̂1
  gdouble* lpg;          // kLpG: [SR] log P̂1 in global memory
  const double* lt;      // kLr: [SR] log T_ref(i, r); else [R + 1] log(c / 2^n)
  const uint16_t* rec;   // kLr: [SR] next * 2^n; else [SR] next << 4 | c
  __host__ __device__ static size_t bytes(int64_t SR) {
    return kLr ? (size_t)SR * 18 * kCp : (size_t)SR * (kLpG ? 2 : 10) + (R + 1) * sizeof(double);
  }
  __device__ void fill(const TabArgs& a, char* smem, int BS) {
    const int SR = (int)a.S * (int)R;
    double* s_lp = reinterpret_cast<double*>(smem);
    double* s_lt = s_lp + (kLpG ? 0 : SR * kCp);
    uint16_t* s_rec = reinterpret_cast<uint16_t*>(s_lt + (kLr ? SR * kCp : (int)R + 1));
    lpg = (gdouble*)a.logp1;
    for (int j = threadIdx.x; j < SR * kCp; j += BS) {
      const int i = j / kCp;
      const uint32_t e = a.rec[i];
      if constexpr (!kLpG) s_lp[j] = a.logp1[i];
      if constexpr (kLr) {
        s_lt[j] = a.ltref[e & 15u];
        s_rec[j] = (uint16_t)((e >> 4) * R * kCp);   // S * 2^n * kCp < 65536 (host-checked)
      } else {
        s_rec[j] = (uint16_t)e;                // next < 4096: next << 4 | c fits 16 bits (host-checked)
      }
    }
    if constexpr (!kLr)
      for (int i = threadIdx.x; i <= (int)R; i += BS) s_lt[i] = a.ltref[i];
    const uint32_t c = kCp > 1 ? (threadIdx.x & (uint32_t)(kCp - 1)) : 0u;
    lp = s_lp + c; lt = s_lt + c; rec = s_rec + c;
  }
  // st: the state's entry base (kLr) or index; state 0 is 0 either way
  __device__ __forceinline__ void step(uint32_t& st, uint32_t r, double& lps, double& lrs) const {
    if constexpr (kLr) {
      const uint32_t idx = st + r * (uint32_t)kCp;
      const uint32_t nx = rec[idx];
      lps += lp[idx];                 // log P̂1[i, j]   (Pd_plotter.py:213)
      lrs += lt[idx];                 // log T_ref[i, j] (Pd_plotter.py:214)
      st = nx;
    } else {
      const uint32_t idx = st * R + r;
      const uint32_t e = rec[idx];
      lps += kLpG ? lpg[idx] : lp[idx];   // log P̂1[i, j]   (Pd_plotter.py:213)
      lrs += lt[e & 15u];             // log T_ref[i, j] = log(c / 2^n) (Pd_plotter.py:214)
      st = e >> 4;
    }
  }
  // the first ns steps of a word (step i in bits n*i .. n*i + n - 1)
  __device__ __forceinline__ void word(uint32_t w, int ns, uint32_t& st, double& lps, double& lrs) const {
    for (int i = 0; i < ns; ++i) step(st, __builtin_amdgcn_ubfe(w, (uint32_t)(n * i), (uint32_t)n), lps, lrs);
  }
};

template <int n, int BS, bool kLr, bool kLpG = false>
__global__ __launch_bounds__(BS) void detect_table16_kernel(TabArgs a) {
  constexpr int SPW = 32 / n;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  LdsModel<n, kLr, 1, kLpG> md;
  md.fill(a, smem, BS);
  __syncthreads();
  const int64_t q = (int64_t)blockIdx.x * BS + threadIdx.x;
  const bool valid = q < a.nseq;
  double lp = 0.0, lr = 0.0;
  if (valid) {
    const int64_t N = a.N, nwords = (N + SPW - 1) / SPW, nchunks = (nwords + 3) / 4;
    const int64_t full = N / (4 * SPW);           // chunks whose 4 words are all full
    const uint4* rc = reinterpret_cast<const uint4*>(a.r) + q;
    const int64_t cs = a.nseq;                    // uint4 stride between chunks of one sequence
    uint4 cur = make_uint4(0u, 0u, 0u, 0u), nxt = cur;
    if (nchunks > 0) cur = rc[0];
    if (nchunks > 1) nxt = rc[cs];
    uint32_t st = 0;                              // D_0 = 0 (first BFS state)
    int dec = 0;                                  // early decision (0 = open)
    for (int64_t c = 0; c < nchunks; ++c) {
      if (a.early && c > 0 && (c & 1) == 0 && c <= full) {   // every 2 chunks (8 words)
        if (!dec) dec = early_decide(lp, lr, N - c * 4 * SPW, a.lt_min, a.lp_min);
        if (__ballot(dec == 0) == 0) break;
      }
      const uint4 ch = cur;
      cur = nxt;
      if (c + 2 < nchunks) nxt = rc[(c + 2) * cs];
      const uint32_t wv[4] = {ch.x, ch.y, ch.z, ch.w};
      if (c < full) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int i = 0; i < SPW; ++i)
            md.step(st, __builtin_amdgcn_ubfe(wv[e], (uint32_t)(n * i), (uint32_t)n), lp, lr);
        }
      } else {
        for (int e = 0; e < 4; ++e) {
          const int64_t t0 = (4 * c + e) * SPW;
          if (t0 >= N) break;
          md.word(wv[e], (int)min((int64_t)SPW, N - t0), st, lp, lr);
        }
      }
    }
    if (a.sums) { a.sums[2 * q] = lp; a.sums[2 * q + 1] = lr; }
    early_final(dec, lp, lr);
  }
  count_decisions(valid, q < a.n_h1, lp, lr, a.counts);
}

// ─────────────── fused trial loop: generator + table automaton ───────────────
//
// The whole trial (Pd_plotter.py:210-223) in one kernel for the LDS-resident table
// path: every lane generates its own sequence's received words four at a time
// (ChunkEncoder: the same encoder and bit-sliced noise as gen_fast_kernel, so the
// same streams bit for bit) and feeds them straight into the table steps of
// detect_table16_kernel, with no stream in HBM.  The table path is LDS-bound and
// the generator VALU-bound, so inside one wave's instruction stream the two
// overlap: the two-kernel pipeline measured 39.6 ms (generator) against 29.7 ms
// (detector) per overlapped m2 step, each ~24 ms alone.  Lanes [0, Tp) are H1
// (encoder G1, sequence 2 (trial_begin + t)), [Tp, 2 Tp) H2 (G2, 2 (...) + 1); Tp is
// the trial count rounded up to whole waves, so every wave is one hypothesis.
struct FusedArgs {
  TabArgs t;               // model tables, N, sums ([T][4]: lp1, lr1, lp2, lr2), counts, early
  GenArgs g[2];            // H1 and H2 encoders, noise threshold, stream key
  int64_t trial_begin, T, Tp;
};

template <int k, int n, int BS, bool kLr, int kT = 0, int kCp = 1>
__global__ __launch_bounds__(BS) void mc_table16_kernel(FusedArgs a) {
  constexpr int SPW = 32 / n;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const TabArgs& ta = a.t;
  LdsModel<n, kLr, kCp> md;
  md.fill(ta, smem, BS);
  // the noise exchange's slot records, 2 x 64 words per wave, after the model
  uint32_t* s_x = reinterpret_cast<uint32_t*>(smem + ((LdsModel<n, kLr, kCp>::bytes(ta.S * (1 << n)) + 15) & ~(size_t)15));
  __syncthreads();
  uint32_t* su = s_x + (threadIdx.x / 64) * 128;
  uint32_t* sm = su + 64;
  // wave-uniform hypothesis (SGPR): the wave's first lane index
  const int64_t wli = (int64_t)blockIdx.x * BS + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  const int h = wli >= a.Tp ? 1 : 0;
  const GenArgs& g = a.g[h];
  const int64_t t0 = wli - (h ? a.Tp : 0);        // trial offset of lane 0
  const uint32_t lane = lane_id();
  const int64_t t = t0 + lane;
  const bool valid = wli < 2 * a.Tp && t < a.T;
  const uint64_t sid0 = 2 * (uint64_t)(a.trial_begin + t0) + (uint64_t)h;
  auto seq = [&](uint32_t l) {
    const uint64_t sd = sid0 + 2 * (uint64_t)l;
    return make_uint2((uint32_t)sd, ctr_hi(sd, kKindNoise));
  };
  ChunkEncoder<k, n, kT, CVD_FUSED_VKEYS != 0> enc;
  enc.init(&g, sid0 + 2 * (uint64_t)lane);
  const uint2 own = seq(lane);
  const int64_t N = ta.N, nwords = (N + SPW - 1) / SPW, nchunks = (nwords + 3) / 4;
  const int64_t full = N / (4 * SPW);             // chunks whose 4 words are all full
  double lp = 0.0, lr = 0.0;
  uint32_t st = 0;                                // D_0 = 0 (first BFS state)
  int dec = 0;                                    // early decision (0 = open)
  // software pipeline: the words of chunk c + 1 are generated while chunk c is walked.
  // The unconditional noise blocks of each next word (straight-line VALU) sit in the
  // same basic block as the walk of a current word (a chain of dependent LDS gathers),
  // so the scheduler overlaps them; the straggler exchange and the encoder follow.
  uint32_t wv[4], U[4], F[4];
  if (nchunks > 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) enc.head(own, e, valid && e < nwords, U[e], F[e]);
    enc.finish(su, sm, seq, 0, U, F, nwords, wv);
  }
  for (int64_t c = 0; c < nchunks; ++c) {
    if (ta.early && c > 0 && (c & 1) == 0 && c <= full) {   // every 2 chunks (8 words)
      if (!dec) dec = early_decide(lp, lr, N - c * 4 * SPW, ta.lt_min, ta.lp_min);
      if (__ballot(dec == 0) == 0) break;         // the whole wave: the exchange stays collective
    }
    const int64_t wn = 4 * (c + 1);               // first word of the next chunk
    const bool more = c + 1 < nchunks;            // wave-uniform
    if (c < full && more) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // walk word e of this chunk with one Philox round of the next chunk's word e
        // after each step (the two blocks of noise_head, by hand: the scheduler keeps
        // source order, and each step waits on its LDS gather)
        uint32_t xv[2][4];
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          xv[b][0] = (uint32_t)(wn + e) * kNoiseBlocksPerWord + (uint32_t)b;
          xv[b][1] = own.x; xv[b][2] = own.y; xv[b][3] = g.tag;
        }
        uint32_t k0 = g.k0, k1 = g.k1;
        uint32_t word = wv[e];
        auto round = [&](int r) {
          if constexpr (CVD_FUSED_VKEYS != 0) {
            philox_round<2>(xv, enc.kv, r);
          } else {
            philox_round<2>(xv, k0, k1);
            k0 += kPhiloxW0;
            k1 += kPhiloxW1;
          }
        };
#pragma unroll
        for (int i = 0; i < SPW; ++i) {
          md.step(st, __builtin_amdgcn_ubfe(word, (uint32_t)(n * i), (uint32_t)n), lp, lr);
          if (i < 10) round(i);
        }
#pragma unroll
        for (int r = SPW; r < 10; ++r) round(r);
        noise_head_planes(g, xv, valid && wn + e < nwords, ChunkEncoder<k, n, kT>::kValid, U[e], F[e]);
      }
    } else {
      for (int e = 0; e < 4; ++e) {
        const int64_t s0 = (4 * c + e) * SPW;
        if (s0 >= N) break;
        md.word(wv[e], (int)min((int64_t)SPW, N - s0), st, lp, lr);
      }
      if (more) {
#pragma unroll
        for (int e = 0; e < 4; ++e) enc.head(own, wn + e, valid && wn + e < nwords, U[e], F[e]);
      }
    }
    if (more) enc.finish(su, sm, seq, wn, U, F, nwords, wv);
  }
  if (valid && ta.sums) { ta.sums[4 * t + 2 * h] = lp; ta.sums[4 * t + 2 * h + 1] = lr; }
  early_final(dec, lp, lr);
  count_decisions(valid, h == 0, lp, lr, ta.counts);
}

// pk16 minimum over L registers as a log-depth tree (independent ops issue back to back)
template <int L>
__device__ __forceinline__ us2 tree_min(const uint32_t (&A)[L]) {
  us2 t[L];
#pragma unroll
  for (int i = 0; i < L; ++i) t[i] = as_us2(A[i]);
#pragma unroll
  for (int w = L / 2; w >= 1; w /= 2)
#pragma unroll
    for (int i = 0; i < w; ++i) t[i] = __builtin_elementwise_min(t[i], t[i + w]);
  return t[0];
}

template <int m, int k, int n>
struct Shape {
  static constexpr int M = 1 << m, K = 1 << k, R = 1 << n, QP = R / 2;
  static constexpr int NG = M / 4;                // groups of 4 states (one 16-bit half)
  static constexpr int NW = M >= 8 ? M / 8 : 1;   // nibble-packed words of a metric vector
  static constexpr int KW = (NW + 1) & ~1;        // record key words (doubles 8-B aligned)
  static constexpr int RW = (KW + 2 * R + 3) & ~3;
  static constexpr int SPW = 32 / n;
  static_assert(m >= 2 && k <= m && n >= 1, "explicit path shape");
};

// D_t of one sequence as 2^m bytes (canonical state order); kDev: Dw is in the
// device key layout (key_nibble), else canonical nibbles
template <int m, int k, int n, bool kDev>
__device__ __forceinline__ void write_trace(uint8_t* tr, int64_t t, int64_t nseq, int64_t q,
                                            const uint32_t (&Dw)[Shape<m, k, n>::NW]) {
  using S = Shape<m, k, n>;
  uint8_t* o = tr + ((size_t)t * nseq + q) * S::M;
#pragma unroll
  for (int s = 0; s < S::M; ++s)
    o[s] = (uint8_t)((Dw[s >> 3] >> (4 * (kDev ? key_nibble(S::M, s) : (s & 7)))) & 15u);
}

template <int NW, int M>
__device__ __forceinline__ void to_key_layout(const uint32_t (&Dw)[NW], uint32_t (&K)[NW]) {
#pragma unroll
  for (int w = 0; w < NW; ++w) K[w] = M >= 8 ? key_swap(Dw[w]) : Dw[w];
}

template <int m, int k, int n>
__global__ __launch_bounds__(kBlock) void detect_explicit_kernel(ExpArgs a) {
  using S = Shape<m, k, n>;
  __shared__ double s_lt[S::R + 1];
  if (threadIdx.x <= S::R) s_lt[threadIdx.x] = a.ltref[threadIdx.x];
  fill_filter_patterns();
  __syncthreads();
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = q < a.nseq;
  double lp = 0.0, lr = 0.0;
  if (valid) {
    uint32_t Dw[S::NW];
#pragma unroll
    for (int w = 0; w < S::NW; ++w) Dw[w] = 0u;
    uint32_t Kw[S::NW];   // Dw in the device key layout (hash keys)
    to_key_layout<S::NW, S::M>(Dw, Kw);
    if (a.trace) write_trace<m, k, n, false>(a.trace, 0, a.nseq, q, Dw);
    StreamReader<n> rd;
    rd.init(a.r, a.nseq, q, a.N);
    RowCursor<S::NW, S::R> cur;
    cur.start(a, rd.peek());
    int dec = 0;   // early decision (0 = open)
    for (int64_t t = 1; t <= a.N; ++t) {
      if (a.early && t > 1 && ((t - 1) & (kEarlyEvery - 1)) == 0) {
        if (!dec) dec = early_decide(lp, lr, a.N - (t - 1), a.lt_min, a.lp_min);
        if (__ballot(dec == 0) == 0) break;
      }
      {
        const uint32_t rr = rd.peek();
        const uint32_t rn = t < a.N ? rd.peek_next() : 0u;
        cur.mid(a, rr);
        // (2) Eq. 4 for every received word q', two per packed-16 instruction.
        uint32_t dup[S::M];
#pragma unroll
        for (int s = 0; s < S::M; ++s) dup[s] = ((Dw[s >> 3] >> (4 * (s & 7))) & 15u) * 0x10001u;
        uint32_t P[S::QP][S::NG];
        cu32* bmp = as_const(a.bmp);
#pragma unroll
        for (int qp = 0; qp < S::QP; ++qp) {
          uint32_t A[S::M];
#pragma unroll
          for (int ns_ = 0; ns_ < S::M; ++ns_) {
            us2 best;
#pragma unroll
            for (int b = 0; b < S::K; ++b) {
              const int pred = (ns_ >> k) | (b << (m - k));
              const us2 c = as_us2(dup[pred]) + as_us2(bmp[(qp * S::M + ns_) * S::K + b]);
              best = b == 0 ? c : __builtin_elementwise_min(best, c);
            }
            A[ns_] = as_u32(best);
          }
          const us2 mu = tree_min<S::M>(A);
#pragma unroll
          for (int g = 0; g < S::NG; ++g)
            P[qp][g] = A[4 * g] | (A[4 * g + 1] << 4) | (A[4 * g + 2] << 8) | (A[4 * g + 3] << 12);
          // Eq. 5: subtract the minimum from every nibble of both halves
          const uint32_t muN = ((uint32_t)mu.x * 0x1111u) | (((uint32_t)mu.y * 0x1111u) << 16);
#pragma unroll
          for (int g = 0; g < S::NG; ++g) P[qp][g] -= muN;
        }
        // (3) the observed successor D_t and c = #{q' : D_t(q') == D_t(r_t)}
        const uint32_t qsel = rr >> 1, hsh = (rr & 1u) * 16u;
        uint32_t obs[S::NG];
#pragma unroll
        for (int g = 0; g < S::NG; ++g) {
          uint32_t x = P[0][g];
#pragma unroll
          for (int qp = 1; qp < S::QP; ++qp) x = (qsel == (uint32_t)qp) ? P[qp][g] : x;
          obs[g] = (x >> hsh) & 0xFFFFu;
        }
        uint32_t c = 0;
#pragma unroll
        for (int qp = 0; qp < S::QP; ++qp) {
          uint32_t acc = 0;
#pragma unroll
          for (int g = 0; g < S::NG; ++g) acc |= P[qp][g] ^ (obs[g] * 0x10001u);
          c += ((acc & 0xFFFFu) == 0u) + ((acc >> 16) == 0u);
        }
        // (4) P̂1 row of D_{t-1}
        const double lpv = cur.resolve(a, Kw, rr);
        lp += lpv;            // Pd_plotter.py:115 with T = P̂1
        lr += s_lt[c];        // Pd_plotter.py:115 with T = T_ref(1/2) = c / 2^n
        // (5) D_t becomes the state
        if (S::NW == 1) {
          Dw[0] = S::NG == 1 ? obs[0] : (obs[0] | (obs[1] << 16));
        } else {
#pragma unroll
          for (int w = 0; w < S::NW; ++w) Dw[w] = obs[2 * w] | (obs[2 * w + 1] << 16);
        }
        to_key_layout<S::NW, S::M>(Dw, Kw);
        if (a.trace) write_trace<m, k, n, false>(a.trace, t, a.nseq, q, Dw);
        cur.prefetch(a, Kw, rn);
        rd.advance();
      }
    }
    if (a.sums) { a.sums[2 * q] = lp; a.sums[2 * q + 1] = lr; }
    early_final(dec, lp, lr);
  }
  count_decisions(valid, q < a.n_h1, lp, lr, a.counts);
}


// ─────────────── k = 1 orbit kernel (the m = 6 headline path) ──────────────
//
// For k = 1, flipping the input bit XORs the branch output with g0 (the tap-0
// column), so the Eq. 4 successor for r ^ g0 is the successor for r with the
// states 2j <-> 2j+1 exchanged (linearity of viterbi_markov.py:82-106).  Only
// the representatives r < r ^ g0 (2^n / 2 words) get an add-compare-select;
// their partners are a nibble swap.  Two representatives share one packed-16
// instruction (lo / hi halves).  This kernel is specialised to n = 2 (one
// representative pair; the (133,171) headline code and every rate-1/2 k=1 code
// with taps[0] != 0 on some output).
//
// Per lane (one sequence):
//   Dp[i]  = (D(2i), D(2i+1)) normalised 16-bit pair; op_sel broadcasts one
//            half into both halves of the packed adds for free
//   key[]  = the normalised D_{t-1}, nibble-packed (hash key of its P̂1 row)
// Per step, everything is produced per group of 4 states as soon as its two
// butterflies are done, so no full 2^m vector of raw ACS outputs stays live:
//   P_g  = raw ACS outputs (<= (ceil(m)+1)n <= 15) nibble-packed, both reps;
//          the minimum is subtracted once per packed word afterwards
//   Dn_i = next metric pairs of the observed representative (v_perm_b32)
#ifndef CVD_K1_WAVES
#define CVD_K1_WAVES 4
#endif
constexpr int kK1WavesPerSimd = CVD_K1_WAVES;   // occupancy target (VGPR budget 512 / waves)

template <int m, int n>
__global__ __launch_bounds__(kBlock, kK1WavesPerSimd) void detect_k1_kernel(ExpArgs a) {
  constexpr int M = 1 << m, H = M / 2, R = 1 << n, NG = M / 4, NP = M / 2;
  constexpr int NW = M >= 8 ? M / 8 : 1;
  constexpr int CH = (H >= 4) ? 4 : H;   // butterflies per branch-metric chunk (16 words)
  static_assert(m >= 2 && n == 2, "k1 orbit kernel shape");
  __shared__ double s_lt[R + 1];
  if (threadIdx.x <= R) s_lt[threadIdx.x] = a.ltref[threadIdx.x];
  fill_filter_patterns();
  __syncthreads();
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = q < a.nseq;
  double lp = 0.0, lr = 0.0;
  if (valid) {
    uint32_t Dp[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) Dp[i] = 0u;
    uint32_t key[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) key[w] = 0u;
    if (a.trace) write_trace<m, 1, n, true>(a.trace, 0, a.nseq, q, key);
    cu32* bmbase = as_const(a.bmp);
    StreamReader<n> rd;
    rd.init(a.r, a.nseq, q, a.N);
    RowCursor<NW, R> cur;
    cur.start(a, rd.peek());
    int dec = 0;   // early decision (0 = open)
    for (int64_t t = 1; t <= a.N; ++t) {
      if (a.early && t > 1 && ((t - 1) & (kEarlyEvery - 1)) == 0) {
        if (!dec) dec = early_decide(lp, lr, a.N - (t - 1), a.lt_min, a.lp_min);
        if (__ballot(dec == 0) == 0) break;
      }
      {
        const uint32_t rr = rd.peek();
        const uint32_t rn = t < a.N ? rd.peek_next() : 0u;
        const uint32_t rep = (a.repmap >> (4u * rr)) & 15u;   // 0 or 1: lo / hi half
        const uint32_t sw = (a.swmap >> rr) & 1u;
        const uint32_t hsh = rep * 16u;

        // (2) Eq. 4 for the two representatives, butterfly by butterfly.
        // Branch metrics: 4 packed words per butterfly, scalar loads from the
        // constant address space, one 16-word chunk ahead; each chunk pointer
        // is laundered through an asm that consumes the previous chunk's
        // outputs, so no pass can hoist the whole table into SGPRs.
        const uint32_t bb = rep * 2u;
        const uint32_t lo_sel = bb | ((bb + 1u) << 8), hi_sel = (bb + 4u) | ((bb + 5u) << 8);
        const uint32_t psel = sw ? (hi_sel | (lo_sel << 16)) : (lo_sel | (hi_sel << 16));
        constexpr int NCH = H / CH;
        uint32_t bmv[2][4 * CH];
        {
          cu32* p0 = bmbase;
          asm volatile("" : "+s"(p0) : "v"(Dp[0]));   // per step: not loop invariant
#pragma unroll
          for (int z = 0; z < 4 * CH; ++z) bmv[0][z] = p0[z];
        }
        uint32_t P[NG], Dn[NP];
        uint32_t zn = 0u;   // per-half "some raw nibble is 0" flags (bit 3 of each nibble)
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const int j0 = c * CH;
          if (c + 1 < NCH) {
            cu32* pn = bmbase + (c + 1) * CH * 4;
            if (c == 0) {
              asm volatile("" : "+s"(pn) : "v"(Dp[0]));
            } else {
              static_assert(CH == 4 || H < 4, "chunk barrier written for 4 butterflies");
              if constexpr (CH == 4) {
                // every value the previous chunk produced (packed words, next-step
                // pairs, running minima) is an operand: it must exist here, so no
                // raw ACS output outlives its chunk
                const int g0 = (j0 - CH) / 2;
                asm volatile("" : "+s"(pn), "+v"(P[g0]), "+v"(P[g0 + 1]), "+v"(Dn[2 * g0]),
                                  "+v"(Dn[2 * g0 + 1]), "+v"(Dn[2 * g0 + 2]), "+v"(Dn[2 * g0 + 3]),
                                  "+v"(zn));
              }
            }
#ifdef CVD_EXPERIMENT_CONST_BM
#pragma unroll
            for (int z = 0; z < 4 * CH; ++z) bmv[(c + 1) & 1][z] = 0x00010001u * ((z + c) % 3);
            (void)pn;
#else
#pragma unroll
            for (int z = 0; z < 4 * CH; ++z) bmv[(c + 1) & 1][z] = pn[z];
#endif
          }
          if (c == NCH / 2) cur.mid(a, rr);          // fingerprint matched: fetch key + row now
#pragma unroll
          for (int gg = 0; gg < CH / 2; ++gg) {       // group g = states 4g..4g+3 = butterflies 2g, 2g+1
            const int g = j0 / 2 + gg;
            uint32_t a4[4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int j = 2 * g + h, jj = j - j0;
              const uint32_t* b4 = &bmv[c & 1][4 * jj];
              const us2 pa = as_us2(Dp[j >> 1]), pb = as_us2(Dp[(j + H) >> 1]);
              const us2 da = (j & 1) ? __builtin_shufflevector(pa, pa, 1, 1) : __builtin_shufflevector(pa, pa, 0, 0);
              const us2 db = ((j + H) & 1) ? __builtin_shufflevector(pb, pb, 1, 1) : __builtin_shufflevector(pb, pb, 0, 0);
              const us2 e0 = __builtin_elementwise_min(da + as_us2(b4[0]), db + as_us2(b4[1]));
              const us2 e1 = __builtin_elementwise_min(da + as_us2(b4[2]), db + as_us2(b4[3]));
              a4[2 * h] = as_u32(e0);
              a4[2 * h + 1] = as_u32(e1);
            }
            P[g] = lshl4_or(lshl4_or(lshl4_or(a4[3], a4[2]), a4[1]), a4[0]);
            // zero-nibble test per 16-bit half (packed subtract: no borrow across halves)
            zn |= as_u32(as_us2(P[g]) - as_us2(0x11111111u)) & ~P[g];
            // next metric pairs (states 4g, 4g+1) and (4g+2, 4g+3) of the observed rep
            Dn[2 * g] = __builtin_amdgcn_perm(a4[1], a4[0], psel);
            Dn[2 * g + 1] = __builtin_amdgcn_perm(a4[3], a4[2], psel);
          }
        }
        // (3) Eq. 5: subtract the per-rep minimum (nibble-wise, no borrows since
        //     every nibble >= the minimum; pairs likewise).  For n = 2 the minimum
        //     is 0 or 1: D_{t-1} has a 0 state, and of its two branches (outputs o,
        //     o ^ g0, g0 != 0) one has metric <= 1.  So mu = [no nibble is 0].
        const uint32_t zm = zn & 0x88888888u;
        const uint32_t mu_lo = (zm & 0xFFFFu) == 0u, mu_hi = (zm >> 16) == 0u;
        const uint32_t muN = (mu_lo * 0x1111u) | (mu_hi * 0x11110000u);
        const uint32_t mo = rep ? mu_hi : mu_lo;
        const us2 mo2 = as_us2(mo * 0x10001u);
#pragma unroll
        for (int i2 = 0; i2 < NP; ++i2) Dp[i2] = as_u32(as_us2(Dn[i2]) - mo2);
        // (4) P̂1 row of D_{t-1}
        const double lpv = cur.resolve(a, key, rr);
        lp += lpv;            // Pd_plotter.py:115, T = P̂1
        // (5) per group: normalised P, its pair swap S (partners r ^ g0), the
        //     T_ref comparisons and the next key.  With obs = half `rep` of
        //     (sw ? S : P):  c = 1 + [P_rep symmetric] + [P.lo == P.hi] + [S.hi == P.lo]
        // (nibble pairs 2i, 2i+1 equal  <=>  (pv ^ pv >> 4) & 0x0F0F0F0F == 0, per half)
        uint32_t acc_sym = 0, acc_eq = 0, acc_x = 0, xs_prev = 0;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          const uint32_t pv = P[g] - muN;
          const uint32_t lsr = pv >> 4;
          uint32_t sv = ((pv << 4) & 0xF0F0F0F0u) | (lsr & 0x0F0F0F0Fu);
          asm("" : "+v"(sv));   // keep the one v_bfi_b32 (else re-expanded into and/and/bitop3 per use)
          const uint32_t rot = __builtin_amdgcn_alignbit(pv, pv, 16);
          acc_sym |= pv ^ lsr;
          acc_eq |= pv ^ rot;
          acc_x |= sv ^ rot;
          const uint32_t xs = sw ? sv : pv;
          if (NW == 1) {
            if (NG == 1) key[0] = (xs >> hsh) & 0xFFFFu;
            else if (g == 1) key[0] = __builtin_amdgcn_perm(xs, xs_prev, lo_sel | ((bb + 4u) << 16) | ((bb + 5u) << 24));
          } else if (g & 1) {
            // key word = (half rep of group g-1) | (half rep of group g) << 16
            key[g >> 1] = __builtin_amdgcn_perm(xs, xs_prev, lo_sel | ((bb + 4u) << 16) | ((bb + 5u) << 24));
          }
          xs_prev = xs;
        }
        const uint32_t c = 1u + ((((acc_sym & 0x0F0F0F0Fu) >> hsh) & 0xFFFFu) == 0u) + ((acc_eq & 0xFFFFu) == 0u) +
                           ((acc_x >> 16) == 0u);
        lr += s_lt[c];        // Pd_plotter.py:115, T = T_ref(1/2) = c / 2^n
        if constexpr (M >= 8) {
#pragma unroll
          for (int w = 0; w < NW; ++w) key[w] = key_swap(key[w]);   // device key layout
        }
        if (a.trace) write_trace<m, 1, n, true>(a.trace, t, a.nseq, q, key);
        cur.prefetch(a, key, rn);
        rd.advance();
      }
    }
    if (a.sums) { a.sums[2 * q] = lp; a.sums[2 * q + 1] = lr; }
    early_final(dec, lp, lr);
  }
  count_decisions(valid, q < a.n_h1, lp, lr, a.counts);
}

// k = 1, n = 2 butterfly detector with the branch metrics read from the
// per-code table (cvd_device.h); hipRTC builds the code-specialised variant
template <int m, bool kTrace>
__global__ __launch_bounds__(kBlock, kK1bWavesPerSimd) void detect_k1b_kernel(ExpArgs a) {
  k1b_body<m, false, 0, kTrace>(a, blockIdx.x);
}

// ──────────── chunked detection: the decisions ────────────
//
// The k1s kernel's chunked launch leaves one record per (time chunk j, sequence q): D at the
// chunk's start and end and the chunk's own fp64 sums.  Per sequence this kernel
//  * checks the chunks join: chunk j's warm-started D at its start equals chunk j-1's D at its
//    end (chunk 0 starts from the true D_0 = 0, so every chunk of a joined sequence ran the
//    reference recursion exactly: the step is a function of D and the word);
//  * adds the chunk sums in chunk order and decides lp > lr (Pd_plotter.py:215, :222) only
//    where the decision is certain for the reference's sequential sum as well: all increments
//    are <= 0 (logs of probabilities), so the sequential sum of N terms and this one are both
//    within gamma-type bounds of the exact sum, |S_seq - S_chunk| <= (N + L + C) u (1 + o(1))
//    |S_chunk| with u = 2^-53; with kappa = 4 (N + L + C + 16) u a gap |lp - lr| > 2 kappa
//    (|lp| + |lr|) decides it;
//  * counts the decided sequences (one 64-bit atomic per wave and hypothesis) and lists the
//    others (chunks that did not join, or a gap too small) for the exact sequential rerun.
__global__ __launch_bounds__(kBlock) void ck_combine_kernel(const uint32_t* ck, int64_t nseq, int64_t n_h1,
                                                            int32_t C, double kappa, int32_t redo_all,
                                                            int64_t* counts, int32_t* redo_n, int32_t* redo) {
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = q < nseq, h1 = q < n_h1;
  bool gt = false, lt = false;
  if (valid) {
    bool joined = true;
    double lp = 0.0, lr = 0.0;
    for (int32_t j = 0; j < C; ++j) {
      const uint4* rec = reinterpret_cast<const uint4*>(ck + ((size_t)j * (size_t)nseq + (size_t)q) * kCkRecWords);
      if (j > 0) {
        const uint4* prv =
            reinterpret_cast<const uint4*>(ck + ((size_t)(j - 1) * (size_t)nseq + (size_t)q) * kCkRecWords);
        const uint4 s0 = rec[0], s1 = rec[1], e0 = prv[2], e1 = prv[3];
        joined = joined && s0.x == e0.x && s0.y == e0.y && s0.z == e0.z && s0.w == e0.w && s1.x == e1.x &&
                 s1.y == e1.y && s1.z == e1.z && s1.w == e1.w;
      }
      const uint4 v = rec[4];
      lp += __hiloint2double((int)v.y, (int)v.x);   // chunk order = t order of the chunks
      lr += __hiloint2double((int)v.w, (int)v.z);
    }
    const double d = lp - lr, e = 2.0 * kappa * (fabs(lp) + fabs(lr));
    if (joined && !redo_all) {
      gt = d > e;
      lt = d < -e;
    }
    if (!gt && !lt) {
      const int k = h1 ? 0 : 1;
      const int32_t i = atomicAdd(redo_n + k, 1);
      redo[(size_t)k * (size_t)nseq + (size_t)i] = (int32_t)q;
    }
  }
  const uint64_t b1 = __ballot(valid && h1 && gt), b2 = __ballot(valid && !h1 && lt);   // Pd_plotter.py:215, :222
  if (lane_id() == 0) {
    if (b1) atomicAdd(reinterpret_cast<unsigned long long*>(counts), (unsigned long long)__popcll(b1));
    if (b2) atomicAdd(reinterpret_cast<unsigned long long*>(counts + 1), (unsigned long long)__popcll(b2));
  }
}

// the listed sequences' streams into a compact buffer (H1 list first, then H2), for the rerun:
// 16-B chunk c of sequence q at r4[c pitch + q] (cvd.h stream layout)
__global__ __launch_bounds__(kBlock) void ck_gather_kernel(const uint4* r4, int64_t pitch, int64_t w4,
                                                           const int32_t* redo, int64_t nseq, int32_t n1, int32_t n2,
                                                           uint4* out) {
  const int64_t nr = (int64_t)n1 + n2;
  const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (idx >= w4 * nr) return;
  const int64_t c = idx / nr, i = idx - c * nr;
  const int64_t q = i < n1 ? redo[i] : redo[nseq + (i - n1)];
  out[c * nr + i] = r4[c * pitch + q];
}

using ExpKernel = void (*)(ExpArgs);
ExpKernel pick_k1b(int m, bool trace) {
  switch (m) {
    case 3: return trace ? detect_k1b_kernel<3, true> : detect_k1b_kernel<3, false>;
    case 4: return trace ? detect_k1b_kernel<4, true> : detect_k1b_kernel<4, false>;
    case 5: return trace ? detect_k1b_kernel<5, true> : detect_k1b_kernel<5, false>;
    case 6: return trace ? detect_k1b_kernel<6, true> : detect_k1b_kernel<6, false>;
  }
  return nullptr;
}
ExpKernel pick_k1(int m, int n) {
  if (n == 2) {
    switch (m) {
      case 2: return detect_k1_kernel<2, 2>;
      case 3: return detect_k1_kernel<3, 2>;
      case 4: return detect_k1_kernel<4, 2>;
      case 5: return detect_k1_kernel<5, 2>;
      case 6: return detect_k1_kernel<6, 2>;
    }
  }
  return nullptr;
}

ExpKernel pick_explicit(int m, int k, int n) {
  if (k == 1 && n == 2) {
    switch (m) {
      case 2: return detect_explicit_kernel<2, 1, 2>;
      case 3: return detect_explicit_kernel<3, 1, 2>;
      case 4: return detect_explicit_kernel<4, 1, 2>;
      case 5: return detect_explicit_kernel<5, 1, 2>;
      case 6: return detect_explicit_kernel<6, 1, 2>;
    }
  }
  if (m == 4 && k == 2 && n == 3) return detect_explicit_kernel<4, 2, 3>;
  return nullptr;
}

template <typename T>
int dev_copy(T*& d, const std::vector<T>& h) {
  if (h.empty()) return CVD_OK;
  HIP_CHECK(hipMalloc(&d, h.size() * sizeof(T)));
  HIP_CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return CVD_OK;
}

// A directory from its occupied slots (cvd_internal.h h_key_rows / h_bkey_rows): every slot
// `fill`, then row i's w dwords at slot slots[i].
__global__ __launch_bounds__(kBlock) void dir_scatter_kernel(const uint32_t* rows, const uint32_t* slots, int64_t n,
                                                             int32_t w, uint32_t* dir) {
  const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (idx >= n * w) return;
  const int64_t i = idx / w, k = idx - i * w;
  dir[(size_t)slots[i] * (size_t)w + (size_t)k] = rows[idx];
}

int dev_directory(uint32_t*& d, const std::vector<uint32_t>& rows, const std::vector<uint32_t>& slots, int64_t cap,
                  int32_t w, uint32_t fill) {
  if (rows.empty() || cap <= 0) return CVD_OK;
  const int64_t n = (int64_t)slots.size();
  if ((int64_t)rows.size() != n * w) { set_error("directory rows / slots mismatch"); return CVD_E_INVALID; }
  HIP_CHECK(hipMalloc(&d, (size_t)cap * (size_t)w * sizeof(uint32_t)));
  HIP_CHECK(hipMemsetD32(d, (int)fill, (size_t)cap * (size_t)w));
  uint32_t *dr = nullptr, *ds = nullptr;
  HIP_CHECK(hipMalloc(&dr, rows.size() * sizeof(uint32_t)));
  HIP_CHECK(hipMalloc(&ds, slots.size() * sizeof(uint32_t)));
  HIP_CHECK(hipMemcpy(dr, rows.data(), rows.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(ds, slots.data(), slots.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  const unsigned grid = (unsigned)((n * w + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(dir_scatter_kernel, dim3(grid), dim3(kBlock), 0, 0, dr, ds, n, w, d);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipFree(dr));
  HIP_CHECK(hipFree(ds));
  return CVD_OK;
}

}  // namespace

// ───────────────────────────── launchers ─────────────────────────────────────

int cvd::check_device(const cvd_model& M) {
  if (M.device < 0) { set_error("model not uploaded (cvd_model_upload)"); return CVD_E_STATE; }
  int cur = -1;
  HIP_CHECK(hipGetDevice(&cur));
  if (cur != M.device) { set_error("current device differs from the model's device"); return CVD_E_INVALID; }
  return CVD_OK;
}

namespace {
// GenArgs of an encoder (the bit-parallel generator's window taps included)
GenArgs gen_args(const CodeDesc& enc, uint32_t k0, uint32_t k1, uint32_t tag, uint64_t thr, int64_t N,
                 int random_input) {
  GenArgs a;
  a.enc = enc; a.k0 = k0; a.k1 = k1; a.tag = tag;
  a.thr_all = thr >= (1ull << 32); a.thr_lo = (uint32_t)std::min<uint64_t>(thr, 0xFFFFFFFFull);
  a.random_input = random_input; a.N = N;
  a.seq_base = 0; a.seq_stride = 1; a.pitch = 0; a.q0 = 0; a.count = 0; a.r = nullptr;
  // bit-parallel generator: window taps per (output j, input phase r)
  a.hs = (enc.m + enc.k - 1) / enc.k;
  for (int j = 0; j < kMaxN; ++j) a.taps[j][0] = a.taps[j][1] = 0u;
  for (int j = 0; j < enc.n; ++j)
    for (int i = 0; i < enc.k; ++i) {
      const uint32_t g = enc.gmask[j * enc.k + i];
      if (g & 1u) a.taps[j][i] ^= 1u << a.hs;                     // u_i(t)
      for (int b = 0; b < enc.m; ++b)                              // s bit b = u_{b%k}(t - 1 - b/k)
        if ((g >> (1 + b)) & 1u) a.taps[j][b % enc.k] ^= 1u << (a.hs - 1 - b / enc.k);
    }
  // the taps as window shifts (ChunkEncoder::encode): spread-first (k = 1) window tap sh
  // is n sh; stride-3 (k = 2, n = 3) tap sh of phase r is 30 - 3 hs + 3 sh + r - j.
  // Padding: k = 1 shifts by 1 (lane 0 of the result reads an empty lane; the lane mask
  // drops what lands elsewhere), stride 3 by 5 - j (lane j reads the empty lane 2).
  a.ntap = 0;
  const bool stride3 = CVD_GEN_K2_STRIDE3 && enc.k == 2 && enc.n == 3;
  for (int j = 0; j < kMaxN; ++j) a.tpk[j][0] = a.tpk[j][1] = 0u;
  if ((enc.k == 1 && (enc.n == 2 || enc.n == 3)) || stride3) {
    for (int j = 0; j < enc.n; ++j) {
      uint32_t sl[kTapSlots];
      int c = 0;
      for (int r = 0; r < enc.k; ++r)
        for (int sh = 0; sh < 32; ++sh)
          if ((a.taps[j][r] >> sh) & 1u) {
            const uint32_t s = stride3 ? (uint32_t)(30 - 3 * a.hs + 3 * sh + r - j) : (uint32_t)(enc.n * sh);
            if (c < kTapSlots) sl[c] = s;
            ++c;
          }
      a.ntap = std::max(a.ntap, c);
      for (; c < kTapSlots; ++c) sl[c] = stride3 ? (uint32_t)(5 - j) : 1u;
      for (int i = 0; i < kTapSlots; ++i) a.tpk[j][i / 6] |= (sl[i] & 31u) << (5 * (i % 6));
    }
    if (a.ntap > kTapSlots) a.ntap = 0;
  }
  {
    // test knob: fewer noise exchange slots per round, so the multi-round path runs
    const char* e = std::getenv("CVD_GEN_SLOTS");
    a.slots = e ? (uint32_t)std::min(64, std::max(1, std::atoi(e))) : 64u;
  }
  return a;
}

// the bit-parallel generator applies: k <= 2 and the window of one word fits 32 bits
bool gen_fast_ok(const CodeDesc& enc) {
  return !std::getenv("CVD_GEN_GENERIC") && enc.m <= kMaxM && enc.k <= 2 &&
         (enc.m + enc.k - 1) / enc.k + 32 / std::max(enc.n, 1) <= 32;
}

// unrolled tap-list length for encoders with at most `ntap` taps per output: the
// instantiated lengths (3..6, 8), 0 = the scalar loop over the tap masks (longer lists,
// the k = 2 per-phase form, or CVD_GEN_TAP_LOOP=1)
int tap_slots(int ntap) {
  if (ntap <= 0 || std::getenv("CVD_GEN_TAP_LOOP")) return 0;
  for (int t : {3, 4, 5, 6, 8})
    if (ntap <= t) return t;
  return 0;
}

template <int k, int n>
void (*gen_fast_variant(int kt))(GenArgs) {
  if constexpr (k == 2 && !CVD_GEN_K2_STRIDE3) return gen_fast_kernel<k, n, 0>;
  switch (kt) {
    case 3: return gen_fast_kernel<k, n, 3>;
    case 4: return gen_fast_kernel<k, n, 4>;
    case 5: return gen_fast_kernel<k, n, 5>;
    case 6: return gen_fast_kernel<k, n, 6>;
    case 8: return gen_fast_kernel<k, n, 8>;
    default: return gen_fast_kernel<k, n, 0>;
  }
}
}  // namespace

int cvd::launch_generate(const CodeDesc& enc, uint32_t k0, uint32_t k1, uint32_t tag, uint64_t thr,
                         int64_t N, int random_input, int64_t seq_base, int64_t seq_stride,
                         uint32_t* d_r, int64_t pitch, int64_t q0, int64_t count, void* stream) {
  if (count <= 0 || N <= 0) return CVD_OK;
  GenArgs a = gen_args(enc, k0, k1, tag, thr, N, random_input);
  a.seq_base = seq_base; a.seq_stride = seq_stride;
  a.pitch = pitch; a.q0 = q0; a.count = count; a.r = d_r;
  const unsigned grid = (unsigned)((count + kBlock - 1) / kBlock);
  const bool fast = gen_fast_ok(enc);
  auto kern = gen_kernel<0, 0>;
  dim3 gdim(grid);
  if (fast) {
    // chunk segments per sequence: about 16 waves per SIMD (1024 SIMDs), >= 16 chunks each
    const int64_t nchunks = (((N + 32 / enc.n - 1) / (32 / enc.n)) + 3) / 4;
    const int64_t waves = (count + 63) / 64;
    const int64_t seg = std::max<int64_t>(1, std::min<int64_t>((16 * 1024 + waves - 1) / waves, nchunks / 16));
    gdim.y = (unsigned)std::min<int64_t>(seg, 65535);
  }
  const int kt = tap_slots(a.ntap);
  if (fast && enc.k == 1 && enc.n == 2) kern = gen_fast_variant<1, 2>(kt);
  else if (fast && enc.k == 1 && enc.n == 3) kern = gen_fast_variant<1, 3>(kt);
  else if (fast && enc.k == 2 && enc.n == 3) kern = gen_fast_variant<2, 3>(kt);
  else if (enc.k == 1 && enc.n == 2) kern = gen_kernel<1, 2>;
  else if (enc.k == 1 && enc.n == 3) kern = gen_kernel<1, 3>;
  else if (enc.k == 2 && enc.n == 3) kern = gen_kernel<2, 3>;
  hipLaunchKernelGGL(kern, gdim, dim3(kBlock), 0, (hipStream_t)stream, a);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}

namespace {
// the small-table LDS image (LdsModel kLr): S 2^n 18 B <= 32 KiB, 256-thread blocks
bool table_lr(const cvd_model& M) {
  const int64_t SR = M.S * ((int64_t)1 << M.dec.n);
  return SR * 18 <= 32 * 1024 && !std::getenv("CVD_TABLE_NOLR");
}
}  // namespace

static int env_i(const char* name, int def) {
  const char* e = std::getenv(name);
  return e && *e ? std::atoi(e) : def;
}

int cvd::launch_detect_table(const cvd_model& M, const uint32_t* d_r, int64_t N, int64_t nseq,
                             int64_t n_h1, double* d_sums, int64_t* d_counts, void* stream, bool early) {
  if (M.kind != 0 || !M.d_rec) { set_error("table path needs a dense (enumerated) model"); return CVD_E_UNSUPPORTED; }
  if (nseq <= 0) return CVD_OK;
  TabArgs a;
  const int R = 1 << M.dec.n;
  a.rec = M.d_rec; a.logp1 = M.d_logp1; a.ltref = M.d_ltref; a.n = M.dec.n;
  a.S = M.S; a.N = N; a.nseq = nseq; a.n_h1 = n_h1; a.r = d_r; a.sums = d_sums; a.counts = d_counts;
  a.early = early && !d_sums; a.lt_min = M.ltref[1]; a.lp_min = M.lp_min;
  const size_t lds = (size_t)M.S * R * (sizeof(double) + sizeof(uint32_t)) + (R + 1) * sizeof(double);
  const unsigned grid = (unsigned)((nseq + kBlock - 1) / kBlock);
  // LDS-resident compact model (16-bit records): 1024-thread blocks when it
  // takes most of a CU's 160 KiB, else 256-thread blocks
  const size_t lds16 = (size_t)M.S * R * (sizeof(double) + sizeof(uint16_t)) + (R + 1) * sizeof(double);
  if (M.S < 4096 && lds16 <= 160 * 1024 && (M.dec.n == 2 || M.dec.n == 3) && !std::getenv("CVD_TABLE_WIDE")) {
    const bool big = lds16 > 40 * 1024;
    const int bs = big ? 1024 : kBlock;
    // (the small-table image measured slower here: in the LDS-bound stand-alone walk its
    // log T_ref gathers spread over S 2^n entries instead of 2^n + 1 broadcast ones --
    // m2 overlapped step 43.6 -> 47.2 ms, profiles/r03f/; the fused kernel, VALU-bound,
    // gains from it)
    size_t lds = lds16;
    void (*kern)(TabArgs) = M.dec.n == 2 ? (big ? detect_table16_kernel<2, 1024, false> : detect_table16_kernel<2, kBlock, false>)
                                         : (big ? detect_table16_kernel<3, 1024, false> : detect_table16_kernel<3, kBlock, false>);
    int bsl = bs;
    // (timing studies: the records in LDS and log P̂1 from global memory, 256-thread blocks)
    if (M.dec.n == 3 && env_i("CVD_T16_LPG", 0) == 1) {
      kern = detect_table16_kernel<3, kBlock, false, true>;
      lds = LdsModel<3, false, 1, true>::bytes((int64_t)M.S * R);
      bsl = kBlock;
    }
    if (lds > 64 * 1024)
      HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3((unsigned)((nseq + bsl - 1) / bsl)), dim3(bsl), lds, (hipStream_t)stream, a);
    HIP_CHECK(hipGetLastError());
    return CVD_OK;
  }
  if (lds <= 64 * 1024) {
    hipLaunchKernelGGL(detect_table_kernel<true>, dim3(grid), dim3(kBlock), lds, (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL(detect_table_kernel<false>, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, a);
  }
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}

namespace {
size_t lds16_bytes(const cvd_model& M) {
  const int R = 1 << M.dec.n;
  return (size_t)M.S * R * (sizeof(double) + sizeof(uint16_t)) + (R + 1) * sizeof(double);
}
}  // namespace

bool cvd::mc_fused_preferred(const cvd_model& M) {
  // C1 (m2, 256-thread blocks): 102.2M vs 96.2M trials/s; C3 (rate 2/3, S = 1,807,
  // 1024-thread blocks, 4 waves/SIMD): 4.80M vs 5.60M (profiles/r03e/)
  const int k = M.dec.k, n = M.dec.n;
  return M.kind == 0 && M.S < 4096 && lds16_bytes(M) <= 40 * 1024 && gen_fast_ok(M.dec) &&
         ((k == 1 && (n == 2 || n == 3)) || (k == 2 && n == 3)) && !std::getenv("CVD_MC_UNFUSED");
}

int cvd::launch_mc_fused(const cvd_model& M, const CodeDesc& e1, const CodeDesc& e2, uint32_t k0, uint32_t k1,
                         uint32_t tag, uint64_t thr, int64_t N, int64_t trial_begin, int64_t T, double* d_sums,
                         int64_t* d_counts, void* stream, bool early) {
  const int R = 1 << M.dec.n;
  const size_t lds16 = (size_t)M.S * R * (sizeof(double) + sizeof(uint16_t)) + (R + 1) * sizeof(double);
  const bool big = lds16 > 40 * 1024;
  const int bs = big ? 1024 : kBlock;
  const bool lr = !big && table_lr(M);
  // interleaved copies of the small image (timing studies, LdsModel kCp): CVD_C1_COPIES =
  // 4, 8 or 16 for rate-1/2 codes of at most 3 taps per output
  const int kt0 = tap_slots(std::max(gen_args(e1, k0, k1, tag, thr, N, 1).ntap, gen_args(e2, k0, k1, tag, thr, N, 1).ntap));
  int cp = env_i("CVD_C1_COPIES", 1);
  if (!(lr && M.dec.k == 1 && M.dec.n == 2 && kt0 == 3 && (cp == 4 || cp == 8 || cp == 16) &&
        (int64_t)M.S * R * cp < 65536))
    cp = 1;
  const size_t limg = lr ? (size_t)M.S * R * 18 * cp : lds16;
  const size_t lds = ((limg + 15) & ~(size_t)15) + (size_t)(bs / 64) * 128 * sizeof(uint32_t);
  const int k = M.dec.k, n = M.dec.n;
  if (M.kind != 0 || !M.d_rec || M.S >= 4096 || lds > 160 * 1024 || std::getenv("CVD_MC_UNFUSED") ||
      !((k == 1 && (n == 2 || n == 3)) || (k == 2 && n == 3)) || !gen_fast_ok(e1) || !gen_fast_ok(e2) ||
      e1.k != k || e2.k != k || e1.n != n || e2.n != n) {
    set_error("fused trial kernel: needs an LDS-resident dense model and (k, n) in {(1,2), (1,3), (2,3)}");
    return CVD_E_UNSUPPORTED;
  }
  if (T <= 0 || N <= 0) return CVD_OK;
  FusedArgs a;
  TabArgs& t = a.t;
  t.rec = M.d_rec; t.logp1 = M.d_logp1; t.ltref = M.d_ltref; t.n = n;
  t.S = M.S; t.N = N; t.nseq = 0; t.n_h1 = 0; t.r = nullptr; t.sums = d_sums; t.counts = d_counts;
  t.early = early && !d_sums; t.lt_min = M.ltref[1]; t.lp_min = M.lp_min;
  a.g[0] = gen_args(e1, k0, k1, tag, thr, N, 1);
  a.g[1] = gen_args(e2, k0, k1, tag, thr, N, 1);
  a.trial_begin = trial_begin; a.T = T; a.Tp = (T + 63) & ~(int64_t)63;
  void (*kern)(FusedArgs) = nullptr;
  // unrolled tap lists for rate 1/2 (C1) with at most 3 or 5 taps per output
  const int kt = tap_slots(std::max(a.g[0].ntap, a.g[1].ntap));
  if (k == 1 && n == 2 && kt == 3 && cp > 1)
    kern = cp == 4 ? mc_table16_kernel<1, 2, kBlock, true, 3, 4> : cp == 8 ? mc_table16_kernel<1, 2, kBlock, true, 3, 8>
                                                                  : mc_table16_kernel<1, 2, kBlock, true, 3, 16>;
  else if (k == 1 && n == 2 && kt == 3)
    kern = big ? mc_table16_kernel<1, 2, 1024, false, 3> : lr ? mc_table16_kernel<1, 2, kBlock, true, 3>
                                                            : mc_table16_kernel<1, 2, kBlock, false, 3>;
  else if (k == 1 && n == 2 && (kt == 4 || kt == 5))
    kern = big ? mc_table16_kernel<1, 2, 1024, false, 5> : lr ? mc_table16_kernel<1, 2, kBlock, true, 5>
                                                            : mc_table16_kernel<1, 2, kBlock, false, 5>;
  else if (k == 1 && n == 2)
    kern = big ? mc_table16_kernel<1, 2, 1024, false> : lr ? mc_table16_kernel<1, 2, kBlock, true>
                                                         : mc_table16_kernel<1, 2, kBlock, false>;
  else if (k == 1 && n == 3)
    kern = big ? mc_table16_kernel<1, 3, 1024, false> : lr ? mc_table16_kernel<1, 3, kBlock, true>
                                                         : mc_table16_kernel<1, 3, kBlock, false>;
  else
    kern = big ? mc_table16_kernel<2, 3, 1024, false> : lr ? mc_table16_kernel<2, 3, kBlock, true>
                                                         : mc_table16_kernel<2, 3, kBlock, false>;
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t lanes = 2 * a.Tp;
  hipLaunchKernelGGL(kern, dim3((unsigned)((lanes + bs - 1) / bs)), dim3(bs), lds, (hipStream_t)stream, a);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}

// Kernel of the explicit path: the butterfly kernel when the code has standard
// butterflies, else the orbit kernel (k = 1), else the generic one.
static int select_explicit(const cvd_model& M, int variant, ExpKernel* kern, const uint32_t** bmp,
                           bool trace = false) {
  *kern = nullptr; *bmp = nullptr;
  if ((variant == cvd::kExplicitBest || variant == cvd::kExplicitButterfly) && M.k1b_ok) {
    *bmp = M.d_bfly;
    // the specialised kernel is built without the (test-only) trace path
    if (variant == cvd::kExplicitBest && M.rtc_fn && !trace) return CVD_KERNEL_BUTTERFLY_RTC;
    if (ExpKernel k = pick_k1b(M.dec.m, trace)) { *kern = k; return CVD_KERNEL_BUTTERFLY; }
  }
  if (variant != cvd::kExplicitGeneric && M.k1_ok)
    if (ExpKernel k = pick_k1(M.dec.m, M.dec.n)) { *kern = k; *bmp = M.d_bmk1; return CVD_KERNEL_ORBIT; }
  if (ExpKernel k = pick_explicit(M.dec.m, M.dec.k, M.dec.n)) { *kern = k; *bmp = M.d_bmp; return CVD_KERNEL_GENERIC; }
  *bmp = nullptr;
  return CVD_KERNEL_NONE;
}

int cvd::explicit_kernel_of(const cvd_model& M) {
  ExpKernel k;
  const uint32_t* b;
  const int which = select_explicit(M, kExplicitBest, &k, &b);
  return which == CVD_KERNEL_BUTTERFLY_RTC && M.rtc_bs ? CVD_KERNEL_BITSLICE_RTC : which;
}

// k1b_walk (cvd_device.h) for the H1 waves of the specialised kernel.  Its walks pay
// only when nearly every H1 step stays in learned rows: the learning chain is the H1
// streams' own process, so rows / learn_len estimates the share of steps that leave
// them (m = 6, learn_len 10^6, with two-step records: 0.030 at p = 0.01, where H1 rows
// hold D_t 98% of the time and the launch takes 529 instead of 617 ms; 0.070 at
// p = 0.02: 614 vs 631; 0.32 at p = 0.05: 1,023 vs 680 -- a lane that leaves its walk
// waits for an ACS step of its wave, and those run with few lanes; profiles/r03i_walk/).  CVD_WALK=0 / 1
// forces it off / on (timing studies; the sums are the same).  Counts-only early decision
// stays lockstep unless forced: there walk mode measured slower (p = 0.01: 700 vs 648 ms
// per 2,621,440-trial launch, profiles/r03i_walk/bench_early_walk.json).
// The specialised kernel reads the Bloom filter from LDS (CVD_K1B_LDSF, 512-thread blocks, two
// per CU) for walking models of <= 32,768 rows, whose filter is built with 64 KiB: in walk mode
// the H2 waves are two per SIMD and their per-step filter read from L2 is what they wait on
// (profiles/r03w: skipping it, timing only, takes p = 0.01 524 -> 466 ms per 655,360-trial
// launch).  Measured (profiles/r03x/ab_block.jsonl, ms per 655,360-trial launch, p = 0.01 /
// 0.02): 256-thread blocks, global filter 531.5 / 612.3; 512 threads, LDS filter of 64 KiB
// 502.4 / 619.4 (p = 0.02's 70,134 rows pass ~3% of non-rows at that size); 1,024 threads, LDS
// filter of 128 KiB 543.8 / 643.4 (blocks of 16 waves wait for their slowest wave: 1,024
// threads with the global filter 570.9 / 668.7, 512 threads 541.6 / 625.7).  CVD_NO_LDSF=1
// keeps the filter in global memory.
// The bit-sliced kernel's lockstep lanes read the whole filter from LDS too (CVD_LDSF_LOCKSTEP,
// default 1 for it): no pre-filter and no L2 filter word per lookup.  p = 0.01 (29,626 rows):
// 1,300-1,309 ms per launch against 1,395-1,397 with the pre-filter and L2 filter and 1,472-1,474
// walking (profiles/r06ai, same sums)
bool cvd::ldsf_wanted(const cvd_model& M) {
  const bool bs = M.rtc_fn ? M.rtc_bs : bitslice_preferred(M);
  return walk_preferred(M) || (env_i("CVD_LDSF_LOCKSTEP", bs ? 1 : 0) == 1);
}
bool cvd::ldsf_preferred(const cvd_model& M) {
  return !std::getenv("CVD_NO_LDSF") && ldsf_wanted(M) && M.n_rows <= ldsf_max_rows(M.bs) &&
         M.fcap <= ((int64_t)1 << ldsf_log2(M.bs)) && M.h_filt_lds.size() == (size_t)M.fcap;
}

bool cvd::walk_preferred(const cvd_model& M, bool early) {
  const int e = env_i("CVD_WALK", -1);
  if (e >= 0) return e != 0;
  // the bit-sliced kernel does not walk by default: its lockstep steps are cheaper (round 5:
  // p = 0.02 1,584 ms lockstep against 1,703 walking, profiles/r05r_p*/), and since round 6's
  // table-form ACS and lockstep LDS filter p = 0.01 too (1,300-1,309 ms against 1,472-1,474
  // walking, profiles/r06ai); the butterfly kernel walks below rows / learn_len = 1/10
  // (keyed on the kernel that runs once the JIT has decided -- a model whose bit-sliced build
  // failed runs the butterfly kernel, ADVICE r05 -- else on the tables' prediction)
  if (M.rtc_fn ? M.rtc_bs : bitslice_preferred(M)) return false;
  return !early && M.kind == 1 && M.learn_len_eff > 0 && 10 * M.n_rows < M.learn_len_eff;
}

// the persistent launch's blocks (CVD_K1S_PERSIST=0: never; CVD_K1S_PERSIST_BLOCKS=b: at most b,
// tests), and the sequences above which a launch is persistent
static int64_t persist_cap(const cvd_model& M) {
  if (!M.rtc_fn || !M.rtc_bs || M.rtc_persist_grid <= 0 || env_i("CVD_K1S_PERSIST", 1) == 0) return 0;
  int64_t g = M.rtc_persist_grid;
  if (const int pb = env_i("CVD_K1S_PERSIST_BLOCKS", 0); pb > 0) g = std::min<int64_t>(g, pb);
  return g;
}
int64_t cvd::persist_seqs(const cvd_model& M) { return persist_cap(M) * M.rtc_block; }
int64_t cvd::persist_grid(const cvd_model& M, int64_t nseq) {
  const int64_t g = persist_cap(M);
  return g > 0 && (nseq + M.rtc_block - 1) / M.rtc_block > g ? g : 0;
}

// dynamic LDS of the specialised kernel: the LDS-resident filter or the k1s pre-filter
static unsigned rtc_dyn_lds(const cvd_model& M) {
  // (the LDS filter, then -- compact walk records -- their value table)
  if (M.rtc_ldsf) return (unsigned)(M.fcap * sizeof(uint32_t) + (M.rtc_t2c ? M.h_vtab.size() * sizeof(double) : 0));
  if (M.rtc_pf) return (unsigned)(M.h_bpf.size() * sizeof(uint32_t));
  return 0u;
}

// The explicit path's launch arguments of one model over one stream buffer.
static ExpArgs exp_args(const cvd_model& M, int which, const uint32_t* d_r, int64_t N, int64_t nseq, int64_t n_h1,
                        double* d_sums, int64_t* d_counts, uint8_t* d_trace, const uint32_t* bmp, bool early) {
  ExpArgs a;
  // the bit-sliced kernel (k1s) reads the bit-sliced tables, every other kernel the nibble ones
  const bool bs = which == CVD_KERNEL_BUTTERFLY_RTC && M.rtc_bs;
  // (the LDS-filter kernel copies its own filter copy, the one with its smaller pattern table)
  a.filt = which == CVD_KERNEL_BUTTERFLY_RTC && M.rtc_ldsf ? (bs ? M.d_bfilt_lds : M.d_filt_lds)
                                                            : (bs ? M.d_bfilt : M.d_filt);
  a.hkey = bs ? M.d_bkey : M.d_hkey; a.drow = M.d_drow; a.ltref = M.d_ltref;
  // directory slots: keys [hcap][h_ssw dwords], records [hcap][h_rsw] or, interleaved
  // (no separate record array), at dword nw of each key slot; bit-sliced: 64-dword slots
  // whose layout the kernel knows (cvd_k1s.h)
  a.hrow = bs ? M.d_bkey : M.d_hrow ? M.d_hrow : M.d_hkey + nib_words(M.dec.m);
  a.ksh = bs ? 8u : (uint32_t)__builtin_ctz((unsigned)(4 * M.h_ssw));
  a.rsh = bs ? 8u : M.d_hrow ? (uint32_t)__builtin_ctz((unsigned)(4 * M.h_rsw)) : a.ksh;
  a.bmp = bmp; a.slot0 = M.slot0;
  a.repmap = M.repmap; a.swmap = M.swmap; a.bfly_uni = M.bfly_uni;
  for (int w = 0; w < 4; ++w) a.bfly_even[w] = M.bfly_even[w];
  a.hmask = (uint32_t)((bs ? M.bhcap : M.hcap) - 1); a.fmask = (uint32_t)(M.fcap / 2 - 1); a.fmask4 = a.fmask << 3;
  a.max_probe = bs ? M.bmax_probe : M.max_probe; a.lp_unseen = M.logp1_unseen;
  a.N = N; a.nseq = nseq; a.n_h1 = n_h1; a.r = d_r; a.sums = d_sums; a.counts = d_counts;
  a.trace = d_trace;
  a.early = early && !d_sums && !d_trace; a.lt_min = M.ltref[1]; a.lp_min = M.lp_min;
  a.dkey = bs ? M.d_bdkey : M.d_dkey;
  a.err = M.d_err;
  a.pf = bs && M.rtc_pf ? M.d_bpf : nullptr;
  a.wq = nullptr;   // (launch_detect_explicit sets it for a persistent launch)
  a.ck_n = 0; a.ck_len = 0; a.ck_warm = 0; a.ck_out = nullptr;   // (ck_submit sets them for a chunked launch)
  // Lockstep k1s units alternate H1 and H2 waves where the H1 sequences mostly walk learned rows
  // (rows < learn_len / 2: p <= 0.05 of the sweep), so that every SIMD holds waves of both
  // kinds: H1 waves there wait on cold directory and record lines, H2 waves mostly on the
  // L2-resident filter.  Measured (profiles/r06k, -DCVD_K1S_MIX=1 on every p): p = 0.05 1,983 ->
  // 1,896 ms, p = 0.1 / 0.15 +1% (their H1 and H2 waves look alike).  CVD_K1S_MIX=0 / 1 forces.
  {
    const int e = env_i("CVD_K1S_MIX", -1);
    a.mix = e >= 0 ? (e != 0) : (M.kind == 1 && M.learn_len_eff > 0 && 2 * M.n_rows < M.learn_len_eff);
  }
  // two-step walk records (CVD_WALK_NOT2=1: one 16-B dense record per step instead, a 1.9-MB table
  // at p = 0.01 against 15 MB; L2 hit rate 0.85 against 0.83, and p = 0.01 1,708-1,730 against
  // 1,502-1,503 ms per launch, H1 waves alone 1,208 against 1,018: profiles/r06r, r06s)
  a.t2 = (!M.h_t2.empty() && !std::getenv("CVD_WALK_NOT2")) ? M.d_t2 : nullptr;
  // the k1s walk with the LDS filter reads the compact 8-B records, their log P̂1 values from a
  // table the block copies into LDS after the filter (rtc_t2c, upload_model)
  a.t2c = 0; a.nvtab = 0; a.vtab_off = 0u; a.vtab = nullptr;
  if (a.t2 && which == CVD_KERNEL_BUTTERFLY_RTC && M.rtc_bs && M.rtc_ldsf && M.rtc_t2c) {
    a.t2 = M.d_t2c;
    a.t2c = 1;
    a.vtab = M.d_vtab;
    a.nvtab = (int32_t)M.h_vtab.size();
    a.vtab_off = (uint32_t)(M.fcap * sizeof(uint32_t));
  }
  a.walk = which == CVD_KERNEL_BUTTERFLY_RTC && !d_trace && N < ((int64_t)1 << 31) && M.d_dkey && walk_preferred(M, a.early);
  // schedule: walk while >= 48 lanes walk (a burst costs its load latency whatever the
  // lanes), or while < 4 lanes wait for the ACS (profiles/r03i_walk/ab_policy.jsonl; with
  // two-step records amin 4 instead of 8: p = 0.01 527.1 -> 524.9 ms, p = 0.02 612.3 -> 610.5
  // per 655,360-trial launch, profiles/r03p/ab_sched2.jsonl)
  a.walk_wmin = env_i("CVD_WALK_WMIN", 48);
  a.walk_amin = env_i("CVD_WALK_AMIN", 4);
  // <= 16 steps per burst (k1b_walk's word buffer); two-step records: <= 7 iterations of 2
  a.walk_burst = a.t2 ? std::max(1, std::min(7, env_i("CVD_WALK_BURST", 7)))
                      : std::max(1, std::min(16, env_i("CVD_WALK_BURST", 16)));
  return a;
}

int cvd::launch_detect_explicit(const cvd_model& M, const uint32_t* d_r, int64_t N, int64_t nseq,
                                int64_t n_h1, double* d_sums, int64_t* d_counts, uint8_t* d_trace,
                                void* stream, int variant, bool early) {
  ExpKernel kern = nullptr;
  const uint32_t* bmp = nullptr;
  const int which = select_explicit(M, variant, &kern, &bmp, d_trace != nullptr);
  if (which == CVD_KERNEL_NONE || !M.d_filt || !bmp) {
    set_error("explicit path: unsupported code shape (m,k,n)");
    return CVD_E_UNSUPPORTED;
  }
  if (nseq <= 0) return CVD_OK;
  ExpArgs a = exp_args(M, which, d_r, N, nseq, n_h1, d_sums, d_counts, d_trace, bmp, early);
  const unsigned grid = (unsigned)((nseq + kBlock - 1) / kBlock);
  if (which == CVD_KERNEL_BUTTERFLY_RTC) {
    void* args[] = {&a};
    const unsigned blk = (unsigned)M.rtc_block;
    unsigned rgrid = (unsigned)((nseq + blk - 1) / blk);
    const unsigned lds = rtc_dyn_lds(M);   // the filter (CVD_K1B_LDSF) or the pre-filter (CVD_K1S_PF)
    // k1s over more blocks than stay resident: one block per resident slot, the waves taking
    // their sequences from a work queue (k1s_body); its counter, one of a ring per model, is
    // zeroed on the launch's stream
    if (const int64_t pgrid = persist_grid(M, nseq); pgrid > 0) {
      // (the counter is the launch's own: allocated, zeroed and freed on its stream, so
      // launches of one model on several streams never share one -- ADVICE r05)
      HIP_CHECK(hipMallocAsync((void**)&a.wq, sizeof(uint32_t), (hipStream_t)stream));
      HIP_CHECK(hipMemsetAsync(a.wq, 0, sizeof(uint32_t), (hipStream_t)stream));
      rgrid = (unsigned)pgrid;
    }
    HIP_CHECK(hipModuleLaunchKernel((hipFunction_t)M.rtc_fn, rgrid, 1, 1, blk, 1, 1, lds,
                                    (hipStream_t)stream, args, nullptr));
    if (a.wq) HIP_CHECK(hipFreeAsync(a.wq, (hipStream_t)stream));
    return CVD_OK;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, a);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}

// Models [i0, i1) of a cvd_detect_multi call in one launch of the specialised kernel's
// multi-model entry (k1b_multi, cvd_device.h); the caller checked they share it.
static int launch_multi(const cvd_model* const* models, int32_t i0, int32_t i1, const uint32_t* const* d_r,
                        int64_t N, const int64_t* nseq, const int64_t* n_h1, double* const* d_sums,
                        int64_t* const* d_counts, void* stream, bool early) {
  const cvd_model& M0 = *models[i0];
  MultiArgs ma;
  ma.nm = 0;
  uint32_t blocks = 0;
  const unsigned blk = (unsigned)M0.rtc_block;
  for (int32_t i = i0; i < i1; ++i) {
    const cvd_model& M = *models[i];
    if (nseq[i] <= 0) continue;
    const int64_t nb = (nseq[i] + blk - 1) / blk;
    if ((int64_t)blocks + nb > (int64_t)UINT32_MAX) { set_error("multi-model launch: grid too large"); return CVD_E_INVALID; }
    ma.a[ma.nm] = exp_args(M, CVD_KERNEL_BUTTERFLY_RTC, d_r[i], N, nseq[i], n_h1[i], d_sums ? d_sums[i] : nullptr,
                           d_counts[i], nullptr, M.d_bfly, early);
    blocks += (uint32_t)nb;
    ma.blk_end[ma.nm] = blocks;
    ++ma.nm;
  }
  if (ma.nm == 0) return CVD_OK;
  for (int j = ma.nm; j < kMultiMax; ++j) ma.blk_end[j] = blocks;
  void* args[] = {&ma};
  const unsigned lds = rtc_dyn_lds(M0);
  HIP_CHECK(hipModuleLaunchKernel((hipFunction_t)M0.rtc_fn_multi, blocks, 1, 1, blk, 1, 1, lds, (hipStream_t)stream,
                                  args, nullptr));
  return CVD_OK;
}

// ──────────── chunked detection: launches ────────────
//
// A launch over fewer sequences than fill the device twice (the reference's own call shape,
// run_experiment with num_iter = 10,000: 20,000 sequences per p against 262,144 resident lanes)
// takes as long as one N-step chain.  Chunked, every sequence's N steps are cut into C time
// chunks of L steps, each started W steps early from D = 0 on a lane of its own (the recursion
// forgets its start: profiles/r06_coalesce_study.py, no restart of 512 per p un-coalesced after
// 768 steps at any p in [0.01, 0.5]), so the launch holds C times the lanes.  The counts are the
// sequential path's exactly: ck_combine_kernel keeps a sequence only if its chunks join and its
// decision is certain under the error bound of both summation orders; every other sequence is
// rerun on the sequential kernel.  Counts only (sums and early decision take the sequential path).
std::array<int64_t, 4> cvd::ck_last = {0, 0, 0, 0};
struct CkPlan {
  int32_t C = 0, L = 0, W = 0;
};
static int64_t round_up192(int64_t x) { return (x + 191) / 192 * 192; }
// CVD_CHUNK: -1 (default) where it pays, 0 never, 1 wherever the kernel allows it (tests);
// CVD_CHUNK_WARM (1152), CVD_CHUNK_UNITS (4 x the resident waves): warm-up steps and target units
static bool ck_plan(const cvd_model& M, int64_t N, int64_t nseq_total, CkPlan* P) {
  const int mode = env_i("CVD_CHUNK", -1);
  if (mode == 0 || !M.rtc_fn || !M.rtc_bs || N <= 0 || N >= ((int64_t)1 << 30) || nseq_total <= 0) return false;
  const int64_t W = round_up192(std::max(0, env_i("CVD_CHUNK_WARM", 1152)));
  const int64_t slots = std::max<int64_t>(1, M.rtc_persist_grid) * (M.rtc_block / 64);   // resident waves
  const int64_t waves = (nseq_total + 63) / 64;
  // small batches (fewer waves than two residency rounds): C x the lanes, ~4 rounds of units,
  // the warm-up at most a third of a chunk (profiles/r06c: 0.0686 s for the reference call at
  // 4 rounds against 0.0761 at 2 and 0.0707 at 8; W = 768 left 5-13 reruns per call, 1152 none)
  int64_t target = 4 * slots, Lmin = std::max<int64_t>(192, 3 * W);
  if (waves >= 2 * slots) {
    // large batches of few residency rounds (C4's N = 1e6: three rounds of ~1 s units): the
    // persistent launch's drain -- its last units finish unevenly -- is a large share; chunks
    // of >= 40 W steps (warm-up <= 2.5%) make the units shorter and the drain with them
    if (mode < 0 && waves >= (int64_t)env_i("CVD_CHUNK_MAX_ROUNDS", 12) * slots) return false;
    target = 16 * slots;
    Lmin = std::max<int64_t>(192, 40 * W);
  }
  if (env_i("CVD_CHUNK_UNITS", 0) > 0) target = env_i("CVD_CHUNK_UNITS", 0);
  int64_t C = std::max<int64_t>(1, (target + waves - 1) / waves);
  int64_t L = round_up192((N + C - 1) / C);
  // (forced: any chunk of >= 192 steps)
  L = std::max<int64_t>(L, mode < 0 ? Lmin : 192);
  C = (N + L - 1) / L;
  if (C < 2 || C * waves > (int64_t)UINT32_MAX / 2) return false;
  P->C = (int32_t)C; P->L = (int32_t)L; P->W = (int32_t)W;
  return true;
}

// A chunked group: its models' launches are queued (ck_submit), the decisions and reruns
// follow once for every group of a call (ck_finish: one stream synchronisation).
struct CkGroup {
  std::vector<const cvd_model*> m;
  std::vector<const uint32_t*> r;
  std::vector<int64_t> nseq, nh1;
  std::vector<int64_t*> counts;
  std::vector<uint32_t*> rec;
  std::vector<int32_t*> redo;   // per model: [2][nseq] lists
  int32_t* redo_n = nullptr;    // [models][2]
  void* ws = nullptr;
  CkPlan P;
  int64_t N = 0;
};

static int ck_submit(CkGroup& g, hipStream_t st) {
  const int32_t nm = (int32_t)g.m.size();
  size_t bytes = 0;
  std::vector<size_t> orec(nm), oredo(nm);
  for (int32_t i = 0; i < nm; ++i) {
    orec[i] = bytes;
    bytes += ((size_t)g.P.C * (size_t)g.nseq[i] * kCkRecWords * 4 + 255) / 256 * 256;
    oredo[i] = bytes;
    bytes += ((size_t)2 * (size_t)g.nseq[i] * 4 + 255) / 256 * 256;
  }
  const size_t on = bytes;
  bytes += (size_t)nm * 2 * 4;
  HIP_CHECK(hipMallocAsync(&g.ws, bytes, st));
  char* w = static_cast<char*>(g.ws);
  g.redo_n = reinterpret_cast<int32_t*>(w + on);
  HIP_CHECK(hipMemsetAsync(g.redo_n, 0, (size_t)nm * 2 * 4, st));
  g.rec.resize(nm);
  g.redo.resize(nm);
  for (int32_t i = 0; i < nm; ++i) {
    g.rec[i] = reinterpret_cast<uint32_t*>(w + orec[i]);
    g.redo[i] = reinterpret_cast<int32_t*>(w + oredo[i]);
  }
  auto args_of = [&](int32_t i) {
    const cvd_model& M = *g.m[i];
    ExpArgs a = exp_args(M, CVD_KERNEL_BUTTERFLY_RTC, g.r[i], g.N, g.nseq[i], g.nh1[i], nullptr, g.counts[i], nullptr,
                         M.d_bfly, false);
    a.walk = 0;
    a.early = 0;
    a.ck_n = g.P.C; a.ck_len = g.P.L; a.ck_warm = g.P.W; a.ck_out = g.rec[i];
    return a;
  };
  const cvd_model& M0 = *g.m[0];
  const unsigned blk = (unsigned)M0.rtc_block;
  const unsigned lds = rtc_dyn_lds(M0);
  const int64_t wpb = blk / 64;   // units (waves) per block
  if (nm == 1) {
    ExpArgs a = args_of(0);
    const int64_t units = (int64_t)g.P.C * ((g.nseq[0] + 63) / 64);
    int64_t grid = (units + wpb - 1) / wpb;
    // more blocks than stay resident: the persistent launch (k1s_body's work queue)
    if (const int64_t cap = persist_cap(M0); cap > 0 && grid > cap) {
      HIP_CHECK(hipMallocAsync((void**)&a.wq, sizeof(uint32_t), st));
      HIP_CHECK(hipMemsetAsync(a.wq, 0, sizeof(uint32_t), st));
      grid = cap;
    }
    void* args[] = {&a};
    HIP_CHECK(hipModuleLaunchKernel((hipFunction_t)M0.rtc_fn, (unsigned)grid, 1, 1, blk, 1, 1, lds, st, args, nullptr));
    if (a.wq) HIP_CHECK(hipFreeAsync(a.wq, st));
  } else {
    MultiArgs ma;
    ma.nm = 0;
    int64_t blocks = 0;
    for (int32_t i = 0; i < nm; ++i) {
      blocks += ((int64_t)g.P.C * ((g.nseq[i] + 63) / 64) + wpb - 1) / wpb;
      if (blocks > (int64_t)UINT32_MAX) { set_error("chunked launch: grid too large"); return CVD_E_INVALID; }
      ma.a[ma.nm] = args_of(i);
      ma.blk_end[ma.nm] = (uint32_t)blocks;
      ++ma.nm;
    }
    for (int j = ma.nm; j < kMultiMax; ++j) ma.blk_end[j] = (uint32_t)blocks;
    void* args[] = {&ma};
    HIP_CHECK(hipModuleLaunchKernel((hipFunction_t)M0.rtc_fn_multi, (unsigned)blocks, 1, 1, blk, 1, 1, lds, st, args,
                                    nullptr));
  }
  const double kappa = 4.0 * (double)(g.N + g.P.L + g.P.C + 16) * 0x1p-53;
  const int32_t redo_all = env_i("CVD_CHUNK_REDO_ALL", 0);   // (tests: the rerun path for every sequence)
  for (int32_t i = 0; i < nm; ++i) {
    const unsigned grid = (unsigned)((g.nseq[i] + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(ck_combine_kernel, dim3(grid), dim3(kBlock), 0, st, g.rec[i], g.nseq[i], g.nh1[i], g.P.C, kappa,
                       redo_all, g.counts[i], g.redo_n + 2 * i, g.redo[i]);
    HIP_CHECK(hipGetLastError());
  }
  return CVD_OK;
}

// a call that fails after queueing chunked groups: their workspaces back to the pool
static void ck_release(std::vector<CkGroup>& gs, hipStream_t st) {
  for (CkGroup& g : gs)
    if (g.ws) {
      (void)hipFreeAsync(g.ws, st);
      g.ws = nullptr;
    }
}

// the decisions' loose ends: the sequences ck_combine_kernel could not keep, rerun sequentially
static int ck_finish(std::vector<CkGroup>& gs, hipStream_t st) {
  if (gs.empty()) return CVD_OK;
  struct Rel {
    std::vector<CkGroup>& gs;
    hipStream_t st;
    ~Rel() { ck_release(gs, st); }   // (every return path: the workspaces back to the pool)
  } rel{gs, st};
  std::vector<std::vector<int32_t>> rn(gs.size());
  for (size_t x = 0; x < gs.size(); ++x) {
    rn[x].resize(2 * gs[x].m.size());
    HIP_CHECK(hipMemcpyAsync(rn[x].data(), gs[x].redo_n, rn[x].size() * 4, hipMemcpyDeviceToHost, st));
  }
  HIP_CHECK(hipStreamSynchronize(st));
  int rc = CVD_OK;
  for (size_t x = 0; x < gs.size() && rc == CVD_OK; ++x) {
    CkGroup& g = gs[x];
    for (size_t i = 0; i < g.m.size() && rc == CVD_OK; ++i) {
      const int32_t n1 = rn[x][2 * i], n2 = rn[x][2 * i + 1];
      if (n1 + n2 == 0) continue;
      const int64_t w4 = ((g.N + 15) / 16 + 3) / 4, nr = (int64_t)n1 + n2;
      void* buf = nullptr;
      HIP_CHECK(hipMallocAsync(&buf, (size_t)(w4 * nr) * 16, st));
      const unsigned grid = (unsigned)((w4 * nr + kBlock - 1) / kBlock);
      hipLaunchKernelGGL(ck_gather_kernel, dim3(grid), dim3(kBlock), 0, st, reinterpret_cast<const uint4*>(g.r[i]),
                         g.nseq[i], w4, g.redo[i], g.nseq[i], n1, n2, static_cast<uint4*>(buf));
      HIP_CHECK(hipGetLastError());
      rc = launch_detect_explicit(*g.m[i], static_cast<const uint32_t*>(buf), g.N, nr, n1, nullptr, g.counts[i], nullptr,
                                  st, kExplicitBest, false);
      HIP_CHECK(hipFreeAsync(buf, st));
    }
  }
  // (the redo counts of the last call, for cvd_chunk_last)
  int64_t tot = 0;
  for (auto& v : rn)
    for (int32_t c : v) tot += c;
  cvd::ck_last[3] = tot;
  return rc;
}

std::string cvd::rtc_variant_defs(int block, bool ldsf, int patbits, bool bs, bool pf, int pf_log2, bool slot3) {
  return "-DCVD_K1B_BLOCK=" + std::to_string(block) + (ldsf ? " -DCVD_K1B_LDSF=1" : "") +
         (patbits != kFilterPatBits ? " -DCVD_FILTER_PAT_BITS=" + std::to_string(patbits) : "") +
         (bs ? " -DCVD_K1B_BITSLICE=1" : "") + (pf ? " -DCVD_K1S_PF=1" : "") +
         (pf && pf_log2 != kBsPfLog2Bits ? " -DCVD_K1S_PF_LOG2=" + std::to_string(pf_log2) : "") +
         (bs && slot3 ? " -DCVD_K1S_SLOT3=1" : "");
}

int cvd::upload_model(cvd_model& M, int device) {
  if (M.device == device) return CVD_OK;
  if (M.device >= 0) free_model_device(M);
  // the caller's current device is restored on every return path
  int cur = 0;
  HIP_CHECK(hipGetDevice(&cur));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{cur};
  HIP_CHECK(hipSetDevice(device));
  int rc;
  if ((rc = dev_copy(M.d_ltref, M.ltref))) return rc;
  if (M.kind == 0) {
    if ((rc = dev_copy(M.d_rec, M.rec))) return rc;
    if ((rc = dev_copy(M.d_logp1, M.logp1))) return rc;
  }
  if (M.hcap > 0) {
    if ((rc = dev_copy(M.d_filt, M.h_filt))) return rc;
    if ((rc = dev_copy(M.d_filt_lds, M.h_filt_lds))) return rc;
    if ((rc = dev_directory(M.d_hkey, M.h_key_rows, M.h_key_slot, M.hcap, M.h_ssw, kEmptyKey))) return rc;
    if ((rc = dev_directory(M.d_hrow, M.h_row_rows, M.h_key_slot, M.hcap, M.h_rsw, 0u))) return rc;
    if ((rc = dev_copy(M.d_drow, M.h_drow))) return rc;
    if ((rc = dev_copy(M.d_dkey, M.h_dkey))) return rc;
    if ((rc = dev_copy(M.d_t2, M.h_t2))) return rc;
    if ((rc = dev_copy(M.d_t2c, M.h_t2c))) return rc;
    if ((rc = dev_copy(M.d_vtab, M.h_vtab))) return rc;
    if ((rc = dev_copy(M.d_bfilt, M.h_bfilt))) return rc;
    if ((rc = dev_copy(M.d_bfilt_lds, M.h_bfilt_lds))) return rc;
    if ((rc = dev_directory(M.d_bkey, M.h_bkey_rows, M.h_bkey_slot, M.bhcap, M.bs_slot_w, 0u))) return rc;
    if ((rc = dev_copy(M.d_bdkey, M.h_bdkey))) return rc;
    if ((rc = dev_copy(M.d_bpf, M.h_bpf))) return rc;
    if ((rc = dev_copy(M.d_bmp, M.bmp))) return rc;
    if ((rc = dev_copy(M.d_bmk1, M.bmk1))) return rc;
    if ((rc = dev_copy(M.d_bfly, M.bfly))) return rc;
  }
  HIP_CHECK(hipMalloc((void**)&M.d_err, sizeof(int32_t)));
  HIP_CHECK(hipMemset(M.d_err, 0, sizeof(int32_t)));
  M.device = device;
  // smallest per-step log P̂1 (early decision bound): every row entry and, for
  // sparse models, the unvisited-row value
  M.lp_min = M.kind == 1 ? M.logp1_unseen : 0.0;
  for (double v : M.logp1) M.lp_min = std::min(M.lp_min, v);
  // code-specialised butterfly kernel (cvd_rtc.cpp); without it the compiled
  // table-driven kernel runs (same results), and the reason is kept for
  // cvd_model_jit_status
  M.rtc_fn = nullptr;
  M.rtc_fn_multi = nullptr;
  M.jit_error.clear();
  M.rtc_ldsf = M.k1b_ok && M.hcap > 0 && ldsf_preferred(M);
  // the bit-sliced form (k1s) for models with the bit-sliced tables, with the LDS pre-filter
  // where the model has one; if it cannot be built, the butterfly kernel on the nibble tables
  M.rtc_bs = false;
  M.rtc_pf = false;
  for (int attempt = M.bs && M.d_bkey ? 0 : 1; attempt < 2 && M.k1b_ok && M.hcap > 0; ++attempt) {
    const bool bs = attempt == 0;
    const bool pf = bs && !M.rtc_ldsf && M.d_bpf != nullptr;
    // block size: 512 threads with the LDS filter (two blocks of 8 waves per CU hold it),
    // 1,024 with the 128-KiB LDS filter or the pre-filter (one block per CU), else 256
    // (CVD_K1B_BLOCK=256/512/1024 overrides the first and last, timing studies)
    M.rtc_block = pf ? (M.bs_pf_log2 >= 20 ? 1024 : 512) : env_i("CVD_K1B_BLOCK", M.rtc_ldsf ? (M.fcap > ((int64_t)1 << 14) ? 1024 : 512) : kBlock);
    if (M.rtc_block != 256 && M.rtc_block != 512 && M.rtc_block != 1024) M.rtc_block = kBlock;
    const int patbits = M.rtc_ldsf ? kFilterPatBitsLds : bs ? M.bs_pat_bits : kFilterPatBits;
    const std::string vdefs = rtc_variant_defs(M.rtc_block, M.rtc_ldsf, patbits, bs, pf, M.bs_pf_log2, M.bs_slot_w == 96);
    if (rtc_k1b_function(device, M.dec.m, M.bfly_x, vdefs.c_str(), &M.rtc_fn, &M.rtc_fn_multi) == 0) {
      M.rtc_bs = bs;
      M.rtc_pf = pf;
      M.jit_error.clear();
      break;
    }
    M.rtc_fn = nullptr;
    M.rtc_fn_multi = nullptr;
    M.jit_error = last_error_copy();
  }
  if (!M.rtc_fn) {
    M.rtc_ldsf = false;
    M.rtc_block = kBlock;
  }
  // compact walk records: where the k1s walk variant runs with the LDS filter and the value
  // table fits beside it and the kernel's static LDS (CVD_WALK_T2C=0 at build: not built)
  M.rtc_t2c = false;
  if (M.rtc_fn && M.rtc_bs && M.rtc_ldsf && M.d_t2c && M.d_vtab) {
    int st = 0, mx = 0;
    if (hipFuncGetAttribute(&st, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, (hipFunction_t)M.rtc_fn) == hipSuccess &&
        hipDeviceGetAttribute(&mx, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) == hipSuccess &&
        (int64_t)st + M.fcap * 4 + (int64_t)M.h_vtab.size() * 8 <= (int64_t)mx)
      M.rtc_t2c = true;
  }
  // persistent launches of k1s: as many blocks as the device keeps resident
  M.rtc_persist_grid = 0;
  if (M.rtc_fn && M.rtc_bs) {
    int nb = 0, ncu = 0;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (hipFunction_t)M.rtc_fn, M.rtc_block,
                                                           rtc_dyn_lds(M)) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && nb > 0 && ncu > 0) {
      M.rtc_persist_grid = (int64_t)nb * ncu;
    }
  }
  return CVD_OK;
}

void cvd::free_model_device(cvd_model& M) {
  if (M.device < 0) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(M.device);
  void* ptrs[] = {M.d_rec, M.d_logp1, M.d_ltref, M.d_filt, M.d_filt_lds, M.d_hkey, M.d_hrow, M.d_drow, M.d_dkey, M.d_t2,
                  M.d_t2c, M.d_vtab, M.d_bmp,
                  M.d_bmk1, M.d_bfly, M.d_err, M.d_bfilt, M.d_bfilt_lds, M.d_bkey, M.d_bdkey, M.d_bpf};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  M.d_rec = nullptr; M.d_logp1 = nullptr; M.d_ltref = nullptr;
  M.d_filt = nullptr; M.d_filt_lds = nullptr; M.d_hkey = nullptr; M.d_hrow = nullptr; M.d_drow = nullptr; M.d_dkey = nullptr; M.d_t2 = nullptr;
  M.d_t2c = nullptr; M.d_vtab = nullptr; M.rtc_t2c = false;
  M.d_bfilt = nullptr; M.d_bfilt_lds = nullptr; M.d_bkey = nullptr; M.d_bdkey = nullptr; M.d_bpf = nullptr;
  M.rtc_persist_grid = 0;
  M.rtc_bs = false;
  M.rtc_pf = false;
  M.d_bmp = nullptr;
  M.d_bmk1 = nullptr;
  M.d_bfly = nullptr;
  M.d_err = nullptr;
  M.rtc_fn = nullptr;
  M.rtc_fn_multi = nullptr;
  M.device = -1;
  (void)hipSetDevice(cur);
}

// ───────────────────────────── ABI: device work ─────────────────────────────

namespace {
int parse_code_dev(const cvd_code* c, CodeDesc& d) {
  if (!c || !c->taps || c->k < 1 || c->k > kMaxK || c->n < 1 || c->n > kMaxN || c->m < 1 || c->m > kMaxM) {
    set_error("bad code description");
    return CVD_E_INVALID;
  }
  d.k = c->k; d.n = c->n; d.m = c->m;
  for (int i = 0; i < kMaxN * kMaxK; ++i) d.gmask[i] = 0;
  const int L = c->m + 1;
  for (int j = 0; j < c->n; ++j)
    for (int i = 0; i < c->k; ++i) {
      uint32_t g = 0;
      for (int t = 0; t < L; ++t) {
        const uint8_t b = c->taps[(j * c->k + i) * L + t];
        if (b > 1) { set_error("taps must be 0/1"); return CVD_E_INVALID; }
        g |= (uint32_t)b << t;
      }
      d.gmask[j * c->k + i] = g;
    }
  return CVD_OK;
}
}  // namespace

extern "C" int cvd_generate(const cvd_code* enc, uint64_t seed, uint32_t tag, double p, int64_t N,
                            int32_t random_input, int64_t seq_base, int64_t seq_stride,
                            uint32_t* d_r, int64_t pitch, int64_t q0, int64_t count, void* stream) {
  CodeDesc d;
  int rc = parse_code_dev(enc, d);
  if (rc) return rc;
  if (!(p >= 0.0 && p <= 1.0)) { set_error("p must lie in [0, 1]"); return CVD_E_INVALID; }
  if (N < 0 || count < 0 || q0 < 0 || q0 + count > pitch || (!d_r && N > 0 && count > 0)) {
    set_error("bad buffer geometry");
    return CVD_E_INVALID;
  }
  return launch_generate(d, (uint32_t)seed, (uint32_t)(seed >> 32), tag, noise_threshold(p), N,
                         random_input, seq_base, seq_stride, d_r, pitch, q0, count, stream);
}

static int detect_one(const cvd_model* model, const uint32_t* d_r, int64_t N, int64_t nseq, int64_t n_h1,
                      double* d_sums, int64_t* d_counts, int32_t path, void* stream);

extern "C" int cvd_detect(const cvd_model* model, const uint32_t* d_r, int64_t N, int64_t nseq,
                          int64_t n_h1, double* d_sums, int64_t* d_counts, int32_t path, void* stream) {
  cvd::ck_last = {0, 0, 0, 0};
  return detect_one(model, d_r, N, nseq, n_h1, d_sums, d_counts, path, stream);
}

static int detect_one(const cvd_model* model, const uint32_t* d_r, int64_t N, int64_t nseq, int64_t n_h1,
                      double* d_sums, int64_t* d_counts, int32_t path, void* stream) {
  if (!model || (!d_r && N > 0 && nseq > 0) || !d_counts || N < 0 || nseq < 0 || n_h1 < 0 || n_h1 > nseq) {
    set_error("bad detect arguments");
    return CVD_E_INVALID;
  }
  int rc = check_device(*model);
  if (rc) return rc;
  const bool early = (path & CVD_DETECT_EARLY_DECISION) != 0;
  path &= ~CVD_DETECT_EARLY_DECISION;
  if (early && d_sums) {
    set_error("early decision stops a trial once its decision is certain: per-trial sums need the full run");
    return CVD_E_INVALID;
  }
  if (path == CVD_PATH_AUTO) path = model->kind == 0 ? CVD_PATH_TABLE : CVD_PATH_EXPLICIT;
  if (path == CVD_PATH_TABLE)
    return launch_detect_table(*model, d_r, N, nseq, n_h1, d_sums, d_counts, stream, early);
  // counts of a batch too small to fill the device: the chunked launch (same counts)
  CkPlan P;
  if (path == CVD_PATH_EXPLICIT && !d_sums && !early && model->kind == 1 && ck_plan(*model, N, nseq, &P)) {
    std::vector<CkGroup> gs(1);
    CkGroup& g = gs[0];
    g.m = {model}; g.r = {d_r}; g.nseq = {nseq}; g.nh1 = {n_h1}; g.counts = {d_counts}; g.P = P; g.N = N;
    cvd::ck_last = {cvd::ck_last[0] + 1, P.C, P.L, 0};
    rc = ck_submit(g, (hipStream_t)stream);
    if (rc) {
      ck_release(gs, (hipStream_t)stream);
      return rc;
    }
    return ck_finish(gs, (hipStream_t)stream);
  }
  if (path == CVD_PATH_EXPLICIT || path == CVD_PATH_EXPLICIT_GENERIC || path == CVD_PATH_EXPLICIT_ORBIT ||
      path == CVD_PATH_EXPLICIT_BUTTERFLY)
    return launch_detect_explicit(*model, d_r, N, nseq, n_h1, d_sums, d_counts, nullptr, stream,
                                  path == CVD_PATH_EXPLICIT ? kExplicitBest
                                  : path == CVD_PATH_EXPLICIT_ORBIT ? kExplicitOrbit
                                  : path == CVD_PATH_EXPLICIT_BUTTERFLY ? kExplicitButterfly : kExplicitGeneric,
                                  early);
  set_error("unknown path");
  return CVD_E_INVALID;
}

// Models i and j can share one multi-model launch: the same specialised kernel variant
// (decoder code, block size, LDS filter) on the same device, explicit best path.
static bool multi_ok(const cvd_model& M) {
  return M.kind == 1 && M.rtc_fn && M.rtc_fn_multi && !std::getenv("CVD_NO_MULTI");
}
static bool multi_same(const cvd_model& A, const cvd_model& B) {
  return A.rtc_fn_multi == B.rtc_fn_multi && A.rtc_block == B.rtc_block && A.rtc_ldsf == B.rtc_ldsf &&
         A.rtc_bs == B.rtc_bs && A.rtc_pf == B.rtc_pf && (!A.rtc_pf || A.bs_pf_log2 == B.bs_pf_log2) && (!A.rtc_bs || A.bs_pat_bits == B.bs_pat_bits) && A.device == B.device &&
         (!A.rtc_ldsf || A.fcap == B.fcap);
}
// the same criterion as one id (cvd_model_info.multi_variant: the Python host groups launches
// for per-launch timing by it): equal for models multi_same merges, 0 if multi_ok fails
int64_t cvd::multi_variant(const cvd_model& M) {
  if (!multi_ok(M)) return 0;
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
  mix((uint64_t)(uintptr_t)M.rtc_fn_multi); mix((uint64_t)M.rtc_block); mix(M.rtc_ldsf ? 1u : 0u);
  mix(M.rtc_bs ? 1u : 0u); mix(M.rtc_pf ? (uint64_t)M.bs_pf_log2 : 0u); mix((uint64_t)(M.device + 1)); mix(M.rtc_ldsf ? (uint64_t)M.fcap : 0u);
  return (int64_t)(h | 1u);
}

extern "C" int cvd_detect_multi(const cvd_model* const* models, int32_t nm, const uint32_t* const* d_r, int64_t N,
                                const int64_t* nseq, const int64_t* n_h1, double* const* d_sums,
                                int64_t* const* d_counts, int32_t path, void* stream) {
  if (!models || nm < 0 || (nm > 0 && (!d_r || !nseq || !n_h1 || !d_counts)) || N < 0) {
    set_error("bad detect_multi arguments");
    return CVD_E_INVALID;
  }
  const bool early = (path & CVD_DETECT_EARLY_DECISION) != 0;
  const int32_t base = path & ~CVD_DETECT_EARLY_DECISION;
  for (int32_t i = 0; i < nm; ++i) {
    if (!models[i] || (!d_r[i] && N > 0 && nseq[i] > 0) || !d_counts[i] || nseq[i] < 0 || n_h1[i] < 0 ||
        n_h1[i] > nseq[i]) {
      set_error("bad detect_multi arguments");
      return CVD_E_INVALID;
    }
    if (early && d_sums && d_sums[i]) {
      set_error("early decision stops a trial once its decision is certain: per-trial sums need the full run");
      return CVD_E_INVALID;
    }
    const int rc = check_device(*models[i]);
    if (rc) return rc;
  }
  int32_t i = 0;
  // a model whose own launch is persistent (a batch past the resident capacity) runs alone:
  // the work queue keeps a CU's waves busy to the end, which a merged block launch does not
  // (cvd_model_info.persist_seqs)
  auto merges = [&](int32_t k) { return multi_ok(*models[k]) && persist_grid(*models[k], nseq[k]) == 0; };
  // groups of batches too small to fill the device: chunked launches (same counts), their
  // decisions and reruns after the last launch of the call (ck_finish)
  std::vector<CkGroup> ck;
  const bool ck_ok = (base == CVD_PATH_AUTO || base == CVD_PATH_EXPLICIT) && !early;
  cvd::ck_last = {0, 0, 0, 0};
  while (i < nm) {
    const cvd_model& M = *models[i];
    const bool mok = (base == CVD_PATH_AUTO || base == CVD_PATH_EXPLICIT) && merges(i);
    int32_t j = i + 1;
    if (mok)
      while (j < nm && j - i < kMultiMax && merges(j) && multi_same(M, *models[j])) ++j;
    int rc;
    bool sums_any = false;
    int64_t ntot = 0;
    for (int32_t x = i; x < (mok ? j : i + 1); ++x) {
      sums_any = sums_any || (d_sums && d_sums[x]);
      ntot += nseq[x];
    }
    CkPlan P;
    if (ck_ok && !sums_any && M.kind == 1 && (mok || j == i + 1) && ck_plan(M, N, ntot, &P)) {
      if (!mok) j = i + 1;
      CkGroup g;
      for (int32_t x = i; x < j; ++x) {
        if (nseq[x] <= 0) continue;
        g.m.push_back(models[x]); g.r.push_back(d_r[x]); g.nseq.push_back(nseq[x]); g.nh1.push_back(n_h1[x]);
        g.counts.push_back(d_counts[x]);
      }
      g.P = P;
      g.N = N;
      if (!g.m.empty()) {
        ck.push_back(std::move(g));
        if ((rc = ck_submit(ck.back(), (hipStream_t)stream))) {
          ck_release(ck, (hipStream_t)stream);
          return rc;
        }
        cvd::ck_last = {cvd::ck_last[0] + 1, P.C, P.L, 0};
      }
      i = j;
      continue;
    }
    if (mok && j - i > 1) {
      rc = launch_multi(models, i, j, d_r, N, nseq, n_h1, d_sums, d_counts, stream, early);
    } else {
      j = i + 1;
      rc = detect_one(models[i], d_r[i], N, nseq[i], n_h1[i], d_sums ? d_sums[i] : nullptr, d_counts[i], path, stream);
    }
    if (rc) {
      ck_release(ck, (hipStream_t)stream);
      return rc;
    }
    i = j;
  }
  return ck_finish(ck, (hipStream_t)stream);
}

extern "C" int cvd_trace(const cvd_model* model, const uint32_t* d_r, int64_t N, int64_t nseq,
                         uint8_t* d_D, void* stream) {
  if (!model || (!d_r && N > 0 && nseq > 0) || (!d_D && nseq > 0) || N < 0 || nseq < 0) {
    set_error("bad trace arguments");
    return CVD_E_INVALID;
  }
  int rc = check_device(*model);
  if (rc) return rc;
  // the counts of a trace launch are discarded into a scratch pair
  int64_t* d_tmp = nullptr;
  HIP_CHECK(hipMallocAsync((void**)&d_tmp, 2 * sizeof(int64_t), (hipStream_t)stream));
  HIP_CHECK(hipMemsetAsync(d_tmp, 0, 2 * sizeof(int64_t), (hipStream_t)stream));
  rc = launch_detect_explicit(*model, d_r, N, nseq, 0, nullptr, d_tmp, d_D, stream, kExplicitBest);
  (void)hipFreeAsync(d_tmp, (hipStream_t)stream);
  return rc;
}

extern "C" int64_t cvd_mc_workspace_bytes(const cvd_code* enc1, int64_t N, int64_t batch) {
  if (!enc1 || enc1->n < 1 || N < 0 || batch < 0) return -1;
  const int64_t spw = 32 / enc1->n;
  const int64_t w4 = ((N + spw - 1) / spw + 3) / 4;
  return w4 * 4 * 2 * batch * (int64_t)sizeof(uint32_t);
}

// Trials per launch of the fused kernel: its grid has 2 Tp lanes (HIP bounds a grid at
// 2^32 work-items), so cvd_mc_run and cvd_mc_fused slice longer ranges; a slice of 2^28
// trials is ~2,000 residency rounds, so the slicing costs nothing measurable.
// CVD_MC_FUSED_SLICE lowers it (tests run the multi-slice path with small ranges).
static int64_t fused_slice() {
  const char* e = std::getenv("CVD_MC_FUSED_SLICE");
  const int64_t v = e && *e ? std::atoll(e) : 0;
  return v > 0 ? std::min<int64_t>(v, (int64_t)1 << 28) : ((int64_t)1 << 28);
}

static int mc_fused_sliced(const cvd_model& M, const CodeDesc& e1, const CodeDesc& e2, uint64_t seed, uint32_t tag,
                           uint64_t thr, int64_t N, int64_t trial_begin, int64_t trial_end, double* d_sums,
                           int64_t* d_counts, void* stream, bool early) {
  const int64_t sl = fused_slice();
  for (int64_t b = trial_begin; b < trial_end; b += sl) {
    const int64_t T = std::min(sl, trial_end - b);
    const int rc = launch_mc_fused(M, e1, e2, (uint32_t)seed, (uint32_t)(seed >> 32), tag, thr, N, b, T,
                                   d_sums ? d_sums + 4 * (b - trial_begin) : nullptr, d_counts, stream, early);
    if (rc) return rc;
  }
  return CVD_OK;
}

// Whether cvd_mc_run (path, model) runs the fused kernel and so needs no workspace.
static bool mc_run_fused(const cvd_model& M, int32_t path) {
  return (path & ~CVD_DETECT_EARLY_DECISION) == CVD_PATH_AUTO && mc_fused_preferred(M);
}

extern "C" int cvd_mc_run(const cvd_model* model, const cvd_code* enc1, const cvd_code* enc2,
                          double p, int64_t N, uint64_t seed, int64_t trial_begin, int64_t trial_end,
                          int64_t batch, void* d_work, int64_t* d_counts, int32_t path, void* stream) {
  if (!model || !d_counts || trial_end < trial_begin || batch <= 0 || N < 0) {
    set_error("bad mc_run arguments");
    return CVD_E_INVALID;
  }
  CodeDesc e1, e2;
  int rc;
  if ((rc = parse_code_dev(enc1, e1)) || (rc = parse_code_dev(enc2, e2))) return rc;
  if (e1.n != model->dec.n || e2.n != model->dec.n || e1.k != model->dec.k || e2.k != model->dec.k) {
    set_error("encoder and decoder must share (k, n)");
    return CVD_E_INVALID;
  }
  if (!(p >= 0.0 && p <= 1.0)) { set_error("p must lie in [0, 1]"); return CVD_E_INVALID; }
  const uint32_t tag = grid_tag(N, p);
  const uint64_t thr = noise_threshold(p);
  const bool early = (path & CVD_DETECT_EARLY_DECISION) != 0;
  if (mc_run_fused(*model, path)) {
    // LDS-resident dense models: the fused trial kernel, no streams in HBM (same counts),
    // in slices of at most fused_slice() trials per launch
    if ((rc = check_device(*model))) return rc;
    rc = mc_fused_sliced(*model, e1, e2, seed, tag, thr, N, trial_begin, trial_end, nullptr, d_counts, stream,
                         early);
    if (rc != CVD_E_UNSUPPORTED) return rc;
  }
  if (!d_work) {
    set_error("cvd_mc_run: this model and path need the stream workspace (cvd_mc_workspace_bytes)");
    return CVD_E_INVALID;
  }
  uint32_t* r = static_cast<uint32_t*>(d_work);
  for (int64_t b = trial_begin; b < trial_end; b += batch) {
    const int64_t T = std::min(batch, trial_end - b);
    if ((rc = launch_generate(e1, (uint32_t)seed, (uint32_t)(seed >> 32), tag, thr, N, 1, 2 * b, 2, r,
                              2 * T, 0, T, stream)))
      return rc;
    if ((rc = launch_generate(e2, (uint32_t)seed, (uint32_t)(seed >> 32), tag, thr, N, 1, 2 * b + 1, 2, r,
                              2 * T, T, T, stream)))
      return rc;
    if ((rc = cvd_detect(model, r, N, 2 * T, T, nullptr, d_counts, path, stream))) return rc;
  }
  return CVD_OK;
}

extern "C" int cvd_mc_fused(const cvd_model* model, const cvd_code* enc1, const cvd_code* enc2, double p, int64_t N,
                            uint64_t seed, int64_t trial_begin, int64_t trial_end, double* d_sums,
                            int64_t* d_counts, int32_t flags, void* stream) {
  if (!model || !d_counts || trial_end < trial_begin || N < 0) {
    set_error("bad mc_fused arguments");
    return CVD_E_INVALID;
  }
  CodeDesc e1, e2;
  int rc;
  if ((rc = parse_code_dev(enc1, e1)) || (rc = parse_code_dev(enc2, e2))) return rc;
  if (!(p >= 0.0 && p <= 1.0)) { set_error("p must lie in [0, 1]"); return CVD_E_INVALID; }
  const bool early = (flags & CVD_DETECT_EARLY_DECISION) != 0;
  if (early && d_sums) {
    set_error("early decision stops a trial once its decision is certain: per-trial sums need the full run");
    return CVD_E_INVALID;
  }
  if ((rc = check_device(*model))) return rc;
  return mc_fused_sliced(*model, e1, e2, seed, grid_tag(N, p), noise_threshold(p), N, trial_begin, trial_end, d_sums,
                         d_counts, stream, early);
}

extern "C" int cvd_chunk_last(int64_t* out4) {
  if (!out4) { set_error("null argument"); return CVD_E_INVALID; }
  for (int i = 0; i < 4; ++i) out4[i] = cvd::ck_last[i];
  return CVD_OK;
}

extern "C" int cvd_model_device_error(cvd_model* model, int32_t* flags_out) {
  if (!model || !flags_out) { set_error("null argument"); return CVD_E_INVALID; }
  *flags_out = 0;
  if (model->device < 0 || !model->d_err) return CVD_OK;
  int cur = 0;
  HIP_CHECK(hipGetDevice(&cur));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{cur};
  HIP_CHECK(hipSetDevice(model->device));
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(flags_out, model->d_err, sizeof(int32_t), hipMemcpyDeviceToHost));
  HIP_CHECK(hipMemset(model->d_err, 0, sizeof(int32_t)));
  if (*flags_out) {
    set_error("detector kernel error flags set (bit 0: walk-mode scheduler guard hit; the launch's counts are void)");
    return CVD_E_STATE;
  }
  return CVD_OK;
}

// ─────────────── the (N, p) grid in one call ───────────────

extern "C" int64_t cvd_mc_grid_workspace_bytes(const cvd_model* const* models, int32_t np, const cvd_code* enc1,
                                               const int64_t* N, int32_t nN, int64_t batch, int32_t path) {
  if (!models || np <= 0 || !enc1 || !N || nN <= 0 || batch <= 0) return -1;
  int32_t need = 0;   // grid points that run generator + detector (one stream slot each)
  for (int32_t i = 0; i < np; ++i) {
    if (!models[i]) return -1;
    need += mc_run_fused(*models[i], path) ? 0 : 1;
  }
  int64_t best = 0;
  for (int32_t j = 0; j < nN; ++j) {
    if (N[j] < 0) return -1;
    best = std::max(best, cvd_mc_workspace_bytes(enc1, N[j], batch));
  }
  return best * need;
}

extern "C" int cvd_mc_run_grid(const cvd_model* const* models, const cvd_code* enc1, const cvd_code* enc2,
                               const double* p, int32_t np, const int64_t* N, int32_t nN, uint64_t seed,
                               int64_t trial_begin, int64_t trial_end, int64_t batch, void* d_work,
                               int64_t* d_counts, int32_t path, void* stream) {
  if (!models || !p || !N || np <= 0 || nN <= 0 || !d_counts || trial_end < trial_begin || batch <= 0) {
    set_error("bad mc_run_grid arguments");
    return CVD_E_INVALID;
  }
  CodeDesc e1, e2;
  int rc;
  if ((rc = parse_code_dev(enc1, e1)) || (rc = parse_code_dev(enc2, e2))) return rc;
  std::vector<int32_t> two;   // grid points on generator + detector (the others run the fused kernel)
  for (int32_t i = 0; i < np; ++i) {
    if (!models[i]) { set_error("mc_run_grid: null model"); return CVD_E_INVALID; }
    if (!(p[i] >= 0.0 && p[i] <= 1.0)) { set_error("p must lie in [0, 1]"); return CVD_E_INVALID; }
    if (e1.n != models[i]->dec.n || e2.n != models[i]->dec.n || e1.k != models[i]->dec.k || e2.k != models[i]->dec.k) {
      set_error("encoder and decoder must share (k, n)");
      return CVD_E_INVALID;
    }
    if ((rc = check_device(*models[i]))) return rc;
    if (!mc_run_fused(*models[i], path)) two.push_back(i);
  }
  int64_t nmax = 0;
  for (int32_t j = 0; j < nN; ++j) {
    if (N[j] < 0) { set_error("N must be >= 0"); return CVD_E_INVALID; }
    nmax = std::max(nmax, N[j]);
  }
  if (!two.empty() && !d_work) {
    set_error("cvd_mc_run_grid: these models and path need the stream workspace (cvd_mc_grid_workspace_bytes)");
    return CVD_E_INVALID;
  }
  const int64_t slot = cvd_mc_workspace_bytes(enc1, nmax, batch);   // bytes per grid point's batch
  const int32_t k = (int32_t)two.size();
  std::vector<const cvd_model*> ms(k);
  std::vector<const uint32_t*> rs(k);
  std::vector<int64_t> ns(k), nh(k);
  std::vector<int64_t*> cs(k);
  // Pd_plotter.py:196-233: N outer, p inner, num_iter trials at every point; the point
  // (N[j], p[i]) accumulates into d_counts[(j * np + i) * 2 .. + 1].  The p row of one N
  // runs batch by batch: every point's streams generated into its own workspace slot,
  // then ONE cvd_detect_multi over the row (the models sharing the specialised kernel
  // variant in one launch, so a row of small batches pays one last-round tail)
  for (int32_t j = 0; j < nN; ++j) {
    for (int32_t i = 0; i < np; ++i)
      if (mc_run_fused(*models[i], path)) {
        rc = cvd_mc_run(models[i], enc1, enc2, p[i], N[j], seed, trial_begin, trial_end, batch, nullptr,
                        d_counts + 2 * ((int64_t)j * np + i), path, stream);
        if (rc) return rc;
      }
    if (k == 0) continue;
    for (int64_t b = trial_begin; b < trial_end; b += batch) {
      const int64_t T = std::min(batch, trial_end - b);
      for (int32_t x = 0; x < k; ++x) {
        const int32_t i = two[x];
        uint32_t* r = reinterpret_cast<uint32_t*>(static_cast<char*>(d_work) + (size_t)x * (size_t)slot);
        const uint32_t tag = grid_tag(N[j], p[i]);
        const uint64_t thr = noise_threshold(p[i]);
        if ((rc = launch_generate(e1, (uint32_t)seed, (uint32_t)(seed >> 32), tag, thr, N[j], 1, 2 * b, 2, r, 2 * T, 0,
                                  T, stream)))
          return rc;
        if ((rc = launch_generate(e2, (uint32_t)seed, (uint32_t)(seed >> 32), tag, thr, N[j], 1, 2 * b + 1, 2, r,
                                  2 * T, T, T, stream)))
          return rc;
        ms[x] = models[i]; rs[x] = r; ns[x] = 2 * T; nh[x] = T;
        cs[x] = d_counts + 2 * ((int64_t)j * np + i);
      }
      rc = cvd_detect_multi(ms.data(), k, rs.data(), N[j], ns.data(), nh.data(), nullptr, cs.data(),
                            path, stream);
      if (rc) return rc;
    }
  }
  return CVD_OK;
}
