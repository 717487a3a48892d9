// Bit-sliced metric vectors of the m = 6, k = 1, n = 2 butterfly decoder: the layout, the
// Eq. 4-5 step in that layout, the T_ref count and the row-table key, shared by the host
// table build (cvd_host.cpp), the host test driver (tests/bs_host_check.cpp) and the
// code-specialised detector k1s (cvd_device.h, compiled at run time by cvd_rtc.cpp).
// Self-contained: no standard-library includes.
//
// Layout.  The 64 relative metrics D(s) <= 12 are four bit-planes of two
// 32-bit words (one bit per state: word r, bit p), 8 registers instead of 32 registers of
// 16-bit pairs.  The 6-bit state index s has its label bits b = 0..5 at six LOCATIONS:
// 0..4 = the bit position's bits, 5 = the word.  A step maps s -> (2s + u) mod 64
// (viterbi_markov.py:82-106): label b of the new state is label b - 1 of its predecessors,
// which differ only in label 5.  So the layout moves with the step instead of the data:
// at phase f (= t mod 6 for D_t) label b sits at location sigma(f, b) = kSig0[(b - f) mod 6],
// the new label 0 takes the location label 5 left, and the step runs in place.  The two
// predecessors of the state at location address A are at A and A ^ (1 << sigma(f, 5));
// with out(j + 32, u) = out(j, u) ^ 3 and out(j, 1) = out(j, 0) ^ 3 (the standard
// butterfly, build_bfly) the own branch costs e(A) = popcount(out(j(A), 0) ^ y) and the
// partner branch 2 - e(A), j(A) = labels 0..4 at A:
//     D'(A) = min(D(A) + e(A), D(A ^ bit) + 2 - e(A)) - mu.
// mu, the step minimum, is 0 or 1 and is known BEFORE the ACS: a normalised vector has a
// zero state, whose better branch costs min(e, 2 - e) <= 1, so mu = 0 iff some zero state
// has e in {0, 2}.  The adds then carry e - mu in 4-bit two's complement and no
// normalisation pass is needed (profiles/r04z: 353 vs ~570 cycles per wave-step).
//
// Row-table key.  The tables must find a row from any of the six layouts.  The Bloom
// filter has to stay L2-resident, so it holds ONE entry per row, hashed from the CANONICAL
// (phase-0) image of the digest plane z = bit0(D) ^ bit1(D): 64 bits that separate the
// learned rows almost as well as the whole vector (profiles/r05_key_study.py: 315,916
// distinct z over 315,953 rows at p = 0.05, 993,055 / 993,088 at p = 0.2).  The kernel
// brings z from phase f to phase 0 with a short network of byte permutes (v_perm_b32) and
// bit swaps (bs_canon: 0 / 14 / 16 / 16 / 16 / 14 VALU for f = 0..5, the cheapest such
// networks for this kSig0, profiles/r05_canon_search.py).  The exact compare, on filter
// positives only, reads the directory slot's image of the lane's own phase: a slot holds
// all six images (192 B) and the row's record (64 B).
#pragma once

#ifndef CVD_HD
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define CVD_HD __host__ __device__ __forceinline__
#else
#define CVD_HD inline
#endif
#endif

#include "cvd_keys.h"

namespace cvd {

typedef unsigned int bs_u32;
typedef unsigned long long bs_u64;

// location of label c at phase 0 (the cycle label b visits: kSig0[b], kSig0[b - 1], ...)
constexpr CVD_HD int bs_sig0(int c) { return c == 0 ? 0 : c == 1 ? 1 : c == 2 ? 3 : c == 3 ? 4 : c == 4 ? 2 : 5; }
constexpr CVD_HD int bs_sigma(int ph, int b) { return bs_sig0(((b - ph) % 6 + 6) % 6); }
// location address (word << 5 | bit) of state s at phase ph
constexpr CVD_HD int bs_addr(int s, int ph) {
  int a = 0;
  for (int b = 0; b < 6; ++b) a |= ((s >> b) & 1) << bs_sigma(ph, b);
  return a;
}
// butterfly index j (labels 0..4) of the state at location address A, phase ph
constexpr CVD_HD int bs_j(int A, int ph) {
  int j = 0;
  for (int b = 0; b < 5; ++b) j |= ((A >> bs_sigma(ph, b)) & 1) << b;
  return j;
}

// Bit planes of out(j(A), 0) over word r at phase ph: bit `bit` of the 2-bit output word,
// XM = out(j, 0) in bits 2j..2j+1 (cvd_model::bfly_x)
constexpr CVD_HD bs_u32 bs_out_plane(bs_u64 xm, int ph, int r, int bit) {
  bs_u32 w = 0u;
  for (int p = 0; p < 32; ++p) w |= (bs_u32)((xm >> (2 * bs_j(r * 32 + p, ph) + bit)) & 1u) << p;
  return w;
}

// ───────────────────── 32-bit primitives (host emulation) ─────────────────────
// v_bitop3_b32 with truth table TT over (a, b, c) = (0xF0, 0xCC, 0xAA)
template <unsigned TT>
CVD_HD bs_u32 bs_bop3(bs_u32 a, bs_u32 b, bs_u32 c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
#else
  bs_u32 r = 0u;
  for (int i = 0; i < 8; ++i)
    if ((TT >> i) & 1u) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
  return r;
#endif
}
// truth tables used below
constexpr unsigned kTtXor3 = 0x96;     // a ^ b ^ c
constexpr unsigned kTtMaj = 0xE8;      // maj(a, b, c)
constexpr unsigned kTtMajNa = 0x8E;    // maj(~a, b, c): borrow of a - b with borrow-in c
constexpr unsigned kTtAndX = 0x60;     // a & (b ^ c)
constexpr unsigned kTtNorX = 0x09;     // ~(a | (b ^ c))
constexpr unsigned kTtXorOr = 0xBE;    // (a ^ b) | c
constexpr unsigned kTtNor3 = 0x01;     // ~(a | b | c)
constexpr unsigned kTtOr3 = 0xFE;      // a | b | c
constexpr unsigned kTtAndXor = 0x28;   // (a ^ b) & c   (not used by the kernel; tests)
constexpr unsigned kTtSel = 0xCA;      // a ? b : c, bitwise (v_bfi_b32)
constexpr unsigned kTtAndNotOr = 0xBA; // (a & ~b) | c

// v_perm_b32(hi, lo, sel): byte i of the result = byte sel_i of the 8-byte hi:lo (sel 12 = 0)
CVD_HD bs_u32 bs_perm(bs_u32 hi, bs_u32 lo, bs_u32 sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const bs_u64 v = ((bs_u64)hi << 32) | lo;
  bs_u32 out = 0u;
  for (int i = 0; i < 4; ++i) {
    const bs_u32 s = (sel >> (8 * i)) & 0xFFu;
    const bs_u32 b = s < 8u ? (bs_u32)(v >> (8 * s)) & 0xFFu : (s == 12u ? 0u : 0xFFu);
    out |= b << (8 * i);
  }
  return out;
#endif
}
// Operand forms for gfx950's VALU issue (profiles/r05an/vib2-3.json, 4 waves per SIMD):
// v_bitop3 / and / or / xor / add / lshrrev with VGPR, inline or literal operands issue at
// ~2.5-2.8 cycles per wave64 instruction, the same with an SGPR (or SGPR-pair / VCC) source
// at ~4.2, and v_lshlrev, v_or3, v_bfi, v_perm, v_cndmask at ~4.2 whatever the operands.  So
// (CVD_BS_VFAST, default on) a bitop3 mask constant is moved into a VGPR once per use site
// group (VOP3 takes no literal here; the compiler's own choice is an SGPR), x << 1 is an add,
// and the step's mu mask is a VGPR value (the compiler's form: v_cndmask on VCC).
// (bits, for A/Bs: 1 the masks, 2 the add, 4 the mu mask, 8 the zero test's OR as a bitop3)
#ifndef CVD_BS_VFAST
#define CVD_BS_VFAST 15
#endif
// CVD_BS_KLDS (timing A/B, default 0): the six flip / canonicalisation masks come from a
// block-shared table (filled with the kernel's other LDS tables) instead of a v_mov per use
// group: an LDS read the compiler may keep in a VGPR across the step loop
#ifndef CVD_BS_KLDS
#define CVD_BS_KLDS 0
#endif
constexpr int bs_kmask_index(bs_u32 C) {
  return C == 0xAAAAAAAAu ? 0 : C == 0xCCCCCCCCu ? 1 : C == 0xF0F0F0F0u ? 2
       : C == 0x55555555u ? 3 : C == 0x33333333u ? 4 : C == 0x0F0F0F0Fu ? 5 : -1;
}
constexpr bs_u32 kBsKmasks[6] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0x55555555u, 0x33333333u, 0x0F0F0F0Fu};
#if defined(__HIPCC__) || defined(__HIPCC_RTC__) || defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ bs_u32* bs_kmask_lds() {
  __shared__ bs_u32 s_km[8];
  return s_km;
}
#endif
template <bs_u32 C>
CVD_HD bs_u32 bs_vconst() {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (CVD_BS_KLDS != 0 && bs_kmask_index(C) >= 0) {
    return bs_kmask_lds()[bs_kmask_index(C)];
  } else if constexpr ((CVD_BS_VFAST & 1) != 0) {
    bs_u32 c;
    asm volatile("v_mov_b32 %0, %1" : "=v"(c) : "i"(C));
    return c;
  }
#endif
  return C;
}
CVD_HD bs_u32 bs_vreg(bs_u32 x) {   // an opaque VGPR copy (no SGPR / VCC-select forms of its uses)
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr ((CVD_BS_VFAST & 4) != 0) asm volatile("" : "+v"(x));
#endif
  return x;
}
template <int S>
CVD_HD bs_u32 bs_shl(bs_u32 x) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr ((CVD_BS_VFAST & 2) != 0 && S == 1) {
    bs_u32 r;
    asm("v_add_u32_e32 %0, %1, %1" : "=v"(r) : "v"(x));
    return r;
  }
#endif
  return x << S;
}
CVD_HD bs_u32 bs_rot16(bs_u32 x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(x, x, 16u);
#else
  return (x >> 16) | (x << 16);
#endif
}

// positions p <-> p ^ (1 << K) within a word (the partner flip of a location 0..4)
// (K < 3: the lower position of each pair, m = bs_flip_mask<K>, as an operand so that a caller
// flipping several planes moves it into a VGPR once)
template <int K>
constexpr bs_u32 bs_flip_mask() { return K == 0 ? 0x55555555u : K == 1 ? 0x33333333u : 0x0F0F0F0Fu; }
template <int K>
CVD_HD bs_u32 bs_flip(bs_u32 x, bs_u32 m = bs_flip_mask<K < 3 ? K : 0>()) {
  if constexpr (K == 4) {
    return bs_rot16(x);
  } else if constexpr (K == 3) {
    return bs_perm(x, x, 0x02030001u);   // bytes 0 <-> 1, 2 <-> 3
  } else {
    constexpr int S = 1 << K;
    return bs_bop3<kTtSel>(m, x >> S, bs_shl<S>(x));
  }
}

// ─────────────── canonicalisation of the digest plane (phase f -> 0) ───────────────
// Address-bit moves on the 64-bit plane (lo = word 0, hi = word 1):
//   swapR<i>: swap location i (< 3) with location 5 (the word): two shifts, two selects;
//   swapW<i, j>: swap two bit-position locations inside both words (delta swap);
//   bperm<q3, q4, q5>: locations 3, 4, 5 (the byte address) go to q3, q4, q5: one v_perm
//   per word.
template <int I>
CVD_HD void bs_swapR(bs_u32& lo, bs_u32& hi) {
  constexpr int D = 1 << I;
  constexpr bs_u32 m1c = I == 0 ? 0xAAAAAAAAu : I == 1 ? 0xCCCCCCCCu : 0xF0F0F0F0u;   // bit I of the position set
  const bs_u32 m1 = bs_vconst<m1c>();
  const bs_u32 l2 = bs_bop3<kTtSel>(m1, bs_shl<D>(hi), lo);
  const bs_u32 h2 = bs_bop3<kTtSel>(m1, hi, lo >> D);
  lo = l2;
  hi = h2;
}
template <int I, int J>
CVD_HD bs_u32 bs_swapW1(bs_u32 x) {
  constexpr int D = (1 << J) - (1 << I);
  // the lower position of each pair: bit I set, bit J clear
  constexpr bs_u32 mA = (I == 1 && J == 2) ? 0x0C0C0C0Cu : 0u;
  static_assert(I == 1 && J == 2, "only the swap the networks use");
  const bs_u32 t = bs_bop3<kTtAndXor>(x, x >> D, mA);
  return bs_bop3<kTtXor3>(x, t, t << D);
}
template <int Q3, int Q4, int Q5>
struct BsBytePerm {
  // output byte B' (B' bits = locations 3, 4, 5) takes input byte B with bit (Qk - 3) of B'
  // = bit (k - 3) of B
  static constexpr int src(int Bp) {
    return (((Bp >> (Q3 - 3)) & 1) << 0) | (((Bp >> (Q4 - 3)) & 1) << 1) | (((Bp >> (Q5 - 3)) & 1) << 2);
  }
  static constexpr bs_u32 sel(int w) {
    return (bs_u32)src(4 * w) | ((bs_u32)src(4 * w + 1) << 8) | ((bs_u32)src(4 * w + 2) << 16) |
           ((bs_u32)src(4 * w + 3) << 24);
  }
};
template <int Q3, int Q4, int Q5>
CVD_HD void bs_bperm(bs_u32& lo, bs_u32& hi) {
  const bs_u32 l2 = bs_perm(hi, lo, BsBytePerm<Q3, Q4, Q5>::sel(0));
  const bs_u32 h2 = bs_perm(hi, lo, BsBytePerm<Q3, Q4, Q5>::sel(1));
  lo = l2;
  hi = h2;
}
template <int I, int J>
CVD_HD void bs_swapW(bs_u32& lo, bs_u32& hi) {
  lo = bs_swapW1<I, J>(lo);
  hi = bs_swapW1<I, J>(hi);
}

// z at phase PH -> z at phase 0 (the networks of profiles/r05_canon_search.py for kSig0)
template <int PH>
CVD_HD void bs_canon(bs_u32& lo, bs_u32& hi) {
  if constexpr (PH == 1) {
    bs_swapR<0>(lo, hi); bs_swapR<1>(lo, hi); bs_bperm<4, 5, 3>(lo, hi); bs_swapR<2>(lo, hi);
  } else if constexpr (PH == 2) {
    bs_swapR<1>(lo, hi); bs_bperm<5, 4, 3>(lo, hi); bs_swapR<2>(lo, hi); bs_swapR<0>(lo, hi); bs_bperm<4, 5, 3>(lo, hi);
  } else if constexpr (PH == 3) {
    bs_bperm<3, 5, 4>(lo, hi); bs_swapR<0>(lo, hi); bs_bperm<5, 3, 4>(lo, hi); bs_swapW<1, 2>(lo, hi);
  } else if constexpr (PH == 4) {
    bs_bperm<5, 3, 4>(lo, hi); bs_swapR<0>(lo, hi); bs_swapR<2>(lo, hi); bs_bperm<5, 4, 3>(lo, hi); bs_swapR<1>(lo, hi);
  } else if constexpr (PH == 5) {
    bs_swapR<2>(lo, hi); bs_bperm<5, 3, 4>(lo, hi); bs_swapR<1>(lo, hi); bs_swapR<0>(lo, hi);
  }
}

// ─────────────────────── host: images, digest, key hash ───────────────────────
// planes of D (64 metric bytes, canonical state order) at phase ph: out[4 r + i] = plane i
// of word r
// (host: the model's table build; bs_addr of every (phase, state) once)
struct BsAddrTab {
  unsigned char a[6][64];
};
inline BsAddrTab bs_addr_tab() {
  BsAddrTab t;
  for (int ph = 0; ph < 6; ++ph)
    for (int s = 0; s < 64; ++s) t.a[ph][s] = (unsigned char)bs_addr(s, ph);
  return t;
}
inline void bs_image(const unsigned char* D, int ph, bs_u32 out[8]) {
  static const BsAddrTab tab = bs_addr_tab();
  for (int i = 0; i < 8; ++i) out[i] = 0u;
  for (int s = 0; s < 64; ++s) {
    const int A = tab.a[ph][s];
    bs_u32* o = out + 4 * (A >> 5);
    const bs_u32 d = D[s];
    for (int i = 0; i < 4; ++i) o[i] |= ((d >> i) & 1u) << (A & 31);
  }
}
// the phase-0 digest plane z = bit0(D) ^ bit1(D)
inline void bs_digest(const unsigned char* D, bs_u32 z[2]) {
  z[0] = z[1] = 0u;
  for (int s = 0; s < 64; ++s) {
    const int A = bs_addr(s, 0);
    if (((D[s] ^ (D[s] >> 1)) & 1) != 0) z[A >> 5] |= 1u << (A & 31);
  }
}

// ───────────────────── the step (host and device) ─────────────────────
// Per received word y and phase, the branch-metric planes of word r: e0 = bit 0 of e
// (e odd), e1 = (e == 2), ez = (e == 0).  The kernel keeps them in an LDS table per (phase,
// y); the host computes them here.
struct BsE {
  bs_u32 e0[2], e1[2], ez[2];
};
CVD_HD BsE bs_eplanes(bs_u64 xm, int ph, bs_u32 y) {
  BsE E{};
  for (int r = 0; r < 2; ++r) {
    const bs_u32 d0 = bs_out_plane(xm, ph, r, 0) ^ (0u - (y & 1u));
    const bs_u32 d1 = bs_out_plane(xm, ph, r, 1) ^ (0u - ((y >> 1) & 1u));
    E.e0[r] = d0 ^ d1;
    E.e1[r] = d0 & d1;
    E.ez[r] = ~(d0 | d1);
  }
  return E;
}

// 4-plane d + addend (b0 ^ M, b1, b23, b23) with b0 ^ M folded into the first two bitop3s
CVD_HD void bs_add(const bs_u32 (&d)[4], bs_u32 e0, bs_u32 M, bs_u32 b1, bs_u32 b23, bs_u32 (&s)[4]) {
  s[0] = bs_bop3<kTtXor3>(d[0], e0, M);
  const bs_u32 c0 = bs_bop3<kTtAndX>(d[0], e0, M);
  s[1] = bs_bop3<kTtXor3>(d[1], b1, c0);
  const bs_u32 c1 = bs_bop3<kTtMaj>(d[1], b1, c0);
  s[2] = bs_bop3<kTtXor3>(d[2], b23, c1);
  const bs_u32 c2 = bs_bop3<kTtMaj>(d[2], b23, c1);
  s[3] = bs_bop3<kTtXor3>(d[3], b23, c2);
}
// o = min(a, b) per 4-bit lane: a < b by a borrow chain (LSB first), then a select per plane
CVD_HD void bs_min(const bs_u32 (&a)[4], const bs_u32 (&b)[4], bs_u32 (&o)[4]) {
  bs_u32 lt = bs_bop3<kTtSel>(a[0], 0u, b[0]);   // ~a0 & b0
  lt = bs_bop3<kTtMajNa>(a[1], b[1], lt);
  lt = bs_bop3<kTtMajNa>(a[2], b[2], lt);
  lt = bs_bop3<kTtMajNa>(a[3], b[3], lt);
  for (int i = 0; i < 4; ++i) o[i] = bs_bop3<kTtSel>(lt, a[i], b[i]);
}

// partner planes of word r (the flip of the location holding label 5 at phase PH)
template <int PH>
CVD_HD void bs_partner(const bs_u32 (&R)[2][4], bs_u32 (&P)[2][4]) {
  constexpr int L5 = bs_sigma(PH, 5);
  const bs_u32 m = L5 < 3 ? bs_vconst<bs_flip_mask<L5 < 3 ? L5 : 0>()>() : 0u;
  for (int i = 0; i < 4; ++i) {
    if constexpr (L5 == 5) {
      P[0][i] = R[1][i];
      P[1][i] = R[0][i];
    } else {
      P[0][i] = bs_flip<L5>(R[0][i], m);
      P[1][i] = bs_flip<L5>(R[1][i], m);
    }
  }
}

// Result of one step beyond the new planes: mu (0 / 1), the T_ref count c of D_t(y)
// among the 2^n words, and the new vector's canonical digest hash (ph, pl).
struct BsStepOut {
  bs_u32 mu, c, hph, hpl;
};

// One Eq. 4-5 step from D_{t-1} (planes R, layout PH) under word y to D_t (planes N, layout
// PH + 1).  uni: every out(j, 0) has even parity (bfly_uni), a code constant.
//   T_ref count (the c of Pd_plotter.py:89-99 for the observed word): D_t(y ^ 3) is D_t(y)
//   with the new label 0 flipped, equal iff every butterfly whose e is even has equal
//   predecessors; D_t(y ^ 1) and D_t(y ^ 2) can equal D_t(y) only if D_{t-1}'s halves are
//   equal and the code is uni: c = 1 + [sym == 0] + 2 [uni and halves equal].
// mid(x): called between the two words' ACS with a value that depends on the first word's
// result (the kernel issues its filter-positive loads there)
struct BsNoMid {
  CVD_HD void operator()(bs_u32) const {}
};
template <int PH, bool kUni, class Mid = BsNoMid>
CVD_HD void bs_step_core(const bs_u32 (&R)[2][4], const bs_u32 (&e0)[2], const bs_u32 (&e1)[2],
                         const bs_u32 (&ez)[2], bs_u32 (&N)[2][4], bs_u32& mu, bs_u32& c, Mid mid = Mid()) {
  constexpr int L5 = bs_sigma(PH, 5);
  // mu first: a zero state with e even
  bs_u32 z[2];
  for (int r = 0; r < 2; ++r) {
    const bs_u32 t = (CVD_BS_VFAST & 8) ? bs_bop3<kTtOr3>(R[r][0], R[r][1], R[r][2]) : R[r][0] | R[r][1] | R[r][2];
    z[r] = bs_bop3<kTtNor3>(t, R[r][3], e0[r]);
  }
  const bool zero_hit = (z[0] | z[1]) != 0u;
  mu = zero_hit ? 0u : 1u;
  const bs_u32 M = bs_vreg(zero_hit ? 0u : ~0u);
  bs_u32 P[2][4];
  bs_partner<PH>(R, P);
  bs_u32 dh[2] = {0u, 0u};
  for (int r = 0; r < 2; ++r) {
    // own branch e - mu, partner branch 2 - e - mu (4-bit two's complement):
    //   mu = 0: own (e0, e1, 0, 0), partner (e0, ez, 0, 0)
    //   mu = 1: own (~e0, ez, ez, ez), partner (~e0, e1, e1, e1)
    const bs_u32 a1 = bs_bop3<kTtSel>(M, ez[r], e1[r]);
    const bs_u32 p1 = bs_bop3<kTtSel>(M, e1[r], ez[r]);
    const bs_u32 a23 = M & ez[r], p23 = M & e1[r];
    bs_u32 a[4], b[4];
    bs_add(R[r], e0[r], M, a1, a23, a);
    bs_add(P[r], e0[r], M, p1, p23, b);
    bs_min(a, b, N[r]);
    // halves differences of D_{t-1} (a state and its partner differ)
    if (L5 != 5 || r == 0) {
      bs_u32 x = R[r][3] ^ P[r][3];
      x = bs_bop3<kTtXorOr>(R[r][2], P[r][2], x);
      x = bs_bop3<kTtXorOr>(R[r][1], P[r][1], x);
      dh[r] = bs_bop3<kTtXorOr>(R[r][0], P[r][0], x);
    } else {
      dh[1] = dh[0];
    }
    if (r == 0) mid(N[0][3]);
  }
  const bs_u32 sym = bs_bop3<kTtAndNotOr>(dh[0], e0[0], dh[1] & ~e0[1]);
  c = 1u + (sym == 0u ? 1u : 0u) + ((kUni && (dh[0] | dh[1]) == 0u) ? 2u : 0u);
}

// The same step with mu's branch-metric planes from a table (CVD_BS_ETAB2): for each (phase,
// y) the planes the adds take once mu is known -- the own and partner addends' bit 0 with mu
// folded in (e0 ^ M), bit 1 and bits 2-3 -- are precomputed for mu = 0 and mu = 1, so the step
// reads them (the kernel: from LDS at a mu-dependent offset) instead of selecting them with M:
// 8 VALU fewer per step, and no M.
struct BsMu {
  bs_u32 e0m[2], a1[2], p1[2], a23[2], p23[2];
};
CVD_HD BsMu bs_mu_planes(const BsE& E, bool mu1) {
  BsMu T{};
  const bs_u32 M = mu1 ? ~0u : 0u;
  for (int r = 0; r < 2; ++r) {
    T.e0m[r] = E.e0[r] ^ M;
    T.a1[r] = mu1 ? E.ez[r] : E.e1[r];
    T.p1[r] = mu1 ? E.e1[r] : E.ez[r];
    T.a23[r] = M & E.ez[r];
    T.p23[r] = M & E.e1[r];
  }
  return T;
}
// 4-plane d + addend (b0, b1, b23, b23), b0 with mu already folded in
CVD_HD void bs_add2(const bs_u32 (&d)[4], bs_u32 b0, bs_u32 b1, bs_u32 b23, bs_u32 (&s)[4]) {
  s[0] = d[0] ^ b0;
  const bs_u32 c0 = d[0] & b0;
  s[1] = bs_bop3<kTtXor3>(d[1], b1, c0);
  const bs_u32 c1 = bs_bop3<kTtMaj>(d[1], b1, c0);
  s[2] = bs_bop3<kTtXor3>(d[2], b23, c1);
  const bs_u32 c2 = bs_bop3<kTtMaj>(d[2], b23, c1);
  s[3] = bs_bop3<kTtXor3>(d[3], b23, c2);
}
// bs_step_core with e0 for the zero test and load(zero_hit) -> BsMu for the adds
template <int PH, bool kUni, class Load, class Mid = BsNoMid>
CVD_HD void bs_step_core_tab(const bs_u32 (&R)[2][4], const bs_u32 (&e0)[2], Load load, bs_u32 (&N)[2][4],
                             bs_u32& mu, bs_u32& c, Mid mid = Mid()) {
  constexpr int L5 = bs_sigma(PH, 5);
  bs_u32 z[2];
  for (int r = 0; r < 2; ++r) {
    const bs_u32 t = (CVD_BS_VFAST & 8) ? bs_bop3<kTtOr3>(R[r][0], R[r][1], R[r][2]) : R[r][0] | R[r][1] | R[r][2];
    z[r] = bs_bop3<kTtNor3>(t, R[r][3], e0[r]);
  }
  const bool zero_hit = (z[0] | z[1]) != 0u;
  mu = zero_hit ? 0u : 1u;
  bs_u32 P[2][4];
  bs_partner<PH>(R, P);
  const BsMu T = load(zero_hit);
  bs_u32 dh[2] = {0u, 0u};
  for (int r = 0; r < 2; ++r) {
    bs_u32 a[4], b[4];
    bs_add2(R[r], T.e0m[r], T.a1[r], T.a23[r], a);
    bs_add2(P[r], T.e0m[r], T.p1[r], T.p23[r], b);
    bs_min(a, b, N[r]);
    if (L5 != 5 || r == 0) {
      bs_u32 x = R[r][3] ^ P[r][3];
      x = bs_bop3<kTtXorOr>(R[r][2], P[r][2], x);
      x = bs_bop3<kTtXorOr>(R[r][1], P[r][1], x);
      dh[r] = bs_bop3<kTtXorOr>(R[r][0], P[r][0], x);
    } else {
      dh[1] = dh[0];
    }
    if (r == 0) mid(N[0][3]);
  }
  const bs_u32 sym = bs_bop3<kTtAndNotOr>(dh[0], e0[0], dh[1] & ~e0[1]);
  c = 1u + (sym == 0u ? 1u : 0u) + ((kUni && (dh[0] | dh[1]) == 0u) ? 2u : 0u);
}

// the bit-sliced tables' key hash of the canonical digest (lo, hi): key_hash's two-word
// fold without its start constant (which only shifted the sum; LLVM added it as one more
// 64-bit VALU op) -- acc = lo K0 + hi K1, x = acc_lo ^ acc_hi, (ph, pl) = x K2
CVD_HD void bs_key_hash(bs_u32 lo, bs_u32 hi, bs_u32& ph, bs_u32& pl) {
  const bs_u64 acc = mul_wide(lo, 0x85EBCA77u) + mul_wide(hi, 0x85EBCA77u + 0x6A09E668u);
  const bs_u32 x = (bs_u32)acc ^ (bs_u32)(acc >> 32);
  const bs_u64 p = mul_wide(x, 0x85EBCA6Bu);
  ph = (bs_u32)(p >> 32);
  pl = (bs_u32)p;
}

// canonical digest hash of planes N at phase PH
template <int PH>
CVD_HD void bs_digest_hash(const bs_u32 (&N)[2][4], bs_u32& ph, bs_u32& pl) {
  bs_u32 lo = N[0][0] ^ N[0][1], hi = N[1][0] ^ N[1][1];
  bs_canon<PH>(lo, hi);
  bs_key_hash(lo, hi, ph, pl);
}

}  // namespace cvd
