// Device code of the explicit path shared by the compiled kernels
// (cvd_kernels.hip) and the code-specialised butterfly kernels hipRTC builds at
// run time (cvd_rtc.cpp embeds this file and cvd_keys.h as source text): the
// launch arguments, the received-word reader, the P̂1 row cursor and the k = 1,
// n = 2 butterfly detector.  Self-contained: no standard-library includes.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#else
// hipRTC keeps its fixed-width types in __hip_internal
typedef unsigned char uint8_t;
typedef int int32_t;
typedef unsigned int uint32_t;
typedef long long int64_t;
typedef unsigned long long uint64_t;
typedef __SIZE_TYPE__ size_t;
#endif
#include "cvd_keys.h"
#include "cvd_bitslice.h"

namespace cvd_dev {

using cvd::kEmptyKey;
using cvd::row_words_c;
using cvd::key_hash;

constexpr int kBlock = 256;
// LDS-resident Bloom filter (walking models, cvd_kernels.hip): the specialised kernel
// copies the filter into dynamic LDS at block start and tests it there; its blocks have
// CVD_K1B_BLOCK threads (the host launches them so)
#ifndef CVD_K1B_LDSF
#define CVD_K1B_LDSF 0
#endif
#ifndef CVD_K1B_BLOCK
#define CVD_K1B_BLOCK 256
#endif
constexpr int kK1bBlock = CVD_K1B_BLOCK;
__device__ __forceinline__ uint32_t* dyn_lds() {
  extern __shared__ uint32_t s_dyn[];
  return s_dyn;
}
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// Uniform read-only tables go through the constant address space so that
// uniform-index loads become scalar (s_load) loads into SGPRs instead of
// per-lane vector loads the compiler would otherwise have to wait on.
typedef const __attribute__((address_space(4))) uint32_t cu32;
__device__ __forceinline__ cu32* as_const(const uint32_t* p) { return (cu32*)p; }

__device__ __forceinline__ us2 as_us2(uint32_t x) { return __builtin_bit_cast(us2, x); }
// (a << 4) | b as one v_lshl_or_b32 (the compiler otherwise splits nibble packs
// into shifts + v_or3)
__device__ __forceinline__ uint32_t lshl4_or(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
__device__ __forceinline__ uint32_t as_u32(us2 x) { return __builtin_bit_cast(uint32_t, x); }

// Received-word layout in HBM (include/cvd.h): words are grouped in 16-byte
// chunks per sequence; word w of sequence q lives at
// r[((w >> 2) * pitch + q) * 4 + (w & 3)], so each lane moves 16 B per load
// and a wave reads / writes 1 KiB contiguously.
__device__ __forceinline__ size_t chunk_index(int64_t w4, int64_t pitch, int64_t q) {
  return ((size_t)w4 * (size_t)pitch + (size_t)q) * 4;
}
__device__ __forceinline__ uint32_t next_word(const uint32_t* r, int64_t pitch, int64_t q, int64_t w,
                                              uint4& cache) {
  if ((w & 3) == 0) cache = *reinterpret_cast<const uint4*>(r + chunk_index(w >> 2, pitch, q));
  const int e = (int)(w & 3);
  return e == 0 ? cache.x : e == 1 ? cache.y : e == 2 ? cache.z : cache.w;
}

// 2-bit field of x at bit s, extracted where it is used: a volatile asm is not
// hoisted, so the four steps of a group do not hold all their words live.
__device__ __forceinline__ uint32_t bits2(uint32_t x, uint32_t s) {
  uint32_t d;
  asm volatile("v_bfe_u32 %0, %1, %2, 2" : "=v"(d) : "v"(x), "v"(s));
  return d;
}

// Lane index in the wave (v_mbcnt; cheap to recompute instead of keeping live:
// the laundered mask keeps LLVM from merging two calls and holding the first
// result across the step loop).
__device__ __forceinline__ uint32_t lane_id() {
  uint32_t all = ~0u;
  asm volatile("" : "+s"(all));
  return __builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
}

// count_decisions with validity and hypothesis given as wave ballots.
__device__ __forceinline__ void count_decisions_masked(uint64_t vmask, uint64_t hmask, double lp, double lr,
                                                       int64_t* counts) {
  const uint64_t gt = __ballot(lp > lr), le = __ballot(lp <= lr);
  const uint64_t b1 = gt & vmask & hmask;     // Pd_plotter.py:215
  const uint64_t b2 = le & vmask & ~hmask;    // Pd_plotter.py:222
  if (lane_id() == 0) {
    if (b1) atomicAdd(reinterpret_cast<unsigned long long*>(counts), (unsigned long long)__popcll(b1));
    if (b2) atomicAdd(reinterpret_cast<unsigned long long*>(counts + 1), (unsigned long long)__popcll(b2));
  }
}

// Wave-level success counting: one 64-bit atomic per wave and hypothesis.
__device__ __forceinline__ void count_decisions(bool valid, bool is_h1, double lp, double lr,
                                                int64_t* counts) {
  const bool s1 = valid && is_h1 && (lp > lr);     // Pd_plotter.py:215
  const bool s2 = valid && !is_h1 && (lp <= lr);   // Pd_plotter.py:222
  const unsigned long long b1 = __ballot(s1), b2 = __ballot(s2);
  if ((threadIdx.x & 63) == 0) {
    if (b1) atomicAdd(reinterpret_cast<unsigned long long*>(counts), (unsigned long long)__popcll(b1));
    if (b2) atomicAdd(reinterpret_cast<unsigned long long*>(counts + 1), (unsigned long long)__popcll(b2));
  }
}

// ───────────────────────── early decision (counts only) ──────────────────────
//
// A trial's decision compares only the FINAL sums (Pd_plotter.py:215, :222:
// success iff logP1 > logTref for H1, logP1 <= logTref for H2).  Every log P̂1
// increment is <= 0 and at least lp_min; every log T_ref increment is <= 0 and
// at least lt_min = log(1/2^n) (the observed word always counts, c >= 1).  With
// rem steps left, in IEEE double with round-to-nearest (u = 2^-53):
//   lp_final <= lp                              (adding a <= 0 never rounds up)
//   lr_final >= (lr + rem * lt_min) (1 + u)^rem  (each rounding enlarges a negative
//                                                 partial sum by at most a factor 1 + u)
// and symmetrically lr_final <= lr, lp_final >= (lp + rem * lp_min)(1 + u)^rem.
// The bounds below use the factor 1 + (4 rem + 32) u, which also covers the
// rounding of the bound's own three operations.  So
//   lp <= (lr + rem lt_min) f   =>  lp_final <= lr_final   (returns 1)
//   (lp + rem lp_min) f > lr    =>  lp_final >  lr_final   (returns 2)
// and the decision is certain from there on: the lane's count is exactly what the
// full recursion gives.  Used only when per-trial sums are not requested; a wave
// stops when every lane has decided.
__device__ __forceinline__ int early_decide(double lp, double lr, int64_t rem, double lt_min, double lp_min) {
  const double f = 1.0 + (double)(4 * rem + 32) * 0x1p-53;
  if (lp <= (lr + (double)rem * lt_min) * f) return 1;
  if ((lp + (double)rem * lp_min) * f > lr) return 2;
  return 0;
}
// (lp, lr) stand-ins with the decided comparison for count_decisions
__device__ __forceinline__ void early_final(int dec, double& lp, double& lr) {
  if (dec == 1) { lp = -1.0; lr = 0.0; }
  if (dec == 2) { lp = 1.0; lr = 0.0; }
}
constexpr int kEarlyEvery = 128;   // steps between checks (the k = 1 butterfly renormalisation period)

// ────────────────────────── explicit metric path ────────────────────────────

struct ExpArgs {
  const uint32_t* filt;     // [fmask + 1][2] Bloom filter blocks over the row keys (filter_pattern)
  const uint32_t* hkey;     // [hcap][NW] nibble-packed metric vectors, word 0 = kEmptyKey if empty
  const uint32_t* hrow;     // [hcap][row_words(n)]: per r, {log P̂1[r] (f64), successor row[r] (i32, -1 = not a row), pad}
  const uint32_t* drow;     // [rows][row_words(n)]: the same records dense by row id (table mode)
  const uint32_t* dkey;     // [rows][NW]: the key of every learned row by row id (k1b_walk: a lane leaving
                            // a table walk rebuilds its metric vector from it)
  const uint32_t* t2;       // [rows][16][8] two-step walk records (k1b_walk; null: one step per load)
  const double* ltref;      // [R + 1]
  const uint32_t* bmp;      // branch-metric table (kernel-specific layout)
  uint32_t repmap, swmap;   // k = 1 orbit kernel: rep index / swap flag per received word
  uint32_t bfly_uni;        // k = 1 butterfly kernel: every out(j, 0), j < 2^(m-1), in one class
  uint32_t bfly_even[4];    // k = 1 butterfly kernel: nibble masks of the butterflies with out(j, 0) in {00, 11}
  uint32_t hmask, fmask, fmask4;   // fmask: filter blocks - 1, fmask4 = fmask << 3 (block byte offsets)
  uint32_t ksh, rsh;        // directory slot strides as byte shifts: key (hkey), record (hrow)
  int32_t max_probe;
  int32_t slot0;            // row of D_0 = 0
  double lp_unseen;
  int64_t N, nseq, n_h1;
  const uint32_t* r;
  double* sums;
  int64_t* counts;
  uint8_t* trace;
  int32_t early;            // early decision (counts only; sums == nullptr)
  int32_t walk;             // k1b_walk for H1 waves (specialised kernel; no trace, no early decision, N < 2^31)
  int32_t walk_wmin, walk_amin, walk_burst;   // k1b_walk schedule (see there)
  double lt_min, lp_min;    // smallest log T_ref / log P̂1 increments (early_decide)
  int32_t* err;             // error flags (nullable): bit 0 = k1b_walk left its loop by the guard
  const uint32_t* pf;       // k1s LDS pre-filter (CVD_K1S_PF): 2^kBsPfLog2Bits bits, copied into dynamic LDS
  uint32_t* wq;             // k1s persistent launch: work-queue counter (zeroed before the launch), else null
  // chunked detection (k1s, counts via ck_combine_kernel): unit u runs time chunk
  // u % ck_n of the 64 sequences of wave u / ck_n -- steps [j ck_len, (j + 1) ck_len), started
  // ck_warm steps early from D = 0 -- and writes its record to ck_out instead of sums / counts
  int32_t mix;              // k1s lockstep: units alternate H1 and H2 waves (walk mode always does)
  int32_t t2c;              // k1s walk with the LDS filter: t2 holds the compact 8-B two-step records
  int32_t nvtab;            // (t2c) values in the log P̂1 table, copied into dynamic LDS at vtab_off
  uint32_t vtab_off;
  const double* vtab;
  int32_t ck_n;             // chunks per sequence (0: off)
  int32_t ck_len, ck_warm;  // steps per chunk and warm-up steps (multiples of 192)
  uint32_t* ck_out;         // [ck_n][nseq][kCkRecWords]: D at the chunk start and end (phase 0), lp, lr
};
constexpr int kCkRecWords = 20;   // chunk record: D_start planes [0, 8), D_end planes [8, 16), lp, lr (f64)

// Received words of one sequence, one word of lookahead (the next step's r is
// known before the current step ends, so its P̂1 row entry can be prefetched).
template <int n>
struct StreamReader {
  static constexpr int SPW = 32 / n;
  static constexpr uint32_t MASK = (1u << n) - 1u;
  const uint32_t* r;
  int64_t pitch, q, N, nwords, wi;
  uint4 cache;
  uint32_t cur, nxt;
  int left;
  __device__ int steps_in(int64_t w) const { return (int)min((int64_t)SPW, N - w * SPW); }
  __device__ void init(const uint32_t* r_, int64_t pitch_, int64_t q_, int64_t N_) {
    r = r_; pitch = pitch_; q = q_; N = N_;
    nwords = (N + SPW - 1) / SPW;
    cur = nxt = 0u; left = 0; wi = 0;
    if (nwords > 0) { cur = next_word(r, pitch, q, 0, cache); left = steps_in(0); }
    wi = 1;
    if (wi < nwords) nxt = next_word(r, pitch, q, wi, cache);
  }
  __device__ uint32_t peek() const { return cur & MASK; }
  __device__ uint32_t peek_next() const { return left > 1 ? ((cur >> n) & MASK) : (nxt & MASK); }
  __device__ void advance() {
    if (left > 1) { cur >>= n; --left; return; }
    cur = nxt;
    left = wi < nwords ? steps_in(wi) : 0;
    ++wi;
    if (wi < nwords) nxt = next_word(r, pitch, q, wi, cache);
  }
};

// 32-bit byte offsets from a uniform base (global_load with an SGPR base: no
// 64-bit address arithmetic per lane)
template <typename T>
__device__ __forceinline__ T ld_off(const void* base, uint32_t byte_off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

// Bloom-filter bit-pattern pairs (cvd_keys.h filter_pattern / filter_pattern_hi)
// in LDS, 8 bytes each: one table per workgroup, filled at kernel start
// (fill_filter_patterns + __syncthreads).
__device__ __forceinline__ uint2* filter_patterns_lds() {
  __shared__ uint2 s_pat[cvd::kFilterPatterns];
  return s_pat;
}
__device__ __forceinline__ void fill_filter_patterns() {
  uint2* t = filter_patterns_lds();
  for (int i = threadIdx.x; i < cvd::kFilterPatterns; i += blockDim.x)
    t[i] = make_uint2(cvd::filter_pattern((unsigned)i), cvd::filter_pattern_hi((unsigned)i));
}

// Ablation knobs for timing studies only (profiles/ab_k1b.py --no-check; results
// differ): bit 0 drops the P̂1 row lookup, bit 1 the T_ref count, bit 2 the
// hashed lookup of states outside the learned rows (table mode only), bit 4 the
// table walk after a hashed hit (the lane hashes again), bit 5 the key and record
// reads of filter-positive lanes (hash and filter test only), bit 6 the filter read of the
// waves of H2 sequences (their lookups end negative).
#ifndef CVD_ABL
#define CVD_ABL 0
#endif
#ifndef CVD_K1B_CMP64
#define CVD_K1B_CMP64 0
#endif
#ifndef CVD_K1B_CMPX
#define CVD_K1B_CMPX 1
#endif
// log P̂1 of an unvisited row held in a VGPR pair across the step loop (the lockstep
// body's resolve selects it with v_cndmask; from its SGPRs each step first copied it
// into VGPRs, two v_mov per step): 211 -> 209 static VALU per step, still 126 VGPRs;
// p = 0.05 / 0.1 / 0.2 675.5 / 705.6 / 678.7 -> 674.1 / 703.8 / 676.3 ms per 655,360-trial
// launch, walk-mode p within 1 ms (profiles/r03v/ab_lpu.txt)
#ifndef CVD_K1B_LPU_VGPR
#define CVD_K1B_LPU_VGPR 1
#endif
#ifndef CVD_K1B_CMPX_WALK
#define CVD_K1B_CMPX_WALK CVD_K1B_CMPX
#endif

// Lookup of the P̂1 row of the current metric state.  A learned row's record
// holds the row of its successor for every received word, so a sequence that
// stays in learned states walks the dense row-indexed records with one small
// prefetched load per step and no hashing ("table mode").  After an unvisited
// state the successor is unknown and the next state is hashed: its Bloom-filter
// word is fetched one step ahead (L2-resident; a negative answer -- almost
// every non-row -- ends the lookup) together with its bit pattern (LDS), the
// key and the directory record of the home slot only on a positive answer
// (mid-step), and the exact key compare, with linear probing past an occupied
// home slot, happens when the step resolves.  slot: >= 0 known row id, -1 known
// unvisited row, -2 pending hash probe (home slot hs, filter word fw, pattern fb).
template <int NW, int R>
struct RowCursor {
  static constexpr uint32_t RSB = 4u * row_words_c(R);   // record bytes
  static_assert(RSB == 16u * R, "record = one 16-byte entry per received word");
  int32_t slot, pnx;
  uint32_t hs, fb, fw, fb1, fw1;   // filter block words and their patterns
  bool h2wave = false;             // (CVD_ABL & 64 timing studies: the wave holds H2 sequences only)
  bool cand;
  double plp;
  uint32_t pc;                     // T_ref count c of the entry (kC loads only: the walk mode of k1b_walk)
  uint32_t pkey[NW];
  // record entry r (log P̂1[r], successor row[r], T_ref count c: 16 bytes, one
  // 12-byte load, 16 with kC) of row s (dense records, table mode) or of directory
  // slot s (a hashed lookup's hit) for word rn; the asm keeps the address one
  // shift-add of the lane's word onto the record offset
  template <bool kC = false>
  __device__ void load_entry(const uint32_t* base, uint32_t off, uint32_t rn) {
    uint32_t o;
    asm("v_lshl_add_u32 %0, %1, 4, %2" : "=v"(o) : "v"(rn), "v"(off));
    if constexpr (kC) {
      // (plp last: a trailing 32-bit store here and the filter words' in prefetch's
      // hashed branch get sunk into one store through a pointer phi, which keeps pc
      // and fw1 in scratch)
      const uint4 v = ld_off<uint4>(base, o);
      pc = v.w;
      pnx = (int32_t)v.z;
      plp = __hiloint2double((int)v.y, (int)v.x);
    } else {
      const uint3 v = ld_off<uint3>(base, o);
      plp = __hiloint2double((int)v.y, (int)v.x);
      pnx = (int32_t)v.z;
    }
  }
  template <bool kC = false>
  __device__ void prefetch_row(const ExpArgs& a, int32_t s, uint32_t rn) { load_entry<kC>(a.drow, (uint32_t)s * RSB, rn); }
  __device__ void prefetch_dir(const ExpArgs& a, int32_t s, uint32_t rn) { load_entry(a.hrow, (uint32_t)s << a.rsh, rn); }
  __device__ void start(const ExpArgs& a, uint32_t r0) {
    // (CVD_ABL & 4: a pattern no filter word passes, so no lane ever becomes a candidate)
    slot = a.slot0; hs = 0u; fb = (CVD_ABL & 4) ? 1u : 0u; fw = 0u; fb1 = 0u; fw1 = 0u; cand = false;
    if (CVD_ABL & 1) return;
    prefetch_row(a, slot, r0);
  }
  // Ordering fences: nothing in mid() / resolve() depends on the ACS, so
  // without these LLVM hoists both to the top of the step, where the loads
  // issued one step (filter word, row) or half a step (key, row) earlier are
  // waited for at once.  Each fence makes the cursor state an output of an asm
  // that consumes an ACS result (the running zero-nibble test, which depends on
  // every butterfly computed so far), so the waits land after that much work.
  __device__ void fence(uint32_t dep) {
    asm volatile("" : "+v"(fw), "+v"(fw1), "+v"(slot), "+v"(pnx), "+v"(plp) : "v"(dep));
  }
  template <int N_>
  __device__ void fence_keys(uint32_t dep) {
#pragma unroll
    for (int w = 0; w < N_; ++w) asm volatile("" : "+v"(pkey[w]) : "v"(dep));
  }
  // key of directory slot s: 16-byte loads when the key is whole 16-byte pieces (a
  // slot's key is aligned to its power-of-two stride), else dword loads
  __device__ static void load_key(const ExpArgs& a, uint32_t s, uint32_t (&k)[NW]) {
    if constexpr (NW % 4 == 0) {
#pragma unroll
      for (int i = 0; i < NW / 4; ++i) {
        const uint4 v = ld_off<uint4>(a.hkey, (s << a.ksh) + 16u * i);
        k[4 * i] = v.x; k[4 * i + 1] = v.y; k[4 * i + 2] = v.z; k[4 * i + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int w = 0; w < NW; ++w) k[w] = ld_off<uint32_t>(a.hkey, (s << a.ksh) + 4u * w);
    }
  }
  __device__ void mid(const ExpArgs& a, uint32_t r) {
    if (CVD_ABL & 1) return;
    cand = slot == -2 && ((fb & ~fw) | (fb1 & ~fw1)) == 0u && !(CVD_ABL & 32);
    if (cand) {
      load_key(a, hs, pkey);
      prefetch_dir(a, (int32_t)hs, r);
    }
  }
  __device__ static bool same_key(const uint32_t (&x)[NW], const uint32_t (&y)[NW]) {
    uint32_t d = 0u;
#pragma unroll
    for (int w = 0; w < NW; ++w) d |= x[w] ^ y[w];
    // keep the xor/or reduction (2-cycle VALU); without the asm LLVM rewrites it
    // into per-word compares materialised through v_cndmask
    asm volatile("" : "+v"(d));
    return d == 0u;
  }
  // stored (canonical) key x == lazy key y - kmu8?  Default (CVD_K1B_CMPX=1): the
  // differences, below; 14 VALU instead of 20 for subtract, xor and or per word
  // (CVD_K1B_CMPX=0): p = 0.1 710.1 -> 703.6 ms, p = 0.05 680.7 -> 675.6, p = 0.2 686.7 ->
  // 680.5 per 655,360-trial launch, p <= 0.02 (walk mode) within +-1.7 ms
  // (profiles/r03o/ab_cmpx.jsonl, profiles/r03p/ab_cmpx_walk.jsonl).  CVD_K1B_CMP64=1:
  // y's words are x + kmu8 with no carry out of any nibble (nibbles <= 14 + 2), so as
  // 64-bit word pairs y = x + K exactly, K = kmu8 *
  // (2^32 + 1): one 64-bit add and one 64-bit compare per pair.  Fewer VALU in the
  // filter-positive block, but measured neutral (p = 0.1: 710.2 vs 709.3 ms per
  // 655,360-trial launch, profiles/r03b/ab_cmp64.jsonl), so it stays off.
  template <bool kX = CVD_K1B_CMPX>
  __device__ static bool same_key_lazy(const uint32_t (&x)[NW], const uint32_t (&y)[NW], uint32_t kmu8) {
#if CVD_K1B_CMP64
    if constexpr (NW % 2 == 0) {
      const uint64_t K = (uint64_t)kmu8 * 0x100000001ull;
      bool eq = true;
#pragma unroll
      for (int i = 0; i < NW / 2; ++i) {
        const uint64_t xi = ((uint64_t)x[2 * i + 1] << 32) | x[2 * i];
        const uint64_t yi = ((uint64_t)y[2 * i + 1] << 32) | y[2 * i];
        eq = eq && (xi + K == yi);
      }
      return eq;
    }
#endif
    // y = x + kmu8 word by word (no borrow: every nibble of y is >= its offset) iff
    // every difference y_w - x_w is kmu8: one subtraction per word, then one v_bitop3
    // per word pair, (d0 ^ k) | (d1 ^ k) (truth table 0x7E), and an or-reduction
    if constexpr (kX && NW % 2 == 0) {
      uint32_t t[NW / 2];
#pragma unroll
      for (int i = 0; i < NW / 2; ++i) {
        const uint32_t d0 = y[2 * i] - x[2 * i], d1 = y[2 * i + 1] - x[2 * i + 1];
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x7e" : "=v"(t[i]) : "v"(d0), "v"(d1), "v"(kmu8));
      }
      uint32_t d = 0u;
#pragma unroll
      for (int i = 0; i < NW / 2; ++i) d |= t[i];
      asm volatile("" : "+v"(d));
      return d == 0u;
    }
    uint32_t key[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) key[w] = y[w] - kmu8;
    return same_key(x, key);
  }
  // log P̂1(row(D_{t-1}), r); afterwards `slot` describes row(D_t)
  // kmu8: the stored key is the canonical key + kmu8 in every nibble (lazy
  // normalisation, CVD_K1B_LAZYKEY); subtracted only where the key is compared
  // or hashed
  template <bool kX = CVD_K1B_CMPX>
  __device__ double resolve(const ExpArgs& a, const uint32_t (&key_in)[NW], uint32_t r, uint32_t kmu8 = 0u,
                            const double* unseen = nullptr) {
    double lpv = unseen ? *unseen : a.lp_unseen;
    if (CVD_ABL & 1) return lpv;
    int32_t ns = -2;
    if (slot >= 0) {
      lpv = plp; ns = pnx;
    } else if (cand) {
      if (same_key_lazy<kX>(pkey, key_in, kmu8)) {
        lpv = plp; ns = (CVD_ABL & 16) ? -2 : pnx;
      } else if (pkey[0] != kEmptyKey) {
        uint32_t key[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) key[w] = key_in[w] - kmu8;
        // home slot holds another row: linear probing up to an empty slot
        uint32_t sl = hs;
        bool found = false;
        for (int pr = 1; pr <= a.max_probe; ++pr) {
          sl = (sl + 1u) & a.hmask;
          uint32_t k[NW];
          load_key(a, sl, k);
          if (k[0] == kEmptyKey) break;
          if (same_key(k, key)) { found = true; break; }
        }
        if (found) {
          const uint3 v = ld_off<uint3>(a.hrow, (sl << a.rsh) + 16u * r);
          lpv = __hiloint2double((int)v.y, (int)v.x);
          ns = (int32_t)v.z;
        }
      }
    }
    slot = ns;
    return lpv;
  }
  // D_t's key is known: issue the next step's loads
  // kmu8: the key's offset c * 0x11111111, c in {kLo, kLo + 1}
  // hi: the offset is kLo + 1 (else kLo), as a flag the caller already has
  template <int kLo = 0, bool kC = false, bool kRow = true>
  __device__ void prefetch(const ExpArgs& a, const uint32_t (&key_in)[NW], uint32_t rn, uint32_t kmu8 = 0u,
                           bool hi = false) {
    if (CVD_ABL & 1) return;
    if (slot >= 0) {
      if (kRow) prefetch_row<kC>(a, slot, rn);
    } else if (slot == -2 && !(CVD_ABL & 4)) {
      uint32_t ph, pl;
      cvd::key_hash_less<kLo>(key_in, NW, kLo + (hi ? 1u : 0u), ph, pl);   // = key_hash(key_in - kmu8)
      // byte offsets straight from the hash bits (cvd_keys.h: filter block (pl >> 3) & fmask,
      // pattern pair (ph >> 3) & (kFilterPatterns - 1)): one AND each
      hs = ph & a.hmask;
      const uint2 pp = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(filter_patterns_lds()) +
                                                       (ph & (uint32_t)((cvd::kFilterPatterns - 1) << 3)));
      fb = pp.x;
      fb1 = pp.y;
      if (CVD_ABL & 64) {   // timing only: waves of H2 sequences skip the filter read (never a candidate)
        if (h2wave) { fw = 0u; fw1 = 0u; return; }
      }
#if CVD_K1B_LDSF
      const uint2 f = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(dyn_lds()) + (pl & a.fmask4));
#else
      const uint2 f = ld_off<uint2>(a.filt, pl & a.fmask4);
#endif
      fw = f.x;
      fw1 = f.y;
    }
  }
};

// D_t of one sequence as 2^m bytes in canonical state order, from nibble keys
// in the device layout (key_nibble)
template <int m>
__device__ __forceinline__ void k1b_trace(uint8_t* tr, int64_t t, int64_t nseq, int64_t q,
                                          const uint32_t (&key)[(1 << m) / 8]) {
  constexpr int M = 1 << m;
  uint8_t* o = tr + ((size_t)t * nseq + q) * M;
#pragma unroll
  for (int s = 0; s < M; ++s) o[s] = (uint8_t)((key[s >> 3] >> (4 * cvd::key_nibble(M, s))) & 15u);
}

// ──────── k = 1, n = 2 single-vector kernel (standard butterfly; m = 6 headline) ────────
//
// For codes whose tap-0 and tap-m columns are both 11 (every good rate-1/2 code,
// (133,171) and (7,5) included), the two ACS candidates of new states (2j, 2j+1)
// come from D(j) with metrics (e, 2-e) and from D(j + 2^(m-1)) with (2-e, e),
// e = popcount(out(j, 0) ^ y).  The lane's own received word y picks e per
// butterfly with ONE v_perm_b32 from a 4-byte constant, and one packed-16
// add/add/min produces the pair (D(2j), D(2j+1)) -- the next step's operand, in
// place.  Only D_t(y) itself is computed: 2^(m-1) butterflies of 4 packed VALU
// ops, against 2 x 2^m ACS for the orbit kernel.
//
// T_ref count without the other words (exact, no fallback).  y ^ 3 flips every
// e to 2 - e, so D_t(y ^ 3) is the pair swap of D_t(y).  For y' = y ^ 1 or
// y ^ 2 the butterfly classes swap (e in {0, 2} <-> e' = 1), and in each
// butterfly the word with e in {0, 2} must give A(2j) == A(2j+1), which holds
// iff D_{t-1}(j) == D_{t-1}(j + 2^(m-1)).  So D_t(y') == D_t(y) (up to the
// normalisation) needs equal halves; with equal halves d_j, A(2j) = A(2j+1) =
// d_j + [e_j == 1] under y and d_j + [e_j != 1] under y', equal up to a constant
// iff [e_j == 1] is constant over j, i.e. every out(j, 0) is in one class
// (a property of the code only: bfly_uni).  Hence
// c = 1 + [D_t(y) == pair swap] + 2 [halves equal and bfly_uni].
//
// Dp carries the metric pairs plus a per-lane offset O (the sum of the step
// minima since the last renormalisation, every kRenorm steps); nibble keys are
// formed with two shift-adds per 4 butterflies and the offset removed by one
// subtraction per word (exact modulo 2^32).  The step minimum is 0 or 1
// (n = 2; D_{t-1} has a 0 state and one of its branches has metric <= 1), so it
// is read off a zero-nibble test.
// Tuning knobs of the run-time compiled kernel (CVD_JIT_DEFINES="-D...",
// cvd_rtc.cpp): occupancy target, and the quarter of the step at which a
// filter-positive lookup issues its key and row loads.
#ifndef CVD_K1B_WAVES
#define CVD_K1B_WAVES 4
#endif
#ifndef CVD_K1B_MID
#define CVD_K1B_MID 2
#endif
#ifndef CVD_K1B_LAZYKEY
#define CVD_K1B_LAZYKEY 1
#endif
constexpr int kK1bWavesPerSimd = CVD_K1B_WAVES;
constexpr int kRenorm = 128;   // O <= 128: raw pair values stay < 256 (byte packing)

// Register layouts of the pair vector.  Layout 0: register i holds
// (D(2i), D(2i+1)).  Layout 1: register i holds (D(x), D(x+2)) with
// x = 4(i >> 1) + (i & 1), so state s is in register 2(s >> 2) + (s & 1), half
// (s >> 1) & 1.  Both keep states 8w..8w+3 / 8w+4..8w+7 in registers 4w, 4w+1 /
// 4w+2, 4w+3, so one v_perm per half-word packs either into the device key.
template <int L>
__device__ constexpr int lay_reg(int s) { return L == 0 ? s >> 1 : (((s >> 2) << 1) | (s & 1)); }
template <int L>
__device__ constexpr int lay_half(int s) { return L == 0 ? (s & 1) : ((s >> 1) & 1); }

// Branch-metric pair (e_j, 2 - e_j) of butterfly j for the lane's word:
// out(j, 0) = bits 2j..2j+1 of XM, e = popcount(out ^ y), so out 3 and 2 give the
// swaps of out 0 and 1 (W0 = (e0, 2 - e0), W1 = (e1, 2 - e1))
template <uint64_t XM>
__device__ __forceinline__ us2 bfly_w(int j, uint32_t W0, uint32_t W1) {
  const int xj = (int)((XM >> (2 * j)) & 3u);
  return xj == 0 ? as_us2(W0) : xj == 1 ? as_us2(W1) : xj == 2 ? __builtin_shufflevector(as_us2(W1), as_us2(W1), 1, 0)
                                                         : __builtin_shufflevector(as_us2(W0), as_us2(W0), 1, 0);
}
// e(out) as the low half it takes in W0 / W1 (v_perm byte selectors)
template <uint64_t XM>
__device__ constexpr uint32_t e_sel(int j) {
  const int xj = (int)((XM >> (2 * j)) & 3u);
  // perm(W1, W0, .): selectors 0-3 = W0 bytes, 4-7 = W1 bytes.  e(out 0) = e0 = W0
  // bytes 0-1, e(3) = 2 - e0 = W0 bytes 2-3, e(1) = e1 = W1 bytes 0-1, e(2) = 2 - e1
  // = W1 bytes 2-3; the complement 2 - e(out) = e(out ^ 3) is selector ^ 0x0202
  return xj == 0 ? 0x0100u : xj == 3 ? 0x0302u : xj == 1 ? 0x0504u : 0x0706u;
}

// Per received word y, the branch-metric registers of the specialised step in
// LDS (filled at kernel start, read once per step instead of two popcounts,
// two multiply-adds and the e-pair perms): [0] W0, [1] W1, [2 + 2c] / [3 + 2c]
// the (e_j, e_{j+1}) / (2 - e_j, 2 - e_{j+1}) pairs of a butterfly pair whose
// out(j, 0), out(j + 1, 0) classes are c & 3, c >> 2.
constexpr int kWtabStride = 64;
__device__ __forceinline__ uint32_t* wtab_lds() {
  __shared__ uint32_t s_wt[8 * kWtabStride];
  return s_wt;
}
template <uint64_t XM>
__device__ constexpr int xm_class(int j) { return (int)((XM >> (2 * j)) & 3u); }
// Row y + 4 mu holds the metrics minus the previous step's minimum mu (the
// specialised step keeps the pairs at D + 1 + mu, see k1b_body): W0 / W1 as
// 16-bit lanes (e - mu may be -1 = 0xFFFF: the packed adds wrap per lane), the
// e-pairs as the 32-bit integer lo + 65536 hi (the plain 32-bit adds of the
// no-broadcast step then give the lane sums, all >= 0, without a borrow
// crossing lanes).
__device__ __forceinline__ uint32_t wtab_entry(uint32_t y, uint32_t mu, int k) {
  const uint32_t e0 = __builtin_popcount(y), e1 = __builtin_popcount(y ^ 1u);
  const uint32_t W0 = e0 | ((2u - e0) << 16), W1 = e1 | ((2u - e1) << 16);
  const uint32_t mm = mu * 0x10001u;
  if (k == 0) return as_u32(as_us2(W0) - as_us2(mm));
  if (k == 1) return as_u32(as_us2(W1) - as_us2(mm));
  const int c = (k - 2) >> 1, x0 = c & 3, x1 = c >> 2;
  const uint32_t s0 = x0 == 0 ? 0x0100u : x0 == 3 ? 0x0302u : x0 == 1 ? 0x0504u : 0x0706u;
  const uint32_t s1 = x1 == 0 ? 0x0100u : x1 == 3 ? 0x0302u : x1 == 1 ? 0x0504u : 0x0706u;
  const uint32_t pr = (k & 1) ? __builtin_amdgcn_perm(W1, W0, ((s1 ^ 0x0202u) << 16) | (s0 ^ 0x0202u))
                              : __builtin_amdgcn_perm(W1, W0, (s1 << 16) | s0);
  return pr - mm;   // (lo - mu) + 65536 (hi - mu) as a 32-bit integer
}
__device__ __forceinline__ void fill_wtab() {
  uint32_t* t = wtab_lds();
  for (int i = threadIdx.x; i < 8 * 34; i += blockDim.x) {
    const int row = i / 34, k = i % 34;
    t[row * kWtabStride + k] = wtab_entry((uint32_t)(row & 3), (uint32_t)(row >> 2), k);
  }
}

// The common step: D_t(y) for the lane's own word, in place in Dp (pair i is
// dead once butterflies 2i, 2i + 1 and 2i - H, 2i + 1 - H have read it), and
// the nibble keys of the raw metrics minus the running offset.
//
// kKind 0 (table-driven and general): layout 0 in and out; each butterfly is
//   one packed add of the broadcast top input, one of the broadcast bottom input
//   and one packed min (three VOP3P).
// kKind 1 (specialised, even steps): layout 0 in, layout 1 out, no broadcast:
//   butterflies j, j+1 (j even) share registers (D(j), D(j+1)) and
//   (D(j+32), D(j+33)); adding (e_j, e_{j+1}) and (2-e_j, 2-e_{j+1}) as plain
//   32-bit adds (two 16-bit lanes, no carry) and two packed mins give
//   (D'(2j), D'(2j+2)) and (D'(2j+1), D'(2j+3)): four VOP2 + two VOP3P per two
//   butterflies instead of six VOP3P.
// kKind 2 (specialised, odd steps): layout 1 in (broadcast picks the half),
//   layout 0 out.
template <int m, bool kSpec, uint64_t XM, int kKind = 0>
__device__ __forceinline__ void k1b_acs(const ExpArgs& a, cu32* tb, RowCursor<(1 << m) / 8, 4>& cur, uint32_t rr,
                                        uint32_t (&Dp)[(1 << m) / 2], uint32_t (&kw)[(1 << m) / 8],
                                        uint32_t sel, uint32_t O8, uint32_t& zn, uint32_t mu_prev = 0u) {
  constexpr int M = 1 << m, H = M / 2;
  constexpr int LIN = kKind == 2 ? 1 : 0;
  constexpr int kMid = ((H * CVD_K1B_MID) / 4) & ~1;   // even: both loops reach it
  uint32_t E[H];
  // specialised (kSpec, out(j, 0) = bits 2j..2j+1 of XM): the lane's pairs
  // (e, 2 - e) for out(j, 0) = 0 and 1; out 3 and 2 are their swaps (op_sel),
  // so no table and no v_perm per butterfly
  uint32_t W0 = 0u, W1 = 0u;
  const uint32_t* wt = nullptr;   // this word's row of the LDS table (wtab_entry)
  if constexpr (kSpec) {
    wt = wtab_lds() + (rr + 4u * mu_prev) * kWtabStride;
    W0 = wt[0];
    W1 = wt[1];
  }
  auto pack = [&](int w, uint32_t sel_pk) {
    // word w = states 8w..8w+7 in nibble order bitrev3 (device key layout):
    // bytes (s0, s2, s1, s3) and (s4, s6, s5, s7) by one v_perm each (metrics + O < 256)
    const uint32_t x = __builtin_amdgcn_perm(E[4 * w + 1], E[4 * w], sel_pk);
    const uint32_t y = __builtin_amdgcn_perm(E[4 * w + 3], E[4 * w + 2], sel_pk);
    // table-driven kernel: nibbles = raw metric - offset (0..14), a zero nibble is
    // the step minimum 0; specialised: the pairs already are D + 1 + mu (1..15) and
    // a nibble < 2 (hasless(v, 2): existence is exact) is the step minimum 0
    const uint32_t v = kSpec ? x + (y << 4) : x + (y << 4) - O8;
    zn |= (v - (kSpec ? 0x22222222u : 0x11111111u)) & ~v;
    kw[w] = v;
  };
  if constexpr (kKind == 1) {
    static_assert(kSpec, "no-broadcast step needs the specialised code");
#pragma unroll
    for (int j = 0; j < H; j += 2) {
      if (j == kMid) {
        cur.fence(zn);
        cur.mid(a, rr);
      }
      const uint32_t ra = Dp[j >> 1], rb = Dp[(j >> 1) + H / 2];
      // (e_j, e_{j+1}) and (2 - e_j, 2 - e_{j+1}) (compile-time selectors; the
      // compiler shares equal ones across butterfly pairs)
      const int c = xm_class<XM>(j) | (xm_class<XM>(j + 1) << 2);   // compile-time after unrolling
      const uint32_t ep = wt[2 + 2 * c], cp = wt[3 + 2 * c];
      E[j] = as_u32(__builtin_elementwise_min(as_us2(ra + ep), as_us2(rb + cp)));       // (D'(2j), D'(2j+2))
      E[j + 1] = as_u32(__builtin_elementwise_min(as_us2(ra + cp), as_us2(rb + ep)));   // (D'(2j+1), D'(2j+3))
      if ((j & 3) == 2) pack(j >> 2, 0x06040200u);
    }
  } else {
#pragma unroll
    for (int j = 0; j < H; ++j) {
      if (j == kMid) {                   // filter positive: key + row loads under the second half
        cur.fence(zn);                    // zn depends on every butterfly so far
        cur.mid(a, rr);
      }
      const us2 pa = as_us2(Dp[lay_reg<LIN>(j)]), pb = as_us2(Dp[lay_reg<LIN>(j + H)]);
      const int h = lay_half<LIN>(j);
      const us2 da = h ? __builtin_shufflevector(pa, pa, 1, 1) : __builtin_shufflevector(pa, pa, 0, 0);
      const us2 db = h ? __builtin_shufflevector(pb, pb, 1, 1) : __builtin_shufflevector(pb, pb, 0, 0);
      us2 W;
      if constexpr (kSpec) {
        W = bfly_w<XM>(j, W0, W1);
      } else {
        const uint32_t T = tb[j];
        W = as_us2(__builtin_amdgcn_perm(T, T, sel));   // (e, 2 - e)
      }
      E[j] = as_u32(__builtin_elementwise_min(da + W, db + __builtin_shufflevector(W, W, 1, 0)));
      if ((j & 3) == 3) pack(j >> 2, 0x06020400u);
    }
  }
#pragma unroll
  for (int j = 0; j < H; ++j) Dp[j] = E[j];
}

// Butterfly parity classes of a specialised code (out(j, 0) = bits 2j..2j+1 of
// XM), as cvd_host.cpp build_bfly derives them at run time: every out(j, 0) of
// even parity (bfly_uni), and the nibble mask of the even-parity butterflies of
// halves-difference word v (bfly_even[v], device key layout).
template <int m, uint64_t XM>
__device__ constexpr bool xm_uni() {
  for (int j = 0; j < (1 << m) / 2; ++j)
    if (__builtin_popcount((unsigned)((XM >> (2 * j)) & 3u)) & 1) return false;
  return true;
}
template <int m, uint64_t XM>
__device__ constexpr uint32_t xm_even(int v) {
  uint32_t w = 0u;
  for (int j = 8 * v; j < 8 * v + 8 && j < (1 << m) / 2; ++j)
    if (!(__builtin_popcount((unsigned)((XM >> (2 * j)) & 3u)) & 1)) w |= 0xFu << (4 * cvd::key_nibble(1 << m, j));
  return w;
}

template <int V>
struct IntC {
  static constexpr int value = V;
};

// ──────── H1 waves that walk learned rows (k1b_walk; specialised kernel) ────────
//
// An H1 sequence (encoder G1, the decoder's own code) spends most of its steps in
// learned rows at small p (rows hold D_t for 98% of the steps at p = 0.01, 96% at
// 0.02, 75% at 0.05, 24% at 0.1, <= 3% at p >= 0.15; m = 6, learn_len 10^6): there
// the successor row, log P̂1 and the T_ref count c of every step are in the row's
// record, and the metric vector is not needed.  The lockstep body still runs the
// whole ACS for such a lane, since its wave's other lanes need it.  Here the lanes
// of an H1 wave keep their own step counts and are in one of four modes:
//   WALK  D_{t-1} is learned row `slot`, its entry for r_t loaded (log P̂1,
//         successor, c): a walk step adds both logs and moves to the successor --
//         one dependent 16-byte load, a dozen VALU, no ACS;
//   PEND  the entry's successor is not a row: the lane needs D_t = ACS(D_{t-1}, r_t)
//         and has started the load of row `slot`'s key (a.dkey) to rebuild its
//         metric vector;
//   ACS   metric vector valid: an ACS step as in k1b_body; a lane whose D_t is a row
//         (successor or hashed hit) goes back to WALK;
//   DONE  t = N.
// The wave alternates walk bursts (up to walk_burst steps of every WALK lane) and
// ACS steps (every PEND / ACS lane), choosing a burst when some lane walks and
// either no lane needs the ACS, or >= walk_wmin lanes walk, or < walk_amin lanes
// need it.  Every iteration moves some lane forward, so the loop ends.  The ACS
// kinds alternate per ACS step of the wave (the layout is the wave's, not the
// lane's), and a PEND lane's vector is rebuilt in the layout of the coming kind with
// mu_prev = 0 (pairs = D + 1).  Per-trial sums are the lockstep body's bit for bit:
// each lane adds the same terms in step order.
enum : uint32_t { kWalkAcs = 0u, kWalkPend = 1u, kWalkWalk = 2u, kWalkDone = 3u };
// timing ablation (CVD_JIT_DEFINES=-DCVD_WALK_ABL=1, results differ): walk-mode waves
// do no work, so the launch times the H2 waves alone
#ifndef CVD_WALK_ABL
#define CVD_WALK_ABL 0
#endif
// the walk loop's guard bound, iterations per step of N (tests: CVD_JIT_DEFINES=-DCVD_WALK_GUARD=0
// trips it at once, so the error flag's path is exercised)
#ifndef CVD_WALK_GUARD
#define CVD_WALK_GUARD 128
#endif

template <int m, uint64_t XM>
__device__ __forceinline__ void k1b_walk(const ExpArgs& a, int64_t qwave, uint64_t vmask, const double* s_lt) {
  constexpr int M = 1 << m, H = M / 2, NW = M / 8, R = 4;
  if (CVD_WALK_ABL & 1) return;
  const bool valid = qwave + lane_id() < a.nseq;
  const uint32_t N = (uint32_t)a.N;
  const uint32_t nwords = (N + 15u) / 16u;
  const size_t cstride = (size_t)a.nseq * 4;
  // received words: the lane's words pos / 16 (curw) and pos / 16 + 1 (nxtw); a lane
  // that moves into nxtw reloads it at the top of the next iteration (need), not
  // inside a walk burst: loads complete in issue order, so a word load issued there
  // would hold up every later record load of the burst (walk_burst <= 16: a lane
  // crosses at most one word per iteration)
  auto load_word = [&](uint32_t wi) -> uint32_t {
    if (wi >= nwords) return 0u;
    return a.r[(size_t)(wi >> 2) * cstride + (size_t)(qwave + lane_id()) * 4 + (wi & 3u)];
  };
  uint32_t pos = 0u, curw = 0u, nxtw = 0u;
  bool need = false;
  // bits 0-1: r of step pos + 1
  auto word_at = [&]() -> uint32_t { return curw >> (2u * (pos & 15u)); };
  auto advance = [&]() {
    ++pos;
    if ((pos & 15u) == 0u) {
      curw = nxtw;
      need = true;
    }
  };
  uint32_t Dp[H];
  uint32_t key[NW];
#pragma unroll
  for (int i = 0; i < H; ++i) Dp[i] = 0x00010001u;
#pragma unroll
  for (int w = 0; w < NW; ++w) key[w] = 0x11111111u;
  uint32_t kmu8 = 0x11111111u, mu_prev = 0u;
  double lp = 0.0, lr = 0.0;
  RowCursor<NW, R> cur;
  cur.slot = -1; cur.pnx = -1; cur.hs = 0u; cur.fb = 0u; cur.fw = 0u; cur.fb1 = 0u; cur.fw1 = 0u;
  cur.cand = false; cur.plp = 0.0; cur.pc = 1u;
  // the entry a walker consumes next: one step (cur.plp / pnx / pc, a drow entry) or, with
  // two-step records and two steps left, {cur.plp, plp2, cur.pnx, cur.pc} = the t2 record
  // {log P̂1 of both steps, (d1 + 1) | c1 << 28, (d2 + 1) | c2 << 28}
  double plp2 = 0.0;
  auto two_steps = [&]() -> bool { return a.t2 != nullptr && pos + 2u <= N; };
  auto walk_prefetch = [&]() {
    const uint32_t x = __builtin_amdgcn_alignbit(nxtw, curw, 2u * (pos & 15u));   // r of steps pos + 1, pos + 2
    if (two_steps()) {
      const uint32_t* e = a.t2 + ((size_t)cur.slot * 16u + (x & 15u)) * 8u;
      const uint4 v = *reinterpret_cast<const uint4*>(e);
      const uint2 w = *reinterpret_cast<const uint2*>(e + 4);
      cur.pc = w.y;
      cur.pnx = (int32_t)w.x;
      plp2 = __hiloint2double((int)v.w, (int)v.z);
      cur.plp = __hiloint2double((int)v.y, (int)v.x);
    } else {
      cur.template prefetch_row<true>(a, cur.slot, x & 3u);
    }
  };
  uint32_t mode = kWalkDone;
  int dec = 0;   // early decision of this lane (counts only): checked every kEarlyEvery of its steps
  // after a step: the lane is done at N, or (early decision) once its decision is certain
  auto finished = [&]() -> bool {
    if (pos == N) return true;
    if (a.early && (pos & (uint32_t)(kEarlyEvery - 1)) == 0u) dec = early_decide(lp, lr, (int64_t)(N - pos), a.lt_min, a.lp_min);
    return dec != 0;
  };
  if (valid && N > 0u) {
    curw = load_word(0u);
    nxtw = load_word(1u);
    cur.slot = a.slot0;   // D_0 = 0 is a learned row: every lane starts walking
    walk_prefetch();
    mode = kWalkWalk;
  }
  // Before an ACS step with PEND lanes: every lane's pairs from a canonical key (no
  // divergent write, so the pairs keep their registers).  A PEND lane's is row
  // `slot`'s key (parked in Dp[0, NW): its pairs are dead); an ACS lane's is its own
  // D_{t-1} (key - kmu8), so its vector is only re-expressed.  Pairs in the layout the
  // coming ACS kind reads (L 0: (D(2i), D(2i+1)); L 1: (D(x), D(x+2)), x = 4(i >> 1) +
  // (i & 1)) as D + 1 (mu_prev = 0), and the lazy key D + 1.
  auto unpack = [&](auto lay) {
    constexpr int L = decltype(lay)::value;
    const bool pend = mode == kWalkPend;
    uint32_t lo[NW], hi[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t k = (pend ? Dp[w] : key[w] - kmu8) + 0x11111111u;
      key[w] = k;
      lo[w] = k & 0x0F0F0F0Fu;           // nibbles 0, 2, 4, 6 as bytes 0..3
      hi[w] = (k >> 4) & 0x0F0F0F0Fu;    // nibbles 1, 3, 5, 7
    }
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const int s0 = L == 0 ? 2 * i : 4 * (i >> 1) + (i & 1), s1 = L == 0 ? s0 + 1 : s0 + 2;
      const int n0 = cvd::key_nibble(M, s0), n1 = cvd::key_nibble(M, s1);
      const uint32_t b0 = (n0 & 1) ? 4u + (uint32_t)(n0 >> 1) : (uint32_t)(n0 >> 1);
      const uint32_t b1 = (n1 & 1) ? 4u + (uint32_t)(n1 >> 1) : (uint32_t)(n1 >> 1);
      Dp[i] = __builtin_amdgcn_perm(hi[s0 >> 3], lo[s0 >> 3], b0 | (0x0Cu << 8) | (b1 << 16) | (0x0Cu << 24));
    }
    kmu8 = 0x11111111u;
    mu_prev = 0u;
    if (pend) mode = kWalkAcs;
  };
  // one ACS step of the wave (every lane computes; ACS lanes keep the result)
  auto acs_step = [&](auto kind) {
    constexpr int KIND = decltype(kind)::value;
    const uint32_t rr = word_at() & 3u;
    uint32_t kw[NW];
    uint32_t zn = 0u;
    k1b_acs<m, true, XM, KIND>(a, nullptr, cur, rr, Dp, kw, 0u, 0u, zn, mu_prev);
    const uint32_t mu = (zn & 0x88888888u) == 0u;
    const uint32_t off8 = mu ? 0x22222222u : 0x11111111u;
    if (mode == kWalkAcs) {
      cur.fence(zn);
      cur.template fence_keys<NW>(zn);
      lp += cur.template resolve<CVD_K1B_CMPX_WALK>(a, key, rr, kmu8);   // Pd_plotter.py:115, T = P̂1
      constexpr int NH = NW / 2;
      const uint32_t pm = (uint32_t)__builtin_amdgcn_sbfe(6, rr, 1);
      uint32_t hx = 0u, sym = 0u;
      constexpr bool kUni = xm_uni<m, XM>();
#pragma unroll
      for (int v = 0; v < NH; ++v) {
        const uint32_t dh = key[v] ^ key[v + NH];
        if (kUni) hx |= dh;
        sym |= dh & (xm_even<m, XM>(v) ^ pm);
      }
      const uint32_t c = 1u + (sym == 0u) + ((kUni && hx == 0u) ? 2u : 0u);
      lr += s_lt[c];                         // Pd_plotter.py:115, T = T_ref(1/2)
#pragma unroll
      for (int v = 0; v < NW; ++v) key[v] = kw[v];
      kmu8 = off8;
      mu_prev = mu;
      advance();
      if (finished()) {
        mode = kWalkDone;
        cur.slot = -1;
      } else {
        cur.template prefetch<1, true, false>(a, key, word_at() & 3u, kmu8, mu != 0u);   // hashed lookups
        if (cur.slot >= 0) {
          mode = kWalkWalk;
          walk_prefetch();
        }
      }
    }
  };
  const uint32_t wmin = (uint32_t)a.walk_wmin, amin = (uint32_t)a.walk_amin;
  const int burst = a.walk_burst;
  // every iteration moves a lane a step or out of a walk: 2 (N + 1) per lane bound it
  // (a guard only: the loop ends by itself)
  int64_t st_acs = 0, st_burst = 0, st_biter = 0, st_unpack = 0, st_lanes_acs = 0, st_lanes_walk = 0;
  for (int64_t it = 0, it_max = CVD_WALK_GUARD * ((int64_t)N + 1); it < it_max; ++it) {
    if (need) {
      nxtw = load_word((pos >> 4) + 1u);
      need = false;
    }
    const uint64_t mA = __ballot(mode <= kWalkPend), mW = __ballot(mode == kWalkWalk);
    if ((mA | mW) == 0u) break;
    const uint32_t nA = (uint32_t)__popcll(mA), nW = (uint32_t)__popcll(mW);
    if (nW != 0u && (nA == 0u || nW >= wmin || nA < amin)) {
      if (CVD_WALK_ABL & 2) { ++st_burst; st_lanes_walk += nW; }
      for (int b = 0; b < burst; ++b) {
        if (CVD_WALK_ABL & 2) ++st_biter;
        if (mode == kWalkWalk) {
          // D_t is not a row: rebuild D_{t-1} (row `slot`) for the ACS; the ACS step takes
          // log P̂1 from cur.plp with successor -1
          auto leave = [&]() {
            mode = kWalkPend;
            cur.pnx = -1;
            const uint32_t* kp = a.dkey + (size_t)cur.slot * NW;
#pragma unroll
            for (int i = 0; i < NW / 4; ++i) {
              const uint4 v = *reinterpret_cast<const uint4*>(kp + 4 * i);
              Dp[4 * i] = v.x; Dp[4 * i + 1] = v.y; Dp[4 * i + 2] = v.z; Dp[4 * i + 3] = v.w;
            }
          };
          auto done = [&]() {
            mode = kWalkDone;
            cur.slot = -1;
          };
          if (two_steps()) {
            const int32_t d1 = (int32_t)((uint32_t)cur.pnx & 0x0FFFFFFFu) - 1;
            if (d1 < 0) {
              leave();
            } else {
              lp += cur.plp;                 // Pd_plotter.py:115, from the row's records
              lr += s_lt[(uint32_t)cur.pnx >> 28];
              cur.slot = d1;
              advance();
              if (finished()) {
                done();
              } else {
                const int32_t d2 = (int32_t)(cur.pc & 0x0FFFFFFFu) - 1;
                if (d2 < 0) {
                  cur.plp = plp2;
                  leave();
                } else {
                  lp += plp2;
                  lr += s_lt[cur.pc >> 28];
                  cur.slot = d2;
                  advance();
                  if (finished()) done();
                  else walk_prefetch();
                }
              }
            }
          } else if (cur.pnx < 0) {
            leave();
          } else {
            lp += cur.plp;                   // Pd_plotter.py:115, from the row's record
            lr += s_lt[cur.pc];
            cur.slot = cur.pnx;
            advance();
            if (finished()) done();
            else walk_prefetch();
          }
        }
        if (__ballot(mode == kWalkWalk) == 0u) break;
      }
      continue;
    }
    // two ACS steps (kinds 1 and 2: layout 0 again after them); a lane the first
    // step sends back to a walk waits out the second
    if (__ballot(mode == kWalkPend) != 0u) {
      if (CVD_WALK_ABL & 2) ++st_unpack;
      unpack(IntC<0>{});
    }
    if (CVD_WALK_ABL & 2) { ++st_acs; st_lanes_acs += nA; }
    acs_step(IntC<1>{});
    acs_step(IntC<2>{});
  }
  // the guard is never reached (every iteration moves a lane); if a scheduling bug ever
  // reaches it, the lanes' partial sums must not pass for results: flag it for the host
  // (cvd_model_device_error), one global atomic from the wave
  if (__ballot(mode != kWalkDone) != 0u && lane_id() == 0 && a.err) atomicOr(a.err, 1);
  // (CVD_WALK_ABL & 2: schedule statistics of the first H1 waves, printed; sums unchanged)
  if ((CVD_WALK_ABL & 2) && qwave < 4 * 64 * 4 && lane_id() == 0)
    printf("walkstats q0=%lld acs_pairs=%lld lanes_per_acs=%.1f bursts=%lld burst_iters=%lld walkers_per_burst=%.1f unpacks=%lld\n",
           (long long)qwave, (long long)st_acs, st_acs ? (double)st_lanes_acs / st_acs : 0.0, (long long)st_burst,
           (long long)st_biter, st_burst ? (double)st_lanes_walk / st_burst : 0.0, (long long)st_unpack);
  if (valid && a.sums) {
    const int64_t qe = qwave + lane_id();
    a.sums[2 * qe] = lp;
    a.sums[2 * qe + 1] = lr;
  }
  early_final(dec, lp, lr);
  count_decisions_masked(vmask, vmask, lp, lr, a.counts);
}

// blk: the block's index within this model's launch range (blockIdx.x, or its offset in a
// multi-model launch, k1b_multi)
template <int m, bool kSpec, uint64_t XM, bool kTrace>
__device__ __forceinline__ void k1b_body(const ExpArgs& a, uint32_t blk) {
  constexpr int M = 1 << m, H = M / 2, NW = M / 8, R = 4;
  static_assert(m >= 3, "k1b kernel: 2^m >= 8 (whole key words)");
  __shared__ double s_lt[R + 1];
  if (threadIdx.x <= R) s_lt[threadIdx.x] = a.ltref[threadIdx.x];
#if defined(CVD_K1B_LDS_PAD) && CVD_K1B_LDS_PAD > 0
  // timing studies only: LDS padding that lowers the blocks per CU (waves per SIMD)
  __shared__ uint32_t s_pad[CVD_K1B_LDS_PAD / 4];
  if (a.N < 0) s_pad[threadIdx.x] = 0u;
#endif
  fill_filter_patterns();
  if constexpr (kSpec) fill_wtab();
#if CVD_K1B_LDSF
  if constexpr (kSpec) {   // the whole filter, 2 (fmask + 1) words, into dynamic LDS
    uint4* d = reinterpret_cast<uint4*>(dyn_lds());
    const uint4* g = reinterpret_cast<const uint4*>(a.filt);
    for (uint32_t i = threadIdx.x; i < (a.fmask + 1u) / 2u; i += blockDim.x) d[i] = g[i];
  }
#endif
  __syncthreads();
  // Sequence index without a VGPR live across the step loop: the wave's first
  // index in SGPRs, the lane from mbcnt, recomputed after the loop; validity
  // and hypothesis as wave ballots (SGPRs)
  constexpr int kBlk = kSpec ? kK1bBlock : kBlock;
  int64_t gw = (int64_t)blk * (kBlk / 64) + (__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6);
  if (!kTrace && a.walk) {
    // H1 and H2 waves alternate (the pair order flips with the block), so every SIMD
    // holds both: the walks' load latency hides under the H2 waves' ACS
    // (waves past 2 * half are the grid's padding and stay past the sequences)
    const int64_t half = ((a.nseq + 63) / 64 + 1) / 2, k = gw >> 1;
    if (gw < 2 * half) gw = ((gw ^ (gw >> 2)) & 1) ? half + k : k;
  }
  const int64_t qwave = gw * 64;
  const int64_t q = qwave + lane_id();
  const bool valid = q < a.nseq;
  const uint64_t vmask = __ballot(valid), hmask = __ballot(q < a.n_h1);
  if constexpr (kSpec && !kTrace) {
    if (a.walk && vmask != 0u && hmask == vmask) {
      k1b_walk<m, XM>(a, qwave, vmask, s_lt);
      return;
    }
  }
  double lp = 0.0, lr = 0.0;
  if (valid) {
    // Pairs (D(2i), D(2i+1)), packed 16-bit.  Table-driven kernel: D + O, O the
    // sum of the step minima since the last renormalisation (every kRenorm
    // steps).  Specialised kernel: D + 1 + mu, mu the last step minimum (0 or 1),
    // kept there by taking mu off the next step's branch metrics (the LDS table
    // row y + 4 mu): the nibble keys need no offset subtraction and nothing is
    // renormalised.
    uint32_t Dp[H];
#pragma unroll
    for (int i = 0; i < H; ++i) Dp[i] = kSpec ? 0x00010001u : 0u;
    uint32_t key[NW];  // D_{t-1}, device key layout (+ kmu8 in every nibble)
#pragma unroll
    for (int w = 0; w < NW; ++w) key[w] = kSpec && CVD_K1B_LAZYKEY ? 0x11111111u : 0u;
    uint32_t O = 0u, O8 = 0u;   // O8 = O * 0x11111111 (table-driven kernel)
    uint32_t mu_prev = 0u;      // step minimum of D_{t-1} (specialised kernel)
    uint32_t kmu8 = kSpec && CVD_K1B_LAZYKEY ? 0x11111111u : 0u;   // nibble offset of the stored key
    double lpu = a.lp_unseen;
    if (CVD_K1B_LPU_VGPR) asm volatile("" : "+v"(lpu));
    if constexpr (kTrace) k1b_trace<m>(a.trace, 0, a.nseq, qwave + lane_id(), key);
    // Received words: word w of this sequence at rbase + (w/4)*cstride + w%4
    // (16-byte chunks, include/cvd.h).  A lane reads its whole chunk at once
    // (one 16-byte load per 64 steps): read a word at a time, the wave's 1 KiB of
    // chunk lines was fetched from HBM up to four times, once per word.  c4 holds
    // the chunk of the next word; it is loaded when the last word of the current
    // chunk starts, 12 steps before its first use (the last group of a word reads
    // the next word's first step).  cw is the current word.
    const int64_t N = a.N, nwords = (N + 15) / 16;
    const size_t cstride = (size_t)a.nseq * 4;   // dwords between chunks of one sequence
    uint32_t c4[4];
    auto load_chunk = [&](int64_t ci) {   // lane address recomputed: no live VGPR pair
      const uint32_t* rb = a.r + (size_t)ci * cstride + (size_t)qwave * 4;
      const uint4 v = 4 * ci < nwords ? *reinterpret_cast<const uint4*>(rb + lane_id() * 4u) : make_uint4(0u, 0u, 0u, 0u);
      c4[0] = v.x; c4[1] = v.y; c4[2] = v.z; c4[3] = v.w;
    };
    // word wi of c4 (wi wave-uniform: three selects on an SGPR index), 0 past the stream
    auto pick = [&](int64_t wi) -> uint32_t {
      const uint32_t e = (uint32_t)wi & 3u;
      const uint32_t v = e == 0u ? c4[0] : e == 1u ? c4[1] : e == 2u ? c4[2] : c4[3];
      return wi < nwords ? v : 0u;
    };
    load_chunk(0);
    uint32_t cw = pick(0);          // current word
    int64_t w = 0;                  // index of the current word
    RowCursor<NW, R> cur;
    cur.start(a, cw & 3u);
    if (CVD_ABL & 64) cur.h2wave = hmask == 0u;

    // one step t (1-based) with received word rr and the next step's word rn;
    // the specialised kernel alternates no-broadcast (layout 0 -> 1) and
    // broadcast (1 -> 0) steps, so every even step leaves layout 0
    auto step = [&](uint32_t rr, uint32_t rn, int64_t t, auto kind) {
      constexpr int KIND = kSpec ? decltype(kind)::value : 0;
      const uint32_t sel = rr | ((rr ^ 3u) << 16) | 0x0C000C00u;
      cu32* tb = as_const(a.bmp);
      asm volatile("" : "+s"(tb));   // per step: the table is re-read (scalar cache), not held in SGPRs
      uint32_t kw[NW];
      uint32_t zn = 0u;
      k1b_acs<m, kSpec, XM, KIND>(a, tb, cur, rr, Dp, kw, sel, O8, zn, mu_prev);
      // Eq. 5: step minimum 0 or 1
      const uint32_t mu = (zn & 0x88888888u) == 0u;
      // offset of kw's nibbles over the normalised D_t
      const uint32_t off8 = kSpec ? (mu ? 0x22222222u : 0x11111111u) : (mu ? 0x11111111u : 0u);
      if constexpr (kSpec) {
        mu_prev = mu;
      } else {
        O += mu;
        O8 += mu ? 0x11111111u : 0u;
      }
      // P̂1 row of D_{t-1}
      cur.fence(zn);                          // zn depends on the whole ACS
      cur.template fence_keys<NW>(zn);
      lp += cur.resolve(a, key, rr, kmu8, CVD_K1B_LPU_VGPR ? &lpu : nullptr);    // Pd_plotter.py:115, T = P̂1
      // halves differences of D_{t-1}: nibble of state j (< 2^(m-1)) is nonzero
      // iff D_{t-1}(j) != D_{t-1}(j + 2^(m-1))
      constexpr int NH = NW >= 2 ? NW / 2 : 1;
      uint32_t dh[NH];
      if constexpr (NW >= 2) {
#pragma unroll
        for (int v = 0; v < NH; ++v) dh[v] = key[v] ^ key[v + NH];
      } else {
        dh[0] = (key[0] ^ (key[0] >> 4)) & 0x0F0F0F0Fu;   // states s, s + 4 = nibbles 2i, 2i + 1
      }
      // pm: all ones when y has odd parity; the butterflies that decide the
      // pair-swap test are those with out(j, 0) of y's parity
      // (bit rr of 0b0110 is y's parity: one sign-extending bit-field extract)
      const uint32_t pm = (uint32_t)__builtin_amdgcn_sbfe(6, rr, 1);
      uint32_t hx = 0u, sym = 0u;
      constexpr bool kUniKnown = kSpec, kUni = kSpec && xm_uni<m, XM>();
#pragma unroll
      for (int v = 0; v < NH; ++v) {
        if (!kUniKnown || kUni) hx |= dh[v];
        sym |= dh[v] & ((kSpec ? xm_even<m, XM>(v) : a.bfly_even[v]) ^ pm);
      }
      // D_t's key.  Lazy form: raw nibbles (canonical + off8 in every nibble, no
      // borrow since every nibble is >= its offset); the halves test only asks
      // which nibbles are equal, which the common offset leaves unchanged
#pragma unroll
      for (int v = 0; v < NW; ++v) key[v] = CVD_K1B_LAZYKEY ? kw[v] : kw[v] - off8;
      kmu8 = CVD_K1B_LAZYKEY ? off8 : 0u;
      // y ^ 3: D_t is the pair swap of D_t(y); y ^ 1, y ^ 2: equal iff halves and uni
      const bool uni = kUniKnown ? kUni : a.bfly_uni != 0u;
      const uint32_t c = (CVD_ABL & 2) ? 1u : 1u + (sym == 0u) + ((uni && hx == 0u) ? 2u : 0u);
      lr += s_lt[c];                          // Pd_plotter.py:115, T = T_ref(1/2) = c / 2^n
      if constexpr (kTrace) {
        uint32_t ck[NW];
#pragma unroll
        for (int v = 0; v < NW; ++v) ck[v] = key[v] - kmu8;
        k1b_trace<m>(a.trace, t, a.nseq, qwave + lane_id(), ck);
      }
      // the key offset is kLo + mu (lazy) or 0 (eager)
      cur.template prefetch<kSpec && CVD_K1B_LAZYKEY ? 1 : 0>(a, key, rn, kmu8, CVD_K1B_LAZYKEY && mu != 0u);
    };

    // groups of 4 steps (a quarter word): the 10 bits they read (4 words and
    // the next step's) come from one window; only the last group of a word
    // needs the next word
    int64_t t = 0;
    int g = 0;
    int dec = 0;   // early decision of this lane (0 = open)
    for (; t + 4 <= N; t += 4) {
      const uint32_t win = g < 3 ? cw >> (8 * g) : __builtin_amdgcn_alignbit(pick(w + 1), cw, 24);
      step(bits2(win, 0), bits2(win, 2), t + 1, IntC<1>{});
      step(bits2(win, 2), bits2(win, 4), t + 2, IntC<2>{});
      step(bits2(win, 4), bits2(win, 6), t + 3, IntC<1>{});
      step(bits2(win, 6), bits2(win, 8), t + 4, IntC<2>{});
      if (++g == 4) {
        g = 0;
        ++w;
        cw = pick(w);
        if (((w + 1) & 3) == 0) load_chunk((w + 1) >> 2);   // the next word opens a chunk
      }
      if (((t + 4) & (kRenorm - 1)) == 0) {
        if constexpr (!kSpec) {
          const us2 o2 = as_us2(O * 0x10001u);
#pragma unroll
          for (int i = 0; i < H; ++i) Dp[i] = as_u32(as_us2(Dp[i]) - o2);
          O = 0u;
          O8 = 0u;
        }
        static_assert(kRenorm == kEarlyEvery, "early checks ride on the renormalisation");
        if (a.early) {
          if (!dec) dec = early_decide(lp, lr, N - (t + 4), a.lt_min, a.lp_min);
          if (__ballot(dec == 0) == 0) {   // every lane decided: the wave is done
            t = N;
            break;
          }
        }
      }
    }
    // last 1-3 steps (inside the current group, so no renormalisation is due)
    if (t < N) {
      const uint32_t win = g < 3 ? cw >> (8 * g) : __builtin_amdgcn_alignbit(pick(w + 1), cw, 24);
      step(bits2(win, 0), bits2(win, 2), t + 1, IntC<1>{});
      if (t + 1 < N) step(bits2(win, 2), bits2(win, 4), t + 2, IntC<2>{});
      if (t + 2 < N) step(bits2(win, 4), bits2(win, 6), t + 3, IntC<1>{});
    }
    if (a.sums) {
      const int64_t qe = qwave + lane_id();
      a.sums[2 * qe] = lp;
      a.sums[2 * qe + 1] = lr;
    }
    early_final(dec, lp, lr);
  }
  count_decisions_masked(vmask, hmask, lp, lr, a.counts);
}

// ──────── several models in ONE launch (cvd_detect_multi; specialised kernel) ────────
//
// A p sweep detects one batch per model (one learned P̂1 per p, Pd_plotter.py:123-169,
// 199-233).  Launched one model at a time, every launch ends with a last residency round
// whose waves finish unevenly (their row lookups differ), which costs ~15-25 ms per
// launch at N = 1e5 (DESIGN.md "Measurement").  Here consecutive block ranges run
// consecutive models -- blocks [blk_end[i-1], blk_end[i]) model i -- so the dispatcher
// starts model i+1's blocks in the CUs model i's last waves leave idle, and a step pays one
// tail instead of one per p.  Blocks are dispatched in order, so at any time the resident
// waves belong to one model or, at a boundary, two: their tables share the caches no
// worse than one model's (concurrent launches of several models on separate queues
// measured 12% slower, profiles/r04a/).  Every model of a launch shares the decoder code
// (the kernel is specialised to it) and the variant (block size, LDS filter).
constexpr int kMultiMax = 8;
struct MultiArgs {
  ExpArgs a[kMultiMax];
  uint32_t blk_end[kMultiMax];   // cumulative block counts
  int32_t nm;
};
template <int m, uint64_t XM>
__device__ __forceinline__ void k1b_multi(const MultiArgs& ma) {
  const uint32_t b = blockIdx.x;
  int i = 0;
  uint32_t b0 = 0u;
  while (i + 1 < ma.nm && b >= ma.blk_end[i]) b0 = ma.blk_end[i++];   // scalar: blockIdx is uniform
  k1b_body<m, true, XM, false>(ma.a[i], b - b0);
}

}  // namespace cvd_dev

// the bit-sliced m = 6 kernel (k1s) and the specialised entries
#include "cvd_k1s.h"
