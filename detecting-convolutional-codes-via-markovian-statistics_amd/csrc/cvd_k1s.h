// The m = 6 bit-sliced detector k1s (the JIT's CVD_K1B_BITSLICE=1 variant of the
// code-specialised kernel, cvd_rtc.cpp).  Included at the end of cvd_device.h (whose
// ExpArgs, filter patterns, walk-mode constants and helpers it uses); the run-time compile
// embeds it after that file.
//
// The detector of k1b_body / k1b_walk, sums identical bit for bit, with the 64 metrics as
// four bit-planes of two words in the rotating layout of cvd_bitslice.h.
// Per step: the branch-metric planes of (phase, y) from an LDS table, mu first, the ACS of
// both words (own and partner adds, a borrow-chain min), the T_ref count off the partner
// planes and, for a lane whose new vector must be hashed, the canonical digest hash.  The
// row tables are the bit-sliced ones (cvd_host.cpp build_hash with bs): the Bloom filter
// over the digest hash, 256-byte directory slots {six phase images, the row's record}, six
// images per learned row by row id (walk mode) and the usual dense records; in front of the
// L2 filter, a 2^20-bit pre-filter in LDS (CVD_K1S_PF).  The layout phase is compile-time in
// the lockstep loop (six steps per iteration) and wave-uniform in walk mode.  A launch over
// more sequences than stay resident is persistent: one block per slot, each wave taking 64
// sequences at a time from a work queue (k1s_body).
#pragma once

#ifndef CVD_K1B_BITSLICE
#define CVD_K1B_BITSLICE 0
#endif

namespace cvd_dev {

constexpr int kBsSlotShift = 6;      // directory slot: 64 dwords
constexpr int kBsRecWord = 48;       // record r at dwords 48 + 4 r of a slot (images 8 x 6 before it)
// Directory slots of three 128-B lines (CVD_K1S_SLOT3, the model's bs_slot_w = 96; cvd_host.cpp
// build_hash): line k = {image of phase 2k, image of phase 2k + 1, the row's record}, so that a
// candidate's image and record share one line (the 256-B slot: 2 lines for phases 0-3)
#ifndef CVD_K1S_SLOT3
#define CVD_K1S_SLOT3 0
#endif
constexpr bool kSlot3 = CVD_K1S_SLOT3 != 0;
template <int PH>
__device__ __forceinline__ constexpr uint32_t bs_img_off() {
  return kSlot3 ? 128u * (PH / 2) + 32u * (PH % 2) : 32u * PH;
}
template <int PH>
__device__ __forceinline__ constexpr uint32_t bs_rec_off() {
  return kSlot3 ? 128u * (PH / 2) + 64u : 4u * kBsRecWord;
}
constexpr int kBsDkeyWords = 48;     // six images per row in a.dkey
constexpr int kBsEarlyGroups = 21;   // early-decision check every 126 steps
// timing ablation (CVD_JIT_DEFINES=-DCVD_K1S_ABL=1; results differ): the waves of H2
// sequences read filter word 0 instead of their own and never take a candidate, so a launch
// times the lockstep kernel without their random L2 requests
#ifndef CVD_K1S_ABL
#define CVD_K1S_ABL 0
#endif
// the LDS pre-filter variant (cvd_kernels.hip upload_model; 1,024-thread blocks, 128 KiB of
// dynamic LDS): a lane tests D_t's pre-filter bit before it requests its L2 filter word
#ifndef CVD_K1S_PF
#define CVD_K1S_PF 0
#endif
// two-step records for the lockstep lanes that walk learned rows (CVD_K1S_T2=1 with the
// model's t2 table, CVD_BS_T2=1): one load per two steps.  Off: +1.5% at p = 0.05, -0.8% to
// -2.6% at p >= 0.1 in block launches (profiles/r05j: the 512-B-per-row table spreads the
// walks over 8x the lines), and with the persistent launch its 4 VGPRs spill: -14% / -22% at
// p = 0.05 / 0.1 (profiles/r05aa)
#ifndef CVD_K1S_T2
#define CVD_K1S_T2 0
#endif
// cursor forms (timing studies; both off: profiles/r05t, p = 0.2 / 0.05 1,949 / 1,953 ms per
// launch against 1,970 / 1,979 with both): bit 0 -- a pre-filter negative marks D_t "not a
// row" at the resolve (else: an all-ones pattern that filter word 0 cannot match); bit 1 --
// the filter offset through an empty asm (the SGPR-base load form)
#ifndef CVD_K1S_TRIM
#define CVD_K1S_TRIM 0
#endif
constexpr bool kK1sT2 = CVD_K1S_T2 != 0;
#ifndef CVD_K1S_MIDPOS
#define CVD_K1S_MIDPOS 0
#endif
// the cursor's per-step selects as sign / bit masks and v_bitop3 (BsCursor::resolve, hash_ahead;
// default on): static loop cost 3,168 -> 3,069 cycles per six steps, the six-p sweep
// 1,383,795-1,384,920 -> 1,389,060-1,390,175 trials/s on one box (profiles/r06ad, three rounds),
// sums identical (119 GPU parity tests)
#ifndef CVD_K1S_AMASK
#define CVD_K1S_AMASK 1
#endif
// the directory / filter masks of the per-step lookup as VGPR copies (BsCursor::masks)
#ifndef CVD_K1S_VMASK
#define CVD_K1S_VMASK 0
#endif
// timing ablation (results unchanged): CVD_K1S_PADV extra VALU instructions per lockstep step,
// independent of the step's own -- the launch's sensitivity to VALU issue
#ifndef CVD_K1S_PADV
#define CVD_K1S_PADV 0
#endif
// chunked launches (-DCVD_K1S_CK=0 compiles them out, for A/Bs of the unchunked
// loop's code: the host then must not chunk, CVD_CHUNK=0)
#ifndef CVD_K1S_CK
#define CVD_K1S_CK 1
#endif
// Word offsets (CVD_K1S_R16, default on): a step's received words enter the cursor and the
// branch-metric table as byte offsets 16 r, each one v_lshrrev and one v_and of the six-step
// group's window shifted once -- both take vector or constant operands at ~2.5 cycles per
// wave64 instruction -- instead of a v_bfe (its shift held in a VGPR) then v_lshlrev /
// v_lshl_add at ~4.2 each (profiles/r05an); and the two-step records' third word is only
// extracted when they are compiled in
#ifndef CVD_K1S_R16
#define CVD_K1S_R16 1
#endif
constexpr bool kR16 = CVD_K1S_R16 != 0;
// a cursor / step word parameter as the byte offset 16 r, and a raw word r as that parameter
__device__ __forceinline__ uint32_t word_off16(uint32_t rp) { return kR16 ? rp : 16u * rp; }
__device__ __forceinline__ uint32_t word_param(uint32_t r) { return kR16 ? 16u * r : r; }

// The lockstep lanes read each 16-B stream chunk once: non-temporal loads (CVD_K1S_NT_STREAM,
// default on) so that the 131 GB per launch do not evict the row tables' lines from L2 (p = 0.1
// / 0.15 2,074 / 2,040 -> 2,041-2,049 / 2,008 ms, profiles/r05y)
#ifndef CVD_K1S_NT_STREAM
#define CVD_K1S_NT_STREAM 1
#endif
// Walk mode's stream words (k1s_walk): 0 (default) -- one 4-B load per word, at the top of the
// loop iteration after the lane moves into its next word; 1 / 2 -- whole 16-B chunks, the next
// chunk requested for the wave's lanes together once one of them is in word >= CVD_WALK_BUF of its
// chunk (bursts move a lane <= 16 steps, so 1 and 2 are the values that load a chunk before it is
// read).  Same sums; p = 0.01 1,579-1,585 (1) / 1,572-1,573 (2) against 1,499-1,505 ms (0) per
// launch on one box (profiles/r06q): the stream words' loads are not what the walk waits on
#ifndef CVD_WALK_BUF
#define CVD_WALK_BUF 0
#endif
static_assert(CVD_WALK_BUF >= 0 && CVD_WALK_BUF <= 2, "CVD_WALK_BUF: 0, 1 or 2");
typedef unsigned int bs_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 stream_load(const uint4* p) {
  if constexpr (CVD_K1S_NT_STREAM != 0) {
    const bs_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const bs_u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}

// LDS: per (phase, y) two uint4 {e0, e1, ez, 0} of word 0 and word 1 (cvd::bs_eplanes)
__device__ __forceinline__ uint4* bs_etab_lds() {
  __shared__ uint4 s_et[6 * 4 * 2];
  return s_et;
}
// CVD_BS_ETAB2 (default 1; cvd_bitslice.h bs_step_core_tab): per (phase, y) e0 of both words for
// the zero test, and the mu-specific addend planes -- {e0m, a1, p1, a23} of word 0, the same of
// word 1, {p23 of word 0, of word 1} -- read at the offset mu selects instead of selecting the
// planes with the mu mask: 8 VALU fewer per step.
// Same sums (119 GPU parity tests); the six-p sweep 1,375,820-1,377,109 -> 1,397,206-1,399,600
// trials/s on one box (profiles/r06ab, three rounds); =2 (the next step's e0 read a step ahead)
// 1,396,238-1,399,600, the same; =0 the select form
#ifndef CVD_BS_ETAB2
#define CVD_BS_ETAB2 1
#endif
// (16-B strides per word y, so that the word parameter 16 y is the byte offset itself and the
// phase and mu parts are the reads' immediate offsets and one add: e0 at [phase][y] in 16-B
// slots; the mu planes in three sub-tables of [phase][mu][y] 16-B slots each)
constexpr uint32_t kBsMtSub = 6 * 2 * 4 * 16;   // bytes per mu sub-table
__device__ __forceinline__ uint4* bs_e0_lds() {
  __shared__ uint4 s_e0[6 * 4];
  return s_e0;
}
__device__ __forceinline__ uint4* bs_mt_lds() {
  __shared__ uint4 s_mt[3 * 6 * 2 * 4];
  return s_mt;
}
template <uint64_t XM>
__device__ __forceinline__ void fill_bs_etab() {
  if constexpr (CVD_BS_KLDS != 0) {
    if (threadIdx.x < 6) cvd::bs_kmask_lds()[threadIdx.x] = cvd::kBsKmasks[threadIdx.x];
  }
  if constexpr (CVD_BS_ETAB2 != 0) {
    uint4* e = bs_e0_lds();
    uint4* t = bs_mt_lds();
    for (int i = threadIdx.x; i < 24; i += blockDim.x) {
      const int ph = i >> 2, y = i & 3;
      const cvd::BsE E = cvd::bs_eplanes(XM, ph, (uint32_t)y);
      e[i] = make_uint4(E.e0[0], E.e0[1], 0u, 0u);
      for (int m = 0; m < 2; ++m) {
        const cvd::BsMu T = cvd::bs_mu_planes(E, m == 1);
        const int k = (ph * 2 + m) * 4 + y;   // 16-B slot in each sub-table
        t[k] = make_uint4(T.e0m[0], T.a1[0], T.p1[0], T.a23[0]);
        t[k + kBsMtSub / 16] = make_uint4(T.e0m[1], T.a1[1], T.p1[1], T.a23[1]);
        t[k + 2 * (kBsMtSub / 16)] = make_uint4(T.p23[0], T.p23[1], 0u, 0u);
      }
    }
  } else {
    uint4* t = bs_etab_lds();
    for (int i = threadIdx.x; i < 24; i += blockDim.x) {
      const cvd::BsE E = cvd::bs_eplanes(XM, i >> 2, (uint32_t)(i & 3));
      t[2 * i] = make_uint4(E.e0[0], E.e1[0], E.ez[0], 0u);
      t[2 * i + 1] = make_uint4(E.e0[1], E.e1[1], E.ez[1], 0u);
    }
  }
}
// the ACS of one step from the mu-specific planes (CVD_BS_ETAB2); mid as bs_step_core's
// e0 of both words at (phase PH, word parameter rr) from the LDS table
template <int PH>
__device__ __forceinline__ uint2 bs_e0_at(uint32_t rr) {
  const char* eb = reinterpret_cast<const char*>(bs_e0_lds()) + PH * 64;
  return *reinterpret_cast<const uint2*>(eb + word_off16(rr));
}
template <int PH, bool kUni, class Mid>
__device__ __forceinline__ void bs_core_tab(const uint32_t (&R)[2][4], uint32_t rr, uint32_t (&N)[2][4], uint32_t& c,
                                            Mid mid, const uint2* e0pre = nullptr) {
  // (CVD_BS_ETAB2=2: the lockstep loop read this step's e0 a step ahead, e0pre)
  const uint2 E0 = e0pre ? *e0pre : bs_e0_at<PH>(rr);
  const uint32_t e0[2] = {E0.x, E0.y};
  uint32_t mu;
  cvd::bs_step_core_tab<PH, kUni>(
      R, e0,
      [&](bool zero_hit) {
        const char* tb = reinterpret_cast<const char*>(bs_mt_lds()) + PH * 128;
        const uint32_t o = word_off16(rr) + (zero_hit ? 0u : 64u);
        const uint4 w0 = *reinterpret_cast<const uint4*>(tb + o);
        const uint4 w1 = *reinterpret_cast<const uint4*>(tb + o + kBsMtSub);
        const uint2 q = *reinterpret_cast<const uint2*>(tb + o + 2u * kBsMtSub);
        cvd::BsMu T;
        T.e0m[0] = w0.x; T.a1[0] = w0.y; T.p1[0] = w0.z; T.a23[0] = w0.w;
        T.e0m[1] = w1.x; T.a1[1] = w1.y; T.p1[1] = w1.z; T.a23[1] = w1.w;
        T.p23[0] = q.x; T.p23[1] = q.y;
        return T;
      },
      N, mu, c, mid);
}

// P̂1 row cursor over the bit-sliced tables (RowCursor's protocol: slot >= 0 known row id,
// -1 known unvisited row, -2 pending hash probe).  The lookup of D_t is issued AHEAD of the
// resolve of D_{t-1} (hash_ahead, right after the ACS): every lane whose D_{t-1} row is not
// known from a successor record (slot < 0) hashes D_t and reads its filter word before the
// step waits for D_{t-1}'s key and record loads; the lanes whose D_{t-1} turns out to be a
// row (a filter-positive candidate that matches) simply do not use it.  So the filter read
// has the rest of the step and half of the next one to land, and the key and record loads
// the second word's ACS plus the hash.
struct BsCursor {
  int32_t slot, pnx;
  uint32_t hs, hsn, fb, fw, fb1, fw1, pc;   // hs: home slot of D_{t-1}'s lookup, hsn: of D_t's
  bool cand;
  bool pfpos = true;     // D_t's pre-filter bit (CVD_K1S_PF; hash_ahead -> resolve)
  bool h2wave = false;   // (CVD_K1S_ABL timing studies: the wave holds H2 sequences only)
  double plp;
  uint32_t pkey[8];
  // (CVD_K1S_VMASK: the directory and filter masks as VGPR copies made once per unit, so that
  // their per-step ANDs take the fast all-vector form instead of an SGPR operand)
  uint32_t vhmask = 0u, vfmask4 = 0u;
  __device__ void masks(const ExpArgs& a) {
    if constexpr (CVD_K1S_VMASK != 0) {
      vhmask = a.hmask;
      vfmask4 = a.fmask4;
      asm volatile("" : "+v"(vhmask), "+v"(vfmask4));
    }
  }
  __device__ uint32_t hmask_v(const ExpArgs& a) const { return CVD_K1S_VMASK != 0 ? vhmask : a.hmask; }
  __device__ uint32_t fmask4_v(const ExpArgs& a) const { return CVD_K1S_VMASK != 0 ? vfmask4 : a.fmask4; }
  // two-step records (a.t2, lockstep lanes that walk learned rows): half 1 = plp / pnx hold the
  // first step of a record whose second is plp2 / pnx2; half 2 = plp / pnx hold that second
  // step, so the next step needs no load
  double plp2;
  int32_t pnx2;
  uint32_t half;
  // entry rn (16 B {log P̂1, successor row, T_ref count c}) of learned row s, dense records
  __device__ void prefetch_row(const ExpArgs& a, int32_t s, uint32_t rn) {
    uint32_t o;
    if constexpr (kR16) asm("v_lshl_add_u32 %0, %1, 6, %2" : "=v"(o) : "v"((uint32_t)s), "v"(rn));
    else asm("v_lshl_add_u32 %0, %1, 4, %2" : "=v"(o) : "v"(rn), "v"((uint32_t)s * 64u));
    const uint4 v = ld_off<uint4>(a.drow, o);
    pc = v.w;
    pnx = (int32_t)v.z;
    plp = __hiloint2double((int)v.y, (int)v.x);
  }
  // the two-step record (learned row s, words rn then rnn): {log P̂1 of both steps, row after
  // one step + 1, row after two + 1} (cvd_host.cpp, t2)
  // (every k1s offset is a 32-bit byte offset from the table's base: the host keeps the
  // bit-sliced tables under 4 GiB)
  __device__ void prefetch_t2(const ExpArgs& a, int32_t s, uint32_t rn, uint32_t rnn) {
    if constexpr (kR16) { rn >>= 4; rnn >>= 4; }
    uint32_t o;
    asm("v_lshl_add_u32 %0, %1, 5, %2" : "=v"(o) : "v"(rn | (rnn << 2)), "v"((uint32_t)s << 9));
    const uint4 v = ld_off<uint4>(a.t2, o);
    const uint2 w = ld_off<uint2>(a.t2, o + 16u);
    plp = __hiloint2double((int)v.y, (int)v.x);
    plp2 = __hiloint2double((int)v.w, (int)v.z);
    pnx = (int32_t)(w.x & 0x0FFFFFFFu) - 1;
    pnx2 = (int32_t)(w.y & 0x0FFFFFFFu) - 1;
    half = 1u;
  }
  __device__ void start(const ExpArgs& a, uint32_t r0, uint32_t r1) {
    masks(a);
    slot = a.slot0; hs = 0u; hsn = 0u; fb = 0u; fw = 0u; fb1 = 0u; fw1 = 0u; cand = false; pc = 1u; half = 0u;
    plp2 = 0.0; pnx2 = -1;
    if (kK1sT2 && a.t2 && !a.t2c) prefetch_t2(a, slot, r0, r1);
    else prefetch_row(a, slot, r0);
  }
  // ordering fences (RowCursor::fence): the waits for the loads issued a step / half a step
  // earlier land after the ACS work the dependency names.  fence_mid: the filter words (the
  // candidate test); fence_resolve: the lookup state of D_{t-1} (its key, record, slot) --
  // not the filter words hash_ahead has just requested
  __device__ void fence_mid(uint32_t dep) {
    asm volatile("" : "+v"(fw), "+v"(fw1), "+v"(slot) : "v"(dep));
  }
  __device__ void fence_resolve(uint32_t dep) {
    asm volatile("" : "+v"(slot), "+v"(pnx), "+v"(plp), "+v"(pc) : "v"(dep));
    if constexpr (kK1sT2) asm volatile("" : "+v"(pnx2), "+v"(plp2) : "v"(dep));
#pragma unroll
    for (int w = 0; w < 8; ++w) asm volatile("" : "+v"(pkey[w]) : "v"(dep));
  }
  __device__ static uint32_t slot_off(uint32_t s) { return kSlot3 ? s * 384u : s << (kBsSlotShift + 2); }
  __device__ static void load_image(const uint32_t* base, uint32_t o, uint32_t (&k)[8]) {
    const uint4 u = ld_off<uint4>(base, o), v = ld_off<uint4>(base, o + 16u);
    k[0] = u.x; k[1] = u.y; k[2] = u.z; k[3] = u.w; k[4] = v.x; k[5] = v.y; k[6] = v.z; k[7] = v.w;
  }
  // filter positive: the home slot's image of phase PH and its record for word r
  template <int PH>
  __device__ void mid(const ExpArgs& a, uint32_t r) {
    // (two v_bitop3: the compiler's form was six VALU)
    cand = slot == -2 && cvd::bs_bop3<cvd::kTtAndNotOr>(fb1, fw1, cvd::bs_bop3<cvd::kTtAndNotOr>(fb, fw, 0u)) == 0u;
    if (cand) {
      const uint32_t so = slot_off(hs);
      load_image(a.hkey, so + bs_img_off<PH>(), pkey);
      const uint4 v = ld_off<uint4>(a.hkey, so + bs_rec_off<PH>() + word_off16(r));
      pc = v.w;
      pnx = (int32_t)v.z;
      plp = __hiloint2double((int)v.y, (int)v.x);
    }
  }
  __device__ static bool same(const uint32_t (&k)[8], const uint32_t (&R)[2][4]) {
    uint32_t d = k[0] ^ R[0][0];
    d = cvd::bs_bop3<cvd::kTtXorOr>(k[1], R[0][1], d);
    d = cvd::bs_bop3<cvd::kTtXorOr>(k[2], R[0][2], d);
    d = cvd::bs_bop3<cvd::kTtXorOr>(k[3], R[0][3], d);
    d = cvd::bs_bop3<cvd::kTtXorOr>(k[4], R[1][0], d);
    d = cvd::bs_bop3<cvd::kTtXorOr>(k[5], R[1][1], d);
    d = cvd::bs_bop3<cvd::kTtXorOr>(k[6], R[1][2], d);
    d = cvd::bs_bop3<cvd::kTtXorOr>(k[7], R[1][3], d);
    asm volatile("" : "+v"(d));
    return d == 0u;
  }
  // log P̂1(row(D_{t-1}), r), D_{t-1} = planes R at phase PH; afterwards `slot` describes row(D_t)
  template <int PH>
  __device__ double resolve(const ExpArgs& a, const uint32_t (&R)[2][4], uint32_t r, double lpu) {
    double lpv = lpu;
    int32_t ns = pfpos ? -2 : -1;   // D_t's lookup pending, or settled by the pre-filter
    const bool known = slot >= 0;
    if constexpr (CVD_K1S_AMASK != 0 && (CVD_K1S_TRIM & 1) == 0) {
      // (the known row's record or the pending state by a sign mask and three v_bitop3 -- not a
      // compare and three selects on it; a candidate implies slot == -2, so it needs no `known`)
      const uint32_t m = (uint32_t)(slot >> 31);   // ~0: D_{t-1}'s row is not known
      ns = (int32_t)cvd::bs_bop3<cvd::kTtSel>(m, (uint32_t)-2, (uint32_t)pnx);
      lpv = __hiloint2double((int)cvd::bs_bop3<cvd::kTtSel>(m, (uint32_t)__double2hiint(lpu), (uint32_t)__double2hiint(plp)),
                             (int)cvd::bs_bop3<cvd::kTtSel>(m, (uint32_t)__double2loint(lpu), (uint32_t)__double2loint(plp)));
    }
    if (CVD_K1S_AMASK != 0 && (CVD_K1S_TRIM & 1) == 0) {
      if (cand) {
        if (same(pkey, R)) {
          lpv = plp; ns = pnx;
        } else if (pc != 0u) {
          uint32_t sl = hs;
          for (int pr = 1; pr <= a.max_probe; ++pr) {
            sl = (sl + 1u) & a.hmask;
            const uint32_t so = slot_off(sl);
            const uint4 v = ld_off<uint4>(a.hkey, so + bs_rec_off<PH>() + word_off16(r));
            if (v.w == 0u) break;
            uint32_t k[8];
            load_image(a.hkey, so + bs_img_off<PH>(), k);
            if (same(k, R)) {
              lpv = __hiloint2double((int)v.y, (int)v.x);
              ns = (int32_t)v.z;
              break;
            }
          }
        }
      }
    } else if (known) {
      lpv = plp; ns = pnx;
    } else if (cand) {
      if (same(pkey, R)) {
        lpv = plp; ns = pnx;
      } else if (pc != 0u) {
        // the home slot holds another row (an empty slot has c = 0): linear probing up to
        // an empty slot
        uint32_t sl = hs;
        for (int pr = 1; pr <= a.max_probe; ++pr) {
          sl = (sl + 1u) & a.hmask;
          const uint32_t so = slot_off(sl);
          const uint4 v = ld_off<uint4>(a.hkey, so + bs_rec_off<PH>() + word_off16(r));
          if (v.w == 0u) break;
          uint32_t k[8];
          load_image(a.hkey, so + bs_img_off<PH>(), k);
          if (same(k, R)) {
            lpv = __hiloint2double((int)v.y, (int)v.x);
            ns = (int32_t)v.z;
            break;
          }
        }
      }
    }
    slot = ns;
    // a two-step record's second step (its row after one step is D_t's): ready for the next
    if (kK1sT2 && known && half == 1u && ns >= 0) {
      plp = plp2; pnx = pnx2; half = 2u;
    } else {
      half = 0u;
    }
    return lpv;
  }
  // D_t (planes N at phase PH) is known, D_{t-1}'s lookup not yet resolved: a lane whose
  // D_{t-1} row is not known from a successor (slot < 0) may need D_t's lookup, so it hashes
  // D_t and requests the filter word now
  // (no divergent branch: a wave hashes whenever one lane needs it anyway, and a load under
  // a divergent branch made the compiler's wait counts conservative -- it waited for this
  // load at the resolve, vmcnt(0).  A lane that does not need the lookup reads filter word 0
  // instead: every such lane of a wave shares that one L2 line; reading each lane's own
  // block measured 26% slower at p = 0.05, where most H1 lanes walk their rows' successors)
  template <int PH>
  __device__ void hash_ahead(const ExpArgs& a, const uint32_t (&N)[2][4]) {
    {
      uint32_t ph, pl;
      cvd::bs_digest_hash<PH>(N, ph, pl);
      hsn = ph & hmask_v(a);
      const uint2 pp = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(filter_patterns_lds()) +
                                                       (ph & (uint32_t)((cvd::kFilterPatterns - 1) << 3)));
      fb = pp.x;
      fb1 = pp.y;
#if CVD_K1S_PF
      // the pre-filter bit of D_t (LDS): clear -- D_t is not a row -- and the lane reads filter
      // word 0 like a lane that needs no lookup; the resolve then marks D_t "not a row" (-1)
      // instead of "pending" (-2), so no candidate test follows
      const uint32_t pfw = reinterpret_cast<const uint32_t*>(dyn_lds())[__builtin_amdgcn_ubfe(
          pl, 32 - cvd::kBsPfLog2Bits + 5, cvd::kBsPfLog2Bits - 5)];
      // (bit (pl >> (32 - kBsPfLog2Bits)) mod 32 of the word: the extract takes the offset's
      // low five bits)
      const uint32_t pbit = __builtin_amdgcn_ubfe(pfw, pl >> (32 - cvd::kBsPfLog2Bits), 1u);
      const bool pos = pbit != 0u;
      uint32_t fo;
      if constexpr (CVD_K1S_AMASK != 0 && (CVD_K1S_TRIM & 1) == 0 && (CVD_K1S_ABL & 1) == 0) {
        // (masks instead of compares and selects: pm = ~0 where the bit is set, sm = ~0 where
        // D_{t-1}'s row is not known; a clear bit makes the pattern all-ones, as below)
        const uint32_t pm = 0u - pbit, sm = (uint32_t)(slot >> 31);
        fb = cvd::bs_bop3<0xF3>(fb, pm, 0u);    // fb | ~pm
        fb1 = cvd::bs_bop3<0xF3>(fb1, pm, 0u);
        fo = cvd::bs_bop3<0x80>(pl, pm, sm) & fmask4_v(a);
      } else {
        if (CVD_K1S_TRIM & 1) {
          pfpos = pos;
        } else if (!pos) {
          fb = ~0u;
          fb1 = ~0u;
        }
        fo = slot < 0 && pos && !((CVD_K1S_ABL & 1) && h2wave) ? (pl & fmask4_v(a)) : 0u;
      }
#else
      constexpr bool pos = true;
      uint32_t fo = slot < 0 && pos && !((CVD_K1S_ABL & 1) && h2wave) ? (pl & fmask4_v(a)) : 0u;
#endif
      if (CVD_K1S_TRIM & 2) asm volatile("" : "+v"(fo));   // a plain 32-bit offset: the SGPR-base load form
#if CVD_K1B_LDSF
      const uint2 f = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(dyn_lds()) + fo);
#else
      const uint2 f = ld_off<uint2>(a.filt, fo);
#endif
      fw = f.x;
      fw1 = f.y;
      if ((CVD_K1S_ABL & 1) && h2wave) { fw = 0u; fw1 = 0u; }
    }
  }
  // after the resolve: a known row's dense record for the next word (kRow; walk mode loads
  // its own), and D_t's home slot becomes the pending lookup's
  template <bool kRow = true>
  __device__ void next(const ExpArgs& a, uint32_t rn, uint32_t rnn = 0u) {
    if (kRow && slot >= 0 && (!kK1sT2 || half != 2u)) {
      if (kK1sT2 && a.t2 && !a.t2c) prefetch_t2(a, slot, rn, rnn);
      else prefetch_row(a, slot, rn);
    }
    hs = hsn;
  }
};

// one bit-sliced step of a lane: D_{t-1} = R (phase PH) -> N (phase PH + 1) under word rr,
// the filter-positive loads issued between the two words' ACS
template <int PH, bool kUni>
__device__ __forceinline__ void bs_step(const ExpArgs& a, BsCursor& cur, const uint32_t (&R)[2][4], uint32_t rr,
                                        uint32_t (&N)[2][4], uint32_t& c, const uint2* e0pre = nullptr) {
  if constexpr (CVD_BS_ETAB2 != 0) {
    static_assert(CVD_K1S_MIDPOS == 0, "CVD_BS_ETAB2 keeps the candidate test between the two words' ACS");
    bs_core_tab<PH, kUni>(R, rr, N, c, [&](uint32_t dep) {
      cur.fence_mid(dep);            // dep: the first word's ACS result
      cur.template mid<PH>(a, rr);
    }, e0pre);
    cur.template hash_ahead<(PH + 1) % 6>(a, N);
    cur.fence_resolve(N[1][3]);
    return;
  }
  const uint4* et = kR16 ? reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(bs_etab_lds()) + PH * 128 +
                                                          cvd::bs_shl<1>(rr))
                        : bs_etab_lds() + (PH * 4 + rr) * 2;
  const uint4 E0 = et[0], E1 = et[1];
  const uint32_t e0[2] = {E0.x, E1.x}, e1[2] = {E0.y, E1.y}, ez[2] = {E0.z, E1.z};
  uint32_t mu;
  // where the candidate test and its directory loads go (CVD_K1S_MIDPOS, timing studies): 0
  // between the two words' ACS (default), 1 at the step's start (the directory lines get the
  // whole ACS, the filter word only the resolve before it), 2 after the ACS
  if constexpr (CVD_K1S_MIDPOS == 1) {
    cur.fence_mid(R[0][3]);
    cur.template mid<PH>(a, rr);
  }
  cvd::bs_step_core<PH, kUni>(R, e0, e1, ez, N, mu, c, [&](uint32_t dep) {
    if constexpr (CVD_K1S_MIDPOS == 0) {
      cur.fence_mid(dep);            // dep: the first word's ACS result
      cur.template mid<PH>(a, rr);
    }
  });
  if constexpr (CVD_K1S_MIDPOS == 2) {
    cur.fence_mid(N[1][3]);
    cur.template mid<PH>(a, rr);
  }
  cur.template hash_ahead<(PH + 1) % 6>(a, N);   // D_t's filter read before D_{t-1}'s loads are waited for
  cur.fence_resolve(N[1][3]);        // N[1][3] depends on the whole ACS
}

// the ACS of one step alone (the deep pipeline's lookups run after it)
template <int PH, bool kUni>
__device__ __forceinline__ void bs_acs(const uint32_t (&R)[2][4], uint32_t rr, uint32_t (&N)[2][4], uint32_t& c) {
  if constexpr (CVD_BS_ETAB2 != 0) {
    bs_core_tab<PH, kUni>(R, rr, N, c, cvd::BsNoMid());
    return;
  }
  const uint4* et = kR16 ? reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(bs_etab_lds()) + PH * 128 +
                                                          cvd::bs_shl<1>(rr))
                        : bs_etab_lds() + (PH * 4 + rr) * 2;
  const uint4 E0 = et[0], E1 = et[1];
  const uint32_t e0[2] = {E0.x, E1.x}, e1[2] = {E0.y, E1.y}, ez[2] = {E0.z, E1.z};
  uint32_t mu;
  cvd::bs_step_core<PH, kUni>(R, e0, e1, ez, N, mu, c);
}

// Two-step lookup pipeline for the lockstep lanes (CVD_K1S_DEEP): every load of a lookup gets a
// whole step of the wave's other work to land, instead of half of one.  At step t (after the ACS
// that makes D_{t+1} from R = D_t):
//   resolve_a -- D_{t-1}'s lookup (planes Rp, loaded during step t-1): log P̂1(row(D_{t-1}), r_{t-1})
//                and D_t's state (a row from the successor record, -1 not a row, -2 pending);
//   mid_b     -- D_t: a known row's record for r_t, or, pending, the candidate test on the filter
//                word requested at step t-1 and on a positive the home slot's image and record;
//   hash_ahead (BsCursor's) -- D_{t+1}'s filter word where row(D_t) is not known.
// So lp takes each P̂1 term one step later (the same terms in the same order), and a drain after
// the last step resolves the last lookup.  The cost: the planes of D_{t-1} stay live for a step.
// =2: D_{t+1}'s hash, pattern and pre-filter test go before the wait, so every load has the ACS
// and the hash (~110 VALU of the step's ~165) to land.  Same sums (the parity, walk, multi,
// config, early, chunked and C0 suites: 119 passed); same-box launches (profiles/r06u, ms, two
// rounds): p = 0.05 / 0.1 / 0.2 1,845-1,849 / 2,051-2,052 / 1,941-1,973 (0), 1,871-1,875 /
// 2,079-2,080 / 2,003-2,004 (1), 1,850 / 2,043-2,044 / 1,956-1,959 (2).  More time for the
// lookups' loads buys nothing, so their latency is not what the lockstep loop waits on; off
#ifndef CVD_K1S_DEEP
#define CVD_K1S_DEEP 0
#endif
struct BsDeep : BsCursor {
  // (the candidate's word rides in the top bits of its home slot, for the probes: hmask < 2^28)
  static constexpr int kWordShift = 28;
  template <int PH>
  __device__ double resolve_a(const ExpArgs& a, const uint32_t (&Rp)[2][4], double lpu, int32_t& ns) {
    double lpv = lpu;
    ns = pfpos ? -2 : -1;   // D_t's lookup pending (its filter word is in), or settled by the pre-filter
    if (slot >= 0) {
      lpv = plp; ns = pnx;
    } else if (cand) {
      if (same(pkey, Rp)) {
        lpv = plp; ns = pnx;
      } else if (pc != 0u) {
        // the home slot holds another row (an empty slot has c = 0): linear probing up to an
        // empty slot
        const uint32_t r16 = word_param(hs >> kWordShift);
        uint32_t sl = hs & a.hmask;
        for (int pr = 1; pr <= a.max_probe; ++pr) {
          sl = (sl + 1u) & a.hmask;
          const uint32_t so = slot_off(sl);
          const uint4 v = ld_off<uint4>(a.hkey, so + bs_rec_off<PH>() + word_off16(r16));
          if (v.w == 0u) break;
          uint32_t k[8];
          load_image(a.hkey, so + bs_img_off<PH>(), k);
          if (same(k, Rp)) {
            lpv = __hiloint2double((int)v.y, (int)v.x);
            ns = (int32_t)v.z;
            break;
          }
        }
      }
    }
    return lpv;
  }
  // D_t (planes at layout PH) in state ns, word r (a cursor word parameter): its lookup's loads
  template <int PH>
  __device__ void mid_b(const ExpArgs& a, int32_t ns, uint32_t r) {
    cand = ns == -2 && cvd::bs_bop3<cvd::kTtAndNotOr>(fb1, fw1, cvd::bs_bop3<cvd::kTtAndNotOr>(fb, fw, 0u)) == 0u;
    slot = ns;
    hs = hsn | (word_off16(r) >> 4 << kWordShift);
    if (ns >= 0) {
      prefetch_row(a, ns, r);
    } else if (cand) {
      const uint32_t so = slot_off(hsn);
      load_image(a.hkey, so + bs_img_off<PH>(), pkey);
      const uint4 v = ld_off<uint4>(a.hkey, so + bs_rec_off<PH>() + word_off16(r));
      pc = v.w;
      pnx = (int32_t)v.z;
      plp = __hiloint2double((int)v.y, (int)v.x);
    }
  }
  // the lookups' loads are waited for after the ACS that does not need them (every plane of
  // the new vector: one plane alone lets the scheduler leave the other word's ACS for later) and,
  // CVD_K1S_DEEP=2, after D_{t+1}'s hash (x2, x3: its results)
  template <class T>
  __device__ static void after(T& x, const uint32_t (&N)[2][4], uint32_t x2, uint32_t x3) {
    asm volatile("" : "+v"(x) : "v"(N[0][0]), "v"(N[0][1]), "v"(N[0][2]), "v"(N[0][3]), "v"(N[1][0]), "v"(N[1][1]),
                 "v"(N[1][2]), "v"(N[1][3]), "v"(x2), "v"(x3));
  }
  __device__ void fence_all(const uint32_t (&N)[2][4], uint32_t x2 = 0u, uint32_t x3 = 0u) {
    after(slot, N, x2, x3); after(pnx, N, x2, x3); after(plp, N, x2, x3); after(pc, N, x2, x3);
    after(fw, N, x2, x3); after(fw1, N, x2, x3);
#pragma unroll
    for (int w = 0; w < 8; ++w) after(pkey[w], N, x2, x3);
  }
  // CVD_K1S_DEEP=2: D_{t+1}'s hash, pattern and pre-filter test before the wait (no loads), its
  // filter word requested after mid_b (whose test reads D_t's)
  struct Prep {
    uint32_t hs, fb, fb1, fo;
  };
  template <int PH>
  __device__ Prep prep(const ExpArgs& a, const uint32_t (&N)[2][4]) const {
    uint32_t ph, pl;
    cvd::bs_digest_hash<PH>(N, ph, pl);
    Prep h;
    h.hs = ph & a.hmask;
    const uint2 pp = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(filter_patterns_lds()) +
                                                     (ph & (uint32_t)((cvd::kFilterPatterns - 1) << 3)));
    h.fb = pp.x;
    h.fb1 = pp.y;
    bool pos = true;
#if CVD_K1S_PF
    const uint32_t pfw = reinterpret_cast<const uint32_t*>(dyn_lds())[__builtin_amdgcn_ubfe(
        pl, 32 - cvd::kBsPfLog2Bits + 5, cvd::kBsPfLog2Bits - 5)];
    pos = __builtin_amdgcn_ubfe(pfw, pl >> (32 - cvd::kBsPfLog2Bits), 1u) != 0u;
    if (!pos) {   // (hash_ahead's form: a pattern that filter word 0 cannot match)
      h.fb = ~0u;
      h.fb1 = ~0u;
    }
#endif
    h.fo = pos ? (pl & a.fmask4) : 0u;
    return h;
  }
  __device__ void issue(const ExpArgs& a, const Prep& h) {
    hsn = h.hs;
    fb = h.fb;
    fb1 = h.fb1;
    const uint32_t fo = slot < 0 ? h.fo : 0u;
#if CVD_K1B_LDSF
    const uint2 f = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(dyn_lds()) + fo);
#else
    const uint2 f = ld_off<uint2>(a.filt, fo);
#endif
    fw = f.x;
    fw1 = f.y;
  }
};

template <bool kDeep>
struct CursorOf {
  using type = BsCursor;
};
template <>
struct CursorOf<true> {
  using type = BsDeep;
};

// H1 waves in walk mode (k1b_walk's schedule; the planes' layout phase is the wave's)
template <uint64_t XM>
__device__ __forceinline__ void k1s_walk(const ExpArgs& a, int64_t qwave, uint64_t vmask, const double* s_lt) {
  constexpr bool kUni = xm_uni<6, XM>();
  if (CVD_WALK_ABL & 1) return;
  const bool valid = qwave + lane_id() < a.nseq;
  const uint32_t N = (uint32_t)a.N;
  const uint32_t nwords = (N + 15u) / 16u;
  const size_t cstride = (size_t)a.nseq * 4;
  auto load_word = [&](uint32_t wi) -> uint32_t {
    if (wi >= nwords) return 0u;
    // (a plain load: walk mode reads a 16-B chunk's four words one at a time, and non-temporal
    // lines were gone before the next word -- p = 0.01 1,411 -> 1,489 ms, profiles/r05y)
    return a.r[(size_t)(wi >> 2) * cstride + (size_t)(qwave + lane_id()) * 4 + (wi & 3u)];
  };
  uint32_t pos = 0u, curw = 0u, nxtw = 0u;
  bool need = false;
  // CVD_WALK_BUF: the lane's stream as two whole 16-B chunks, ca (holding word pos / 16) and cb
  // (the next one), read by one non-temporal load each.  A lane that moves into cb's chunk needs
  // the chunk after it (needb); the wave requests those chunks together, at the top of the first
  // loop iteration where such a lane has reached its chunk's word 1 -- 32 steps before the lane
  // can read cb -- so that one stream load holds up the waits of the record loads behind it
  // (loads complete in issue order) every few iterations instead of every iteration
  uint4 ca = make_uint4(0u, 0u, 0u, 0u), cb = make_uint4(0u, 0u, 0u, 0u);
  bool needb = false;
  auto load_chunk = [&](uint32_t ci) -> uint4 {
    if (4u * ci >= nwords) return make_uint4(0u, 0u, 0u, 0u);
    return stream_load(reinterpret_cast<const uint4*>(a.r + (size_t)ci * cstride + (size_t)(qwave + lane_id()) * 4));
  };
  // the words pos / 16 and pos / 16 + 1 (CVD_WALK_BUF: picked from the chunks at each use, so that
  // the chunks take 6 VGPRs more than the two words instead of 8; the words of a chunk past the
  // stream's end are never read for a step < N)
  auto cur_word = [&]() -> uint32_t {
    if constexpr (CVD_WALK_BUF == 0) return curw;
    const uint32_t i = (pos >> 4) & 3u;
    return i == 0u ? ca.x : i == 1u ? ca.y : i == 2u ? ca.z : ca.w;
  };
  auto nxt_word = [&]() -> uint32_t {
    if constexpr (CVD_WALK_BUF == 0) return nxtw;
    const uint32_t i = (pos >> 4) & 3u;
    return i == 0u ? ca.y : i == 1u ? ca.z : i == 2u ? ca.w : cb.x;
  };
  auto word_at = [&]() -> uint32_t { return cur_word() >> (2u * (pos & 15u)); };
  auto advance = [&]() {
    ++pos;
    if ((pos & 15u) == 0u) {
      if constexpr (CVD_WALK_BUF != 0) {
        if (((pos >> 4) & 3u) == 0u) {
          ca = cb;
          needb = true;
        }
      } else {
        curw = nxtw;
        need = true;
      }
    }
  };
  uint32_t R[2][4] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
  double lp = 0.0, lr = 0.0;
  BsCursor cur;
  cur.slot = -1; cur.pnx = -1; cur.hs = 0u; cur.hsn = 0u; cur.fb = 0u; cur.fw = 0u; cur.fb1 = 0u; cur.fw1 = 0u;
  cur.cand = false; cur.plp = 0.0; cur.pc = 1u; cur.half = 0u; cur.plp2 = 0.0; cur.pnx2 = -1;
  cur.masks(a);
  double plp2 = 0.0;
  auto two_steps = [&]() -> bool { return a.t2 != nullptr && pos + 2u <= N; };
  auto walk_prefetch = [&]() {
    const uint32_t x = __builtin_amdgcn_alignbit(nxt_word(), cur_word(), 2u * (pos & 15u));   // r of steps pos + 1, pos + 2
    if (two_steps() && a.t2c) {
      // the compact record (8 B, cvd_host.cpp t2c): both steps' log P̂1 as indices into the
      // model's value table, copied into LDS by the block; rows + 1 in 16 bits, c in 3
      uint32_t o;
      asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(o) : "v"(x & 15u), "v"((uint32_t)cur.slot << 7));
      const uint2 e = ld_off<uint2>(a.t2, o);
      const double* vt = reinterpret_cast<const double*>(reinterpret_cast<const char*>(dyn_lds()) + a.vtab_off);
      cur.plp = vt[e.x & 0xFFFu];
      plp2 = vt[(e.x >> 12) & 0xFFFu];
      cur.pnx = (int32_t)(__builtin_amdgcn_alignbit(e.y, e.x, 24u) & 0xFFFFu) | (int32_t)(((e.y >> 8) & 7u) << 28);
      cur.pc = ((e.y >> 11) & 0xFFFFu) | (((e.y >> 27) & 7u) << 28);
    } else if (two_steps()) {
      uint32_t o;
      asm("v_lshl_add_u32 %0, %1, 5, %2" : "=v"(o) : "v"(x & 15u), "v"((uint32_t)cur.slot << 9));
      const uint4 v = ld_off<uint4>(a.t2, o);
      const uint2 w = ld_off<uint2>(a.t2, o + 16u);
      cur.pc = w.y;
      cur.pnx = (int32_t)w.x;
      plp2 = __hiloint2double((int)v.w, (int)v.z);
      cur.plp = __hiloint2double((int)v.y, (int)v.x);
    } else {
      cur.prefetch_row(a, cur.slot, word_param(x & 3u));
    }
  };
  uint32_t mode = kWalkDone;
  int dec = 0;
  auto finished = [&]() -> bool {
    if (pos == N) return true;
    if (a.early && (pos & (uint32_t)(kEarlyEvery - 1)) == 0u) dec = early_decide(lp, lr, (int64_t)(N - pos), a.lt_min, a.lp_min);
    return dec != 0;
  };
  if (valid && N > 0u) {
    if constexpr (CVD_WALK_BUF != 0) {
      ca = load_chunk(0u);
      cb = load_chunk(1u);
    } else {
      curw = load_word(0u);
      nxtw = load_word(1u);
    }
    cur.slot = a.slot0;   // D_0 = 0 is a learned row: every lane starts walking
    walk_prefetch();
    mode = kWalkWalk;
  }
  uint32_t phw = 0u;   // layout phase of the ACS lanes' planes (wave-uniform)
  // one ACS step of the wave at phase PH (every lane computes; ACS lanes keep the result)
  auto acs_step = [&](auto phc) {
    constexpr int PH = decltype(phc)::value;
    const uint32_t rr = word_param(word_at() & 3u);
    uint32_t Nn[2][4], c;
    bs_step<PH, kUni>(a, cur, R, rr, Nn, c);
    if (mode == kWalkAcs) {
      lp += cur.template resolve<PH>(a, R, rr, a.lp_unseen);   // Pd_plotter.py:115, T = P̂1
      lr += s_lt[c];                                            // Pd_plotter.py:115, T = T_ref(1/2)
      advance();
      cur.template next<false>(a, 0u);
      if (finished()) {
        mode = kWalkDone;
        cur.slot = -1;
      } else if (cur.slot >= 0) {
        mode = kWalkWalk;
        walk_prefetch();
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) R[r][i] = Nn[r][i];
  };
  const uint32_t wmin = (uint32_t)a.walk_wmin, amin = (uint32_t)a.walk_amin;
  const int burst = a.walk_burst;
  for (int64_t it = 0, it_max = CVD_WALK_GUARD * ((int64_t)N + 1); it < it_max; ++it) {
    if constexpr (CVD_WALK_BUF != 0) {
      // (a burst moves a lane <= 16 steps, so a lane in word 0 of its chunk at one iteration's
      // top is past word 1 at a later top before it reaches word 3, where it reads cb)
      if (__ballot(needb && ((pos >> 4) & 3u) >= (uint32_t)CVD_WALK_BUF) != 0u && needb) {
        cb = load_chunk((pos >> 6) + 1u);
        needb = false;
      }
    } else if (need) {
      nxtw = load_word((pos >> 4) + 1u);
      need = false;
    }
    const uint64_t mA = __ballot(mode == kWalkAcs), mW = __ballot(mode == kWalkWalk);
    if ((mA | mW) == 0u) break;
    const uint32_t nA = (uint32_t)__popcll(mA), nW = (uint32_t)__popcll(mW);
    if (nW != 0u && (nA == 0u || nW >= wmin || nA < amin)) {
      for (int b = 0; b < burst; ++b) {
        if (mode == kWalkWalk) {
          // D_t is not a row: the lane joins the ACS steps with D_{t-1} = row `slot`, its
          // planes the row's image at the wave's phase; that step takes log P̂1 from
          // cur.plp with successor -1
          auto leave = [&]() {
            // (timing ablation, CVD_WALK_ABL & 8: a lane that leaves its rows skips that step and
            // walks on from row 0 -- the walk's own cost without the leavers' ACS steps; every
            // leave still advances the lane, so the loop ends)
            if (CVD_WALK_ABL & 8) {
              cur.slot = a.slot0;
              advance();
              if (finished()) {
                mode = kWalkDone;
                cur.slot = -1;
              } else {
                walk_prefetch();
              }
              return;
            }
            mode = kWalkAcs;
            cur.pnx = -1;
            const uint32_t ko = (uint32_t)cur.slot * (4u * kBsDkeyWords) + 32u * phw;
            const uint4 u = ld_off<uint4>(a.dkey, ko), v = ld_off<uint4>(a.dkey, ko + 16u);
            R[0][0] = u.x; R[0][1] = u.y; R[0][2] = u.z; R[0][3] = u.w;
            R[1][0] = v.x; R[1][1] = v.y; R[1][2] = v.z; R[1][3] = v.w;
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
    // two ACS steps of the wave (phases phw, phw + 1; phw is even); a lane the first sends
    // back to a walk waits out the second
    if (phw == 0u) {
      acs_step(IntC<0>{});
      acs_step(IntC<1>{});
    } else if (phw == 2u) {
      acs_step(IntC<2>{});
      acs_step(IntC<3>{});
    } else {
      acs_step(IntC<4>{});
      acs_step(IntC<5>{});
    }
    phw = phw == 4u ? 0u : phw + 2u;
  }
  // the guard is never reached (every iteration moves a lane); if it were, the partial
  // sums must not pass for results (k1b_walk)
  if (__ballot(mode != kWalkDone) != 0u && lane_id() == 0 && a.err) atomicOr(a.err, 1);
  if (valid && a.sums) {
    const int64_t qe = qwave + lane_id();
    a.sums[2 * qe] = lp;
    a.sums[2 * qe + 1] = lr;
  }
  early_final(dec, lp, lr);
  count_decisions_masked(vmask, vmask, lp, lr, a.counts);
}

// one wave's 64 sequences [64 gw, 64 gw + 64) through the lockstep loop, or walk mode
// chunked detection (a.ck_n > 0): a lane's 8 plane words into its chunk record
// (dword `off`: 0 = D at the chunk start, 8 = D at its end; both in layout phase 0)
__device__ __forceinline__ void ck_store(const ExpArgs& a, int64_t qwave, int32_t j, uint32_t off,
                                         const uint32_t (&R)[2][4]) {
  uint32_t l = lane_id();
  asm volatile("" : "+v"(l));   // (keeps the address arithmetic in the rarely taken branch)
  uint4* p = reinterpret_cast<uint4*>(a.ck_out + ((size_t)j * (size_t)a.nseq + (size_t)qwave + l) * kCkRecWords + off);
  p[0] = make_uint4(R[0][0], R[0][1], R[0][2], R[0][3]);
  p[1] = make_uint4(R[1][0], R[1][1], R[1][2], R[1][3]);
}

// (kCk: a chunked launch's unit; a separate instantiation, so that the unchunked loop keeps its
// registers and scalar state exactly)
template <uint64_t XM, bool kCk = false>
__device__ __forceinline__ void k1s_wave(const ExpArgs& a, int64_t gw, const double* s_lt, int32_t ck_j = 0) {
  constexpr bool kUni = xm_uni<6, XM>();
  if (a.walk || (a.mix && !kCk)) {
    // H1 and H2 waves alternate on every SIMD (k1b_body; lockstep too where a.mix: the units of
    // a persistent launch are taken in order, so that without it the first half of the launch
    // runs H1 waves only and the second H2 waves only)
    const int64_t half = ((a.nseq + 63) / 64 + 1) / 2, k = gw >> 1;
    if (gw < 2 * half) gw = ((gw ^ (gw >> 2)) & 1) ? half + k : k;
  }
  const int64_t qwave = gw * 64;
  const int64_t q = qwave + lane_id();
  const bool valid = q < a.nseq;
  const uint64_t vmask = __ballot(valid), hmask = __ballot(q < a.n_h1);
  if (a.walk && vmask != 0u && hmask == vmask) {
    k1s_walk<XM>(a, qwave, vmask, s_lt);
    return;
  }
  // (timing ablation, CVD_WALK_ABL & 4: a walk launch's lockstep (H2) waves do nothing)
  if ((CVD_WALK_ABL & 4) && a.walk) return;
  double lp = 0.0, lr = 0.0;
  if (valid) {
    uint32_t R[2][4] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};   // D_0 = 0
    double lpu = a.lp_unseen;
    asm volatile("" : "+v"(lpu));
    const int64_t N = a.N, nwords = (N + 15) / 16;
    const size_t cstride = (size_t)a.nseq * 4;
    // the steps this unit runs: all of them, or (chunked) its chunk [t_sum, t_end) after
    // t_sum - t_begin warm-up steps from D = 0 whose sums it drops (every bound but N a multiple
    // of 192: whole 16-B stream chunks and six-step groups, the planes in layout phase 0)
    constexpr bool ck = kCk;
    int64_t t_begin = 0, t_sum = 0, t_end = N;
    if (ck) {
      t_sum = (int64_t)ck_j * a.ck_len;
      t_end = min(N, t_sum + (int64_t)a.ck_len);
      t_begin = max((int64_t)0, t_sum - (int64_t)a.ck_warm);
    }
    uint32_t c4[4];
    auto load_chunk = [&](int64_t ci) {
      const uint32_t* rb = a.r + (size_t)ci * cstride + (size_t)qwave * 4;
      const uint4 v = 4 * ci < nwords ? stream_load(reinterpret_cast<const uint4*>(rb + lane_id() * 4u))
                                      : make_uint4(0u, 0u, 0u, 0u);
      c4[0] = v.x; c4[1] = v.y; c4[2] = v.z; c4[3] = v.w;
    };
    auto pick = [&](int64_t wi) -> uint32_t {
      const uint32_t e = (uint32_t)wi & 3u;
      const uint32_t v = e == 0u ? c4[0] : e == 1u ? c4[1] : e == 2u ? c4[2] : c4[3];
      return wi < nwords ? v : 0u;
    };
    // the received words as a 64-bit window (words wi, wi + 1) and the bit offset of the
    // next step in it (< 32 at the top of a six-step group): one funnel shift per group,
    // one bit-field extract per step
    int64_t wi = t_begin / 16;
    load_chunk(wi >> 2);
    uint32_t cw = pick(wi), nw = pick(wi + 1);
    uint32_t sh = 0u;
    // (the deep pipeline: the unchunked lockstep loop; chunk units keep the one-step cursor)
    constexpr bool kDeep = CVD_K1S_DEEP != 0 && !kCk;
    typename CursorOf<kDeep>::type cur;
    uint32_t Rp[2][4] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};   // (deep) D_{t-1}
    if constexpr (kDeep) {
      // "D_{-1}" is a known row whose record adds 0.0 (lp = 0.0 + 0.0 + term_0: the same bits)
      // and names D_0 = 0's row as its successor
      cur.slot = 0; cur.pnx = a.slot0; cur.plp = 0.0; cur.pc = 1u; cur.cand = false;
      cur.hs = 0u; cur.hsn = 0u; cur.fb = 0u; cur.fw = 0u; cur.fb1 = 0u; cur.fw1 = 0u; cur.half = 0u;
      cur.masks(a);
    } else {
      cur.start(a, word_param(cw & 3u), word_param((cw >> 2) & 3u));
    }
    if (CVD_K1S_ABL & 1) cur.h2wave = hmask == 0u;
    // (CVD_BS_ETAB2=2: each step reads the next step's e0 from LDS, so the zero test does not
    // wait for it)
    uint2 e0c = make_uint2(0u, 0u);
    if constexpr (CVD_BS_ETAB2 == 2 && !kDeep) e0c = bs_e0_at<0>(word_param(cw & 3u));
    auto step = [&](auto phc, uint32_t rr, uint32_t rn, uint32_t rnn) {
      constexpr int PH = decltype(phc)::value;
      uint32_t Nn[2][4], c;
      if constexpr (kDeep) {
        bs_acs<PH, kUni>(R, rr, Nn, c);
        int32_t ns;
        if constexpr (CVD_K1S_DEEP == 2) {
          const typename BsDeep::Prep h = cur.template prep<(PH + 1) % 6>(a, Nn);
          cur.fence_all(Nn, h.fo, h.fb1);
          lp += cur.template resolve_a<(PH + 5) % 6>(a, Rp, lpu, ns);   // Pd_plotter.py:115, T = P̂1 (step t - 1)
          lr += s_lt[c];                                                // Pd_plotter.py:115, T = T_ref(1/2)
          cur.template mid_b<PH>(a, ns, rr);
          cur.issue(a, h);
        } else {
          cur.fence_all(Nn);
          lp += cur.template resolve_a<(PH + 5) % 6>(a, Rp, lpu, ns);   // Pd_plotter.py:115, T = P̂1 (step t - 1)
          lr += s_lt[c];                                                // Pd_plotter.py:115, T = T_ref(1/2)
          cur.template mid_b<PH>(a, ns, rr);
          cur.template hash_ahead<(PH + 1) % 6>(a, Nn);
        }
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int i = 0; i < 4; ++i) Rp[r][i] = R[r][i];
      } else {
        if constexpr (CVD_BS_ETAB2 == 2) {
          const uint2 e0u = e0c;
          e0c = bs_e0_at<(PH + 1) % 6>(rn);   // the next step's (its word rn, its phase)
          bs_step<PH, kUni>(a, cur, R, rr, Nn, c, &e0u);
        } else {
          bs_step<PH, kUni>(a, cur, R, rr, Nn, c);
        }
#if CVD_K1S_PADV
        {   // (timing ablation, sums unchanged: CVD_K1S_PADV independent v_bitop3 per step, two chains)
          uint32_t x = Nn[0][0], y = Nn[1][0];
#pragma unroll
          for (int i = 0; i < CVD_K1S_PADV; ++i) {
            if (i & 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(y) : "v"(Nn[1][1]), "v"(Nn[0][2]));
            else asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(Nn[0][1]), "v"(Nn[1][2]));
          }
          asm volatile("" ::"v"(x), "v"(y));
        }
#endif
        lp += cur.template resolve<PH>(a, R, rr, lpu);   // Pd_plotter.py:115, T = P̂1
        lr += s_lt[c];                                   // Pd_plotter.py:115, T = T_ref(1/2) = c / 2^n
      }
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) R[r][i] = Nn[r][i];
      if constexpr (!kDeep) cur.next(a, rn, rnn);
    };
    int64_t t = t_begin;
    int grp = 0, dec = 0;
    // word k / 2 of the group's window as the step's parameter (kR16: bits k, k + 1 of win sit
    // at k + 5, k + 6 of w5 = win << 5, so (w5 >> (k + 1)) & 0x30 = 16 r)
    auto wk = [&](uint32_t win, uint32_t w5, auto kc) -> uint32_t {
      constexpr uint32_t k = decltype(kc)::value;
      if constexpr (kR16) return (w5 >> (k + 1)) & 0x30u;
      else return bits2(win, k);
    };
    auto w3 = [&](uint32_t win, uint32_t w5, auto kc) -> uint32_t {   // the T2 records' third word
      if constexpr (kK1sT2 || !kR16) return wk(win, w5, kc);
      else return 0u;
    };
    for (; t + 6 <= t_end; t += 6) {
      if (ck && t == t_sum) {   // (wave-uniform) the chunk's first summed step: D_t is its start
        ck_store(a, qwave, ck_j, 0u, R);
        lp = 0.0;
        lr = 0.0;
      }
      const uint32_t win = __builtin_amdgcn_alignbit(nw, cw, sh);
      const uint32_t w5 = kR16 ? win << 5 : 0u;
      step(IntC<0>{}, wk(win, w5, IntC<0>{}), wk(win, w5, IntC<2>{}), w3(win, w5, IntC<4>{}));
      step(IntC<1>{}, wk(win, w5, IntC<2>{}), wk(win, w5, IntC<4>{}), w3(win, w5, IntC<6>{}));
      step(IntC<2>{}, wk(win, w5, IntC<4>{}), wk(win, w5, IntC<6>{}), w3(win, w5, IntC<8>{}));
      step(IntC<3>{}, wk(win, w5, IntC<6>{}), wk(win, w5, IntC<8>{}), w3(win, w5, IntC<10>{}));
      step(IntC<4>{}, wk(win, w5, IntC<8>{}), wk(win, w5, IntC<10>{}), w3(win, w5, IntC<12>{}));
      step(IntC<5>{}, wk(win, w5, IntC<10>{}), wk(win, w5, IntC<12>{}), w3(win, w5, IntC<14>{}));
      sh += 12u;
      if (sh >= 32u) {
        sh -= 32u;
        ++wi;
        cw = nw;
        nw = pick(wi + 1);
        if (((wi + 1) & 3) == 3) load_chunk((wi + 2) >> 2);   // the word after nw opens a chunk
      }
      if (a.early && ++grp == kBsEarlyGroups) {
        grp = 0;
        // (deep: lp still lacks step t + 5's P̂1 term, so one more remaining increment)
        if (!dec) dec = early_decide(lp, lr, N - (t + 6) + (kDeep ? 1 : 0), a.lt_min, a.lp_min);
        if (__ballot(dec == 0) == 0) {   // every lane decided: the wave is done
          t = N;
          break;
        }
      }
    }
    // last 1-5 steps
    const int ntail = (int)(t_end - t);   // (0 after an early exit)
    if (t < t_end) {
      if (ck && t == t_sum) {   // (a last chunk of fewer than six steps)
        ck_store(a, qwave, ck_j, 0u, R);
        lp = 0.0;
        lr = 0.0;
      }
      const uint32_t win = __builtin_amdgcn_alignbit(nw, cw, sh);
      const uint32_t w5 = kR16 ? win << 5 : 0u;
      step(IntC<0>{}, wk(win, w5, IntC<0>{}), wk(win, w5, IntC<2>{}), w3(win, w5, IntC<4>{}));
      if (t + 1 < t_end) step(IntC<1>{}, wk(win, w5, IntC<2>{}), wk(win, w5, IntC<4>{}), w3(win, w5, IntC<6>{}));
      if (t + 2 < t_end) step(IntC<2>{}, wk(win, w5, IntC<4>{}), wk(win, w5, IntC<6>{}), w3(win, w5, IntC<8>{}));
      if (t + 3 < t_end) step(IntC<3>{}, wk(win, w5, IntC<6>{}), wk(win, w5, IntC<8>{}), w3(win, w5, IntC<10>{}));
      if (t + 4 < t_end) step(IntC<4>{}, wk(win, w5, IntC<8>{}), wk(win, w5, IntC<10>{}), w3(win, w5, IntC<12>{}));
    }
    if constexpr (kDeep) {   // the drain: the last step's lookup (Rp in that step's layout phase)
      int32_t ns;
      switch (ntail > 0 ? ntail - 1 : 5) {
        case 0: lp += cur.template resolve_a<0>(a, Rp, lpu, ns); break;
        case 1: lp += cur.template resolve_a<1>(a, Rp, lpu, ns); break;
        case 2: lp += cur.template resolve_a<2>(a, Rp, lpu, ns); break;
        case 3: lp += cur.template resolve_a<3>(a, Rp, lpu, ns); break;
        case 4: lp += cur.template resolve_a<4>(a, Rp, lpu, ns); break;
        default: lp += cur.template resolve_a<5>(a, Rp, lpu, ns); break;
      }
    }
    if (ck) {   // the chunk's record: D at its end (phase 0 unless it is the last) and its sums
      ck_store(a, qwave, ck_j, 8u, R);
      uint32_t l = lane_id();
      asm volatile("" : "+v"(l));
      double* ps = reinterpret_cast<double*>(
          a.ck_out + ((size_t)ck_j * (size_t)a.nseq + (size_t)qwave + l) * kCkRecWords + 16u);
      ps[0] = lp;
      ps[1] = lr;
      return;   // (the decisions: ck_combine_kernel)
    }
    if (a.sums) {
      const int64_t qe = qwave + lane_id();
      a.sums[2 * qe] = lp;
      a.sums[2 * qe + 1] = lr;
    }
    early_final(dec, lp, lr);
  }
  if constexpr (kCk) return;
  count_decisions_masked(vmask, hmask, lp, lr, a.counts);
}

// The block's LDS tables, then its waves' sequences: by block index, or -- a.wq set, the
// persistent launch of cvd_kernels.hip (one block per resident slot) -- from a work queue,
// each wave taking the next 64 sequences until none are left, so that a CU's waves finish
// together whatever their lookups cost and the LDS tables are filled once per block
template <uint64_t XM>
__device__ __forceinline__ void k1s_body(const ExpArgs& a, uint32_t blk) {
  __shared__ double s_lt[5];
  if (threadIdx.x <= 4) s_lt[threadIdx.x] = a.ltref[threadIdx.x];
  fill_filter_patterns();
  fill_bs_etab<XM>();
#if CVD_K1B_LDSF
  {   // the whole filter, 2 (fmask + 1) words, into dynamic LDS
    uint4* d = reinterpret_cast<uint4*>(dyn_lds());
    const uint4* g = reinterpret_cast<const uint4*>(a.filt);
    for (uint32_t i = threadIdx.x; i < (a.fmask + 1u) / 2u; i += blockDim.x) d[i] = g[i];
  }
  if (a.t2c) {   // the compact walk records' value table, after the filter
    double* d = reinterpret_cast<double*>(reinterpret_cast<char*>(dyn_lds()) + a.vtab_off);
    for (int32_t i = (int32_t)threadIdx.x; i < a.nvtab; i += (int32_t)blockDim.x) d[i] = a.vtab[i];
  }
#elif CVD_K1S_PF
  {   // the pre-filter, 2^kBsPfLog2Bits bits, into dynamic LDS
    uint4* d = reinterpret_cast<uint4*>(dyn_lds());
    const uint4* g = reinterpret_cast<const uint4*>(a.pf);
    for (uint32_t i = threadIdx.x; i < (1u << (cvd::kBsPfLog2Bits - 7)); i += blockDim.x) d[i] = g[i];
  }
#endif
  __syncthreads();
  // every wave leaves once the queue is past the last unit (no block barrier below)
  // units: waves of 64 sequences; walk mode's H1 / H2 interleave (k1s_wave) permutes
  // [0, 2 ceil(units / 2)), whose last unit may hold no sequence
  uint32_t nunits = (uint32_t)((a.nseq + 63) / 64);   // < 2^32 (host: grid and queue limits)
  if (a.walk || (a.mix && a.ck_n <= 0)) nunits = (nunits + 1u) & ~1u;
  // chunked: ck_n units (time chunks) per wave of sequences (no walk mode)
  const uint32_t ckn = a.ck_n > 0 ? (uint32_t)a.ck_n : 1u;
  nunits *= ckn;
  auto take = [&]() -> uint32_t {
    uint32_t u = 0u;
    if (lane_id() == 0) u = atomicAdd(a.wq, 1u);
    return __builtin_amdgcn_readfirstlane(u);
  };
  uint32_t u = a.wq ? take() : blk * (uint32_t)(kK1bBlock / 64) + (__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6);
  while (u < nunits) {
    if (CVD_K1S_CK && a.ck_n > 0) k1s_wave<XM, true>(a, (int64_t)(u / ckn), s_lt, (int32_t)(u % ckn));
    else k1s_wave<XM>(a, (int64_t)u, s_lt);
    if (!a.wq) break;
    u = take();
  }
}

template <uint64_t XM>
__device__ __forceinline__ void k1s_multi(const MultiArgs& ma) {
  const uint32_t b = blockIdx.x;
  int i = 0;
  uint32_t b0 = 0u;
  while (i + 1 < ma.nm && b >= ma.blk_end[i]) b0 = ma.blk_end[i++];   // scalar: blockIdx is uniform
  k1s_body<XM>(ma.a[i], b - b0);
}

// the specialised kernel's entries (cvd_rtc.cpp): the butterfly kernel, or for m = 6 its
// bit-sliced form when the model's tables are the bit-sliced ones
template <int m, uint64_t XM>
__device__ __forceinline__ void k1b_spec_entry(const ExpArgs& a) {
  if constexpr (CVD_K1B_BITSLICE && m == 6) k1s_body<XM>(a, blockIdx.x);
  else k1b_body<m, true, XM, false>(a, blockIdx.x);
}
template <int m, uint64_t XM>
__device__ __forceinline__ void k1b_spec_multi_entry(const MultiArgs& ma) {
  if constexpr (CVD_K1B_BITSLICE && m == 6) k1s_multi<XM>(ma);
  else k1b_multi<m, XM>(ma);
}

}  // namespace cvd_dev
