// Microbenchmark for the design study of DESIGN.md §11 (profiles/bitslice_acs_study.py):
// the m = 6 rate-1/2 Eq. 4-5 step (ACS + normalisation) in bit-sliced form -- 64 relative
// metrics as W = 4 bit-planes of two 32-bit registers per lane, in the rotating in-place
// layout -- on the GPU, one sequence per lane, received words from a per-lane xorshift.
// It times the step alone and writes each lane's final planes and step-minimum sum so the
// host can check them against the Python restatement (profiles/bitslice_acs_run.py).
// Not part of the product; built and run by profiles/bitslice_acs_run.py.
#include <hip/hip_runtime.h>
#include <cstdint>

constexpr int W = 4;

struct Masks {        // per phase and register: positions whose out(j,0) bit 0 / bit 1 is 1
  uint32_t o0[6][2], o1[6][2];
};

// positions p <-> p ^ 2^k in a register (k = 4: one rotate)
template <int K>
__device__ __forceinline__ uint32_t flip(uint32_t x) {
  if constexpr (K == 4) {
    return __builtin_amdgcn_alignbit(x, x, 16u);
  } else {
    constexpr uint32_t S = 1u << K;
    constexpr uint32_t m = K == 0 ? 0x55555555u : K == 1 ? 0x33333333u : K == 2 ? 0x0F0F0F0Fu : 0x00FF00FFu;
    return ((x >> S) & m) | ((x & m) << S);
  }
}

// d + e, e in {0, 1, 2} as planes (e0, e1), four planes (metrics <= 13)
__device__ __forceinline__ void add2(const uint32_t (&d)[W], uint32_t e0, uint32_t e1, uint32_t (&s)[W]) {
  s[0] = d[0] ^ e0;
  uint32_t c = d[0] & e0;
  s[1] = d[1] ^ e1 ^ c;
  c = (d[1] & e1) | (d[1] & c) | (e1 & c);
  s[2] = d[2] ^ c;
  c = d[2] & c;
  s[3] = d[3] ^ c;
}

__device__ __forceinline__ void min4(const uint32_t (&a)[W], const uint32_t (&b)[W], uint32_t (&o)[W]) {
  uint32_t lt = 0u;
#pragma unroll
  for (int i = 0; i < W; ++i) lt = (~a[i] & b[i]) | ((~a[i] | b[i]) & lt);   // a < b, LSB first
#pragma unroll
  for (int i = 0; i < W; ++i) o[i] = (a[i] & lt) | (b[i] & ~lt);
}

// one step at layout phase PH: partner location L5 = 0 (other register) or position bit L5-1
template <int PH>
__device__ __forceinline__ void step(uint32_t (&R)[2][W], uint32_t y, const Masks& mk, uint32_t& musum) {
  constexpr int L5tab[6] = {0, 5, 4, 3, 2, 1};
  constexpr int L5 = L5tab[PH];
  const uint32_t Y0 = 0u - (y & 1u), Y1 = 0u - ((y >> 1) & 1u);
  uint32_t N[2][W];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint32_t P[W];
#pragma unroll
    for (int i = 0; i < W; ++i) {
      if constexpr (L5 == 0) P[i] = R[1 - r][i];
      else P[i] = flip<L5 - 1>(R[r][i]);
    }
    const uint32_t d0 = mk.o0[PH][r] ^ Y0, d1 = mk.o1[PH][r] ^ Y1;   // bits of out(j,0) ^ y
    const uint32_t e0 = d0 ^ d1, e1 = d0 & d1;                        // e = popcount
    const uint32_t n1 = ~(d0 | d1);                                   // 2 - e: bit 0 = e0, bit 1 = (e == 0)
    uint32_t a[W], b[W];
    add2(R[r], e0, e1, a);
    add2(P, e0, n1, b);
    min4(a, b, N[r]);
  }
  // normalisation: the minimum is 0, 1 or 2
  uint32_t z = 0u, o = 0u;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    z |= ~(N[r][0] | N[r][1] | N[r][2] | N[r][3]);
    o |= N[r][0] & ~(N[r][1] | N[r][2] | N[r][3]);
  }
  const uint32_t mu = z ? 0u : (o ? 1u : 2u);
  musum += mu;
  // d - mu (mu in {0, 1, 2}): borrow chain
  const uint32_t m0 = 0u - (mu & 1u), m1 = 0u - (mu >> 1);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint32_t bw = 0u;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      const uint32_t mi = i == 0 ? m0 : i == 1 ? m1 : 0u;
      const uint32_t x = N[r][i];
      R[r][i] = x ^ mi ^ bw;
      bw = (~x & (mi | bw)) | (mi & bw);
    }
  }
}

__device__ __forceinline__ uint32_t xs(uint32_t& s) {
  s ^= s << 13; s ^= s >> 17; s ^= s << 5;
  return s;
}

extern "C" __global__ __launch_bounds__(256) void bitslice_acs(Masks mk, int64_t nsix, uint32_t seed,
                                                               uint32_t* out, int64_t nlanes) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t R[2][W] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
  uint32_t s = seed ^ (uint32_t)(q * 0x9E3779B9u), musum = 0u;
  if (s == 0u) s = 1u;
  for (int64_t t = 0; t < nsix; ++t) {
    uint32_t w = xs(s);   // 12 received words of 2 bits, six steps used
    step<0>(R, w & 3u, mk, musum);
    step<1>(R, (w >> 2) & 3u, mk, musum);
    step<2>(R, (w >> 4) & 3u, mk, musum);
    step<3>(R, (w >> 6) & 3u, mk, musum);
    step<4>(R, (w >> 8) & 3u, mk, musum);
    step<5>(R, (w >> 10) & 3u, mk, musum);
  }
  if (q < nlanes) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < W; ++i) out[q * 9 + r * W + i] = R[r][i];
    out[q * 9 + 8] = musum;
  }
}

// The same step with every 3-input function written as one v_bitop3_b32 (inline asm) and
// the 2-input ones as VOP2, as a hand-scheduled kernel would issue them: the count the
// design study's model gives (~100 VALU per step), against what the compiler makes of the
// plain form above.
#define BOP3(out, a, b, c, tt) asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:" #tt : "=v"(out) : "v"(a), "v"(b), "v"(c))

__device__ __forceinline__ void add2a(const uint32_t (&d)[W], uint32_t e0, uint32_t e1, uint32_t (&s)[W]) {
  s[0] = d[0] ^ e0;
  uint32_t c = d[0] & e0, c2;
  BOP3(s[1], d[1], e1, c, 0x96);     // xor3
  BOP3(c2, d[1], e1, c, 0xe8);       // maj
  s[2] = d[2] ^ c2;
  c = d[2] & c2;
  s[3] = d[3] ^ c;
}

__device__ __forceinline__ void min4a(const uint32_t (&a)[W], const uint32_t (&b)[W], uint32_t (&o)[W]) {
  uint32_t lt = 0u;
#pragma unroll
  for (int i = 0; i < W; ++i) BOP3(lt, a[i], b[i], lt, 0x8e);   // MAJ(~a, b, lt)
#pragma unroll
  for (int i = 0; i < W; ++i) o[i] = __builtin_amdgcn_ubfe(0u, 0u, 0u) | ((a[i] & lt) | (b[i] & ~lt));
}

template <int K>
__device__ __forceinline__ uint32_t flipa(uint32_t x) {
  if constexpr (K == 4) {
    return __builtin_amdgcn_alignbit(x, x, 16u);
  } else {
    constexpr uint32_t S = 1u << K;
    constexpr uint32_t m = K == 0 ? 0x55555555u : K == 1 ? 0x33333333u : K == 2 ? 0x0F0F0F0Fu : 0x00FF00FFu;
    const uint32_t hi = x >> S, lo = x << S;
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(hi), "v"(lo));   // (m & hi) | (~m & lo)
    return r;
  }
}

template <int PH>
__device__ __forceinline__ void stepa(uint32_t (&R)[2][W], uint32_t y, const Masks& mk, uint32_t& musum) {
  constexpr int L5tab[6] = {0, 5, 4, 3, 2, 1};
  constexpr int L5 = L5tab[PH];
  const uint32_t Y0 = 0u - (y & 1u), Y1 = 0u - ((y >> 1) & 1u);
  uint32_t N[2][W];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint32_t P[W];
#pragma unroll
    for (int i = 0; i < W; ++i) {
      if constexpr (L5 == 0) P[i] = R[1 - r][i];
      else P[i] = flipa<L5 - 1>(R[r][i]);
    }
    const uint32_t d0 = mk.o0[PH][r] ^ Y0, o1 = mk.o1[PH][r];
    uint32_t e0, e1, n1;
    BOP3(e0, d0, o1, Y1, 0x96);        // d0 ^ d1
    BOP3(e1, d0, o1, Y1, 0x60);        // d0 & (o1 ^ Y1)
    BOP3(n1, d0, o1, Y1, 0x09);        // ~(d0 | (o1 ^ Y1))
    uint32_t a[W], b[W];
    add2a(R[r], e0, e1, a);
    add2a(P, e0, n1, b);
    min4a(a, b, N[r]);
  }
  uint32_t zA, zB, oA, oB, tA, tB;
  asm("v_or3_b32 %0, %1, %2, %3" : "=v"(tA) : "v"(N[0][1]), "v"(N[0][2]), "v"(N[0][3]));
  asm("v_or3_b32 %0, %1, %2, %3" : "=v"(tB) : "v"(N[1][1]), "v"(N[1][2]), "v"(N[1][3]));
  zA = ~(tA | N[0][0]); zB = ~(tB | N[1][0]);
  oA = N[0][0] & ~tA; oB = N[1][0] & ~tB;
  const uint32_t mu = (zA | zB) ? 0u : ((oA | oB) ? 1u : 2u);
  musum += mu;
  const uint32_t m0 = 0u - (mu & 1u), m1 = 0u - (mu >> 1);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const uint32_t x0 = N[r][0], x1 = N[r][1], x2 = N[r][2], x3 = N[r][3];
    uint32_t b0, b1, b2;
    R[r][0] = x0 ^ m0;
    b0 = ~x0 & m0;
    BOP3(R[r][1], x1, m1, b0, 0x96);
    BOP3(b1, x1, m1, b0, 0x8e);        // MAJ(~x1, m1, b0)
    R[r][2] = x2 ^ b1;
    b2 = ~x2 & b1;
    R[r][3] = x3 ^ b2;
  }
}

extern "C" __global__ __launch_bounds__(256) void bitslice_acs_asm(Masks mk, int64_t nsix, uint32_t seed,
                                                                   uint32_t* out, int64_t nlanes) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t R[2][W] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
  uint32_t s = seed ^ (uint32_t)(q * 0x9E3779B9u), musum = 0u;
  if (s == 0u) s = 1u;
  for (int64_t t = 0; t < nsix; ++t) {
    uint32_t w = xs(s);
    stepa<0>(R, w & 3u, mk, musum);
    stepa<1>(R, (w >> 2) & 3u, mk, musum);
    stepa<2>(R, (w >> 4) & 3u, mk, musum);
    stepa<3>(R, (w >> 6) & 3u, mk, musum);
    stepa<4>(R, (w >> 8) & 3u, mk, musum);
    stepa<5>(R, (w >> 10) & 3u, mk, musum);
  }
  if (q < nlanes) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < W; ++i) out[q * 9 + r * W + i] = R[r][i];
    out[q * 9 + 8] = musum;
  }
}

// Third form: the step minimum known BEFORE the ACS.  A normalised vector has a zero
// state, whose better branch costs min(e, 2 - e) <= 1, so the new minimum mu is 0 or 1,
// and 0 exactly when some zero state has e in {0, 2} (bit 0 of e clear).  The ACS then
// adds E - mu in 4-bit two's complement (every candidate stays >= 0) and needs no
// normalisation pass.
__device__ __forceinline__ void add4s(const uint32_t (&d)[W], uint32_t b0, uint32_t b1, uint32_t b23,
                                      uint32_t (&s)[W]) {
  s[0] = d[0] ^ b0;
  uint32_t c = d[0] & b0, c1, c2;
  BOP3(s[1], d[1], b1, c, 0x96);
  BOP3(c1, d[1], b1, c, 0xe8);
  BOP3(s[2], d[2], b23, c1, 0x96);
  BOP3(c2, d[2], b23, c1, 0xe8);
  BOP3(s[3], d[3], b23, c2, 0x96);
}

template <int PH>
__device__ __forceinline__ void stepb(uint32_t (&R)[2][W], uint32_t y, const Masks& mk, uint32_t& musum) {
  constexpr int L5tab[6] = {0, 5, 4, 3, 2, 1};
  constexpr int L5 = L5tab[PH];
  const uint32_t Y0 = 0u - (y & 1u), Y1 = 0u - ((y >> 1) & 1u);
  uint32_t e0[2], e1[2], ez[2], hit = 0u;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const uint32_t d0 = mk.o0[PH][r] ^ Y0, o1 = mk.o1[PH][r];
    BOP3(e0[r], d0, o1, Y1, 0x96);      // bit 0 of e
    BOP3(e1[r], d0, o1, Y1, 0x60);      // bit 1 of e (e == 2)
    BOP3(ez[r], d0, o1, Y1, 0x09);      // e == 0
    uint32_t t, z;
    asm("v_or3_b32 %0, %1, %2, %3" : "=v"(t) : "v"(R[r][0]), "v"(R[r][1]), "v"(R[r][2]));
    BOP3(z, t, R[r][3], e0[r], 0x01);   // zero state with e in {0, 2}: ~t & ~d3 & ~e0
    hit |= z;
  }
  const uint32_t M = hit ? 0u : ~0u;    // mu = 1 on every position
  musum += hit ? 0u : 1u;
  uint32_t N[2][W];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    uint32_t P[W];
#pragma unroll
    for (int i = 0; i < W; ++i) {
      if constexpr (L5 == 0) P[i] = R[1 - r][i];
      else P[i] = flipa<L5 - 1>(R[r][i]);
    }
    // own branch e - mu, partner branch (2 - e) - mu, as 4-bit two's complement planes
    const uint32_t b0 = e0[r] ^ M;
    uint32_t a1, p1;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(a1) : "v"(M), "v"(ez[r]), "v"(e1[r]));   // M ? (e == 0) : e1
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(p1) : "v"(M), "v"(e1[r]), "v"(ez[r]));   // M ? (e == 2) : (e == 0)
    const uint32_t a23 = M & ez[r], p23 = M & e1[r];
    uint32_t a[W], b[W];
    add4s(R[r], b0, a1, a23, a);
    add4s(P, b0, p1, p23, b);
    min4a(a, b, N[r]);
  }
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int i = 0; i < W; ++i) R[r][i] = N[r][i];
}

extern "C" __global__ __launch_bounds__(256) void bitslice_acs_mu(Masks mk, int64_t nsix, uint32_t seed,
                                                                  uint32_t* out, int64_t nlanes) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t R[2][W] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
  uint32_t s = seed ^ (uint32_t)(q * 0x9E3779B9u), musum = 0u;
  if (s == 0u) s = 1u;
  for (int64_t t = 0; t < nsix; ++t) {
    uint32_t w = xs(s);
    stepb<0>(R, w & 3u, mk, musum);
    stepb<1>(R, (w >> 2) & 3u, mk, musum);
    stepb<2>(R, (w >> 4) & 3u, mk, musum);
    stepb<3>(R, (w >> 6) & 3u, mk, musum);
    stepb<4>(R, (w >> 8) & 3u, mk, musum);
    stepb<5>(R, (w >> 10) & 3u, mk, musum);
  }
  if (q < nlanes) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < W; ++i) out[q * 9 + r * W + i] = R[r][i];
    out[q * 9 + 8] = musum;
  }
}

// host launcher (ctypes): masks = o0[6][2] then o1[6][2]; returns the kernel's ms
extern "C" int bitslice_run(const uint32_t* masks, int64_t nsix, uint32_t seed, uint32_t* d_out, int64_t nlanes,
                            float* ms_out, int variant) {
  Masks mk;
  for (int ph = 0; ph < 6; ++ph)
    for (int r = 0; r < 2; ++r) {
      mk.o0[ph][r] = masks[ph * 2 + r];
      mk.o1[ph][r] = masks[12 + ph * 2 + r];
    }
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1;
  const unsigned grid = (unsigned)((nlanes + 255) / 256);
  hipEventRecord(e0, nullptr);
  if (variant == 2) hipLaunchKernelGGL(bitslice_acs_mu, dim3(grid), dim3(256), 0, nullptr, mk, nsix, seed, d_out, nlanes);
  else if (variant) hipLaunchKernelGGL(bitslice_acs_asm, dim3(grid), dim3(256), 0, nullptr, mk, nsix, seed, d_out, nlanes);
  else hipLaunchKernelGGL(bitslice_acs, dim3(grid), dim3(256), 0, nullptr, mk, nsix, seed, d_out, nlanes);
  hipEventRecord(e1, nullptr);
  if (hipEventSynchronize(e1) != hipSuccess) return -2;
  hipEventElapsedTime(ms_out, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
