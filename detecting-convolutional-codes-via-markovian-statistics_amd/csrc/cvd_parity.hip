// Parity-template baseline detector (comp_parity.py:90-128) for gfx950: the
// fraction of anchors t in [max_delay, N) at which the received streams satisfy
// a parity template  XOR_{(j, s) in S} y_j[t - s] = 0,  and the threshold test
// P̂ >= gamma, over the same bit-packed received-word buffers the Markov
// detector reads (include/cvd.h layout).
//
// One sequence per lane.  Per 32-bit word (SPW = 32/n steps) the n output
// streams are de-interleaved into SPW-bit words and shifted into a 64-bit
// window per output (bit 64 - SPW + i = y_j[t0 + i]); every template term is
// one shift of its output's window, so a word costs n de-interleaves, n window
// updates and one shift + xor per term, and SPW anchors are tested at once
// (popcount of the zero bits).  The kernel is a streaming read of the received
// words: 16-byte chunks per lane, two chunks in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <type_traits>

#include "../../include/cvd.h"
#include "cvd_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kMaxTerms = 32;   // per output stream (n = 3) / in total (n <= 2)
constexpr int kMaxOut = 3;

struct ParArgs {
  const uint32_t* r;
  int64_t N, nseq, n_h1;
  int64_t first;               // first anchor: max delay of the template
  double gamma;
  // n <= 2 (interleaved words): a term reads stream bit (n*t0 + n*i) - o,
  // o = n*s - j, as alignbit(hi, lo, sh) of word pair g: 0 = (cur, prev),
  // 1 = (prev, prev2), 2 = (cur, cur) for o <= 0; sh[g][k], cnt[g] terms.
  // n = 3 (de-interleaved): term k of output j shifts its 64-bit window by sh[j][k]
  uint32_t sh[kMaxOut][kMaxTerms];
  uint32_t mk[kMaxOut][kMaxTerms];   // n <= 2: all ones for a term, 0 for padding
  int32_t cnt[kMaxOut];
  int32_t* sat;
  int64_t* counts;
};

// bits 3i + j of x -> bit i (output j of step i)
__device__ __forceinline__ uint32_t output_bits3(uint32_t x, int j) {
  x = (x >> j) & 0x09249249u;
  x = (x | (x >> 2)) & 0x030C30C3u;
  x = (x | (x >> 4)) & 0x0300F00Fu;
  x = (x | (x >> 8)) & 0xFF0000FFu;
  return (x | (x >> 16)) & 0x000003FFu;
}

// n <= 2: T0 / T1 / T2 term slots of the word pairs (cur, prev) / (prev, prev2) /
// (cur, cur), unrolled with compile-time indices so the shift amounts and masks
// stay in SGPRs for the whole kernel; a padding slot has mask 0 (one bitop3
// P ^ (x & mask) per slot).  n = 3: uniform runtime loops.
template <int n, int T0 = 0, int T1 = 0, int T2 = 0>
__global__ __launch_bounds__(kBlock) void parity_kernel(ParArgs a) {
  constexpr int SPW = 32 / n;
  // anchor bits of a word: bit n*i for step i (n <= 2, interleaved), bit i (n = 3)
  constexpr uint32_t LANES = n == 1 ? ~0u : n == 2 ? 0x55555555u : 0x3FFu;
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = q < a.nseq;
  int64_t sat = 0;
  const int64_t N = a.N;
  if (valid) {
    const int64_t nwords = (N + SPW - 1) / SPW, nchunks = (nwords + 3) / 4;
    const uint4* rc = reinterpret_cast<const uint4*>(a.r) + q;
    const int64_t cs = a.nseq;   // uint4 stride between chunks of one sequence
    uint4 c0 = make_uint4(0u, 0u, 0u, 0u), c1 = c0, c2 = c0;
    if (nchunks > 0) c0 = rc[0];
    if (nchunks > 1) c1 = rc[cs];
    if (nchunks > 2) c2 = rc[2 * cs];
    uint32_t prev = 0u, prev2 = 0u;   // n <= 2: the two words before the current one
    uint64_t win[n == 3 ? 3 : 1];     // n = 3: per-output windows, bit 64 - SPW + i = y_j[t0 + i]
#pragma unroll
    for (int j = 0; j < (n == 3 ? 3 : 1); ++j) win[j] = 0ull;
    // one chunk (4 words); kEdge: mask the anchors outside [first, N)
    auto chunk = [&](const uint4& ch, int64_t c, auto edge) {
      constexpr bool kEdge = decltype(edge)::value;
      const uint32_t wv[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t cur = wv[e];
        uint32_t P = 0u;
        if constexpr (n <= 2) {
#pragma unroll
          for (int k = 0; k < T0; ++k) P ^= __builtin_amdgcn_alignbit(cur, prev, a.sh[0][k]) & a.mk[0][k];
#pragma unroll
          for (int k = 0; k < T1; ++k) P ^= __builtin_amdgcn_alignbit(prev, prev2, a.sh[1][k]) & a.mk[1][k];
#pragma unroll
          for (int k = 0; k < T2; ++k) P ^= __builtin_amdgcn_alignbit(cur, cur, a.sh[2][k]) & a.mk[2][k];
          prev2 = prev;
          prev = cur;
        } else {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            win[j] = (win[j] >> SPW) | ((uint64_t)output_bits3(cur, j) << (64 - SPW));
#pragma nounroll
            for (int k = 0; k < a.cnt[j]; ++k) P ^= (uint32_t)(win[j] >> a.sh[j][k]);
          }
        }
        uint32_t vm = LANES;
        if constexpr (kEdge) {
          // anchors of this word: first <= t0 + i < N
          const int64_t t0 = (4 * c + e) * SPW;
          const int64_t lo_i = a.first > t0 ? a.first - t0 : 0;
          const int64_t hi_i = N - t0 < SPW ? N - t0 : SPW;
          vm = 0u;
          for (int64_t i = lo_i; i < hi_i; ++i) vm |= 1u << (uint32_t)((n <= 2 ? n : 1) * i);
        }
        sat += __builtin_popcount(~P & vm);
      }
    };
    // chunks [0, head) may hold steps before the first anchor, chunks from
    // `tail` on steps at or after N; the body needs no masking
    constexpr int64_t CS = 4 * SPW;   // steps per chunk
    const int64_t head = (a.first + CS - 1) / CS, tail = N / CS;
    for (int64_t c = 0; c < nchunks; ++c) {
      const uint4 ch = c0;
      c0 = c1;
      c1 = c2;
      if (c + 3 < nchunks) c2 = rc[(c + 3) * cs];
      if (c < head || c >= tail) chunk(ch, c, std::true_type{});
      else chunk(ch, c, std::false_type{});
    }
    if (a.sat) a.sat[q] = (int32_t)sat;
  }
  // comp_parity.py:107-117: P̂ = satisfied / total (0.0 without anchors); H1 iff P̂ >= gamma
  const int64_t total = N > a.first ? N - a.first : 0;
  const double ph = total > 0 ? (double)sat / (double)total : 0.0;
  const bool h1 = q < a.n_h1;
  const bool ok = valid && (h1 ? (ph >= a.gamma) : !(ph >= a.gamma));
  const uint64_t b1 = __ballot(ok && h1), b2 = __ballot(ok && !h1);
  if ((threadIdx.x & 63) == 0) {
    if (b1) atomicAdd(reinterpret_cast<unsigned long long*>(a.counts), (unsigned long long)__popcll(b1));
    if (b2) atomicAdd(reinterpret_cast<unsigned long long*>(a.counts + 1), (unsigned long long)__popcll(b2));
  }
}

#define HIP_CHECK(x)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      cvd::set_error(std::string("HIP error '") + hipGetErrorString(e_) + "' at " #x);     \
      return CVD_E_HIP;                                                                   \
    }                                                                                     \
  } while (0)

}  // namespace

extern "C" int cvd_parity_detect(const uint32_t* d_r, int32_t n, int64_t N, int64_t nseq, int64_t n_h1,
                                 const int32_t* terms, int32_t n_terms, double gamma, int32_t* d_sat,
                                 int64_t* d_counts, void* stream) {
  if (n < 1 || n > kMaxOut || N < 0 || nseq < 0 || n_h1 < 0 || n_h1 > nseq || !d_counts ||
      (!d_r && N > 0 && nseq > 0) || n_terms < 1 || n_terms > kMaxOut * kMaxTerms || !terms) {
    cvd::set_error("bad parity_detect arguments (1 <= n <= 3, 1 <= n_terms <= 96)");
    return CVD_E_INVALID;
  }
  if (N > 0x7FFFFFFF) { cvd::set_error("parity_detect: N must fit 31 bits"); return CVD_E_INVALID; }
  const int spw = 32 / n;
  ParArgs a{};
  a.r = d_r; a.N = N; a.nseq = nseq; a.n_h1 = n_h1; a.gamma = gamma; a.sat = d_sat; a.counts = d_counts;
  int64_t first = 0;
  for (int e = 0; e < n_terms; ++e) {
    const int tj = terms[2 * e], ts = terms[2 * e + 1];
    const int smax = n <= 2 ? (64 + tj) / n : 64 - spw;   // n <= 2: o = n*s - j <= 64
    if (tj < 0 || tj >= n || ts < 0 || ts > smax) {
      cvd::set_error("parity_detect: term (j, s) needs 0 <= j < n and n*s - j <= 64 (n <= 2) / s <= 54 (n = 3)");
      return CVD_E_INVALID;
    }
    first = std::max<int64_t>(first, ts);
    if (n <= 2) {
      const int o = n * ts - tj;   // bits back from the anchor bit n*i
      const int g = o <= 0 ? 2 : o <= 32 ? 0 : 1;
      const uint32_t sh = o <= 0 ? (uint32_t)(-o) : o <= 32 ? (uint32_t)(32 - o) : (uint32_t)(64 - o);
      int& c = a.cnt[g];
      if (c >= kMaxTerms) { cvd::set_error("parity_detect: more than 32 terms per word pair"); return CVD_E_INVALID; }
      a.mk[g][c] = ~0u;
      a.sh[g][c++] = sh;
    } else {
      int& c = a.cnt[tj];
      if (c >= kMaxTerms) { cvd::set_error("parity_detect: more than 32 terms per output"); return CVD_E_INVALID; }
      a.sh[tj][c++] = (uint32_t)(64 - spw - ts);
    }
  }
  a.first = first;
  if (nseq == 0) return CVD_OK;
  const unsigned grid = (unsigned)((nseq + kBlock - 1) / kBlock);
  void (*kern)(ParArgs) = parity_kernel<3>;
  if (n <= 2) {
    // padded slot counts: T0 in {4, 8, 16, 32}, T1 in {0, 32}, T2 = 2
    const int c0 = a.cnt[0], c1 = a.cnt[1];
    const int T0 = c0 <= 4 ? 4 : c0 <= 8 ? 8 : c0 <= 16 ? 16 : 32;
    using K = void (*)(ParArgs);
    static const K k1[2][4] = {{parity_kernel<1, 4, 0, 2>, parity_kernel<1, 8, 0, 2>, parity_kernel<1, 16, 0, 2>,
                                parity_kernel<1, 32, 0, 2>},
                               {parity_kernel<1, 4, 32, 2>, parity_kernel<1, 8, 32, 2>, parity_kernel<1, 16, 32, 2>,
                                parity_kernel<1, 32, 32, 2>}};
    static const K k2[2][4] = {{parity_kernel<2, 4, 0, 2>, parity_kernel<2, 8, 0, 2>, parity_kernel<2, 16, 0, 2>,
                                parity_kernel<2, 32, 0, 2>},
                               {parity_kernel<2, 4, 32, 2>, parity_kernel<2, 8, 32, 2>, parity_kernel<2, 16, 32, 2>,
                                parity_kernel<2, 32, 32, 2>}};
    const int i0 = T0 == 4 ? 0 : T0 == 8 ? 1 : T0 == 16 ? 2 : 3;
    kern = (n == 1 ? k1 : k2)[c1 > 0 ? 1 : 0][i0];
    if (a.cnt[2] > 2) { cvd::set_error("parity_detect: duplicate terms"); return CVD_E_INVALID; }
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, a);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}
