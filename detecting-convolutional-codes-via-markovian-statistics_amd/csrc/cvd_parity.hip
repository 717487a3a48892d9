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

#include "../../include/cvd.h"
#include "cvd_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kMaxTerms = 64;
constexpr int kMaxOut = 3;

struct ParArgs {
  const uint32_t* r;
  int64_t N, nseq, n_h1;
  int64_t first;               // first anchor: max delay of the template
  double gamma;
  uint32_t sh[kMaxTerms];      // window shift of each term: 64 - SPW - s, grouped by output
  int32_t tbeg[kMaxOut + 1];   // terms of output j: [tbeg[j], tbeg[j+1])
  int32_t* sat;
  int64_t* counts;
};

// bits n*i + j of x -> bit i (output j of step i)
template <int n>
__device__ __forceinline__ uint32_t output_bits(uint32_t x, int j) {
  x >>= j;
  if constexpr (n == 1) {
    return x;
  } else if constexpr (n == 2) {
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    return (x | (x >> 8)) & 0x0000FFFFu;
  } else {
    static_assert(n == 3, "parity kernel: n in 1..3");
    x &= 0x09249249u;
    x = (x | (x >> 2)) & 0x030C30C3u;
    x = (x | (x >> 4)) & 0x0300F00Fu;
    x = (x | (x >> 8)) & 0xFF0000FFu;
    return (x | (x >> 16)) & 0x000003FFu;
  }
}

template <int n>
__global__ __launch_bounds__(kBlock) void parity_kernel(ParArgs a) {
  constexpr int SPW = 32 / n;
  constexpr uint32_t LOW = SPW == 32 ? ~0u : (1u << SPW) - 1u;
  const int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = q < a.nseq;
  int64_t sat = 0;
  const int64_t N = a.N;
  if (valid) {
    const int64_t nwords = (N + SPW - 1) / SPW, nchunks = (nwords + 3) / 4;
    const uint4* rc = reinterpret_cast<const uint4*>(a.r) + q;
    const int64_t cs = a.nseq;   // uint4 stride between chunks of one sequence
    uint4 cur = make_uint4(0u, 0u, 0u, 0u), nxt = cur;
    if (nchunks > 0) cur = rc[0];
    if (nchunks > 1) nxt = rc[cs];
    uint64_t win[n];
#pragma unroll
    for (int j = 0; j < n; ++j) win[j] = 0ull;
    for (int64_t c = 0; c < nchunks; ++c) {
      const uint4 ch = cur;
      cur = nxt;
      if (c + 2 < nchunks) nxt = rc[(c + 2) * cs];
      const uint32_t wv[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t t0 = (4 * c + e) * SPW;
        uint32_t P = 0u;
#pragma unroll
        for (int j = 0; j < n; ++j) {
          win[j] = (win[j] >> SPW) | ((uint64_t)output_bits<n>(wv[e], j) << (64 - SPW));
          for (int k = a.tbeg[j]; k < a.tbeg[j + 1]; ++k) P ^= (uint32_t)(win[j] >> a.sh[k]);
        }
        // anchors of this word: first <= t0 + i < N
        uint32_t vm = LOW;
        if (t0 < a.first) vm = a.first - t0 >= SPW ? 0u : vm & ~((1u << (a.first - t0)) - 1u);
        if (t0 + SPW > N) vm = t0 >= N ? 0u : vm & ((1u << (N - t0)) - 1u);
        sat += __builtin_popcount(~P & vm);
      }
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
      (!d_r && N > 0 && nseq > 0) || n_terms < 1 || n_terms > kMaxTerms || !terms) {
    cvd::set_error("bad parity_detect arguments (1 <= n <= 3, 1 <= n_terms <= 64)");
    return CVD_E_INVALID;
  }
  if (N > 0x7FFFFFFF) { cvd::set_error("parity_detect: N must fit 31 bits"); return CVD_E_INVALID; }
  const int spw = 32 / n;
  ParArgs a{};
  a.r = d_r; a.N = N; a.nseq = nseq; a.n_h1 = n_h1; a.gamma = gamma; a.sat = d_sat; a.counts = d_counts;
  int64_t first = 0;
  int k = 0;
  for (int j = 0; j < n; ++j) {
    a.tbeg[j] = k;
    for (int e = 0; e < n_terms; ++e) {
      const int tj = terms[2 * e], ts = terms[2 * e + 1];
      if (tj < 0 || tj >= n || ts < 0 || ts > 64 - spw) {
        cvd::set_error("parity_detect: term (j, s) needs 0 <= j < n and 0 <= s <= 64 - 32/n");
        return CVD_E_INVALID;
      }
      if (tj != j) continue;
      a.sh[k++] = (uint32_t)(64 - spw - ts);
      first = std::max<int64_t>(first, ts);
    }
  }
  for (int j = n; j <= kMaxOut; ++j) a.tbeg[j] = k;
  a.first = first;
  if (nseq == 0) return CVD_OK;
  const unsigned grid = (unsigned)((nseq + kBlock - 1) / kBlock);
  void (*kern)(ParArgs) = n == 1 ? parity_kernel<1> : n == 2 ? parity_kernel<2> : parity_kernel<3>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, a);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}
