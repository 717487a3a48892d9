// Device helpers of the host-layout metric vector shared by the P̂1 learning chain
// (cvd_learn.hip) and the GPU state enumeration (cvd_bfs.hip): the received word
// of step t of a pitch-1 stream, the Eq. 4-5 step in predecessor form on 2^m
// bytes, and the nibble packing of cvd::pack_nibbles (state s in nibble s % 8 of
// word s / 8).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cvd_chain {

__device__ __forceinline__ uint32_t word_at(const uint32_t* r, int64_t t, int n) {
  const int spw = 32 / n;
  return (r[t / spw] >> (n * (int)(t % spw))) & ((1u << n) - 1u);
}

// Eq. 4-5 in predecessor form (viterbi_markov.py:139-159): state x is reached from
// s = (x >> k) | (b << (m - k)) with input U = x & (2^k - 1); bm[r][s][U] = popcount(out ^ r)
template <int m, int k>
__device__ __forceinline__ void step_vec(uint8_t (&D)[1 << m], const uint8_t* bm_r) {
  constexpr int M = 1 << m, K = 1 << k;
  uint8_t nd[M];
  uint8_t mn = 255;
#pragma unroll
  for (int x = 0; x < M; ++x) {
    uint8_t best = 255;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      const int s = (x >> k) | (b << (m - k));
      const uint8_t v = (uint8_t)(D[s] + bm_r[s * K + (x & (K - 1))]);
      best = v < best ? v : best;
    }
    nd[x] = best;
    mn = best < mn ? best : mn;
  }
#pragma unroll
  for (int x = 0; x < M; ++x) D[x] = (uint8_t)(nd[x] - mn);
}

// host key layout (cvd::pack_nibbles): state s in nibble s % 8 of word s / 8
template <int m>
__device__ __forceinline__ void pack_key(const uint8_t (&D)[1 << m], uint32_t* out) {
  constexpr int M = 1 << m, NW = M >= 8 ? M / 8 : 1;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    uint32_t v = 0u;
#pragma unroll
    for (int s = 0; s < 8 && 8 * w + s < M; ++s) v |= (uint32_t)D[8 * w + s] << (4 * s);
    out[w] = v;
  }
}

template <int m>
__device__ __forceinline__ void unpack_key(const uint32_t* in, uint8_t (&D)[1 << m]) {
  constexpr int M = 1 << m;
#pragma unroll
  for (int s = 0; s < M; ++s) D[s] = (uint8_t)((in[s / 8] >> (4 * (s % 8))) & 15u);
}

}  // namespace cvd_chain
