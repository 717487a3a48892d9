// P̂1 learning chain on the GPU.
//
// Reference: Pd_plotter.py:143-167 (learn_P1_empirical): ONE long G1-encoded
// chain D_0..D_L of the Eq. 4-5 recursion on the learning stream; the state
// index is the order of first visit; counts C[i][r] over t in [learn_burn, L).
// The chain is sequential in t, but its input (the received words) is
// counter-based, so every step's word is known up front, and the relative-
// metric recursion forgets its start: two chains started from different
// metric vectors merge once their survivor paths do (the min-plus product of
// the steps' transfer matrices becomes rank one).  So the chain is cut into
// blocks, one per lane; each lane starts `warm` steps before its block from
// D = 0 and walks through its block (speculative), and the block boundaries are
// then VERIFIED: block b is exact iff block b-1 is exact and its end state
// equals the state block b computed at its start.  Blocks that fail are re-run
// from their predecessor's end state (a pass fixes at least the first failing
// block, so the loop terminates; with a few hundred warm-up steps it never
// runs in practice).  The result is identical to the sequential chain.
//
// Sparse models (non-enumerable codes): the chain writes every
// D_t as a nibble-packed key; first visits come from a stable radix sort of
// (64-bit key hash, t) -- equal hashes are checked key by key, and a collision
// (two keys, one hash) re-runs the sort with another hash seed -- then a scan
// over t numbers the first visits in t order (= the host map's insertion
// order), and counts are integer atomics.  Dense models walk the BFS automaton
// (next index per received word) the same way.
//
// The host then computes successors and the P̂1 rows exactly as for the host
// chain (cvd_host.cpp), so the model is bit-identical.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/cvd.h"
#include "cvd_common.h"
#include "cvd_chain.h"
#include "cvd_internal.h"

using namespace cvd;
using namespace cvd_chain;

#define LHIP(x)                                                                           \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      set_error(std::string("HIP error '") + hipGetErrorString(e_) + "' at " #x);          \
      return e_ == hipErrorOutOfMemory ? CVD_E_CAPACITY : CVD_E_HIP;                      \
    }                                                                                     \
  } while (0)

namespace {

constexpr int kLB = 256;

struct ChainArgs {
  const uint32_t* r;       // learning stream, word w at r[w] (pitch 1), steps_per_word(n) steps per word
  int64_t L, blen, warm, nblocks;
  const int32_t* list;     // blocks to run (nullptr: block = thread index)
  int64_t nlist;
  const uint32_t* start;   // exact start state of list[i] (nullptr: speculative from D = 0)
  int32_t seq;             // 1: one lane runs list[0..nlist) in order, each block from its
                           // predecessor's end (the bounded sequential tail of run_chain)
  uint32_t* states;        // sparse: [(L+1)][NW] keys; dense: [(L+1)] indices
  uint32_t* ends;          // [nblocks][NW or 1]: state at the block's end
  const int32_t* next;     // dense: [S][R] automaton
  const uint8_t* bm;       // sparse: [R][M][K] branch metrics popcount(out(s, U) ^ r), staged in LDS
};

template <int m, int k, int n>
__global__ __launch_bounds__(kLB) void chain_sparse_kernel(ChainArgs a) {
  constexpr int M = 1 << m, K = 1 << k, R = 1 << n, NW = M >= 8 ? M / 8 : 1;
  __shared__ uint8_t s_bm[R * M * K];
  for (int j = threadIdx.x; j < R * M * K; j += kLB) s_bm[j] = a.bm[j];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kLB + threadIdx.x;
  const int64_t nb = a.list ? a.nlist : a.nblocks;
  if (i >= nb || (a.seq && i > 0)) return;
  // seq: this lane walks every listed block in order; block list[j] starts from
  // the end state the lane has just written for list[j] - 1
  for (int64_t j = a.seq ? 0 : i; j < (a.seq ? nb : i + 1); ++j) {
    const int64_t b = a.list ? a.list[j] : j;
    const int64_t s0 = b * a.blen, e0 = min(s0 + a.blen, a.L);
    uint8_t D[M];
    int64_t t;
    if (a.seq) {
      unpack_key<m>(a.ends + (size_t)(b - 1) * NW, D);
      t = s0;
    } else if (a.start) {
      unpack_key<m>(a.start + j * NW, D);
      t = s0;
    } else {
#pragma unroll
      for (int x = 0; x < M; ++x) D[x] = 0;
      t = max((int64_t)0, s0 - a.warm);
      for (; t < s0; ++t) step_vec<m, k>(D, s_bm + word_at(a.r, t, n) * (M * K));
    }
    for (; t < e0; ++t) {
      pack_key<m>(D, a.states + (size_t)t * NW);
      step_vec<m, k>(D, s_bm + word_at(a.r, t, n) * (M * K));
    }
    pack_key<m>(D, a.ends + (size_t)b * NW);
    if (e0 == a.L) pack_key<m>(D, a.states + (size_t)a.L * NW);
  }
}

template <int n>
__global__ __launch_bounds__(kLB) void chain_dense_kernel(ChainArgs a) {
  constexpr int R = 1 << n;
  const int64_t i = (int64_t)blockIdx.x * kLB + threadIdx.x;
  const int64_t nb = a.list ? a.nlist : a.nblocks;
  if (i >= nb || (a.seq && i > 0)) return;
  for (int64_t j = a.seq ? 0 : i; j < (a.seq ? nb : i + 1); ++j) {
    const int64_t b = a.list ? a.list[j] : j;
    const int64_t s0 = b * a.blen, e0 = min(s0 + a.blen, a.L);
    int32_t s;
    int64_t t;
    if (a.seq) {
      s = (int32_t)a.ends[b - 1];
      t = s0;
    } else if (a.start) {
      s = (int32_t)a.start[j];
      t = s0;
    } else {
      s = 0;   // D_0 = 0 is BFS index 0
      t = max((int64_t)0, s0 - a.warm);
      for (; t < s0; ++t) s = a.next[(size_t)s * R + word_at(a.r, t, n)];
    }
    for (; t < e0; ++t) {
      a.states[t] = (uint32_t)s;
      s = a.next[(size_t)s * R + word_at(a.r, t, n)];
    }
    a.ends[b] = (uint32_t)s;
    if (e0 == a.L) a.states[a.L] = (uint32_t)s;
  }
}

// bad[b] = block b's start state differs from block b-1's end state (b >= 1)
__global__ void verify_kernel(const uint32_t* states, const uint32_t* ends, int64_t blen, int64_t nblocks, int nw,
                              uint8_t* bad) {
  const int64_t b = (int64_t)blockIdx.x * kLB + threadIdx.x;
  if (b >= nblocks) return;
  uint8_t d = 0;
  if (b > 0)
    for (int w = 0; w < nw; ++w) d |= states[(size_t)(b * blen) * nw + w] != ends[(size_t)(b - 1) * nw + w];
  bad[b] = d;
}

__global__ void gather_starts_kernel(const uint32_t* ends, const int32_t* list, int64_t nlist, int nw,
                                     uint32_t* start) {
  const int64_t i = (int64_t)blockIdx.x * kLB + threadIdx.x;
  if (i >= nlist) return;
  for (int w = 0; w < nw; ++w) start[i * nw + w] = ends[(size_t)(list[i] - 1) * nw + w];
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void hash_kernel(const uint32_t* keys, int64_t n, int nw, uint64_t seed, uint64_t* h, uint32_t* v) {
  const int64_t t = (int64_t)blockIdx.x * kLB + threadIdx.x;
  if (t >= n) return;
  uint64_t x = seed;
  for (int w = 0; w < nw; w += 2) {
    const uint64_t lo = keys[(size_t)t * nw + w], hi = w + 1 < nw ? keys[(size_t)t * nw + w + 1] : 0u;
    x = mix64(x ^ (lo | (hi << 32)));
  }
  h[t] = x;
  v[t] = (uint32_t)t;
}

// sorted (hs, vs): segment heads, first visits, key check of equal hashes
__global__ void heads_kernel(const uint64_t* hs, const uint32_t* vs, int64_t n, const uint32_t* keys, int nw,
                             uint32_t* isfirst, uint32_t* headpos, uint32_t* collision) {
  const int64_t i = (int64_t)blockIdx.x * kLB + threadIdx.x;
  if (i >= n) return;
  const bool head = i == 0 || hs[i] != hs[i - 1];
  if (head) {
    isfirst[vs[i]] = 1u;
  } else {
    uint32_t d = 0u;
    for (int w = 0; w < nw; ++w) d |= keys[(size_t)vs[i] * nw + w] ^ keys[(size_t)vs[i - 1] * nw + w];
    if (d) atomicOr(collision, 1u);
  }
  headpos[i] = head ? (uint32_t)i : 0u;
}

__global__ void index_kernel(const uint32_t* vs, const uint32_t* segstart, const uint32_t* rowof, int64_t n,
                             uint32_t* idx) {
  const int64_t i = (int64_t)blockIdx.x * kLB + threadIdx.x;
  if (i >= n) return;
  idx[vs[i]] = rowof[vs[segstart[i]]];
}

__global__ void rowkeys_kernel(const uint32_t* keys, const uint32_t* isfirst, const uint32_t* rowof, int64_t n,
                               int nw, uint32_t* rowkeys) {
  const int64_t t = (int64_t)blockIdx.x * kLB + threadIdx.x;
  if (t >= n || !isfirst[t]) return;
  for (int w = 0; w < nw; ++w) rowkeys[(size_t)rowof[t] * nw + w] = keys[(size_t)t * nw + w];
}

__global__ void count_kernel(const uint32_t* r, const uint32_t* idx, int64_t burn, int64_t L, int n,
                             uint32_t* cnt) {
  const int64_t t = burn + (int64_t)blockIdx.x * kLB + threadIdx.x;
  if (t >= L) return;
  atomicAdd(&cnt[(size_t)idx[t] * (1u << n) + word_at(r, t, n)], 1u);
}

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + kLB - 1) / kLB); }

using SparseKernel = void (*)(ChainArgs);
SparseKernel pick_sparse(int m, int k, int n) {
  if (k == 1 && n == 2) {
    switch (m) {
      case 2: return chain_sparse_kernel<2, 1, 2>;
      case 3: return chain_sparse_kernel<3, 1, 2>;
      case 4: return chain_sparse_kernel<4, 1, 2>;
      case 5: return chain_sparse_kernel<5, 1, 2>;
      case 6: return chain_sparse_kernel<6, 1, 2>;
    }
  }
  if (m == 4 && k == 2 && n == 3) return chain_sparse_kernel<4, 2, 3>;
  return nullptr;
}

struct DevGuard {
  int cur = 0;
  DevGuard() { (void)hipGetDevice(&cur); }
  ~DevGuard() { (void)hipSetDevice(cur); }
};

// stream-ordered scratch allocations, freed on every return path
struct Scratch {
  hipStream_t st;
  std::vector<void*> ptrs;
  explicit Scratch(hipStream_t s) : st(s) {}
  template <typename T>
  hipError_t alloc(T*& p, size_t count) {
    void* q = nullptr;
    hipError_t e = hipMallocAsync(&q, std::max<size_t>(count, 1) * sizeof(T), st);
    if (e == hipSuccess) ptrs.push_back(q);
    p = static_cast<T*>(q);
    return e;
  }
  ~Scratch() {
    (void)hipStreamSynchronize(st);
    for (void* p : ptrs) (void)hipFreeAsync(p, st);
    (void)hipStreamSynchronize(st);
  }
};

int64_t env_int(const char* name, int64_t def) {
  const char* e = std::getenv(name);
  return e && e[0] ? std::atoll(e) : def;
}

// Speculative chain + boundary verification + re-runs (see file comment).
// states_per_t = NW (sparse keys) or 1 (dense indices).
int run_chain(ChainArgs a, int nw, void (*kern)(ChainArgs), size_t lds, hipStream_t st, Scratch& sc,
              LearnStats* stats) {
  a.nblocks = (a.L + a.blen - 1) / a.blen;
  a.list = nullptr; a.start = nullptr; a.nlist = 0; a.seq = 0;
  hipLaunchKernelGGL(kern, dim3(grid_of(a.nblocks)), dim3(kLB), lds, st, a);
  LHIP(hipGetLastError());
  uint8_t* bad = nullptr;
  int32_t* d_list = nullptr;
  uint32_t* d_start = nullptr;
  LHIP(sc.alloc(bad, (size_t)a.nblocks));
  LHIP(sc.alloc(d_list, (size_t)a.nblocks));
  LHIP(sc.alloc(d_start, (size_t)a.nblocks * nw));
  std::vector<uint8_t> h_bad((size_t)a.nblocks);
  std::vector<int32_t> list;
  // parallel re-run passes before the sequential tail (CVD_LEARN_MAX_PASSES: tests)
  const int64_t max_passes = std::max<int64_t>(0, env_int("CVD_LEARN_MAX_PASSES", 8));
  for (int pass = 0;; ++pass) {
    hipLaunchKernelGGL(verify_kernel, dim3(grid_of(a.nblocks)), dim3(kLB), 0, st, a.states, a.ends, a.blen,
                       a.nblocks, nw, bad);
    LHIP(hipGetLastError());
    LHIP(hipMemcpyAsync(h_bad.data(), bad, h_bad.size(), hipMemcpyDeviceToHost, st));
    LHIP(hipStreamSynchronize(st));
    list.clear();
    for (int64_t b = 0; b < a.nblocks; ++b)
      if (h_bad[(size_t)b]) list.push_back((int32_t)b);
    if (stats) {
      if (pass == 0) stats->mismatched_blocks = (int64_t)list.size();
      stats->fix_passes = pass;
    }
    if (list.empty()) return CVD_OK;
    // each pass makes the first failing block exact (its predecessor is); to stay
    // bounded when mismatches cascade, re-run from the first failing block to the
    // end once the passes exceed a few
    if (pass >= max_passes) {
      // sequential tail: ONE launch in which one lane re-runs every block from the
      // first failing one to the end, in order, each from its predecessor's end
      // (bounded: one kernel, L - first * blen steps; timed in LearnStats)
      const auto t0 = std::chrono::steady_clock::now();
      const int32_t first = list.front();
      list.clear();
      for (int64_t b = first; b < a.nblocks; ++b) list.push_back((int32_t)b);
      LHIP(hipMemcpyAsync(d_list, list.data(), list.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
      ChainArgs f = a;
      f.list = d_list; f.nlist = (int64_t)list.size(); f.start = nullptr; f.seq = 1;
      hipLaunchKernelGGL(kern, dim3(1), dim3(kLB), lds, st, f);
      LHIP(hipGetLastError());
      LHIP(hipStreamSynchronize(st));
      if (stats) {
        stats->sequential_blocks = (int64_t)list.size();
        stats->sequential_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      }
      return CVD_OK;
    }
    LHIP(hipMemcpyAsync(d_list, list.data(), list.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(gather_starts_kernel, dim3(grid_of((int64_t)list.size())), dim3(kLB), 0, st, a.ends, d_list,
                       (int64_t)list.size(), nw, d_start);
    ChainArgs f = a;
    f.list = d_list; f.nlist = (int64_t)list.size(); f.start = d_start;
    hipLaunchKernelGGL(kern, dim3(grid_of(f.nlist)), dim3(kLB), lds, st, f);
    LHIP(hipGetLastError());
  }
}

void chain_geometry(int64_t L, ChainArgs& a) {
  // ~32k lanes (blocks), at least 256 steps each; warm-up before every block
  a.blen = std::max<int64_t>(env_int("CVD_LEARN_BLOCK", 0), 0);
  if (a.blen == 0) a.blen = std::max<int64_t>(256, (L + 32767) / 32768);
  a.warm = std::max<int64_t>(0, env_int("CVD_LEARN_WARM", 512));
}

int learn_stream(const CodeDesc& dec, int64_t L, uint64_t seed, double p, hipStream_t st, Scratch& sc,
                 uint32_t*& d_r) {
  const int64_t spw = 32 / dec.n;
  const int64_t words = (((L + spw - 1) / spw) + 3) / 4 * 4;
  LHIP(sc.alloc(d_r, (size_t)words));
  // the learning chain's stream: encoder = decoder G1, seq 0, CVD_LEARN_TAG (cvd_model_create)
  return launch_generate(dec, (uint32_t)seed, (uint32_t)(seed >> 32), kLearnTag, noise_threshold(p), L, 1, 0, 1,
                         d_r, 1, 0, 1, st);
}

std::vector<uint8_t> bm_table(const CodeDesc& d) {
  const int M = 1 << d.m, K = 1 << d.k, R = 1 << d.n;
  std::vector<uint8_t> bm((size_t)R * M * K);
  for (int r = 0; r < R; ++r)
    for (int s = 0; s < M; ++s)
      for (int U = 0; U < K; ++U)
        bm[((size_t)r * M + s) * K + U] = (uint8_t)__builtin_popcount(enc_out(d, (uint32_t)s, (uint32_t)U) ^ (uint32_t)r);
  return bm;
}

}  // namespace

int cvd::device_learn_sparse(const CodeDesc& dec, int64_t L, int64_t burn, uint64_t seed, double p, int device,
                             void* stream, std::vector<uint8_t>& keys_out, std::vector<int64_t>& cnt_out,
                             int64_t& S_out, LearnStats* stats) {
  const int m = dec.m, k = dec.k, n = dec.n, M = 1 << m, R = 1 << n, nw = M >= 8 ? M / 8 : 1;
  if (!pick_sparse(m, k, n)) { set_error("GPU learning: unsupported code shape"); return CVD_E_UNSUPPORTED; }
  if (L < 1 || L >= ((int64_t)1 << 31)) { set_error("GPU learning: learn_len must be in [1, 2^31)"); return CVD_E_UNSUPPORTED; }
  DevGuard guard;
  LHIP(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  Scratch sc(st);
  uint32_t* d_r = nullptr;
  int rc = learn_stream(dec, L, seed, p, st, sc, d_r);
  if (rc) return rc;
  const std::vector<uint8_t> bm = bm_table(dec);
  uint8_t* d_bm = nullptr;
  LHIP(sc.alloc(d_bm, bm.size()));
  LHIP(hipMemcpyAsync(d_bm, bm.data(), bm.size(), hipMemcpyHostToDevice, st));
  ChainArgs a{};
  a.r = d_r; a.L = L;
  chain_geometry(L, a);
  const int64_t nbl = (L + a.blen - 1) / a.blen;
  LHIP(sc.alloc(a.states, (size_t)(L + 1) * nw));
  LHIP(sc.alloc(a.ends, (size_t)nbl * nw));
  a.bm = d_bm;
  rc = run_chain(a, nw, pick_sparse(m, k, n), 0, st, sc, stats);
  if (rc) return rc;

  // first visits: stable radix sort of (hash(key_t), t)
  const int64_t nt = L + 1;
  uint64_t *h = nullptr, *hs = nullptr;
  uint32_t *v = nullptr, *vs = nullptr, *isfirst = nullptr, *headpos = nullptr, *segstart = nullptr, *rowof = nullptr,
           *idx = nullptr, *coll = nullptr;
  LHIP(sc.alloc(h, (size_t)nt)); LHIP(sc.alloc(hs, (size_t)nt));
  LHIP(sc.alloc(v, (size_t)nt)); LHIP(sc.alloc(vs, (size_t)nt));
  LHIP(sc.alloc(isfirst, (size_t)nt)); LHIP(sc.alloc(headpos, (size_t)nt));
  LHIP(sc.alloc(segstart, (size_t)nt)); LHIP(sc.alloc(rowof, (size_t)nt));
  LHIP(sc.alloc(idx, (size_t)nt)); LHIP(sc.alloc(coll, 1));
  size_t tmp_sort = 0, tmp_scan1 = 0, tmp_scan2 = 0;
  LHIP(rocprim::radix_sort_pairs(nullptr, tmp_sort, h, hs, v, vs, (size_t)nt, 0, 64, st));
  LHIP(rocprim::inclusive_scan(nullptr, tmp_scan1, headpos, segstart, (size_t)nt, rocprim::maximum<uint32_t>(), st));
  LHIP(rocprim::exclusive_scan(nullptr, tmp_scan2, isfirst, rowof, 0u, (size_t)nt, rocprim::plus<uint32_t>(), st));
  void* tmp = nullptr;
  LHIP(sc.alloc(reinterpret_cast<uint8_t*&>(tmp), std::max({tmp_sort, tmp_scan1, tmp_scan2})));
  uint64_t hseed = 0x243F6A8885A308D3ull;
  uint32_t h_coll = 1;
  for (int attempt = 0; h_coll && attempt < 4; ++attempt, hseed = hseed * 0x9E3779B97F4A7C15ull + 1) {
    hipLaunchKernelGGL(hash_kernel, dim3(grid_of(nt)), dim3(kLB), 0, st, a.states, nt, nw, hseed, h, v);
    size_t ts = tmp_sort;
    LHIP(rocprim::radix_sort_pairs(tmp, ts, h, hs, v, vs, (size_t)nt, 0, 64, st));
    LHIP(hipMemsetAsync(isfirst, 0, (size_t)nt * sizeof(uint32_t), st));
    LHIP(hipMemsetAsync(coll, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(heads_kernel, dim3(grid_of(nt)), dim3(kLB), 0, st, hs, vs, nt, a.states, nw, isfirst, headpos,
                       coll);
    LHIP(hipGetLastError());
    LHIP(hipMemcpyAsync(&h_coll, coll, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    LHIP(hipStreamSynchronize(st));
    if (stats) stats->hash_attempts = attempt + 1;
  }
  if (h_coll) { set_error("GPU learning: persistent 64-bit key hash collisions"); return CVD_E_STATE; }
  size_t t1 = tmp_scan1, t2 = tmp_scan2;
  LHIP(rocprim::inclusive_scan(tmp, t1, headpos, segstart, (size_t)nt, rocprim::maximum<uint32_t>(), st));
  LHIP(rocprim::exclusive_scan(tmp, t2, isfirst, rowof, 0u, (size_t)nt, rocprim::plus<uint32_t>(), st));
  uint32_t last[2] = {0, 0};
  LHIP(hipMemcpyAsync(&last[0], rowof + (nt - 1), sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  LHIP(hipMemcpyAsync(&last[1], isfirst + (nt - 1), sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  LHIP(hipStreamSynchronize(st));
  const int64_t S = (int64_t)last[0] + last[1];
  hipLaunchKernelGGL(index_kernel, dim3(grid_of(nt)), dim3(kLB), 0, st, vs, segstart, rowof, nt, idx);
  uint32_t *rowkeys = nullptr, *cnt = nullptr;
  LHIP(sc.alloc(rowkeys, (size_t)S * nw));
  LHIP(sc.alloc(cnt, (size_t)S * R));
  LHIP(hipMemsetAsync(cnt, 0, (size_t)S * R * sizeof(uint32_t), st));
  hipLaunchKernelGGL(rowkeys_kernel, dim3(grid_of(nt)), dim3(kLB), 0, st, a.states, isfirst, rowof, nt, nw, rowkeys);
  if (L > burn)
    hipLaunchKernelGGL(count_kernel, dim3(grid_of(L - burn)), dim3(kLB), 0, st, d_r, idx, burn, L, n, cnt);
  LHIP(hipGetLastError());
  std::vector<uint32_t> h_keys((size_t)S * nw), h_cnt((size_t)S * R);
  LHIP(hipMemcpyAsync(h_keys.data(), rowkeys, h_keys.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  LHIP(hipMemcpyAsync(h_cnt.data(), cnt, h_cnt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  LHIP(hipStreamSynchronize(st));
  keys_out.assign((size_t)S * M, 0);
  for (int64_t s = 0; s < S; ++s)
    for (int x = 0; x < M; ++x)
      keys_out[(size_t)s * M + x] = (uint8_t)((h_keys[(size_t)s * nw + x / 8] >> (4 * (x % 8))) & 15u);
  cnt_out.assign(h_cnt.begin(), h_cnt.end());
  S_out = S;
  return CVD_OK;
}

int cvd::device_learn_dense(const CodeDesc& dec, const std::vector<int32_t>& next, int64_t S, int64_t L,
                            int64_t burn, uint64_t seed, double p, int device, void* stream,
                            std::vector<int64_t>& cnt_out, LearnStats* stats) {
  const int n = dec.n, R = 1 << n;
  if (n < 1 || n > 3) { set_error("GPU learning: n must be 1..3"); return CVD_E_UNSUPPORTED; }
  if (L < 1 || L >= ((int64_t)1 << 31)) { set_error("GPU learning: learn_len must be in [1, 2^31)"); return CVD_E_UNSUPPORTED; }
  DevGuard guard;
  LHIP(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  Scratch sc(st);
  uint32_t* d_r = nullptr;
  int rc = learn_stream(dec, L, seed, p, st, sc, d_r);
  if (rc) return rc;
  int32_t* d_next = nullptr;
  LHIP(sc.alloc(d_next, next.size()));
  LHIP(hipMemcpyAsync(d_next, next.data(), next.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
  ChainArgs a{};
  a.r = d_r; a.L = L; a.next = d_next;
  chain_geometry(L, a);
  const int64_t nbl = (L + a.blen - 1) / a.blen;
  LHIP(sc.alloc(a.states, (size_t)(L + 1)));
  LHIP(sc.alloc(a.ends, (size_t)nbl));
  void (*kern)(ChainArgs) = n == 1 ? chain_dense_kernel<1> : n == 2 ? chain_dense_kernel<2> : chain_dense_kernel<3>;
  rc = run_chain(a, 1, kern, 0, st, sc, stats);
  if (rc) return rc;
  uint32_t* cnt = nullptr;
  LHIP(sc.alloc(cnt, (size_t)S * R));
  LHIP(hipMemsetAsync(cnt, 0, (size_t)S * R * sizeof(uint32_t), st));
  if (L > burn)
    hipLaunchKernelGGL(count_kernel, dim3(grid_of(L - burn)), dim3(kLB), 0, st, d_r, a.states, burn, L, n, cnt);
  LHIP(hipGetLastError());
  std::vector<uint32_t> h_cnt((size_t)S * R);
  LHIP(hipMemcpyAsync(h_cnt.data(), cnt, h_cnt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  LHIP(hipStreamSynchronize(st));
  cnt_out.assign(h_cnt.begin(), h_cnt.end());
  return CVD_OK;
}
