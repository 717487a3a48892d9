// State enumeration on the GPU: the reference's BFS
// enumerate_markov_states_allzero (viterbi_markov.py:166-195) as a
// level-synchronous search over a hash set in HBM, sized for the codes whose
// state count the host BFS (cvd_enumerate) cannot reach -- (133,171) passes 2e8.
//
// The reference pops states FIFO and appends each unseen successor, trying the
// received words in itertools.product order (the LAST output bit fastest).  So
// a state's index is its level's first index plus its rank among that level's
// new states ordered by their FIRST discovery (parent index, word order q): the
// search runs level by level, every (parent, q) of a level is a candidate with
// the code g = parent * 2^n + q, and a new state keeps the smallest g of the
// candidates that reach it (atomicMin).  Sorting a level's new states by that g
// gives exactly the reference's discovery order.
//
// The set: open addressing over 16-byte slots {h, v}, h = a 64-bit hash of the
// nibble-packed metric vector (never 0; 0 = empty), v = the state index (or,
// while its level runs, NEW | staging index).  A candidate claims the first
// slot on its probe path that is empty or carries its hash (one 64-bit CAS;
// no locks, so no lane ever waits on another).  Whether it is the SAME state is
// decided in a second launch, after every claim of the pass is visible: the
// candidate's key is compared with the key of the slot's owner (a state of an
// earlier level, or a staged new state).  A 64-bit hash collision (two states,
// one hash) is therefore never merged: the candidate probes on from the next
// slot in another claim pass.  Every state counted is a distinct reachable
// metric vector.
//
// Past the memory budget the search stops with CVD_E_CAPACITY: the states of the
// completed levels plus the new states staged so far are then a certified lower
// bound on S (all distinct, all reachable), reported with the per-level sizes.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cvd.h"
#include "cvd_chain.h"
#include "cvd_common.h"
#include "cvd_internal.h"

using namespace cvd;
using namespace cvd_chain;

#define BHIP(x)                                                                           \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      set_error(std::string("HIP error '") + hipGetErrorString(e_) + "' at " #x);          \
      return CVD_E_HIP;                                                                   \
    }                                                                                     \
  } while (0)

namespace {

constexpr int kBB = 256;
constexpr uint64_t kNew = 1ull << 63;
constexpr uint64_t kVMask = kNew - 1;

struct BfsArgs {
  const uint8_t* bm;        // [R][M][K] branch metrics
  uint32_t* states;         // [cap][NW] keys by state index (discovery order)
  uint64_t* th;             // [slots] slot hashes (0 = empty)
  uint64_t* tv;             // [slots] state index, or kNew | staging index while its level runs
  uint64_t mask;            // slots - 1
  uint64_t hkeep;           // hash bits kept (all; CVD_BFS_HASH_BITS narrows them to force collisions in tests)
  int64_t lo, hi;           // this level's parents: states [lo, hi)
  int64_t g0, nc;           // candidates g0 .. g0 + nc - 1 of this chunk (g = parent * R + q)
  uint32_t* ckey;           // [chunk][NW] candidate keys
  uint64_t* ch;             // [chunk] candidate hashes
  uint64_t* cslot;          // [chunk] slot the candidate claimed or matched (probe start on a retry)
  const uint32_t* list;     // retry pass: candidates (chunk offsets) to probe again, else nullptr
  int64_t nlist;
  uint32_t* retry;          // [chunk] offsets of candidates that met another state's hash
  uint32_t* nretry;
  uint32_t* nkey;           // [stage][NW] staged new states of this level
  uint64_t* ncode;          // [stage] smallest candidate code g reaching it
  uint64_t* nslot;          // [stage] its slot
  uint32_t* nnew;           // staged count
  int64_t stage;            // staging capacity
  uint32_t* overflow;       // staging full
  int64_t* next;            // nullable: [cap][R] successor (new states as -(staging index + 1) until ranked)
};

__device__ __forceinline__ uint64_t mix64b(uint64_t x) {
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <int NW>
__device__ __forceinline__ uint64_t key_hash64(const uint32_t (&k)[NW]) {
  uint64_t x = 0x2545F4914F6CDD1Dull;
#pragma unroll
  for (int w = 0; w < NW; w += 2) {
    const uint64_t lo = k[w], hi = w + 1 < NW ? k[w + 1] : 0u;
    x = mix64b(x ^ (lo | (hi << 32)));
  }
  return x ? x : 0x9E3779B97F4A7C15ull;
}

// The received word of candidate order q: itertools.product order, the last
// output bit varies fastest (viterbi_markov.py:175), i.e. r = bit-reverse of q.
template <int n>
__device__ __forceinline__ uint32_t word_of_order(uint32_t q) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < n; ++j) r |= ((q >> (n - 1 - j)) & 1u) << j;
  return r;
}

// claim pass: expand (first pass of a chunk) and probe for a slot that is empty
// (claim it with a CAS) or carries the candidate's hash
template <int m, int k, int n>
__global__ __launch_bounds__(kBB) void bfs_claim_kernel(BfsArgs a) {
  constexpr int M = 1 << m, K = 1 << k, R = 1 << n, NW = M >= 8 ? M / 8 : 1;
  __shared__ uint8_t s_bm[R * M * K];
  for (int j = threadIdx.x; j < R * M * K; j += kBB) s_bm[j] = a.bm[j];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kBB + threadIdx.x;
  if (i >= (a.list ? a.nlist : a.nc)) return;
  const int64_t c = a.list ? (int64_t)a.list[i] : i;
  uint32_t key[NW];
  uint64_t h, s;
  if (!a.list) {
    const int64_t g = a.g0 + c, parent = g / R;
    const uint32_t r = word_of_order<n>((uint32_t)(g % R));
    uint8_t D[M];
    unpack_key<m>(a.states + (size_t)parent * NW, D);
    step_vec<m, k>(D, s_bm + r * (M * K));
    pack_key<m>(D, key);
#pragma unroll
    for (int w = 0; w < NW; ++w) a.ckey[(size_t)c * NW + w] = key[w];
    h = key_hash64<NW>(key) & a.hkeep;
    h = h ? h : 1u;
    a.ch[c] = h;
    s = h & a.mask;
  } else {
#pragma unroll
    for (int w = 0; w < NW; ++w) key[w] = a.ckey[(size_t)c * NW + w];
    h = a.ch[c];
    s = (a.cslot[c] + 1) & a.mask;   // past the slot whose state had this hash but another key
  }
  for (;;) {
    const uint64_t cur = a.th[s];
    if (cur == h) break;
    if (cur == 0) {
      const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long*>(a.th + s), 0ull, (unsigned long long)h);
      if (old == 0) {
        const uint32_t ni = atomicAdd(a.nnew, 1u);
        if ((int64_t)ni >= a.stage) {
          atomicOr(a.overflow, 1u);
          a.tv[s] = kNew | kVMask;   // no staged key: resolve skips it, the search stops after this pass
          a.cslot[c] = s | kNew;
          return;
        }
#pragma unroll
        for (int w = 0; w < NW; ++w) a.nkey[(size_t)ni * NW + w] = key[w];
        a.ncode[ni] = (uint64_t)(a.g0 + c);
        a.nslot[ni] = s;
        a.tv[s] = kNew | ni;
        a.cslot[c] = s | kNew;   // (bit 63: this candidate created the slot's state)
        if (a.next) a.next[a.g0 + c] = -(int64_t)ni - 1;
        return;
      }
      if (old == h) break;
    }
    s = (s + 1) & a.mask;
  }
  a.cslot[c] = s;
}

// resolve pass (every claim of the pass visible): the candidate is the slot
// owner's state iff the keys are equal; else it probes on (retry list)
template <int NW>
__global__ __launch_bounds__(kBB) void bfs_resolve_kernel(BfsArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kBB + threadIdx.x;
  if (i >= (a.list ? a.nlist : a.nc)) return;
  const int64_t c = a.list ? (int64_t)a.list[i] : i;
  const uint64_t cs = a.cslot[c];
  if (cs & kNew) return;   // created the state
  const uint64_t v = a.tv[cs];
  if ((v & kNew) && (int64_t)(v & kVMask) >= a.stage) return;   // staging overflowed: the search stops
  const uint32_t* other = (v & kNew) ? a.nkey + (size_t)(v & kVMask) * NW : a.states + (size_t)v * NW;
  uint32_t d = 0u;
#pragma unroll
  for (int w = 0; w < NW; ++w) d |= a.ckey[(size_t)c * NW + w] ^ other[w];
  if (d) {   // 64-bit hash collision: another state owns this hash
    const uint32_t ri = atomicAdd(a.nretry, 1u);
    a.retry[ri] = (uint32_t)c;
    return;
  }
  const int64_t g = a.g0 + c;
  if (v & kNew) {
    atomicMin(reinterpret_cast<unsigned long long*>(a.ncode + (v & kVMask)), (unsigned long long)g);
    if (a.next) a.next[g] = -(int64_t)(v & kVMask) - 1;
  } else if (a.next) {
    a.next[g] = (int64_t)v;
  }
}

// a level's new states in discovery order: state hi + pos is the staged state
// order[pos] (sorted by smallest candidate code)
template <int NW>
__global__ __launch_bounds__(kBB) void bfs_place_kernel(const uint32_t* order, int64_t nnew, int64_t hi,
                                                        const uint32_t* nkey, const uint64_t* nslot, uint64_t* tv,
                                                        uint32_t* states, int64_t* rank) {
  const int64_t pos = (int64_t)blockIdx.x * kBB + threadIdx.x;
  if (pos >= nnew) return;
  const uint32_t ni = order[pos];
#pragma unroll
  for (int w = 0; w < NW; ++w) states[(size_t)(hi + pos) * NW + w] = nkey[(size_t)ni * NW + w];
  tv[nslot[ni]] = (uint64_t)(hi + pos);
  if (rank) rank[ni] = hi + pos;
}

__global__ void bfs_fix_next_kernel(int64_t* next, int64_t g0, int64_t g1, const int64_t* rank) {
  const int64_t g = g0 + (int64_t)blockIdx.x * kBB + threadIdx.x;
  if (g >= g1) return;
  const int64_t v = next[g];
  if (v < 0) next[g] = rank[-v - 1];
}

__global__ void bfs_iota_kernel(uint32_t* v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kBB + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + kBB - 1) / kBB); }

struct Kern {
  void (*claim)(BfsArgs);
  void (*resolve)(BfsArgs);
  void (*place)(const uint32_t*, int64_t, int64_t, const uint32_t*, const uint64_t*, uint64_t*, uint32_t*, int64_t*);
};

template <int m, int k, int n>
Kern kern_of() {
  constexpr int NW = (1 << m) >= 8 ? (1 << m) / 8 : 1;
  return {bfs_claim_kernel<m, k, n>, bfs_resolve_kernel<NW>, bfs_place_kernel<NW>};
}

bool pick(int m, int k, int n, Kern& K) {
  if (k == 1 && n == 2) {
    switch (m) {
      case 2: K = kern_of<2, 1, 2>(); return true;
      case 3: K = kern_of<3, 1, 2>(); return true;
      case 4: K = kern_of<4, 1, 2>(); return true;
      case 5: K = kern_of<5, 1, 2>(); return true;
      case 6: K = kern_of<6, 1, 2>(); return true;
    }
  }
  if (m == 4 && k == 2 && n == 3) { K = kern_of<4, 2, 3>(); return true; }
  return false;
}

struct DevMem {
  std::vector<void*> ptrs;
  template <typename T>
  hipError_t alloc(T*& p, size_t count) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) ptrs.push_back(q);
    p = static_cast<T*>(q);
    return e;
  }
  ~DevMem() {
    (void)hipDeviceSynchronize();
    for (void* p : ptrs) (void)hipFree(p);
  }
};

int64_t env_i64(const char* name, int64_t def) {
  const char* e = std::getenv(name);
  return e && e[0] ? std::atoll(e) : def;
}

}  // namespace

extern "C" int cvd_enumerate_device(const cvd_code* dec, int32_t device, int64_t cap, int64_t mem_bytes,
                                    int64_t* S_out, uint8_t* states_out, int32_t* next_out, int64_t* level_sizes,
                                    int32_t max_levels, int32_t* n_levels_out, void* stream) {
  if (!dec || !S_out || cap < 1 || device < 0) { set_error("bad cvd_enumerate_device arguments"); return CVD_E_INVALID; }
  // CVD_E_CAPACITY always comes with S_out >= 1 (the states certified so far); any other
  // failure leaves S_out = 0, which no caller may read as a bound
  *S_out = 0;
  if (n_levels_out) *n_levels_out = 0;
  if (dec->k < 1 || dec->k > kMaxK || dec->n < 1 || dec->n > kMaxN || dec->m < 1 || dec->m > kMaxM || !dec->taps) {
    set_error("code shape out of range");
    return CVD_E_INVALID;
  }
  CodeDesc d{};
  d.k = dec->k; d.n = dec->n; d.m = dec->m;
  const int L = d.m + 1;
  for (int j = 0; j < d.n; ++j)
    for (int i = 0; i < d.k; ++i) {
      uint32_t g = 0;
      for (int t = 0; t < L; ++t) g |= (uint32_t)(dec->taps[(j * d.k + i) * L + t] & 1u) << t;
      d.gmask[j * d.k + i] = g;
    }
  Kern K;
  if (!pick(d.m, d.k, d.n, K)) { set_error("GPU enumeration: unsupported code shape"); return CVD_E_UNSUPPORTED; }
  const int M = 1 << d.m, Kk = 1 << d.k, R = 1 << d.n, NW = M >= 8 ? M / 8 : 1;
  int cur_dev = 0;
  (void)hipGetDevice(&cur_dev);
  struct Restore {
    int dv;
    ~Restore() { (void)hipSetDevice(dv); }
  } restore{cur_dev};
  BHIP(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  // memory plan (bytes per state): key 4 NW, slots 16 / load (<= 1/2), staging
  // (a level's new states: key, code, slot, sort buffers, rank) ~ 4 NW + 40 for up
  // to half the states, next 8 R if requested; the candidate chunk apart
  size_t freeb = 0, totb = 0;
  BHIP(hipMemGetInfo(&freeb, &totb));
  const int64_t budget = mem_bytes > 0 ? std::min<int64_t>(mem_bytes, (int64_t)freeb) : (int64_t)(freeb * 0.9);
  const int64_t chunk = std::max<int64_t>(1024, env_i64("CVD_BFS_CHUNK", (int64_t)1 << 26));
  const int64_t chunk_bytes = chunk * (4 * NW + 8 + 8 + 4);
  const bool want_next = next_out != nullptr;
  // per state beside the slots: its key, and staging for up to half of them (key,
  // code, sorted code, slot, order in / out, rank)
  const double per_state = 4.0 * NW + 0.5 * (4.0 * NW + 8 + 8 + 8 + 4 + 4 + 8) + (want_next ? 8.0 * R : 0.0);
  const int64_t avail = budget - chunk_bytes - ((int64_t)512 << 20);
  // slots: a power of two at load <= 0.6; pick the count that admits the most states
  int64_t scap = 0, slots = 64;
  for (int64_t sl = 64; sl <= ((int64_t)1 << 36); sl <<= 1) {
    const int64_t fit = (int64_t)((double)(avail - sl * 16) / per_state);
    const int64_t sc = std::min<int64_t>({cap + 1, (int64_t)(0.6 * (double)sl), fit});
    if (sc > scap) { scap = sc; slots = sl; }
    if ((double)sl * 0.6 > (double)(cap + 1)) break;
  }
  if (scap < 2) { set_error("GPU enumeration: not enough device memory to start"); return CVD_E_HIP; }
  // staging for a level's new states: all of scap while that is small, half beyond
  const int64_t stage = std::max<int64_t>(1024, scap <= ((int64_t)1 << 26) ? scap : scap / 2);
  DevMem dm;
  uint8_t* d_bm = nullptr;
  uint32_t *d_states = nullptr, *d_ckey = nullptr, *d_retry = nullptr, *d_cnt = nullptr, *d_nkey = nullptr,
           *d_order_in = nullptr, *d_order = nullptr;
  uint64_t *d_th = nullptr, *d_tv = nullptr, *d_ch = nullptr, *d_cslot = nullptr, *d_ncode = nullptr,
           *d_ncode_s = nullptr, *d_nslot = nullptr;
  int64_t *d_next = nullptr, *d_rank = nullptr;
  BHIP(dm.alloc(d_states, (size_t)scap * NW));
  BHIP(dm.alloc(d_th, (size_t)slots));
  BHIP(dm.alloc(d_tv, (size_t)slots));
  BHIP(dm.alloc(d_ckey, (size_t)chunk * NW));
  BHIP(dm.alloc(d_ch, (size_t)chunk));
  BHIP(dm.alloc(d_cslot, (size_t)chunk));
  BHIP(dm.alloc(d_retry, (size_t)chunk));
  BHIP(dm.alloc(d_cnt, 4));   // [0] staged, [1] retries, [2] overflow
  BHIP(dm.alloc(d_nkey, (size_t)stage * NW));
  BHIP(dm.alloc(d_ncode, (size_t)stage));
  BHIP(dm.alloc(d_ncode_s, (size_t)stage));
  BHIP(dm.alloc(d_nslot, (size_t)stage));
  BHIP(dm.alloc(d_order_in, (size_t)stage));
  BHIP(dm.alloc(d_order, (size_t)stage));
  if (want_next) {
    BHIP(dm.alloc(d_next, (size_t)scap * R));
    BHIP(dm.alloc(d_rank, (size_t)stage));
  }
  size_t sort_tmp = 0;
  BHIP(rocprim::radix_sort_pairs(nullptr, sort_tmp, d_ncode, d_ncode_s, d_order_in, d_order, (size_t)stage, 0, 64, st));
  uint8_t* d_sort_tmp = nullptr;
  BHIP(dm.alloc(d_sort_tmp, sort_tmp));
  {
    std::vector<uint8_t> bm((size_t)R * M * Kk);
    for (int r = 0; r < R; ++r)
      for (int s = 0; s < M; ++s)
        for (int U = 0; U < Kk; ++U)
          bm[((size_t)r * M + s) * Kk + U] = (uint8_t)__builtin_popcount(enc_out(d, (uint32_t)s, (uint32_t)U) ^ (uint32_t)r);
    BHIP(dm.alloc(d_bm, bm.size()));
    BHIP(hipMemcpyAsync(d_bm, bm.data(), bm.size(), hipMemcpyHostToDevice, st));
  }
  BHIP(hipMemsetAsync(d_th, 0, (size_t)slots * 8, st));
  const int64_t hbits = env_i64("CVD_BFS_HASH_BITS", 64);
  const uint64_t hkeep = hbits >= 64 ? ~0ull : ((1ull << std::max<int64_t>(1, hbits)) - 1);
  // D_0 = 0 is state 0 (viterbi_markov.py:177-180)
  {
    std::vector<uint32_t> z((size_t)NW, 0u);
    BHIP(hipMemcpyAsync(d_states, z.data(), (size_t)NW * 4, hipMemcpyHostToDevice, st));
    uint64_t h = 0x2545F4914F6CDD1Dull;   // key_hash64 of the zero key (host restatement)
    auto mix = [](uint64_t x) {
      x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
      x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
      return x ^ (x >> 31);
    };
    for (int w = 0; w < NW; w += 2) h = mix(h ^ 0ull);
    if (!h) h = 0x9E3779B97F4A7C15ull;
    h &= hkeep;
    if (!h) h = 1u;
    const uint64_t s0 = h & (uint64_t)(slots - 1), v0 = 0;
    BHIP(hipMemcpyAsync(d_th + s0, &h, 8, hipMemcpyHostToDevice, st));
    BHIP(hipMemcpyAsync(d_tv + s0, &v0, 8, hipMemcpyHostToDevice, st));
  }
  BfsArgs a{};
  a.bm = d_bm; a.states = d_states; a.th = d_th; a.tv = d_tv; a.mask = (uint64_t)(slots - 1); a.hkeep = hkeep;
  a.ckey = d_ckey; a.ch = d_ch; a.cslot = d_cslot; a.retry = d_retry; a.nretry = d_cnt + 1;
  a.nkey = d_nkey; a.ncode = d_ncode; a.nslot = d_nslot; a.nnew = d_cnt; a.stage = stage; a.overflow = d_cnt + 2;
  a.next = d_next;
  int64_t lo = 0, hi = 1;
  int32_t nlev = 0;
  if (level_sizes && max_levels > 0) level_sizes[0] = 1;
  nlev = 1;
  const bool verbose = std::getenv("CVD_BFS_VERBOSE") != nullptr;
  const double tlimit = (double)env_i64("CVD_BFS_SECONDS", 0);
  const auto t_start = std::chrono::steady_clock::now();
  while (lo < hi) {
    BHIP(hipMemsetAsync(d_cnt, 0, 16, st));
    const int64_t G = (hi - lo) * R;
    for (int64_t c0 = 0; c0 < G; c0 += chunk) {
      a.lo = lo; a.hi = hi;
      a.g0 = lo * R + c0;
      a.nc = std::min<int64_t>(chunk, G - c0);
      a.list = nullptr; a.nlist = 0;
      hipLaunchKernelGGL(K.claim, dim3(grid_of(a.nc)), dim3(kBB), 0, st, a);
      BHIP(hipGetLastError());
      uint32_t cnt[3] = {0, 0, 0};
      for (int pass = 0;; ++pass) {
        BHIP(hipMemsetAsync(d_cnt + 1, 0, 4, st));
        hipLaunchKernelGGL(K.resolve, dim3(grid_of(a.list ? a.nlist : a.nc)), dim3(kBB), 0, st, a);
        BHIP(hipGetLastError());
        BHIP(hipMemcpyAsync(cnt, d_cnt, 12, hipMemcpyDeviceToHost, st));
        BHIP(hipStreamSynchronize(st));
        if (cnt[2]) break;   // staging full
        if (cnt[1] == 0) break;
        // hash collisions: probe on past the other state's slot (the retry list
        // becomes this pass's list; rare -- two states sharing a 64-bit hash)
        if (pass > 4096) { set_error("GPU enumeration: unbounded hash-collision retries"); return CVD_E_STATE; }
        uint32_t* lst = nullptr;
        BHIP(dm.alloc(lst, cnt[1]));
        BHIP(hipMemcpyAsync(lst, d_retry, (size_t)cnt[1] * 4, hipMemcpyDeviceToDevice, st));
        a.list = lst; a.nlist = cnt[1];
        hipLaunchKernelGGL(K.claim, dim3(grid_of(a.nlist)), dim3(kBB), 0, st, a);
        BHIP(hipGetLastError());
      }
      if (cnt[2]) break;
    }
    uint32_t cnt[3] = {0, 0, 0};
    BHIP(hipMemcpyAsync(cnt, d_cnt, 12, hipMemcpyDeviceToHost, st));
    BHIP(hipStreamSynchronize(st));
    const int64_t nnew = std::min<int64_t>((int64_t)cnt[0], stage);
    if (cnt[2] || hi + nnew > scap || hi + nnew > cap) {
      // capacity: the staged states are distinct and reachable -> a lower bound
      if (level_sizes && nlev < max_levels) level_sizes[nlev] = nnew;
      ++nlev;
      *S_out = hi + nnew;
      if (n_levels_out) *n_levels_out = nlev;
      set_error("GPU enumeration: state count exceeds the capacity (S_out is a lower bound)");
      return CVD_E_CAPACITY;
    }
    if (nnew == 0) break;
    hipLaunchKernelGGL(bfs_iota_kernel, dim3(grid_of(nnew)), dim3(kBB), 0, st, d_order_in, nnew);
    size_t ts = sort_tmp;
    BHIP(rocprim::radix_sort_pairs(d_sort_tmp, ts, d_ncode, d_ncode_s, d_order_in, d_order, (size_t)nnew, 0, 64, st));
    hipLaunchKernelGGL(K.place, dim3(grid_of(nnew)), dim3(kBB), 0, st, d_order, nnew, hi, d_nkey, d_nslot, d_tv,
                       d_states, d_rank);
    BHIP(hipGetLastError());
    if (want_next) {
      hipLaunchKernelGGL(bfs_fix_next_kernel, dim3(grid_of(G)), dim3(kBB), 0, st, d_next, lo * R, hi * R, d_rank);
      BHIP(hipGetLastError());
    }
    if (level_sizes && nlev < max_levels) level_sizes[nlev] = nnew;
    ++nlev;
    if (verbose)
      std::fprintf(stderr, "[cvd bfs] level %d: %lld new, %lld states, %.1f s\n", nlev - 1, (long long)nnew,
                   (long long)(hi + nnew),
                   std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
    lo = hi;
    hi += nnew;
    if (tlimit > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() > tlimit &&
        lo < hi) {
      // time budget spent (CVD_BFS_SECONDS): the completed levels are a lower bound
      *S_out = hi;
      if (n_levels_out) *n_levels_out = nlev;
      set_error("GPU enumeration: time budget spent (S_out is a lower bound)");
      return CVD_E_CAPACITY;
    }
  }
  *S_out = hi;
  if (n_levels_out) *n_levels_out = nlev;
  if (states_out || next_out) {
    if (hi > cap) { set_error("GPU enumeration: S exceeds cap"); return CVD_E_CAPACITY; }
    if (states_out) {
      std::vector<uint32_t> keys((size_t)hi * NW);
      BHIP(hipMemcpyAsync(keys.data(), d_states, keys.size() * 4, hipMemcpyDeviceToHost, st));
      BHIP(hipStreamSynchronize(st));
      for (int64_t s = 0; s < hi; ++s)
        for (int x = 0; x < M; ++x)
          states_out[(size_t)s * M + x] = (uint8_t)((keys[(size_t)s * NW + x / 8] >> (4 * (x % 8))) & 15u);
    }
    if (next_out) {
      std::vector<int64_t> nx((size_t)hi * R);
      BHIP(hipMemcpyAsync(nx.data(), d_next, nx.size() * 8, hipMemcpyDeviceToHost, st));
      BHIP(hipStreamSynchronize(st));
      // next_out[i * 2^n + r] for the received word r (cvd_enumerate layout); the
      // search stored it by candidate order q
      for (int64_t s = 0; s < hi; ++s)
        for (int q = 0; q < R; ++q) {
          uint32_t r = 0;
          for (int j = 0; j < d.n; ++j) r |= ((uint32_t)(q >> (d.n - 1 - j)) & 1u) << j;
          next_out[(size_t)s * R + r] = (int32_t)nx[(size_t)s * R + q];
        }
    }
  }
  return CVD_OK;
}
