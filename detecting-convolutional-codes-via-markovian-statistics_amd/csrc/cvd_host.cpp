// Host-side native setup behind the C-ABI: code algebra, Eq. 4-5 step on the
// host, BFS state enumeration, the P̂1 learning chain, T_ref(1/2), the row
// tables and the explicit-path hash.  None of this is the hot path (the trial
// loop runs in cvd_kernels.hip); it is the analogue of the reference's table
// construction (viterbi_markov.py:118-230, Pd_plotter.py:123-169).
#include <atomic>
#include <chrono>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <cstdlib>
#include <exception>
#include <cstdio>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include <sys/stat.h>
#include <unistd.h>

#include "../../include/cvd.h"
#include "cvd_internal.h"
#include "cvd_bitslice.h"

using namespace cvd;

static thread_local std::string g_err;
void cvd::set_error(const std::string& msg) { g_err = msg; }
std::string cvd::last_error_copy() { return g_err; }

namespace {
// CVD_SETUP_TIMING=1: phase times of cvd_model_create on stderr
struct PhaseTimer {
  bool on = std::getenv("CVD_SETUP_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  void mark(const char* what) {
    if (!on) return;
    const auto t1 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[cvd setup] %-28s %8.3f s\n", what, std::chrono::duration<double>(t1 - t0).count());
    t0 = t1;
  }
};
}  // namespace

#define CVD_TRY try {
#define CVD_CATCH                                          \
  }                                                        \
  catch (const std::bad_alloc&) {                          \
    set_error("out of host memory");                       \
    return CVD_E_CAPACITY;                                 \
  }                                                        \
  catch (const std::exception& e) {                        \
    set_error(std::string("internal error: ") + e.what()); \
    return CVD_E_INVALID;                                  \
  }

extern "C" int cvd_version(void) { return CVD_ABI_VERSION; }
extern "C" const char* cvd_last_error(void) { return g_err.c_str(); }
extern "C" uint32_t cvd_grid_tag(int64_t N, double p) { return grid_tag(N, p); }

// ───────────────────────────── code algebra ─────────────────────────────────

namespace {

struct Tabs {
  int m, k, n, M, K, R;
  std::vector<uint8_t> out;   // [M][K] output word
  std::vector<uint16_t> nxt;  // [M][K]
};

int parse_code(const cvd_code* c, CodeDesc& d) {
  if (!c || !c->taps) { set_error("null code"); return CVD_E_INVALID; }
  if (c->k < 1 || c->k > kMaxK || c->n < 1 || c->n > kMaxN || c->m < 1 || c->m > kMaxM) {
    set_error("code shape out of range (1<=k<=4, 1<=n<=8, 1<=m<=8)");
    return CVD_E_INVALID;
  }
  d.k = c->k; d.n = c->n; d.m = c->m;
  std::memset(d.gmask, 0, sizeof(d.gmask));
  const int L = c->m + 1;
  for (int j = 0; j < c->n; ++j)
    for (int i = 0; i < c->k; ++i) {
      uint32_t g = 0;
      for (int t = 0; t < L; ++t) {
        uint8_t b = c->taps[(j * c->k + i) * L + t];
        if (b > 1) { set_error("taps must be 0/1"); return CVD_E_INVALID; }
        g |= (uint32_t)b << t;   // taps[d] multiplies x[d]: d=0 input bit, d>=1 state bit d-1
      }
      d.gmask[j * c->k + i] = g;
    }
  return CVD_OK;
}

Tabs make_tabs(const CodeDesc& d) {
  Tabs T;
  T.m = d.m; T.k = d.k; T.n = d.n; T.M = 1 << d.m; T.K = 1 << d.k; T.R = 1 << d.n;
  T.out.resize((size_t)T.M * T.K);
  T.nxt.resize((size_t)T.M * T.K);
  for (int s = 0; s < T.M; ++s)
    for (int U = 0; U < T.K; ++U) {
      T.out[s * T.K + U] = (uint8_t)enc_out(d, s, U);
      T.nxt[s * T.K + U] = (uint16_t)enc_next(d, s, U);
    }
  return T;
}

// Eq. 4-5 on the host (viterbi_markov.py:139-159).
inline void step_host(const Tabs& T, const uint8_t* D, uint32_t r, uint8_t* out) {
  uint8_t best[256];
  std::memset(best, 0xFF, (size_t)T.M);
  for (int s = 0; s < T.M; ++s) {
    const int ds = D[s];
    for (int U = 0; U < T.K; ++U) {
      const int v = ds + __builtin_popcount((unsigned)(T.out[s * T.K + U] ^ r));
      uint8_t& b = best[T.nxt[s * T.K + U]];
      if (v < b) b = (uint8_t)v;
    }
  }
  uint8_t mn = 255;
  for (int i = 0; i < T.M; ++i) mn = std::min(mn, best[i]);
  for (int i = 0; i < T.M; ++i) out[i] = (uint8_t)(best[i] - mn);
}

// The same step in predecessor form for k = 1 (next(s, u) = (2s + u) mod 2^m,
// viterbi_markov.py:102-104): state x has predecessors x >> 1 and
// (x >> 1) + 2^(m-1) with input x & 1.  bm[r][s][u] = popcount(out(s, u) ^ r).
struct StepK1 {
  int M;
  std::vector<uint8_t> bm;   // [R][M][2]
  explicit StepK1(const Tabs& T) : M(T.M), bm((size_t)T.R * T.M * 2) {
    for (int r = 0; r < T.R; ++r)
      for (int s = 0; s < T.M; ++s)
        for (int u = 0; u < 2; ++u)
          bm[((size_t)r * T.M + s) * 2 + u] = (uint8_t)__builtin_popcount((unsigned)(T.out[s * 2 + u] ^ r));
  }
  void operator()(const uint8_t* D, uint32_t r, uint8_t* out) const {
    const uint8_t* b = bm.data() + (size_t)r * M * 2;
    const int H = M / 2;
    uint8_t mn = 255;
    for (int x = 0; x < M; ++x) {
      const int s0 = x >> 1, s1 = s0 + H, u = x & 1;
      const int a = D[s0] + b[s0 * 2 + u], c = D[s1] + b[s1 * 2 + u];
      const uint8_t v = (uint8_t)(a < c ? a : c);
      out[x] = v;
      mn = v < mn ? v : mn;
    }
    for (int x = 0; x < M; ++x) out[x] = (uint8_t)(out[x] - mn);
  }
};

// Eq. 4-5 through the fastest form the code admits (identical results).
struct HostStep {
  const Tabs& T;
  bool k1;
  StepK1 s1;
  explicit HostStep(const Tabs& t) : T(t), k1(t.k == 1), s1(t.k == 1 ? t : Tabs{1, 1, 1, 2, 2, 2, {0, 0, 0, 0}, {0, 0, 0, 0}}) {}
  void operator()(const uint8_t* D, uint32_t r, uint8_t* out) const {
    if (k1) s1(D, r, out);
    else step_host(T, D, r, out);
  }
};

// Run f(i) for i in [0, n) on up to `threads` std::threads (contiguous ranges).
template <typename F>
void parallel_for(int64_t n, F f) {
  unsigned hw = std::thread::hardware_concurrency();
  if (const char* e = std::getenv("CVD_HOST_THREADS")) hw = (unsigned)std::max(1, std::atoi(e));
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({(int64_t)hw, (int64_t)32, n / 4096 + 1}));
  if (nt == 1) { for (int64_t i = 0; i < n; ++i) f(i, 0); return; }
  std::vector<std::thread> th;
  std::exception_ptr err;
  std::mutex mu;
  for (int64_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      try {
        for (int64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) f(i, (int)t);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu);
        err = std::current_exception();
      }
    });
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
}

// Open-addressing map from metric vectors (M bytes) to row indices.
struct StateMap {
  int M;
  std::vector<uint8_t>* store;  // rows of M bytes
  std::vector<int32_t> slots;
  uint64_t mask = 0;
  int64_t count = 0;
  StateMap(int M_, std::vector<uint8_t>* st) : M(M_), store(st) { rehash(1024); }
  // room for n keys without rehashing or moving the key store
  void reserve(int64_t n) {
    store->reserve((size_t)n * M);
    uint64_t cap = mask + 1;
    while ((uint64_t)n * 2 > cap) cap *= 2;
    if (cap != mask + 1) rehash(cap);
  }
  static uint64_t hb(const uint8_t* p, int M) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < M; i += 8) {
      uint64_t w = 0;
      std::memcpy(&w, p + i, (size_t)std::min(8, M - i));
      h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
      h ^= h >> 31;
    }
    return h;
  }
  void rehash(uint64_t cap) {
    slots.assign(cap, -1);
    mask = cap - 1;
    for (int64_t i = 0; i < count; ++i) {
      uint64_t h = hb(store->data() + (size_t)i * M, M) & mask;
      while (slots[h] >= 0) h = (h + 1) & mask;
      slots[h] = (int32_t)i;
    }
  }
  int64_t find(const uint8_t* key) const {
    uint64_t h = hb(key, M) & mask;
    while (true) {
      int32_t v = slots[h];
      if (v < 0) return -1;
      if (!std::memcmp(store->data() + (size_t)v * M, key, (size_t)M)) return v;
      h = (h + 1) & mask;
    }
  }
  // returns index; inserted=true if new (appended to store)
  int64_t insert(const uint8_t* key, bool& inserted) {
    int64_t f = find(key);
    if (f >= 0) { inserted = false; return f; }
    if ((uint64_t)(count + 1) * 2 > mask + 1) rehash((mask + 1) * 2);
    store->insert(store->end(), key, key + M);
    uint64_t h = hb(key, M) & mask;
    while (slots[h] >= 0) h = (h + 1) & mask;
    slots[h] = (int32_t)count;
    inserted = true;
    return count++;
  }
};

// BFS from D_0 = 0 over all 2^n received words (viterbi_markov.py:166-195):
// index = discovery order, successors in received-word order.
int bfs(const Tabs& T, int64_t cap, std::vector<uint8_t>& states, std::vector<int32_t>& next,
        int64_t& S) {
  states.clear();
  next.clear();
  StateMap map(T.M, &states);
  std::vector<uint8_t> zero((size_t)T.M, 0), nb((size_t)T.M);
  const HostStep step(T);
  bool ins;
  map.insert(zero.data(), ins);
  int64_t head = 0;
  while (head < map.count) {
    next.resize((size_t)(head + 1) * T.R);
    // received words in itertools.product order (viterbi_markov.py:175): the
    // LAST output bit varies fastest, i.e. bit-reversed integer order.
    for (int i = 0; i < T.R; ++i) {
      uint32_t r = 0;
      for (int j = 0; j < T.n; ++j) r |= ((uint32_t)(i >> (T.n - 1 - j)) & 1u) << j;
      step(states.data() + (size_t)head * T.M, r, nb.data());
      int64_t j = map.insert(nb.data(), ins);
      if (map.count > cap) { S = map.count; return CVD_E_CAPACITY; }
      next[(size_t)head * T.R + r] = (int32_t)j;
    }
    ++head;
  }
  S = map.count;
  return CVD_OK;
}

// The build's simulator spec (oracle/philox.py) on the host: received words of
// one sequence, encoder `enc`, BSC(thr).
struct HostStream {
  const CodeDesc& enc;
  const Tabs& T;
  StreamKey key;
  uint64_t seq_id;
  uint64_t thr;
  bool random_input;
  uint32_t s = 0;
  int64_t nword = -1, iblk = -1;
  uint32_t nmask = 0;
  U4 ival{};
  HostStream(const CodeDesc& e, const Tabs& t, uint64_t seed, uint32_t tag, uint64_t sid,
             double p, bool ri)
      : enc(e), T(t), key{(uint32_t)seed, (uint32_t)(seed >> 32), tag}, seq_id(sid),
        thr(noise_threshold(p)), random_input(ri) {}
  // flips of step t's n code bits: bits of received word t / spw (noise_word)
  uint32_t noise_bits(int64_t t) {
    const int spw = 32 / T.n;
    const int64_t w = t / spw;
    if (w != nword) {
      const int nb = spw * T.n;
      nmask = noise_word(key, seq_id, (uint64_t)w, thr, nb >= 32 ? ~0u : (1u << nb) - 1u);
      nword = w;
    }
    return (nmask >> (uint32_t)((t - w * spw) * T.n)) & ((1u << T.n) - 1u);
  }
  uint32_t input_bit(int64_t bi) {
    const int64_t b = bi >> 7;
    if (b != iblk) {
      ival = philox((uint32_t)b, (uint32_t)seq_id, ctr_hi(seq_id, kKindInput), key.tag, key.k0, key.k1);
      iblk = b;
    }
    return (u4_get(ival, (uint32_t)((bi >> 5) & 3)) >> (bi & 31)) & 1u;
  }
  uint32_t next_word(int64_t t) {
    uint32_t U = 0;
    if (random_input)
      for (int i = 0; i < T.k; ++i) U |= input_bit(t * T.k + i) << i;
    uint32_t r = T.out[s * T.K + U];
    s = T.nxt[s * T.K + U];
    return r ^ noise_bits(t);
  }
};

// numpy's float64 add.reduce along a contiguous axis: 0 + pairwise_sum(row)
// (8 accumulators, 128-element blocks; verified against numpy 2.2 in tests).
// The row is virtual: lam everywhere except `pos` (ascending) where it is val.
struct VirtualRow {
  double lam;
  const std::vector<std::pair<int64_t, double>>* sp;
  std::unordered_map<int64_t, double>* memo;
  bool has_special(int64_t off, int64_t n) const {
    auto it = std::lower_bound(sp->begin(), sp->end(), std::make_pair(off, -1e308));
    return it != sp->end() && it->first < off + n;
  }
  double leaf(int64_t off, int64_t n) const {
    // the block's values materialised once (lam, with the few specials patched in),
    // then numpy's leaf arithmetic on them, in numpy's order
    double v[128];
    for (int64_t i = 0; i < n; ++i) v[i] = lam;
    for (auto it = std::lower_bound(sp->begin(), sp->end(), std::make_pair(off, -1e308));
         it != sp->end() && it->first < off + n; ++it)
      v[it->first - off] = it->second;
    if (n < 8) {
      double res = 0.;
      for (int64_t i = 0; i < n; ++i) res += v[i];
      return res;
    }
    double r[8];
    for (int e = 0; e < 8; ++e) r[e] = v[e];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int e = 0; e < 8; ++e) r[e] += v[i + e];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += v[i];
    return res;
  }
  double pw(int64_t off, int64_t n) const {
    if (!has_special(off, n)) {
      auto it = memo->find(n);
      if (it != memo->end()) return it->second;
      double v = (n <= 128) ? leaf(off, n) : 0.0;
      if (n > 128) {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        v = pw(off, n2) + pw(off + n2, n - n2);
      }
      (*memo)[n] = v;
      return v;
    }
    if (n <= 128) return leaf(off, n);
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pw(off, n2) + pw(off + n2, n - n2);
  }
};

double ltref_value(int c, int R) { return std::log(std::max((double)c / (double)R, 1e-300)); }

// Row of P̂1 (Pd_plotter.py:166-167) for one state: counts per successor
// index; returns log P for each received word.
double p1_row(int64_t S, double lam, std::unordered_map<int64_t, double>& memo,
              const int64_t* succ /*[R], -1 = unvisited successor*/, const int64_t* cnt_r /*[R]*/,
              int R, double* logp_out, std::vector<std::pair<int64_t, double>>* nz = nullptr) {
  std::vector<std::pair<int64_t, double>> sp;
  for (int r = 0; r < R; ++r) {
    if (succ[r] < 0 || cnt_r[r] == 0) continue;
    bool found = false;
    for (auto& e : sp)
      if (e.first == succ[r]) { e.second += (double)cnt_r[r]; found = true; }
    if (!found) sp.emplace_back(succ[r], (double)cnt_r[r]);
  }
  std::sort(sp.begin(), sp.end());
  for (auto& e : sp) e.second = e.second + lam;   // counts + laplace (elementwise)
  VirtualRow vr{lam, &sp, &memo};
  const double rowsum = 0.0 + vr.pw(0, S);
  for (int r = 0; r < R; ++r) {
    double v = lam;
    if (succ[r] >= 0)
      for (auto& e : sp)
        if (e.first == succ[r]) v = e.second;
    logp_out[r] = std::log(std::max(v / rowsum, 1e-300));
  }
  if (nz) *nz = sp;
  return rowsum;
}

}  // namespace

void cvd::pack_nibbles(const uint8_t* D, int M, uint32_t* out) {
  const int nw = M >= 8 ? M / 8 : 1;
  for (int w = 0; w < nw; ++w) out[w] = 0;
  for (int s = 0; s < M; ++s) out[s / 8] |= (uint32_t)(D[s] & 15) << (4 * (s % 8));
}

// ───────────────────────────── ABI: algebra ─────────────────────────────────

extern "C" int cvd_code_tables(const cvd_code* code, int32_t* out_sym, int32_t* next_state) {
  CVD_TRY
  CodeDesc d;
  int rc = parse_code(code, d);
  if (rc) return rc;
  Tabs T = make_tabs(d);
  for (int i = 0; i < T.M * T.K; ++i) {
    if (out_sym) out_sym[i] = T.out[i];
    if (next_state) next_state[i] = T.nxt[i];
  }
  return CVD_OK;
  CVD_CATCH
}

extern "C" int cvd_metric_step(const cvd_code* dec, const uint8_t* D_prev, int32_t r, uint8_t* D_out) {
  CVD_TRY
  CodeDesc d;
  int rc = parse_code(dec, d);
  if (rc) return rc;
  if (!D_prev || !D_out || r < 0 || r >= (1 << d.n)) { set_error("bad step arguments"); return CVD_E_INVALID; }
  Tabs T = make_tabs(d);
  step_host(T, D_prev, (uint32_t)r, D_out);
  return CVD_OK;
  CVD_CATCH
}

extern "C" int cvd_enumerate(const cvd_code* dec, int64_t cap, int64_t* S_out, uint8_t* states_out,
                             int32_t* next_out) {
  CVD_TRY
  CodeDesc d;
  int rc = parse_code(dec, d);
  if (rc) return rc;
  Tabs T = make_tabs(d);
  std::vector<uint8_t> states;
  std::vector<int32_t> next;
  int64_t S = 0;
  rc = bfs(T, cap, states, next, S);
  if (S_out) *S_out = S;
  if (rc) { set_error("state enumeration exceeded cap"); return rc; }
  if (states_out) std::memcpy(states_out, states.data(), states.size());
  if (next_out) std::memcpy(next_out, next.data(), next.size() * sizeof(int32_t));
  return CVD_OK;
  CVD_CATCH
}

// ───────────────────────────── ABI: model ───────────────────────────────────

namespace {

void build_hash(cvd_model& Mo) {
  // Explicit-path row table:
  //  * a blocked Bloom filter over the row keys (filter_pattern);
  //  * an open-addressing directory (linear probing) of the nibble-packed metric
  //    vectors with, per slot, the row's record {log P̂1[r], row of successor(r)
  //    or -1} -- read when a hashed lookup hits;
  //  * the same records dense by row id (h_drow), which a sequence walking
  //    learned rows reads without hashing (table mode): the rows a walk visits
  //    sit together in first-visit order instead of scattered over the
  //    directory (load <= 1/16).
  PhaseTimer pt;
  const int m = Mo.dec.m, M = 1 << m, R = 1 << Mo.dec.n, nw = nib_words(m);
  Mo.h_rsw = row_words(Mo.dec.n);
  // Key and record of a slot in one power-of-two slot (128 B at m = 6, n = 2): a
  // hit reads one line instead of a key line and a record line (p = 0.1 launch
  // 3,122 -> 2,969 ms, profiles/r02z5_il/).  h_row_rows stays empty and the device
  // record base is the key base + nw dwords.  CVD_SLOT_IL=0: separate key and
  // record arrays (timing studies).
  const char* il = std::getenv("CVD_SLOT_IL");
  const bool interleave = !(il && std::atoi(il) == 0);
  int ssw = nw;
  if (interleave)
    for (ssw = 1; ssw < nw + Mo.h_rsw;) ssw <<= 1;
  Mo.h_ssw = ssw;
  // Load factor <= 1/16: a hit is at its home slot ~97% of the time, and every
  // probe past it is a dependent line read (p = 0.1: 2,972 ms at 1/8, 2,925 at
  // 1/16, 3,095 at 1/4, profiles/r02z6_dir/).  Device offsets are 32-bit byte
  // offsets, so a table past 4 GiB runs at a higher load (down to 1/2).
  // (CVD_DIR_LOAD_LOG2=s: load <= 2^-s, for timing studies)
  int load_log2 = 4;
  if (const char* e = std::getenv("CVD_DIR_LOAD_LOG2")) load_log2 = std::max(1, std::min(5, std::atoi(e)));
  int64_t cap = 64;
  while (cap < ((int64_t)1 << load_log2) * Mo.n_rows) cap <<= 1;
  const int64_t slot_bytes = 4 * (int64_t)std::max(ssw, interleave ? 0 : Mo.h_rsw);
  while (cap * slot_bytes > ((int64_t)1 << 32) && cap / 2 >= 2 * Mo.n_rows && cap > 64) cap >>= 1;
  if (cap * slot_bytes > ((int64_t)1 << 32) || cap < 2 * Mo.n_rows)
    throw std::length_error("explicit-path row table over 4 GiB (too many learned rows)");
  Mo.hcap = cap;
  int64_t fcap = 64;
  // >= 32 filter bits per row: a non-row passes the one-word filter ~0.25% of the
  // time (~1% at 16 bits), and every false positive costs the wave the key and
  // record loads and the key compare.  But at most 2 MiB: the filter must stay
  // L2-resident beside the streams (4 MiB at p = 0.1, 8.2e5 rows, measured 9%
  // slower per launch than 2 MiB, profiles/r02h/filter.jsonl).
  // (CVD_FILTER_SCALE=s: filter words >= rows * 2^s, CVD_FILTER_MAX_LOG2: the
  // cap, for timing studies)
  // Walking models of <= 32,768 rows (p = 0.01 in the sweep: 29,626): 2^14 words, 64 KiB,
  // so that the specialised kernel keeps the whole filter in LDS (ldsf_preferred,
  // cvd_kernels.hip): up to 4 keys per two-word block, ~0.06% false positives, against an
  // L2 read per H2 step.
  const bool bsp = bitslice_preferred(Mo);
  const bool ldsf = ldsf_wanted(Mo) && Mo.n_rows <= ldsf_max_rows(bsp) && !std::getenv("CVD_NO_LDSF");
  int fscale = 0, fmax_log2 = ldsf ? ldsf_log2(bsp) : 19;
  if (const char* e = std::getenv("CVD_FILTER_SCALE")) fscale = std::max(-3, std::min(3, std::atoi(e)));
  if (const char* e = std::getenv("CVD_FILTER_MAX_LOG2")) fmax_log2 = std::max(8, std::min(28, std::atoi(e)));
  while ((fscale >= 0 ? fcap >> fscale : fcap << -fscale) < Mo.n_rows && fcap < ((int64_t)1 << fmax_log2)) fcap <<= 1;
  Mo.fcap = fcap;
  Mo.h_filt.assign((size_t)fcap, 0u);
  Mo.h_filt_lds.assign(ldsf ? (size_t)fcap : 0u, 0u);
  const unsigned npat = (unsigned)kFilterPatterns;   // the kernels' pattern table (cvd_keys.h)
  Mo.h_key_rows.assign((size_t)Mo.n_rows * ssw, kEmptyKey);
  Mo.h_key_slot.assign((size_t)Mo.n_rows, 0u);
  Mo.h_row_rows.assign(interleave ? 0 : (size_t)Mo.n_rows * Mo.h_rsw, 0u);
  Mo.h_drow.assign((size_t)Mo.n_rows * Mo.h_rsw, 0u);
  Mo.max_probe = 0;
  pt.mark("  nibble tables: allocate");
  // Device row ids (drow index, successor fields, slot0): rows by descending visit count
  // of the learning chain, which is the trial streams' own process (encoder G1, BSC(p)),
  // so the rows table walks read most sit together in few cache lines instead of in
  // first-visit order (CVD_ROW_ORDER=first keeps first-visit order).  Only the device
  // numbering changes; lookups resolve to the same rows.
  std::vector<int64_t> dev_of((size_t)Mo.n_rows);
  for (int64_t i = 0; i < Mo.n_rows; ++i) dev_of[(size_t)i] = i;
  {
    const char* ro = std::getenv("CVD_ROW_ORDER");
    const bool hot = !(ro && std::string(ro) == "first");
    if (hot && (int64_t)Mo.visits.size() == Mo.n_rows) {
      std::vector<int64_t> order((size_t)Mo.n_rows);
      for (int64_t i = 0; i < Mo.n_rows; ++i) order[(size_t)i] = i;
      std::stable_sort(order.begin(), order.end(),
                       [&](int64_t x, int64_t y) { return Mo.visits[(size_t)x] > Mo.visits[(size_t)y]; });
      for (int64_t k = 0; k < Mo.n_rows; ++k) dev_of[(size_t)order[(size_t)k]] = k;
    }
  }
  std::vector<int64_t> slot_of((size_t)Mo.n_rows);
  std::vector<uint32_t> kws((size_t)Mo.n_rows * nw), phs((size_t)Mo.n_rows), pls((size_t)Mo.n_rows);
  parallel_for(Mo.n_rows, [&](int64_t i, int) {
    uint32_t* kw = kws.data() + (size_t)i * nw;
    pack_nibbles(Mo.keys.data() + (size_t)i * M, M, kw);
    if (M >= 8)
      for (int w = 0; w < nw; ++w) kw[w] = key_swap(kw[w]);   // device key layout
    key_hash(kw, nw, phs[(size_t)i], pls[(size_t)i]);
  });
  std::vector<uint8_t> occupied((size_t)cap, 0);
  for (int64_t i = 0; i < Mo.n_rows; ++i) {
    const uint32_t* kw = kws.data() + (size_t)i * nw;
    const uint32_t ph = phs[(size_t)i], pl = pls[(size_t)i];
    const size_t fb = (size_t)filter_block_index(pl, (uint32_t)(fcap / 2 - 1));
    Mo.h_filt[2 * fb] |= filter_pattern(filter_pattern_index(ph, npat));
    Mo.h_filt[2 * fb + 1] |= filter_pattern_hi(filter_pattern_index(ph, npat), npat);
    if (ldsf) {
      const unsigned nl = 1u << kFilterPatBitsLds;
      Mo.h_filt_lds[2 * fb] |= filter_pattern(filter_pattern_index(ph, nl));
      Mo.h_filt_lds[2 * fb + 1] |= filter_pattern_hi(filter_pattern_index(ph, nl), nl);
    }
    uint64_t slot = ph & (uint64_t)(cap - 1);
    int probe = 0;
    while (occupied[slot]) { slot = (slot + 1) & (uint64_t)(cap - 1); ++probe; }
    occupied[slot] = 1;
    Mo.max_probe = std::max(Mo.max_probe, probe);
    for (int w = 0; w < nw; ++w) Mo.h_key_rows[(size_t)i * ssw + w] = kw[w];
    Mo.h_key_slot[(size_t)i] = (uint32_t)slot;
    slot_of[(size_t)i] = (int64_t)slot;
  }
  pt.mark("  nibble tables: hash + insert");
  // row keys by device row id (the walk mode of the specialised kernel rebuilds a
  // lane's metric vector from the key of the last row it walked)
  Mo.h_dkey.assign((size_t)Mo.n_rows * nw, 0u);
  const Tabs T = make_tabs(Mo.dec);
  parallel_for(Mo.n_rows, [&](int64_t i, int) {
    // entry r = 16 bytes {log P̂1[r] (f64), successor row (i32, -1: none), T_ref count
    // c(r)}: one 12-byte device load per step (16 in walk mode).  c(r) = the words q
    // with successor(q) == successor(r) as metric vectors (Pd_plotter.py:89-99, the
    // |Y| the butterfly kernel derives from the halves test).
    uint32_t* dw = Mo.h_drow.data() + (size_t)dev_of[(size_t)i] * Mo.h_rsw;
    const uint8_t* D = Mo.keys.data() + (size_t)i * M;
    uint8_t succ[16][256];
    for (int r = 0; r < R; ++r) step_host(T, D, (uint32_t)r, succ[r]);
    for (int r = 0; r < R; ++r) {
      std::memcpy(dw + 4 * r, Mo.logp1.data() + (size_t)i * R + r, sizeof(double));
      const int64_t j = Mo.row_next[(size_t)i * R + r];
      dw[4 * r + 2] = (uint32_t)(j >= 0 ? (int32_t)dev_of[(size_t)j] : -1);
      uint32_t c = 0u;
      for (int q2 = 0; q2 < R; ++q2) c += std::memcmp(succ[q2], succ[r], (size_t)M) == 0;
      dw[4 * r + 3] = c;
    }
    std::memcpy(Mo.h_dkey.data() + (size_t)dev_of[(size_t)i] * nw, kws.data() + (size_t)i * nw,
                sizeof(uint32_t) * (size_t)nw);
    uint32_t* hw = interleave ? Mo.h_key_rows.data() + (size_t)i * ssw + nw
                              : Mo.h_row_rows.data() + (size_t)i * Mo.h_rsw;
    std::memcpy(hw, dw, sizeof(uint32_t) * Mo.h_rsw);
  });
  Mo.slot0 = (int32_t)dev_of[0];   // D_0 = 0 is row 0 in both model kinds
  pt.mark("  nibble tables: records");
  // Bit-sliced tables of the m = 6 kernel k1s (cvd_bitslice.h): the same rows and records,
  // found by the hash of the canonical digest plane z = bit0(D) ^ bit1(D) (one filter entry
  // per row whatever the lane's layout phase); a directory slot holds the row's image at
  // each of the six phases (the exact compare) and its record; a.dkey the six images by
  // device row id (walk mode).  Load <= 1/8 by default (CVD_BS_LOAD_LOG2): 256-B slots, so
  // the directory stays within 2 GiB at 10^6 rows; the kernel addresses it by 32-bit byte offsets.
  Mo.bs = bitslice_preferred(Mo);
  int bload = 3;
  if (const char* e = std::getenv("CVD_BS_LOAD_LOG2")) bload = std::max(1, std::min(5, std::atoi(e)));
  int64_t bcap = 64;
  while (bcap < ((int64_t)1 << bload) * Mo.n_rows) bcap <<= 1;
  // the kernel addresses the directory, the two-step records and the images by 32-bit byte
  // offsets: past 4 GiB (over ~2·10^6 rows) the model keeps the nibble tables
  // directory slots of 256 B, or three 128-B lines {two phase images, record} (CVD_BS_SLOT3=1)
  const char* s3 = std::getenv("CVD_BS_SLOT3");
  Mo.bs_slot_w = s3 && s3[0] == '1' ? 96 : 64;
  if (bcap * 4 * Mo.bs_slot_w > ((int64_t)1 << 32) || Mo.n_rows * 512 > ((int64_t)1 << 32)) Mo.bs = false;
  Mo.h_bfilt.clear(); Mo.h_bfilt_lds.clear(); Mo.h_bkey_rows.clear(); Mo.h_bkey_slot.clear(); Mo.h_bdkey.clear();
  Mo.h_bpf.clear();
  Mo.bhcap = 0; Mo.bmax_probe = 0;
  if (Mo.bs) {
    // the filter's pattern table (kernel LDS: 8 B per pattern pair); CVD_BS_PAT_BITS 8..12
    Mo.bs_pat_bits = kFilterPatBits;
    if (const char* e = std::getenv("CVD_BS_PAT_BITS")) Mo.bs_pat_bits = std::max(8, std::min(kFilterPatBits, std::atoi(e)));
    // the LDS pre-filter (a 1,024-thread block holds it beside the pattern table, which then
    // has 1,024 pairs)
    const bool bpf = bs_pf_preferred(Mo, ldsf);
    if (bpf) {
      Mo.bs_pat_bits = std::min(Mo.bs_pat_bits, (int32_t)kFilterPatBitsLds);
      Mo.bs_pf_log2 = kBsPfLog2Bits;
      if (const char* e = std::getenv("CVD_BS_PF_LOG2")) Mo.bs_pf_log2 = std::max(16, std::min(20, std::atoi(e)));
      Mo.h_bpf.assign((size_t)1 << (Mo.bs_pf_log2 - 5), 0u);
    }
    const unsigned bnpat = 1u << Mo.bs_pat_bits;
    Mo.bhcap = bcap;
    constexpr int kRecW = 48, kImgW = 48;
    const int kSlotW = Mo.bs_slot_w;
    Mo.h_bkey_rows.assign((size_t)Mo.n_rows * kSlotW, 0u);   // (the empty slots: zero, c = 0 in every record)
    Mo.h_bkey_slot.assign((size_t)Mo.n_rows, 0u);
    Mo.h_bfilt.assign((size_t)fcap, 0u);
    Mo.h_bfilt_lds.assign(ldsf ? (size_t)fcap : 0u, 0u);
    Mo.h_bdkey.assign((size_t)Mo.n_rows * kImgW, 0u);
    pt.mark("  bit-sliced tables: allocate");
    std::vector<uint32_t> bph((size_t)Mo.n_rows), bpl((size_t)Mo.n_rows);
    parallel_for(Mo.n_rows, [&](int64_t i, int) {
      uint32_t z[2];
      bs_digest(Mo.keys.data() + (size_t)i * M, z);
      bs_key_hash(z[0], z[1], bph[(size_t)i], bpl[(size_t)i]);
    });
    std::vector<uint8_t> used((size_t)bcap, 0);
    for (int64_t i = 0; i < Mo.n_rows; ++i) {
      const uint32_t ph = bph[(size_t)i], pl = bpl[(size_t)i];
      const size_t fb = (size_t)filter_block_index(pl, (uint32_t)(fcap / 2 - 1));
      Mo.h_bfilt[2 * fb] |= filter_pattern(filter_pattern_index(ph, bnpat));
      Mo.h_bfilt[2 * fb + 1] |= filter_pattern_hi(filter_pattern_index(ph, bnpat), bnpat);
      if (ldsf) {
        const unsigned nl = 1u << kFilterPatBitsLds;
        Mo.h_bfilt_lds[2 * fb] |= filter_pattern(filter_pattern_index(ph, nl));
        Mo.h_bfilt_lds[2 * fb + 1] |= filter_pattern_hi(filter_pattern_index(ph, nl), nl);
      }
      if (bpf) {
        const uint32_t b = pl >> (32 - Mo.bs_pf_log2);
        Mo.h_bpf[b >> 5] |= 1u << (b & 31u);
      }
      uint64_t slot = ph & (uint64_t)(bcap - 1);
      int probe = 0;
      while (used[slot]) { slot = (slot + 1) & (uint64_t)(bcap - 1); ++probe; }
      used[slot] = 1;
      Mo.bmax_probe = std::max(Mo.bmax_probe, probe);
      Mo.h_bkey_slot[(size_t)i] = (uint32_t)slot;
    }
    pt.mark("  bit-sliced tables: hash + insert");
    parallel_for(Mo.n_rows, [&](int64_t i, int) {
      uint32_t* sp = Mo.h_bkey_rows.data() + (size_t)i * kSlotW;
      uint32_t* dk = Mo.h_bdkey.data() + (size_t)dev_of[(size_t)i] * kImgW;
      const uint32_t* rec = Mo.h_drow.data() + (size_t)dev_of[(size_t)i] * Mo.h_rsw;
      for (int ph = 0; ph < 6; ++ph) {
        bs_image(Mo.keys.data() + (size_t)i * M, ph, dk + 8 * ph);
        // (slot3: image of phase ph at dword 32 (ph / 2) + 8 (ph % 2) of the line ph / 2)
        std::memcpy(sp + (kSlotW == 96 ? 32 * (ph / 2) + 8 * (ph % 2) : 8 * ph), dk + 8 * ph, 8 * sizeof(uint32_t));
      }
      if (kSlotW == 96)
        for (int k = 0; k < 3; ++k) std::memcpy(sp + 32 * k + 16, rec, sizeof(uint32_t) * 16);
      else
        std::memcpy(sp + kRecW, rec, sizeof(uint32_t) * 16);
    });
  }
  pt.mark("  bit-sliced tables: images + records");
  // two-step walk records (k1b_walk), for models that walk: per device row d and word pair
  // (r1, r2), 32 B {log P̂1(d, r1), log P̂1(d1, r2), (d1 + 1) | c(d, r1) << 28,
  // (d2 + 1) | c(d1, r2) << 28}, d1 / d2 the rows after one / two steps (0 = not a row)
  Mo.h_t2.clear();
  Mo.h_t2c.clear();
  Mo.h_vtab.clear();
  // (CVD_BS_T2=1: for the bit-sliced lockstep lanes too, whose kernel reads them with
  // -DCVD_K1S_T2=1 in CVD_JIT_DEFINES; timing studies, cvd_k1s.h)
  const char* bt2 = std::getenv("CVD_BS_T2");
  if (Mo.dec.k == 1 && R == 4 && (walk_preferred(Mo) || (Mo.bs && bt2 && bt2[0] == '1'))) {
    Mo.h_t2.assign((size_t)Mo.n_rows * 16 * 8, 0u);
    parallel_for(Mo.n_rows, [&](int64_t d, int) {
      const uint32_t* a0 = Mo.h_drow.data() + (size_t)d * Mo.h_rsw;
      for (int r1 = 0; r1 < 4; ++r1) {
        const int32_t d1 = (int32_t)a0[4 * r1 + 2];
        for (int r2 = 0; r2 < 4; ++r2) {
          uint32_t* e = Mo.h_t2.data() + ((size_t)d * 16 + (size_t)(r1 | (r2 << 2))) * 8;
          e[0] = a0[4 * r1];
          e[1] = a0[4 * r1 + 1];
          e[4] = (uint32_t)(d1 + 1) | (a0[4 * r1 + 3] << 28);
          if (d1 >= 0) {
            const uint32_t* a1 = Mo.h_drow.data() + (size_t)d1 * Mo.h_rsw;
            e[2] = a1[4 * r2];
            e[3] = a1[4 * r2 + 1];
            e[5] = (uint32_t)((int32_t)a1[4 * r2 + 2] + 1) | (a1[4 * r2 + 3] << 28);
          }
        }
      }
    });
    // the compact form (CVD_WALK_T2C=1; 8 B per record for the k1s walk, a quarter of the
    // table's bytes: at p = 0.01's 29,626 rows 3.8 MB instead of 15 MB) where rows + 1 fit 16
    // bits and the distinct log P̂1 values 12.  Same sums; p = 0.01 1,498 against 1,500-1,505 ms
    // per launch (profiles/r06p): the walk waits on its dependent chain, not on the table's
    // size, so it is not the default
    const char* t2c = std::getenv("CVD_WALK_T2C");
    if (Mo.bs && Mo.n_rows < 65535 && t2c && t2c[0] == '1') {
      std::vector<uint64_t> bits(Mo.logp1.size());
      std::memcpy(bits.data(), Mo.logp1.data(), bits.size() * sizeof(double));
      std::sort(bits.begin(), bits.end());
      bits.erase(std::unique(bits.begin(), bits.end()), bits.end());
      if (bits.size() <= 4096) {
        Mo.h_vtab.resize(bits.size());
        std::memcpy(Mo.h_vtab.data(), bits.data(), bits.size() * sizeof(double));
        auto idx = [&](uint32_t lo, uint32_t hi) -> uint64_t {
          const uint64_t b = (uint64_t)lo | ((uint64_t)hi << 32);
          return (uint64_t)(std::lower_bound(bits.begin(), bits.end(), b) - bits.begin());
        };
        Mo.h_t2c.assign((size_t)Mo.n_rows * 16 * 2, 0u);
        parallel_for(Mo.n_rows, [&](int64_t d, int) {
          for (int q = 0; q < 16; ++q) {
            const uint32_t* e = Mo.h_t2.data() + ((size_t)d * 16 + (size_t)q) * 8;
            const uint64_t d1 = e[4] & 0x0FFFFFFFu, c1 = e[4] >> 28, d2 = e[5] & 0x0FFFFFFFu, c2 = e[5] >> 28;
            const uint64_t i1 = idx(e[0], e[1]), i2 = d1 ? idx(e[2], e[3]) : 0u;
            const uint64_t w = i1 | (i2 << 12) | (d1 << 24) | (c1 << 40) | (d2 << 43) | (c2 << 59);
            Mo.h_t2c[((size_t)d * 16 + (size_t)q) * 2] = (uint32_t)w;
            Mo.h_t2c[((size_t)d * 16 + (size_t)q) * 2 + 1] = (uint32_t)(w >> 32);
          }
        });
      }
    }
  }
}

void build_bmk1(cvd_model& Mo, const Tabs& T) {
  // g0 = output word of (state 0, input 1): the tap-0 column over the outputs
  const uint32_t g0 = T.out[0 * T.K + 1];
  if (T.k != 1 || T.n < 2 || T.n > 3 || g0 == 0) return;
  std::vector<int> reps;
  for (int r = 0; r < T.R; ++r)
    if ((uint32_t)r < ((uint32_t)r ^ g0)) reps.push_back(r);
  Mo.repmap = 0; Mo.swmap = 0;
  for (int r = 0; r < T.R; ++r) {
    const int rep = std::min<int>(r, r ^ (int)g0);
    const int idx = (int)(std::find(reps.begin(), reps.end(), rep) - reps.begin());
    Mo.repmap |= (uint32_t)idx << (4 * r);
    Mo.swmap |= (uint32_t)(r != rep) << r;
  }
  const int QP = (int)reps.size() / 2;
  Mo.bmk1.assign((size_t)QP * T.M * 2, 0u);
  for (int qp = 0; qp < QP; ++qp)
    for (int ns = 0; ns < T.M; ++ns)
      for (int b = 0; b < 2; ++b) {
        const int pred = (ns >> 1) | (b << (T.m - 1));
        const uint32_t o = T.out[pred * T.K + (ns & 1)];
        const uint32_t b0 = __builtin_popcount(o ^ (uint32_t)reps[2 * qp]);
        const uint32_t b1 = __builtin_popcount(o ^ (uint32_t)reps[2 * qp + 1]);
        Mo.bmk1[((size_t)qp * T.M + ns) * 2 + b] = b0 | (b1 << 16);
      }
  Mo.k1_ok = true;
}

void build_bfly(cvd_model& Mo, const Tabs& T) {
  // Standard butterfly: out(j, 1) = out(j, 0) ^ 3 and out(j + 2^(m-1), u) =
  // out(j, u) ^ 3 for every j (tap-0 and tap-m columns both 11).  Then the two
  // ACS candidates of states (2j, 2j+1) carry metrics (e, 2-e) and (2-e, e),
  // e = popcount(out(j, 0) ^ y).
  if (T.k != 1 || T.n != 2 || T.m < 3) return;
  const int H = T.M / 2;
  for (int j = 0; j < H; ++j) {
    const uint32_t x = T.out[j * T.K + 0];
    if (T.out[j * T.K + 1] != (x ^ 3u) || T.out[(j + H) * T.K + 0] != (x ^ 3u) ||
        T.out[(j + H) * T.K + 1] != x)
      return;
  }
  Mo.bfly.assign((size_t)H, 0u);
  Mo.bfly_uni = 1u;
  Mo.bfly_x = 0u;
  for (uint32_t& w : Mo.bfly_even) w = 0u;
  for (int j = 0; j < H; ++j) {
    const uint32_t x = T.out[j * T.K + 0];
    for (uint32_t y = 0; y < 4; ++y) Mo.bfly[(size_t)j] |= (uint32_t)__builtin_popcount(x ^ y) << (8 * y);
    // class of out(j, 0): {00, 11} or {01, 10}; out(0, 0) = 00
    Mo.bfly_x |= (uint64_t)x << (2 * j);
    if (__builtin_popcount(x) & 1) Mo.bfly_uni = 0u;
    // nibble of state j in the halves-difference words (device key layout)
    else Mo.bfly_even[j / 8] |= 0xFu << (4 * key_nibble(T.M, j));
  }
  Mo.k1b_ok = true;
}

void build_bmp(cvd_model& Mo, const Tabs& T) {
  if (!explicit_supported(T.m, T.k, T.n)) return;
  build_bmk1(Mo, T);
  build_bfly(Mo, T);
  const int QP = T.R / 2;
  Mo.bmp.assign((size_t)QP * T.M * T.K, 0u);
  for (int qp = 0; qp < QP; ++qp)
    for (int ns = 0; ns < T.M; ++ns)
      for (int b = 0; b < T.K; ++b) {
        const int pred = (ns >> T.k) | (b << (T.m - T.k));
        const int U = ns & (T.K - 1);
        const uint32_t o = T.out[pred * T.K + U];
        const uint32_t b0 = __builtin_popcount(o ^ (uint32_t)(2 * qp));
        const uint32_t b1 = __builtin_popcount(o ^ (uint32_t)(2 * qp + 1));
        Mo.bmp[((size_t)qp * T.M + ns) * T.K + b] = b0 | (b1 << 16);
      }
}

}  // namespace

int cvd::ldsf_log2(bool bs) {
  // the bit-sliced kernel's persistent blocks hold a 128-KiB filter one block per CU (p = 0.01:
  // 1,440 vs 1,511 ms per launch with 64 KiB in two 512-thread blocks, profiles/r05l); the
  // nibble kernel keeps 64 KiB (profiles/r03x)
  const char* e = std::getenv("CVD_LDSF_LOG2");
  return e && *e ? std::max(13, std::min(15, std::atoi(e))) : (bs ? 15 : kLdsFilterLog2);
}
// (the bit-sliced kernel's lockstep lanes gain from the 128-KiB LDS filter up to p = 0.02's
// 70,134 rows: 1,442-1,443 ms per launch against 1,497-1,499 with the pre-filter and L2 filter,
// profiles/r06ak; at p = 0.05's 315,953 rows it is saturated, 4,770-4,789 against 1,860,
// profiles/r06al: so up to 3 x 32,768 rows)
int64_t cvd::ldsf_max_rows(bool bs) {
  const char* e = std::getenv("CVD_LDSF_MAX_ROWS");
  return e && *e ? (int64_t)std::atoll(e)
                 : (bs ? 3 : 1) * (kLdsFilterMaxRows << std::max(0, ldsf_log2(bs) - (bs ? 15 : kLdsFilterLog2)));
}

bool cvd::bs_pf_preferred(const cvd_model& M, bool ldsf) {
  const char* e = std::getenv("CVD_BS_PF");
  if (e && e[0] == '0') return false;
  return M.bs && !ldsf;
}

bool cvd::bitslice_preferred(const cvd_model& M) {
  const char* e = std::getenv("CVD_BITSLICE");
  if (e && e[0] == '0') return false;
  return M.k1b_ok && M.dec.k == 1 && M.dec.n == 2 && M.dec.m == 6;
}

bool cvd::explicit_supported(int m, int k, int n) {
  // nibble storage of un-normalised metrics: D <= ceil(m/k)*n, plus one branch (<= n)
  const int L = (m + k - 1) / k;
  const bool shape = (m == 2 && k == 1 && n == 2) || (m == 3 && k == 1 && n == 2) ||
                     (m == 4 && k == 1 && n == 2) || (m == 5 && k == 1 && n == 2) ||
                     (m == 6 && k == 1 && n == 2) || (m == 4 && k == 2 && n == 3);
  return shape && (L + 1) * n <= 15;
}

namespace {
// The GPU chain refused the model (a shape or chain length it does not take, or
// too little device memory for its scratch): the host chain, which gives the
// same model bit for bit, runs instead (recorded in LearnStats).  Any other
// device error is returned as is.
bool device_refused(int rc, LearnStats* stats) {
  if (rc != CVD_E_UNSUPPORTED && rc != CVD_E_CAPACITY) return false;
  if (stats) stats->host_fallback = 1;
  return true;
}

// cvd_model_create / cvd_model_create_device: the learning chain on the host
// (device < 0) or on a GPU (cvd_learn.hip; same outputs), everything else shared.
int model_create(const cvd_code* dec, const cvd_learn_params* prm, int device, void* stream, cvd_model** out,
                 LearnStats* stats) {
  CVD_TRY
  if (!prm || !out) { set_error("null argument"); return CVD_E_INVALID; }
  *out = nullptr;
  if (!(prm->p >= 0.0 && prm->p <= 1.0)) { set_error("p must lie in [0, 1]"); return CVD_E_INVALID; }
  if (!(prm->laplace >= 0.0) || prm->learn_burn < 0) { set_error("bad learning parameters"); return CVD_E_INVALID; }
  std::unique_ptr<cvd_model> Mo(new cvd_model());
  int rc = parse_code(dec, Mo->dec);
  if (rc) return rc;
  Tabs T = make_tabs(Mo->dec);
  const int M = T.M, R = T.R;
  Mo->laplace = prm->laplace;
  Mo->ltref.resize((size_t)R + 1);
  for (int c = 0; c <= R; ++c) Mo->ltref[c] = ltref_value(c, R);
  const uint64_t seed = prm->seed;

  PhaseTimer pt;
  std::vector<uint8_t> states;
  std::vector<int32_t> next;
  int64_t S = 0;
  const int64_t cap = prm->enum_cap > 0 ? prm->enum_cap : 0;
  // a code whose BFS outgrew the cap once always will: remember it per
  // process (the model is built once per p, the BFS outcome is p-independent)
  static std::mutex bfs_mu;
  static std::map<std::tuple<int, int, int, std::vector<uint32_t>>, int64_t> bfs_too_big;   // -> largest cap tried
  const auto ckey = std::make_tuple(T.m, T.k, T.n,
                                    std::vector<uint32_t>(Mo->dec.gmask, Mo->dec.gmask + T.n * T.k));
  // (the lock is held over the BFS: models of one code built on several threads at once --
  // Detector.prepare_models -- wait for the first thread's verdict instead of each running the
  // capped BFS, 0.2-0.5 s of CPU per model of the m = 6 code)
  {
    std::lock_guard<std::mutex> lk(bfs_mu);
    auto it = bfs_too_big.find(ckey);
    const bool known_big = it != bfs_too_big.end() && it->second >= cap;
    rc = (cap > 0 && !known_big) ? bfs(T, cap, states, next, S) : CVD_E_CAPACITY;
    if (rc == CVD_E_CAPACITY && cap > 0 && !known_big) {
      int64_t& c = bfs_too_big[ckey];
      c = std::max(c, cap);
    }
  }
  pt.mark("bfs");
  std::unordered_map<int64_t, double> memo;

  if (rc == CVD_OK && prm->laplace_states > 0 && prm->laplace_states != S) {
    set_error("laplace_states: an enumerable code's Laplace denominator is its BFS state count");
    return CVD_E_INVALID;
  }
  if (rc == CVD_OK) {
    // ── dense model: the reference's exact semantics (Pd_plotter.py:123-169) ──
    Mo->kind = 0;
    Mo->S = S;
    const int64_t L = prm->learn_len < 0 ? std::max<int64_t>(5000, 200 * S) : prm->learn_len;
    Mo->learn_len_eff = L;
    std::vector<int64_t> cnt((size_t)S * R, 0);
    bool on_host = true;
    if (device >= 0 && L >= 1) {   // (an empty chain, L = 0, has nothing to run)
      rc = device_learn_dense(Mo->dec, next, S, L, prm->learn_burn, seed, prm->p, device, stream, cnt, stats);
      on_host = device_refused(rc, stats);
      if (rc && !on_host) return rc;
      if (on_host) cnt.assign((size_t)S * R, 0);
    }
    if (on_host) {
      HostStream hs(Mo->dec, T, seed, kLearnTag, 0, prm->p, true);
      int64_t i = 0;   // D_0 = 0 is BFS index 0
      for (int64_t t = 0; t < L; ++t) {
        const uint32_t r = hs.next_word(t);
        if (t >= prm->learn_burn) cnt[(size_t)i * R + r]++;
        i = next[(size_t)i * R + r];
      }
    }
    pt.mark("chain");
    Mo->n_rows = S;
    Mo->keys = std::move(states);
    Mo->visits.assign((size_t)S, 0);
    for (int64_t s2 = 0; s2 < S; ++s2)
      for (int r = 0; r < R; ++r) Mo->visits[(size_t)s2] += cnt[(size_t)s2 * R + r];
    Mo->logp1.assign((size_t)S * R, 0.0);
    Mo->rec.assign((size_t)S * R, 0u);
    std::vector<int64_t> succ((size_t)R);
    std::vector<std::pair<int64_t, double>> nz;
    Mo->rowsum.assign((size_t)S, 0.0);
    for (int64_t s = 0; s < S; ++s) {
      for (int r = 0; r < R; ++r) succ[r] = next[(size_t)s * R + r];
      for (int r = 0; r < R; ++r) Mo->row_next.push_back(succ[r]);
      Mo->rowsum[(size_t)s] = p1_row(S, prm->laplace, memo, succ.data(), cnt.data() + (size_t)s * R, R,
                                     Mo->logp1.data() + (size_t)s * R, &nz);
      for (auto& e : nz) Mo->p1_nz.push_back({s, e.first, e.second});
      for (int r = 0; r < R; ++r) {
        int c = 0;
        for (int q = 0; q < R; ++q) c += succ[q] == succ[r];
        Mo->rec[(size_t)s * R + r] = ((uint32_t)succ[r] << 4) | (uint32_t)c;
      }
    }
    {
      std::vector<int64_t> none((size_t)R, -1), zc((size_t)R, 0);
      std::vector<double> lp((size_t)R);
      p1_row(S, prm->laplace, memo, none.data(), zc.data(), R, lp.data());
      Mo->logp1_unseen = lp[0];
    }
  } else if (rc == CVD_E_CAPACITY) {
    // ── sparse model: rows = states visited by the learning chain ──
    // The reference's semantics need the full BFS index (Pd_plotter.py:136-139,
    // 166-167), infeasible here (m = 6: > 2e8 states).  Declared policy
    // (deviation D4): the state set is the chain's visited states
    // D_0..D_L in first-visit order, S = their number, unvisited rows are the
    // all-zero-count row λ / (S λ).
    Mo->kind = 1;
    const int64_t L = prm->learn_len >= 0 ? prm->learn_len
                                          : (prm->default_learn_len > 0 ? prm->default_learn_len : 1000000);
    Mo->learn_len_eff = L;
    std::vector<uint8_t> keys;
    StateMap map(M, &keys);
    std::vector<int64_t> cnt;
    bool on_host = true;
    if (device >= 0 && L >= 1) {
      // the chain on the GPU: rows in first-visit order + counts; the host map is
      // rebuilt from the rows (insertion order = row order) for the successors
      std::vector<uint8_t> rows;
      int64_t Sd = 0;
      rc = device_learn_sparse(Mo->dec, L, prm->learn_burn, seed, prm->p, device, stream, rows, cnt, Sd, stats);
      on_host = device_refused(rc, stats);
      if (rc && !on_host) return rc;
      if (!on_host) {
        map.reserve(Sd);
        bool ins;
        for (int64_t s = 0; s < Sd; ++s) {
          map.insert(rows.data() + (size_t)s * M, ins);
          if (!ins) { set_error("GPU learning: duplicate row key"); return CVD_E_STATE; }
        }
      } else {
        cnt.clear();
      }
    }
    if (on_host) {
      map.reserve(std::min<int64_t>(L + 1, (int64_t)1 << 26));
      std::vector<uint8_t> D((size_t)M, 0), Dn((size_t)M);
      const HostStep step(T);
      bool ins;
      int64_t i = map.insert(D.data(), ins);
      cnt.resize((size_t)R, 0);
      HostStream hs(Mo->dec, T, seed, kLearnTag, 0, prm->p, true);
      for (int64_t t = 0; t < L; ++t) {
        const uint32_t r = hs.next_word(t);
        if (t >= prm->learn_burn) cnt[(size_t)i * R + r]++;
        step(D.data(), r, Dn.data());
        int64_t j = map.insert(Dn.data(), ins);
        if (ins) cnt.resize((size_t)map.count * R, 0);
        std::swap(D, Dn);
        i = j;
      }
    }
    pt.mark("chain");
    const HostStep step(T);
    const int64_t rows = map.count;
    // Laplace denominator S * laplace (Pd_plotter.py:166-167): the visited rows (D4),
    // or a state count the caller measured / bounded (laplace_states)
    if (prm->laplace_states > 0 && prm->laplace_states < rows) {
      set_error("laplace_states below the number of visited states");
      return CVD_E_INVALID;
    }
    S = prm->laplace_states > 0 ? prm->laplace_states : rows;
    Mo->S = S;
    Mo->n_rows = rows;
    Mo->logp1.assign((size_t)rows * R, 0.0);
    Mo->row_next.assign((size_t)rows * R, -1);
    // successors and P̂1 rows: independent per row (read-only map), on host threads
    std::vector<std::unordered_map<int64_t, double>> memos(32);
    parallel_for(rows, [&](int64_t s, int tid) {
      uint8_t nb[256];
      int64_t succ[16];
      for (int r = 0; r < R; ++r) {
        step(keys.data() + (size_t)s * M, (uint32_t)r, nb);
        succ[r] = map.find(nb);
      }
      for (int r = 0; r < R; ++r) Mo->row_next[(size_t)s * R + r] = succ[r];
      p1_row(S, prm->laplace, memos[(size_t)tid], succ, cnt.data() + (size_t)s * R, R,
             Mo->logp1.data() + (size_t)s * R);
    });
    pt.mark("successors + P1 rows");
    Mo->keys = std::move(keys);
    Mo->visits.assign((size_t)rows, 0);
    for (int64_t s2 = 0; s2 < rows; ++s2)
      for (int r = 0; r < R; ++r) Mo->visits[(size_t)s2] += cnt[(size_t)s2 * R + r];
    std::vector<int64_t> none((size_t)R, -1), zc((size_t)R, 0);
    std::vector<double> lp((size_t)R);
    p1_row(S, prm->laplace, memo, none.data(), zc.data(), R, lp.data());
    Mo->logp1_unseen = lp[0];
  } else {
    return rc;
  }
  if (explicit_supported(T.m, T.k, T.n)) {
    build_bmp(*Mo, T);   // (first: the butterfly check decides the bit-sliced tables)
    build_hash(*Mo);
    pt.mark("row table");
  }
  *out = Mo.release();
  return CVD_OK;
  CVD_CATCH
}

// ───────────────────────── ABI: on-disk model cache ──────────────────────────
// A learned model is the reference's lru_cache entry (Pd_plotter.py:123-127) made
// persistent: the learned rows (keys, log P̂1, successors, dense extras) are
// written as length-prefixed blobs; the device-side tables (row hash, branch
// metrics) are rebuilt from them at load, exactly as cvd_model_create does.

namespace {
constexpr char kMagic[4] = {'C', 'V', 'D', 'M'};
constexpr uint32_t kFileVersion = 2;   // 2: + visits

struct Writer {
  FILE* f;
  bool ok = true;
  void raw(const void* p, size_t n) { ok = ok && std::fwrite(p, 1, n, f) == n; }
  template <typename T>
  void pod(const T& v) { raw(&v, sizeof(T)); }
  template <typename T>
  void vec(const std::vector<T>& v) {
    const uint64_t n = v.size();
    pod(n);
    if (n) raw(v.data(), n * sizeof(T));
  }
};

struct Reader {
  FILE* f;
  bool ok = true;
  void raw(void* p, size_t n) { ok = ok && std::fread(p, 1, n, f) == n; }
  template <typename T>
  void pod(T& v) { raw(&v, sizeof(T)); }
  template <typename T>
  void vec(std::vector<T>& v, uint64_t max_elems = (uint64_t)1 << 34) {
    uint64_t n = 0;
    pod(n);
    if (!ok || n > max_elems) { ok = false; return; }
    v.resize((size_t)n);
    if (n) raw(v.data(), (size_t)n * sizeof(T));
  }
};
}  // namespace

extern "C" int cvd_model_save(const cvd_model* Mo, const char* path) {
  CVD_TRY
  if (!Mo || !path) { set_error("null argument"); return CVD_E_INVALID; }
  // a tmp name of this process and thread (ranks sharing a cache directory save
  // the same model at once), then an atomic rename over the target
  static std::atomic<uint64_t> serial{0};
  const std::string tmp = std::string(path) + ".tmp." + std::to_string((long long)getpid()) + "." +
                          std::to_string((unsigned long long)std::hash<std::thread::id>()(std::this_thread::get_id())) +
                          "." + std::to_string((unsigned long long)serial++);
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) { set_error(std::string("cannot write ") + tmp); return CVD_E_INVALID; }
  Writer w{f};
  w.raw(kMagic, 4);
  w.pod(kFileVersion);
  w.pod((int32_t)CVD_ABI_VERSION);
  w.pod(Mo->dec);
  w.pod(Mo->kind); w.pod(Mo->S); w.pod(Mo->learn_len_eff); w.pod(Mo->laplace); w.pod(Mo->logp1_unseen);
  w.pod(Mo->n_rows);
  w.vec(Mo->ltref); w.vec(Mo->keys); w.vec(Mo->logp1); w.vec(Mo->rec); w.vec(Mo->rowsum);
  w.vec(Mo->p1_nz); w.vec(Mo->row_next); w.vec(Mo->visits);
  const bool ok = w.ok && std::fclose(f) == 0;
  // (a rename onto an existing file is atomic on POSIX: concurrent writers of one cache
  // entry never fail here, so a failure is real -- EACCES, EXDEV, ... -- and is reported)
  if (!ok || std::rename(tmp.c_str(), path) != 0) {
    std::remove(tmp.c_str());
    set_error(std::string("cannot write ") + path);
    return CVD_E_INVALID;
  }
  return CVD_OK;
  CVD_CATCH
}

extern "C" int cvd_model_load(const char* path, cvd_model** out) {
  CVD_TRY
  if (!path || !out) { set_error("null argument"); return CVD_E_INVALID; }
  *out = nullptr;
  FILE* f = std::fopen(path, "rb");
  if (!f) { set_error(std::string("cannot open ") + path); return CVD_E_INVALID; }
  std::unique_ptr<FILE, int (*)(FILE*)> guard(f, std::fclose);
  Reader r{f};
  char magic[4];
  uint32_t ver = 0;
  int32_t abi = 0;
  r.raw(magic, 4); r.pod(ver); r.pod(abi);
  if (!r.ok || std::memcmp(magic, kMagic, 4) != 0 || ver != kFileVersion || abi != CVD_ABI_VERSION) {
    set_error(std::string("not a model file of this build: ") + path);
    return CVD_E_INVALID;
  }
  std::unique_ptr<cvd_model> Mo(new cvd_model());
  r.pod(Mo->dec);
  r.pod(Mo->kind); r.pod(Mo->S); r.pod(Mo->learn_len_eff); r.pod(Mo->laplace); r.pod(Mo->logp1_unseen);
  r.pod(Mo->n_rows);
  r.vec(Mo->ltref); r.vec(Mo->keys); r.vec(Mo->logp1); r.vec(Mo->rec); r.vec(Mo->rowsum);
  r.vec(Mo->p1_nz); r.vec(Mo->row_next); r.vec(Mo->visits);
  const CodeDesc& d = Mo->dec;
  const bool shape_ok = d.k >= 1 && d.k <= kMaxK && d.n >= 1 && d.n <= kMaxN && d.m >= 1 && d.m <= kMaxM;
  const size_t M = shape_ok ? (size_t)1 << d.m : 0, R = shape_ok ? (size_t)1 << d.n : 0;
  bool valid = r.ok && shape_ok && (Mo->kind == 0 || Mo->kind == 1) && Mo->n_rows >= 1 &&
               Mo->n_rows < ((int64_t)1 << 31) && Mo->keys.size() == (size_t)Mo->n_rows * M &&
               Mo->logp1.size() == (size_t)Mo->n_rows * R && Mo->row_next.size() == (size_t)Mo->n_rows * R &&
               Mo->ltref.size() == R + 1 && Mo->visits.size() == (size_t)Mo->n_rows;
  // dense models: S rows, one 32-bit record and one row sum per (row, word) / row,
  // every record's successor a row; sparse: S = rows.  Successors must be rows or
  // -1, and every metric byte a nibble: the device tables are built from these
  // without further checks
  if (valid && Mo->kind == 0)
    valid = Mo->S == Mo->n_rows && Mo->rec.size() == (size_t)Mo->n_rows * R &&
            Mo->rowsum.size() == (size_t)Mo->n_rows;
  if (valid && Mo->kind == 1) valid = Mo->S >= Mo->n_rows;
  for (size_t i = 0; valid && i < Mo->row_next.size(); ++i)
    valid = Mo->row_next[i] >= -1 && Mo->row_next[i] < Mo->n_rows && (Mo->kind == 1 || Mo->row_next[i] >= 0);
  for (size_t i = 0; valid && i < Mo->rec.size(); ++i)
    valid = (int64_t)(Mo->rec[i] >> 4) < Mo->n_rows && (Mo->rec[i] & 15u) >= 1 && (Mo->rec[i] & 15u) <= R;
  for (size_t i = 0; valid && i < Mo->keys.size(); ++i) valid = Mo->keys[i] < 15;
  for (size_t i = 0; valid && i < Mo->p1_nz.size(); ++i)
    valid = Mo->p1_nz[i].row >= 0 && Mo->p1_nz[i].row < Mo->n_rows && Mo->p1_nz[i].col >= 0 &&
            Mo->p1_nz[i].col < Mo->n_rows;
  if (!valid) {
    set_error(std::string("corrupt model file: ") + path);
    return CVD_E_INVALID;
  }
  if (explicit_supported(d.m, d.k, d.n)) {
    Tabs T = make_tabs(Mo->dec);
    build_bmp(*Mo, T);
    build_hash(*Mo);
  }
  *out = Mo.release();
  return CVD_OK;
  CVD_CATCH
}
}  // namespace

extern "C" int cvd_model_create(const cvd_code* dec, const cvd_learn_params* prm, cvd_model** out) {
  return model_create(dec, prm, -1, nullptr, out, nullptr);
}

extern "C" int cvd_model_create_device(const cvd_code* dec, const cvd_learn_params* prm, int32_t device,
                                       void* stream, cvd_model** out, double* stats_out) {
  if (device < 0) { set_error("device must be >= 0"); return CVD_E_INVALID; }
  LearnStats st;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = model_create(dec, prm, device, stream, out, &st);
  st.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (stats_out) {
    stats_out[0] = st.seconds;
    stats_out[1] = (double)st.mismatched_blocks;
    stats_out[2] = (double)st.fix_passes;
    stats_out[3] = (double)st.sequential_blocks;
    stats_out[4] = (double)st.hash_attempts;
    stats_out[5] = (double)st.host_fallback;
    stats_out[6] = st.sequential_seconds;
  }
  return rc;
}

// The code-specialised kernel's default variants for a decoder, compiled now (no device
// needed) into `dir`, the prebuilt cache the run-time compile looks in first (cvd_rtc.cpp): a
// fresh box then loads them instead of compiling ~10 s per variant at model upload.  The
// bit-sliced codes' (m = 6) lockstep variant (pre-filter, 1,024-thread blocks) and the walking
// models' LDS-filter variants (1,024 and 512 threads).
extern "C" int cvd_jit_prebuild(const cvd_code* dec, const char* arch, const char* dir, int32_t* n_built) {
  CVD_TRY
  if (!dec || !arch || !dir || !n_built) { set_error("null argument"); return CVD_E_INVALID; }
  *n_built = 0;
  cvd_model Mo;
  int rc = parse_code(dec, Mo.dec);
  if (rc) return rc;
  const Tabs T = make_tabs(Mo.dec);
  build_bmp(Mo, T);
  if (!Mo.k1b_ok || !bitslice_preferred(Mo)) return CVD_OK;   // (only the bit-sliced codes)
  const std::string vs[] = {
      rtc_variant_defs(kBsPfLog2Bits >= 20 ? 1024 : 512, false, kFilterPatBitsLds, true, true, kBsPfLog2Bits),
      rtc_variant_defs(1024, true, kFilterPatBitsLds, true, false, kBsPfLog2Bits),
      rtc_variant_defs(512, true, kFilterPatBitsLds, true, false, kBsPfLog2Bits)};
  std::vector<std::thread> th;
  std::vector<int> res(3, 0);
  std::vector<std::string> errs(3);
  for (int i = 0; i < 3; ++i)
    th.emplace_back([&, i] {
      res[i] = rtc_prebuild(Mo.dec.m, Mo.bfly_x, vs[i].c_str(), arch, dir);
      if (res[i]) errs[i] = last_error_copy();
    });
  for (auto& t : th) t.join();
  for (int i = 0; i < 3; ++i) {
    if (res[i]) { set_error(errs[i]); return CVD_E_UNSUPPORTED; }
    ++*n_built;
  }
  return CVD_OK;
  CVD_CATCH
}

extern "C" int cvd_model_info_get(const cvd_model* Mo, cvd_model_info* info) {
  if (!Mo || !info) { set_error("null argument"); return CVD_E_INVALID; }
  info->kind = Mo->kind;
  info->k = Mo->dec.k; info->n = Mo->dec.n; info->m = Mo->dec.m;
  info->S = Mo->S;
  info->n_rows = Mo->n_rows;
  info->learn_len_eff = Mo->learn_len_eff;
  info->hash_capacity = Mo->hcap;
  info->max_probe = Mo->max_probe;
  info->device = Mo->device;
  info->logp1_unseen = Mo->logp1_unseen;
  info->explicit_kernel = explicit_kernel_of(*Mo);
  info->mc_fused = mc_fused_preferred(*Mo) ? 1 : 0;
  // walk mode runs only on the specialised kernel: once uploaded, report what runs (no JIT
  // kernel -> lockstep), before upload what would
  info->walk = Mo->k1b_ok && Mo->hcap > 0 && walk_preferred(*Mo) && (Mo->device < 0 || Mo->rtc_fn) ? 1 : 0;
  info->lds_filter = Mo->device >= 0 ? (Mo->rtc_fn && Mo->rtc_ldsf ? 1 : 0)
                                     : (Mo->k1b_ok && Mo->hcap > 0 && ldsf_preferred(*Mo) ? 1 : 0);
  info->walk_compact = Mo->device >= 0 && Mo->rtc_t2c ? 1 : 0;
  info->multi_variant = multi_variant(*Mo);
  info->persist_seqs = persist_seqs(*Mo);
  return CVD_OK;
}

extern "C" int cvd_model_dense_P1(const cvd_model* Mo, double* P_out, int64_t S) {
  CVD_TRY
  if (!Mo || !P_out) { set_error("null argument"); return CVD_E_INVALID; }
  if (Mo->kind != 0 || S != Mo->S) { set_error("dense P1 only for dense models with matching S"); return CVD_E_INVALID; }
  for (int64_t i = 0; i < S; ++i) {
    const double base = Mo->laplace / Mo->rowsum[(size_t)i];
    for (int64_t j = 0; j < S; ++j) P_out[(size_t)i * S + j] = base;
  }
  for (const auto& e : Mo->p1_nz)
    P_out[(size_t)e.row * S + e.col] = e.val / Mo->rowsum[(size_t)e.row];
  return CVD_OK;
  CVD_CATCH
}

extern "C" int cvd_model_rows(const cvd_model* Mo, double* logp1_out, uint8_t* keys_out, int64_t n_rows) {
  if (!Mo) { set_error("null model"); return CVD_E_INVALID; }
  if (n_rows != Mo->n_rows) { set_error("n_rows mismatch"); return CVD_E_INVALID; }
  const int R = 1 << Mo->dec.n, M = 1 << Mo->dec.m;
  if (logp1_out) std::memcpy(logp1_out, Mo->logp1.data(), (size_t)n_rows * R * sizeof(double));
  if (keys_out) std::memcpy(keys_out, Mo->keys.data(), (size_t)n_rows * M);
  return CVD_OK;
}

extern "C" int cvd_model_jit_status(const cvd_model* Mo, char* msg_out, int64_t msg_len) {
  if (!Mo) { set_error("null model"); return CVD_E_INVALID; }
  if (msg_out && msg_len > 0) {
    const size_t n = std::min<size_t>(Mo->jit_error.size(), (size_t)msg_len - 1);
    std::memcpy(msg_out, Mo->jit_error.data(), n);
    msg_out[n] = 0;
  }
  if (Mo->device < 0 || !Mo->k1b_ok || Mo->hcap == 0) return 0;   // not applicable
  return Mo->rtc_fn ? 1 : -1;
}

extern "C" int cvd_model_taps(const cvd_model* Mo, uint8_t* taps_out, int64_t len) {
  if (!Mo || !taps_out) { set_error("null argument"); return CVD_E_INVALID; }
  const CodeDesc& d = Mo->dec;
  const int L = d.m + 1;
  if (len != (int64_t)d.n * d.k * L) { set_error("taps buffer size must be n*k*(m+1)"); return CVD_E_INVALID; }
  for (int j = 0; j < d.n; ++j)
    for (int i = 0; i < d.k; ++i)
      for (int t = 0; t < L; ++t) taps_out[(j * d.k + i) * L + t] = (uint8_t)((d.gmask[j * d.k + i] >> t) & 1u);
  return CVD_OK;
}

extern "C" int cvd_model_upload(cvd_model* Mo, int device) {
  if (!Mo) { set_error("null model"); return CVD_E_INVALID; }
  return upload_model(*Mo, device);
}

extern "C" void cvd_model_destroy(cvd_model* Mo) {
  if (!Mo) return;
  free_model_device(*Mo);
  delete Mo;
}
