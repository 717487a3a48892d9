/*
 * cvd_oracle.c — plain-C restatement of the reference's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (the oracle).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / the reported CPU baseline.  The product never links it.
 *
 * Restates, function by function (reference = So-bonkers/Detecting-Convolutional-
 * Codes-Via-Markovian-Statistics):
 *   oc_branch            viterbi_markov.py:82-106  branch_output_and_next_state
 *   oc_step              viterbi_markov.py:139-159 viterbi_metric_step (Eq. 4-5)
 *   oc_bfs               viterbi_markov.py:166-195 enumerate_markov_states_allzero
 *   oc_model_create      Pd_plotter.py:123-169     learn_P1_empirical (+ T(1/2), Pd:89-99)
 *   oc_stream            the missing simulate_markov_sequence (build spec, oracle/philox.py)
 *   oc_log_prob          Pd_plotter.py:106-116     log_prob_sequence
 *   oc_run_trials        Pd_plotter.py:198-233     trial loop + decisions
 * The state index is a hash map keyed by the full metric vector, exactly the
 * reference's dict (Pd_plotter.py:139); rows are Laplace-smoothed count rows.
 * Row sums use the closed form R_i + S*laplace, equal to numpy's pairwise sum
 * for integral laplace (the only case the C oracle is used for).
 * Non-enumerable codes (m = 6) use the build's declared sparse policy
 * (DESIGN.md deviation D4): states = those visited by the learning chain.
 * Pinned against the Python restatement (tests/test_c_oracle.py), which is
 * pinned bit-exactly to the reference's golden vectors.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { int32_t k, n, m; const uint8_t* taps; } oc_code;

/* ───────────────────────── Philox4x32-10 spec ───────────────────────────── */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
#define LEARN_TAG 0xC0DE1EA7u

uint32_t oc_grid_tag(int64_t N, double p) {
  uint64_t bits; memcpy(&bits, &p, 8);
  uint64_t x = (uint64_t)N * 0x9E3779B97F4A7C15ull + bits;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)((x ^ (x >> 32)) & 0x7FFFFFFFu);
}

/* ───────────────────────── encoder (vm:82-106) ───────────────────────────── */
typedef struct { int k, n, m, M, K, R; uint8_t out[256 * 16]; uint16_t nxt[256 * 16]; } Tabs;

static void oc_branch(const oc_code* c, int s, int U, int* out, int* ns) {
  int o = 0;
  for (int j = 0; j < c->n; ++j) {
    int bit = 0;
    for (int i = 0; i < c->k; ++i) {
      /* x = [input_bits[i]] + state_bits[:m]; taps[d] & x[d] */
      const uint8_t* taps = c->taps + (j * c->k + i) * (c->m + 1);
      bit ^= taps[0] & ((U >> i) & 1);
      for (int d = 1; d <= c->m; ++d) bit ^= taps[d] & ((s >> (d - 1)) & 1);
    }
    o |= bit << j;
  }
  /* new_regs = input_bits + state_bits[:m-k], truncated to m */
  int nsv = 0;
  for (int b = 0; b < c->m; ++b) {
    int v = b < c->k ? ((U >> b) & 1) : ((s >> (b - c->k)) & 1);
    nsv |= v << b;
  }
  *out = o; *ns = nsv;
}

static void make_tabs(const oc_code* c, Tabs* T) {
  T->k = c->k; T->n = c->n; T->m = c->m; T->M = 1 << c->m; T->K = 1 << c->k; T->R = 1 << c->n;
  for (int s = 0; s < T->M; ++s)
    for (int U = 0; U < T->K; ++U) {
      int o, ns;
      oc_branch(c, s, U, &o, &ns);
      T->out[s * T->K + U] = (uint8_t)o; T->nxt[s * T->K + U] = (uint16_t)ns;
    }
}

/* ───────────────────────── Eq. 4-5 (vm:139-159) ──────────────────────────── */
static void oc_step(const Tabs* T, const uint8_t* D, int r, uint8_t* out) {
  int best[256];
  for (int i = 0; i < T->M; ++i) best[i] = 1 << 30;
  for (int s = 0; s < T->M; ++s)
    for (int U = 0; U < T->K; ++U) {
      int v = D[s] + __builtin_popcount((unsigned)(T->out[s * T->K + U] ^ r));
      int ns = T->nxt[s * T->K + U];
      if (v < best[ns]) best[ns] = v;
    }
  int mn = 1 << 30;
  for (int i = 0; i < T->M; ++i) if (best[i] < mn) mn = best[i];
  for (int i = 0; i < T->M; ++i) out[i] = (uint8_t)(best[i] - mn);
}

/* ───────────────────────── state index (dict) ────────────────────────────── */
typedef struct { int M; uint8_t* keys; int64_t n, cap_keys; int32_t* slot; uint64_t mask; } Index;

static uint64_t hkey(const uint8_t* p, int M) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < M; ++i) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}
static void idx_init(Index* I, int M) {
  I->M = M; I->n = 0; I->cap_keys = 1024; I->keys = malloc((size_t)I->cap_keys * M);
  I->mask = 2047; I->slot = malloc(sizeof(int32_t) * 2048);
  memset(I->slot, 0xFF, sizeof(int32_t) * 2048);
}
static void idx_free(Index* I) { free(I->keys); free(I->slot); }
static int64_t idx_find(const Index* I, const uint8_t* k) {
  uint64_t h = hkey(k, I->M) & I->mask;
  for (;;) {
    int32_t v = I->slot[h];
    if (v < 0) return -1;
    if (!memcmp(I->keys + (size_t)v * I->M, k, (size_t)I->M)) return v;
    h = (h + 1) & I->mask;
  }
}
static int64_t idx_insert(Index* I, const uint8_t* k, int* ins) {
  int64_t f = idx_find(I, k);
  if (f >= 0) { *ins = 0; return f; }
  if (I->n == I->cap_keys) { I->cap_keys *= 2; I->keys = realloc(I->keys, (size_t)I->cap_keys * I->M); }
  if ((uint64_t)(I->n + 1) * 2 > I->mask + 1) {
    uint64_t nc = (I->mask + 1) * 2;
    free(I->slot); I->slot = malloc(sizeof(int32_t) * nc); memset(I->slot, 0xFF, sizeof(int32_t) * nc);
    I->mask = nc - 1;
    for (int64_t i = 0; i < I->n; ++i) {
      uint64_t h = hkey(I->keys + (size_t)i * I->M, I->M) & I->mask;
      while (I->slot[h] >= 0) h = (h + 1) & I->mask;
      I->slot[h] = (int32_t)i;
    }
  }
  memcpy(I->keys + (size_t)I->n * I->M, k, (size_t)I->M);
  uint64_t h = hkey(k, I->M) & I->mask;
  while (I->slot[h] >= 0) h = (h + 1) & I->mask;
  I->slot[h] = (int32_t)I->n;
  *ins = 1;
  return I->n++;
}

/* ───────────────────────── simulator spec ────────────────────────────────── */
typedef struct {
  const Tabs* T; uint32_t k0, k1, tag; uint64_t sid, thr; int s;
  int64_t nw, ib; uint32_t nmask, iv[4], iv_noise[4];
} Stream;

static void stream_init(Stream* S, const Tabs* T, uint64_t seed, uint32_t tag, uint64_t sid, double p) {
  S->T = T; S->k0 = (uint32_t)seed; S->k1 = (uint32_t)(seed >> 32); S->tag = tag; S->sid = sid;
  S->thr = (uint64_t)(p * 4294967296.0); S->s = 0; S->nw = -1; S->ib = -1;
}
static uint32_t chi(uint64_t sid, uint32_t kind) { return (uint32_t)((sid >> 32) & 0xFFFF) | (kind << 16); }
static int stream_next(Stream* S, int64_t t) {
  const Tabs* T = S->T;
  int U = 0;
  for (int i = 0; i < T->k; ++i) {
    int64_t b = t * T->k + i, blk = b >> 7;
    if (blk != S->ib) {
      S->iv[0] = (uint32_t)blk; S->iv[1] = (uint32_t)S->sid; S->iv[2] = chi(S->sid, 1); S->iv[3] = S->tag;
      philox(S->iv, S->k0, S->k1); S->ib = blk;
    }
    U |= (int)((S->iv[(b >> 5) & 3] >> (b & 31)) & 1u) << i;
  }
  int r = T->out[S->s * T->K + U];
  S->s = T->nxt[S->s * T->K + U];
  /* BSC flips, bit-sliced (oracle/philox.py noise_bits): the uniform of bit b of
     received word w is sum_i bit_b(P_i) 2^(31-i) over the bit-planes
     P_i = word i%4 of philox(8w + i/4, ...); decided plane by plane, MSB first */
  const int spw = 32 / T->n, nb = spw * T->n;
  const int64_t w = t / spw;
  if (w != S->nw) {
    uint32_t und = nb >= 32 ? 0xFFFFFFFFu : (1u << nb) - 1u, flp = 0;
    if (S->thr >= 4294967296ull) flp = und, und = 0;
    if (S->thr == 0) und = 0;
    for (int i = 0; i < 32 && und; ++i) {
      if ((i & 3) == 0) {
        uint32_t c[4];
        c[0] = (uint32_t)(w * 8 + i / 4); c[1] = (uint32_t)S->sid; c[2] = chi(S->sid, 0); c[3] = S->tag;
        philox(c, S->k0, S->k1);
        memcpy(S->iv_noise, c, sizeof c);
      }
      const uint32_t pl = S->iv_noise[i & 3];
      if ((S->thr >> (31 - i)) & 1u) { flp |= und & ~pl; und &= pl; }
      else und &= ~pl;
    }
    S->nmask = flp; S->nw = w;
  }
  r ^= (int)((S->nmask >> ((t - w * spw) * T->n)) & ((1u << T->n) - 1u));
  return r;
}

/* ───────────────────────── model (Pd:123-169) ────────────────────────────── */
typedef struct {
  Tabs T; int kind; int64_t S, L; double lam, unseen;
  Index idx;            /* rows: dense = BFS order, sparse = first visit */
  double* logp1;        /* [S][R] */
  uint8_t* cnt_c;       /* dense: [S][R] T_ref count c; sparse: NULL */
} Model;

static int oc_bfs(const Tabs* T, int64_t cap, Index* I, int32_t** next_out) {
  idx_init(I, T->M);
  uint8_t z[256] = {0}, nb[256];
  int ins;
  idx_insert(I, z, &ins);
  int64_t head = 0, ncap = 1024;
  int32_t* next = malloc(sizeof(int32_t) * ncap * T->R);
  while (head < I->n) {
    if (head >= ncap) { ncap *= 2; next = realloc(next, sizeof(int32_t) * ncap * T->R); }
    for (int i = 0; i < T->R; ++i) {
      int r = 0;   /* itertools.product order: last output bit fastest */
      for (int j = 0; j < T->n; ++j) r |= ((i >> (T->n - 1 - j)) & 1) << j;
      uint8_t cur[256];
      memcpy(cur, I->keys + (size_t)head * T->M, (size_t)T->M);
      oc_step(T, cur, r, nb);
      int64_t jx = idx_insert(I, nb, &ins);
      if (I->n > cap) { free(next); return -1; }
      next[head * T->R + r] = (int32_t)jx;
    }
    ++head;
  }
  *next_out = next;
  return 0;
}

/* S_lap > 0 (non-enumerable codes): the S of the Laplace denominator S*lam
 * (Pd:166-167) instead of the number of visited rows -- the product's
 * cvd_learn_params.laplace_states, restated */
void* oc_model_create(const oc_code* dec, double p, int64_t learn_len, int64_t burn, double lam,
                      uint64_t seed, int64_t enum_cap, int64_t sparse_default_len, int64_t S_lap) {
  Model* Mo = calloc(1, sizeof(Model));
  make_tabs(dec, &Mo->T);
  const Tabs* T = &Mo->T;
  const int R = T->R, M = T->M;
  Mo->lam = lam;
  int32_t* next = NULL;
  int64_t* cnt;
  Stream st;
  stream_init(&st, T, seed, LEARN_TAG, 0, p);
  if (enum_cap > 0 && oc_bfs(T, enum_cap, &Mo->idx, &next) == 0) {
    Mo->kind = 0;
    const int64_t S = Mo->idx.n;
    Mo->S = S;
    Mo->L = learn_len < 0 ? (200 * S > 5000 ? 200 * S : 5000) : learn_len;
    cnt = calloc((size_t)S * R, sizeof(int64_t));
    int64_t i = 0;
    for (int64_t t = 0; t < Mo->L; ++t) {
      int r = stream_next(&st, t);
      if (t >= burn) cnt[i * R + r]++;
      i = next[i * R + r];
    }
    Mo->cnt_c = malloc((size_t)S * R);
    for (int64_t s = 0; s < S; ++s)
      for (int r = 0; r < R; ++r) {
        int c = 0;
        for (int q = 0; q < R; ++q) c += next[s * R + q] == next[s * R + r];
        Mo->cnt_c[s * R + r] = (uint8_t)c;
      }
  } else {
    if (Mo->idx.keys) idx_free(&Mo->idx);
    Mo->kind = 1;
    idx_init(&Mo->idx, M);
    Mo->L = learn_len >= 0 ? learn_len : sparse_default_len;
    int64_t ccap = 1024;
    cnt = calloc((size_t)ccap * R, sizeof(int64_t));
    uint8_t D[256] = {0}, Dn[256];
    int ins;
    int64_t i = idx_insert(&Mo->idx, D, &ins);
    for (int64_t t = 0; t < Mo->L; ++t) {
      int r = stream_next(&st, t);
      if (t >= burn) cnt[i * R + r]++;
      oc_step(T, D, r, Dn);
      int64_t j = idx_insert(&Mo->idx, Dn, &ins);
      if (Mo->idx.n > ccap) {
        cnt = realloc(cnt, sizeof(int64_t) * (size_t)ccap * 2 * R);
        memset(cnt + ccap * R, 0, sizeof(int64_t) * (size_t)ccap * R);
        ccap *= 2;
      }
      memcpy(D, Dn, (size_t)M);
      i = j;
    }
    Mo->S = Mo->idx.n;
    next = malloc(sizeof(int32_t) * (size_t)Mo->S * R);
    for (int64_t s = 0; s < Mo->S; ++s)
      for (int r = 0; r < R; ++r) {
        uint8_t cur[256];
        memcpy(cur, Mo->idx.keys + (size_t)s * M, (size_t)M);
        oc_step(T, cur, r, Dn);
        next[s * R + r] = (int32_t)idx_find(&Mo->idx, Dn);
      }
  }
  /* P = (counts + laplace) / rowsum  (Pd:166-167), logs as in Pd:114-115 */
  const int64_t S = Mo->S;
  const int64_t SL = (Mo->kind == 1 && S_lap > 0) ? S_lap : S;   /* Laplace denominator's S */
  Mo->logp1 = malloc(sizeof(double) * (size_t)S * R);
  for (int64_t s = 0; s < S; ++s) {
    int64_t rs = 0;
    for (int r = 0; r < R; ++r) rs += cnt[s * R + r];
    const double rowsum = (double)rs + (double)SL * lam;
    for (int r = 0; r < R; ++r) {
      int64_t c = 0;
      if (next[s * R + r] >= 0)
        for (int q = 0; q < R; ++q) if (next[s * R + q] == next[s * R + r]) c += cnt[s * R + q];
      double v = (next[s * R + r] >= 0 ? (double)c + lam : lam) / rowsum;
      Mo->logp1[s * R + r] = log(v > 1e-300 ? v : 1e-300);
    }
  }
  Mo->unseen = log(lam / ((double)SL * lam));
  free(cnt);
  free(next);
  return Mo;
}

int64_t oc_model_S(void* m) { return ((Model*)m)->S; }
int oc_model_kind(void* m) { return ((Model*)m)->kind; }
int64_t oc_model_learn_len(void* m) { return ((Model*)m)->L; }
void oc_model_rows(void* m, double* logp1, uint8_t* keys) {
  Model* Mo = m;
  memcpy(logp1, Mo->logp1, sizeof(double) * (size_t)Mo->S * Mo->T.R);
  memcpy(keys, Mo->idx.keys, (size_t)Mo->S * Mo->T.M);
}
void oc_model_destroy(void* m) {
  Model* Mo = m;
  idx_free(&Mo->idx); free(Mo->logp1); free(Mo->cnt_c); free(Mo);
}

/* ───────────────────────── one sequence (Pd:106-116) ─────────────────────── */
static void oc_sequence(const Model* Mo, const Tabs* Te, int64_t N, double p, uint64_t seed, uint32_t tag,
                        uint64_t sid, double* lp_out, double* lr_out) {
  const Tabs* T = &Mo->T;
  const int M = T->M, R = T->R;
  Stream st;
  stream_init(&st, Te, seed, tag, sid, p);
  uint8_t D[256] = {0}, succ[16][256];
  double lp = 0.0, lr = 0.0;
  for (int64_t t = 0; t < N; ++t) {
    const int r = stream_next(&st, t);
    const int64_t i = idx_find(&Mo->idx, D);          /* state_index[metrics[t]] */
    int c = 0;
    if (Mo->kind == 0) {
      oc_step(T, D, r, succ[r]);
      c = Mo->cnt_c[i * R + r];                        /* |Y(i,j)| */
    } else {
      for (int q = 0; q < R; ++q) oc_step(T, D, q, succ[q]);
      for (int q = 0; q < R; ++q) c += !memcmp(succ[q], succ[r], (size_t)M);
    }
    const double pij = i >= 0 ? Mo->logp1[i * R + r] : Mo->unseen;
    const double tij = (double)c / (double)R;
    lp += pij;
    lr += log(tij > 1e-300 ? tij : 1e-300);
    memcpy(D, succ[r], (size_t)M);
  }
  *lp_out = lp;
  *lr_out = lr;
}

/* Trials [t0, t1) of one (N, p) grid point; sums [T][4] (nullable), counts[2]. */
int oc_run_trials(void* model, const oc_code* enc1, const oc_code* enc2, int64_t N, double p,
                  uint64_t seed, int64_t t0, int64_t t1, double* sums, int64_t* counts, int nthreads) {
  const Model* Mo = model;
  Tabs T1, T2;
  make_tabs(enc1, &T1);
  make_tabs(enc2, &T2);
  const uint32_t tag = oc_grid_tag(N, p);
  int64_t s1 = 0, s2 = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : s1, s2)
#endif
  for (int64_t t = t0; t < t1; ++t) {
    double a, b, c, d;
    oc_sequence(Mo, &T1, N, p, seed, tag, (uint64_t)(2 * t), &a, &b);
    oc_sequence(Mo, &T2, N, p, seed, tag, (uint64_t)(2 * t + 1), &c, &d);
    s1 += a > b;
    s2 += c <= d;
    if (sums) { double* o = sums + 4 * (t - t0); o[0] = a; o[1] = b; o[2] = c; o[3] = d; }
  }
  counts[0] += s1;
  counts[1] += s2;
  return 0;
}

/* Received words of one sequence (spec check). */
void oc_stream(const oc_code* enc, int64_t N, double p, uint64_t seed, uint32_t tag, uint64_t sid,
               int32_t* out) {
  Tabs T;
  make_tabs(enc, &T);
  Stream st;
  stream_init(&st, &T, seed, tag, sid, p);
  for (int64_t t = 0; t < N; ++t) out[t] = stream_next(&st, t);
}

int oc_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
