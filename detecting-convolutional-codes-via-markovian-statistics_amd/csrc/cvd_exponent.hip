// Error-exponent engine for gfx950 (alpha_exponent.py, Eq. 7 of the paper):
//
//   count_transitions_kernel  joint counts C[i, r] of (state, received word) along
//                             received streams (learn_transition_tensor,
//                             alpha_exponent.py:83-156), walking the enumerated
//                             automaton with LDS-resident 16-bit records and
//                             LDS histograms
//   chernoff_build_kernel     M(u) = sum_r P1(i->j, r)^u P2(i->j, r)^(1-u) for a
//                             grid of u, in the structure the learned tensors
//                             have: with Laplace smoothing every cell of P is
//                             (C + lambda) / rowsum and C[i, j, r] is nonzero only
//                             for j = next(i, r), so
//                               M(u) = a(u) 1^T + sum_r V_r(u),
//                             a_i = 2^n T0_i, T0_i = (lambda/rs1_i)^u (lambda/rs2_i)^(1-u),
//                             V_r[i, next(i, r)] = T_ir - T0_i: O(K 2^n) per u
//                             instead of the K x K x 2^n dense sum
//   dense_build_kernel        the dense sum for arbitrary P1, P2 (the reference's
//                             compute_error_exponent signature, alpha_exponent.py:159-188)
//   spectral_radius_kernel    rho(M(u)) for a batch of u, one workgroup each: power
//                             iteration on the positive matrix with Collatz-
//                             Wielandt bounds  min_i (Mx)_i/x_i <= rho <= max_i (Mx)_i/x_i
//                             until they agree to `tol` (Perron-Frobenius: M > 0)
//   rho_*_kernel              the same iteration for K above the LDS limit (the
//                             m = 4 rate-1/2 automata, K = 150,743): vectors in
//                             HBM, every u at once, one launch per phase
//   count_transitions_global_kernel  the joint counts for S >= 4096 (records read
//                             from L2, global atomics)
//
// These are the math of alpha_exponent.py; the reference's np.linalg.eigvals
// (alpha_exponent.py:69-76) is replaced by the Perron root, which equals the
// spectral radius for the nonnegative matrices Eq. 7 produces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/cvd.h"
#include "cvd_internal.h"

namespace {

#define HIP_CHECK(x)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      cvd::set_error(std::string("HIP error '") + hipGetErrorString(e_) + "' at " #x);     \
      return CVD_E_HIP;                                                                   \
    }                                                                                     \
  } while (0)

// ─────────────────────────── transition counts ──────────────────────────────

constexpr int kCountBlock = 1024;

struct CountArgs {
  const uint32_t* rec;   // [S*R] next << 4 | c
  const uint32_t* r;     // received words, include/cvd.h layout, pitch nseq
  int64_t S, N, nseq, burn;
  int32_t n;
  unsigned long long* cnt;   // [S*R]
  int32_t lds_hist;      // histogram in LDS (else global atomics)
};

template <int n>
__global__ __launch_bounds__(kCountBlock) void count_transitions_kernel(CountArgs a) {
  constexpr int R = 1 << n, SPW = 32 / n;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int SR = (int)a.S * R;
  uint32_t* s_hist = reinterpret_cast<uint32_t*>(smem);
  uint16_t* s_rec = reinterpret_cast<uint16_t*>(s_hist + (a.lds_hist ? SR : 0));
  for (int i = threadIdx.x; i < SR; i += kCountBlock) {
    s_rec[i] = (uint16_t)a.rec[i];   // next < 4096 (host-checked)
    if (a.lds_hist) s_hist[i] = 0u;
  }
  __syncthreads();
  const int64_t q = (int64_t)blockIdx.x * kCountBlock + threadIdx.x;
  if (q < a.nseq) {
    const int64_t nwords = (a.N + SPW - 1) / SPW;
    uint32_t st = 0;   // D_0 = 0 is BFS index 0
    for (int64_t w = 0; w < nwords; ++w) {
      uint32_t word = a.r[((w >> 2) * a.nseq + q) * 4 + (w & 3)];
      const int64_t t0 = w * SPW;
      const int ns = (int)min((int64_t)SPW, a.N - t0);
      for (int i = 0; i < ns; ++i) {
        const uint32_t rr = word & (uint32_t)(R - 1);
        word >>= n;
        const uint32_t idx = st * (uint32_t)R + rr;
        if (t0 + i >= a.burn) {
          if (a.lds_hist) atomicAdd(&s_hist[idx], 1u);
          else atomicAdd(&a.cnt[idx], 1ull);
        }
        st = (uint32_t)s_rec[idx] >> 4;
      }
    }
  }
  if (a.lds_hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < SR; i += kCountBlock)
      if (s_hist[i]) atomicAdd(&a.cnt[i], (unsigned long long)s_hist[i]);
  }
}

// S >= 4096: the 32-bit records stay in global memory (L2-resident: 2.4 MB at
// S = 150,743, n = 2) and every count is a global atomic
template <int n>
__global__ __launch_bounds__(256) void count_transitions_global_kernel(CountArgs a) {
  constexpr int R = 1 << n, SPW = 32 / n;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= a.nseq) return;
  const int64_t nwords = (a.N + SPW - 1) / SPW;
  uint32_t st = 0;
  for (int64_t w = 0; w < nwords; ++w) {
    uint32_t word = a.r[((w >> 2) * a.nseq + q) * 4 + (w & 3)];
    const int64_t t0 = w * SPW;
    const int ns = (int)min((int64_t)SPW, a.N - t0);
    for (int i = 0; i < ns; ++i) {
      const uint32_t rr = word & (uint32_t)(R - 1);
      word >>= n;
      const uint64_t idx = (uint64_t)st * R + rr;
      if (t0 + i >= a.burn) atomicAdd(&a.cnt[idx], 1ull);
      st = a.rec[idx] >> 4;
    }
  }
}

// ─────────────────────────────── M(u) build ─────────────────────────────────

struct BuildArgs {
  int32_t K, R, U;
  const double* cnt1;   // [K*R]
  const double* cnt2;
  double lam;
  const double* u;      // [U]
  double* a;            // [U*K]
  double* vals;         // [U*K*R]
};

// one thread per (u, i); rowsum over the dense K x K x R tensor incl. Laplace
// (alpha_exponent.py:152-154)
__global__ void chernoff_build_kernel(BuildArgs b) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)b.U * b.K) return;
  const int ui = (int)(g / b.K), i = (int)(g % b.K);
  const double u = b.u[ui], v = 1.0 - u;
  double s1 = 0.0, s2 = 0.0;
  for (int r = 0; r < b.R; ++r) {
    s1 += b.cnt1[(int64_t)i * b.R + r];
    s2 += b.cnt2[(int64_t)i * b.R + r];
  }
  const double cells = (double)b.K * (double)b.R;
  const double rs1 = fmax(s1 + cells * b.lam, 1.0), rs2 = fmax(s2 + cells * b.lam, 1.0);
  // P^u with P clipped to [1e-300, 1] as alpha_exponent.py:171-172
  auto term = [&](double c1, double c2) {
    const double p1 = fmin(fmax((c1 + b.lam) / rs1, 1e-300), 1.0);
    const double p2 = fmin(fmax((c2 + b.lam) / rs2, 1e-300), 1.0);
    return pow(p1, u) * pow(p2, v);
  };
  const double t0 = term(0.0, 0.0);
  b.a[g] = (double)b.R * t0;
  for (int r = 0; r < b.R; ++r)
    b.vals[g * b.R + r] = term(b.cnt1[(int64_t)i * b.R + r], b.cnt2[(int64_t)i * b.R + r]) - t0;
}

struct DenseArgs {
  int32_t K, R, U;
  const double* P1;   // [K*K*R]
  const double* P2;
  const double* u;
  double* vals;       // [U*K*K]
};

// M(u)[i, j] = sum_r P1^u P2^(1-u), P clipped to [1e-300, 1] (alpha_exponent.py:171-180)
__global__ void dense_build_kernel(DenseArgs d) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t KK = (int64_t)d.K * d.K;
  if (g >= (int64_t)d.U * KK) return;
  const int ui = (int)(g / KK);
  const int64_t ij = g % KK;
  const double u = d.u[ui], v = 1.0 - u;
  double s = 0.0;
  for (int r = 0; r < d.R; ++r) {
    const double p1 = fmin(fmax(d.P1[ij * d.R + r], 1e-300), 1.0);
    const double p2 = fmin(fmax(d.P2[ij * d.R + r], 1e-300), 1.0);
    s += pow(p1, u) * pow(p2, v);
  }
  d.vals[g] = s;
}

// ───────────────────────────── spectral radius ──────────────────────────────

constexpr int kRhoBlock = 1024;

struct RhoArgs {
  int32_t K, E;          // E entries per row (dense: E = K, cols = NULL)
  const double* a;       // [U*K] rank-one row coefficients (NULL: none)
  const double* vals;    // [U*K*E]
  const int32_t* cols;   // [K*E] (NULL: dense, column e)
  double tol;
  int32_t max_iter;
  double* rho;           // [U*3]: estimate, lower, upper bound
  int32_t* iters;        // [U]
};

__device__ __forceinline__ double block_reduce(double v, double* s_red, int op) {   // 0 sum, 1 min, 2 max
  for (int o = 32; o > 0; o >>= 1) {
    const double w = __shfl_xor(v, o);
    v = op == 0 ? v + w : op == 1 ? fmin(v, w) : fmax(v, w);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s_red[wid] = v;
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6;
  v = s_red[0];
  for (int k = 1; k < nw; ++k) v = op == 0 ? v + s_red[k] : op == 1 ? fmin(v, s_red[k]) : fmax(v, s_red[k]);
  return v;
}

__global__ __launch_bounds__(kRhoBlock) void spectral_radius_kernel(RhoArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int K = p.K, E = p.E, ub = blockIdx.x;
  double* x = reinterpret_cast<double*>(smem);
  double* y = x + K;
  double* s_red = y + K;
  const double* av = p.a ? p.a + (int64_t)ub * K : nullptr;
  const double* vv = p.vals + (int64_t)ub * K * E;
  for (int i = threadIdx.x; i < K; i += kRhoBlock) x[i] = 1.0;
  __syncthreads();
  // x > 0 with max x = 1: for any nonnegative M, min_i (Mx)_i/x_i <= rho <=
  // max_i (Mx)_i/x_i; the bounds meet for irreducible M (every M(u) of Eq. 7
  // is positive).  A reducible M (dense input) can keep them apart: then the
  // estimate is max_i (Mx)_i, the power-iteration norm ratio, once it is
  // stable to tol / 100 between iterations.
  double lo = 0.0, hi = 0.0, sx = (double)K, est = 0.0, prev = -1.0;
  bool met = false;
  int it = 0;
  for (; it < p.max_iter; ++it) {
    double rmin = 1e308, rmax = 0.0, ymax = 0.0;
    for (int i = threadIdx.x; i < K; i += kRhoBlock) {
      double s = av ? av[i] * sx : 0.0;
      const double* row = vv + (int64_t)i * E;
      if (p.cols) {
        const int32_t* cr = p.cols + (int64_t)i * E;
        for (int e = 0; e < E; ++e) s += row[e] * x[cr[e]];
      } else {
        for (int e = 0; e < E; ++e) s += row[e] * x[e];
      }
      y[i] = s;
      const double ratio = s / x[i];
      rmin = fmin(rmin, ratio);
      rmax = fmax(rmax, ratio);
      ymax = fmax(ymax, s);
    }
    lo = block_reduce(rmin, s_red, 1);
    hi = block_reduce(rmax, s_red, 2);
    ymax = block_reduce(ymax, s_red, 2);
    est = ymax;   // ||M x||_inf with ||x||_inf = 1
    if (hi - lo <= p.tol * hi) { met = true; ++it; break; }
    if (!(ymax > 0.0) || fabs(est - prev) <= 0.01 * p.tol * est) { ++it; break; }
    prev = est;
    double sl = 0.0;
    for (int i = threadIdx.x; i < K; i += kRhoBlock) {
      const double v = y[i] / ymax;
      x[i] = v;
      sl += v;
    }
    sx = block_reduce(sl, s_red, 0);
  }
  if (threadIdx.x == 0) {
    p.rho[3 * ub] = met ? 0.5 * (lo + hi) : est;
    p.rho[3 * ub + 1] = lo;
    p.rho[3 * ub + 2] = hi;
    p.iters[ub] = it;
  }
}

// ─────────────── spectral radius for K above the LDS limit ───────────────
// The iteration of spectral_radius_kernel with x, y in HBM for all u at once:
// rho_matvec (y = M x, per-block Collatz-Wielandt min / max and max y), rho_step
// (per u: the bounds, the stopping tests, the next scale), rho_scale (x = y /
// ymax, per-block sums), rho_sum (per u: 1^T x for the rank-one part).  State
// per u in st[8]: 0 sx, 1 est, 2 prev, 3 lo, 4 hi, 5 ymax, 6 done (1 bounds met,
// 2 stopped on the norm ratio), 7 iterations.
constexpr int kGBlock = 256;

struct GRhoArgs {
  int32_t K, E, nb;
  const double* a;
  const double* vals;
  const int32_t* cols;
  double* x;
  double* y;
  double* part;   // [U][nb][3]
  double* st;     // [U][8]
  double tol;
};

__global__ __launch_bounds__(kGBlock) void rho_matvec_kernel(GRhoArgs g) {
  __shared__ double s_red[kGBlock / 64];
  const int u = blockIdx.y;
  const double* st = g.st + 8 * u;
  if (st[6] != 0.0) return;   // uniform per block
  const int i = blockIdx.x * kGBlock + threadIdx.x;
  double rmin = 1e308, rmax = 0.0, ym = 0.0;
  if (i < g.K) {
    const int64_t ui = (int64_t)u * g.K + i;
    const double* xu = g.x + (int64_t)u * g.K;
    double s = g.a ? g.a[ui] * st[0] : 0.0;
    const double* row = g.vals + ui * g.E;
    const int32_t* cr = g.cols + (int64_t)i * g.E;
    for (int e = 0; e < g.E; ++e) s += row[e] * xu[cr[e]];
    g.y[ui] = s;
    rmin = rmax = s / xu[i];
    ym = s;
  }
  rmin = block_reduce(rmin, s_red, 1);
  rmax = block_reduce(rmax, s_red, 2);
  ym = block_reduce(ym, s_red, 2);
  if (threadIdx.x == 0) {
    double* pp = g.part + ((int64_t)u * g.nb + blockIdx.x) * 3;
    pp[0] = rmin; pp[1] = rmax; pp[2] = ym;
  }
}

__global__ __launch_bounds__(kGBlock) void rho_step_kernel(GRhoArgs g) {
  __shared__ double s_red[kGBlock / 64];
  const int u = blockIdx.x;
  double* st = g.st + 8 * u;
  if (st[6] != 0.0) return;
  double lo = 1e308, hi = 0.0, ym = 0.0;
  for (int b = threadIdx.x; b < g.nb; b += kGBlock) {
    const double* pp = g.part + ((int64_t)u * g.nb + b) * 3;
    lo = fmin(lo, pp[0]); hi = fmax(hi, pp[1]); ym = fmax(ym, pp[2]);
  }
  lo = block_reduce(lo, s_red, 1);
  hi = block_reduce(hi, s_red, 2);
  ym = block_reduce(ym, s_red, 2);
  if (threadIdx.x == 0) {
    st[3] = lo; st[4] = hi; st[1] = ym; st[5] = ym;
    st[7] += 1.0;
    if (hi - lo <= g.tol * hi) st[6] = 1.0;
    else if (!(ym > 0.0) || fabs(ym - st[2]) <= 0.01 * g.tol * ym) st[6] = 2.0;
    else st[2] = ym;
  }
}

__global__ __launch_bounds__(kGBlock) void rho_scale_kernel(GRhoArgs g) {
  __shared__ double s_red[kGBlock / 64];
  const int u = blockIdx.y;
  const double* st = g.st + 8 * u;
  if (st[6] != 0.0) return;
  const int i = blockIdx.x * kGBlock + threadIdx.x;
  double v = 0.0;
  if (i < g.K) {
    const int64_t ui = (int64_t)u * g.K + i;
    v = g.y[ui] / st[5];
    g.x[ui] = v;
  }
  v = block_reduce(v, s_red, 0);
  if (threadIdx.x == 0) g.part[((int64_t)u * g.nb + blockIdx.x) * 3] = v;
}

__global__ void rho_sum_kernel(GRhoArgs g, int32_t U) {   // one thread per u, blocks in order
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U || g.st[8 * u + 6] != 0.0) return;
  double s = 0.0;
  for (int b = 0; b < g.nb; ++b) s += g.part[((int64_t)u * g.nb + b) * 3];
  g.st[8 * u] = s;
}

__global__ void rho_init_kernel(GRhoArgs g, int32_t U) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (int64_t)U * g.K) g.x[t] = 1.0;
  if (t < U) {
    double* st = g.st + 8 * t;
    st[0] = (double)g.K; st[1] = 0.0; st[2] = -1.0; st[3] = 0.0; st[4] = 0.0; st[5] = 0.0; st[6] = 0.0; st[7] = 0.0;
  }
}

__global__ void rho_out_kernel(GRhoArgs g, int32_t U, double* rho, int32_t* iters) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  const double* st = g.st + 8 * u;
  rho[3 * u] = st[6] == 1.0 ? 0.5 * (st[3] + st[4]) : st[1];
  rho[3 * u + 1] = st[3];
  rho[3 * u + 2] = st[4];
  iters[u] = (int32_t)st[7];
}

int spectral_radius_global(int32_t K, int32_t E, const double* d_a, const double* d_vals, const int32_t* d_cols,
                           int32_t U, double tol, int32_t max_iter, double* d_rho, int32_t* d_iters,
                           hipStream_t stream) {
  GRhoArgs g{};
  g.K = K; g.E = E; g.nb = (K + kGBlock - 1) / kGBlock;
  g.a = d_a; g.vals = d_vals; g.cols = d_cols; g.tol = tol;
  const size_t nx = (size_t)U * K;
  HIP_CHECK(hipMallocAsync((void**)&g.x, sizeof(double) * (2 * nx + (size_t)U * g.nb * 3 + (size_t)U * 8), stream));
  g.y = g.x + nx;
  g.part = g.y + nx;
  g.st = g.part + (size_t)U * g.nb * 3;
  const unsigned ni = (unsigned)((std::max<size_t>(nx, (size_t)U) + 255) / 256);
  hipLaunchKernelGGL(rho_init_kernel, dim3(ni), dim3(256), 0, stream, g, U);
  std::vector<double> st((size_t)U * 8);
  const dim3 grid((unsigned)g.nb, (unsigned)U);
  const unsigned gu = (unsigned)((U + 255) / 256);
  int rc = CVD_OK;
  for (int it = 0; it < max_iter; ++it) {
    hipLaunchKernelGGL(rho_matvec_kernel, grid, dim3(kGBlock), 0, stream, g);
    hipLaunchKernelGGL(rho_step_kernel, dim3((unsigned)U), dim3(kGBlock), 0, stream, g);
    hipLaunchKernelGGL(rho_scale_kernel, grid, dim3(kGBlock), 0, stream, g);
    hipLaunchKernelGGL(rho_sum_kernel, dim3(gu), dim3(256), 0, stream, g, U);
    if ((it & 31) == 31 || it + 1 == max_iter) {   // every u stopped?
      if (hipMemcpyAsync(st.data(), g.st, sizeof(double) * st.size(), hipMemcpyDeviceToHost, stream) != hipSuccess ||
          hipStreamSynchronize(stream) != hipSuccess) {
        cvd::set_error("spectral_radius: HIP error in the global iteration");
        rc = CVD_E_HIP;
        break;
      }
      bool all = true;
      for (int u = 0; u < U && all; ++u) all = st[(size_t)u * 8 + 6] != 0.0;
      if (all) break;
    }
  }
  if (rc == CVD_OK) hipLaunchKernelGGL(rho_out_kernel, dim3(gu), dim3(256), 0, stream, g, U, d_rho, d_iters);
  const hipError_t e = hipGetLastError();
  (void)hipFreeAsync(g.x, stream);
  if (rc == CVD_OK && e != hipSuccess) {
    cvd::set_error(std::string("HIP error '") + hipGetErrorString(e) + "' in spectral_radius (global)");
    rc = CVD_E_HIP;
  }
  return rc;
}

}  // namespace

// ───────────────────────────────── ABI ──────────────────────────────────────

extern "C" int cvd_count_transitions(const cvd_model* model, const uint32_t* d_r, int64_t N, int64_t nseq,
                                     int64_t burn_in, uint64_t* d_cnt, void* stream) {
  if (!model || !d_cnt || N < 0 || nseq < 0 || burn_in < 0 || (!d_r && N > 0 && nseq > 0)) {
    cvd::set_error("bad count_transitions arguments");
    return CVD_E_INVALID;
  }
  int rc = cvd::check_device(*model);
  if (rc) return rc;
  const cvd_model& M = *model;
  if (M.kind != 0 || !M.d_rec) { cvd::set_error("count_transitions needs an enumerated (dense) model"); return CVD_E_UNSUPPORTED; }
  const int n = M.dec.n, R = 1 << n;
  if (n != 2 && n != 3) {
    cvd::set_error("count_transitions: n in {2, 3}");
    return CVD_E_UNSUPPORTED;
  }
  if (nseq == 0 || N == 0) return CVD_OK;
  CountArgs a;
  a.rec = M.d_rec; a.r = d_r; a.S = M.S; a.N = N; a.nseq = nseq; a.burn = burn_in; a.n = n;
  a.cnt = reinterpret_cast<unsigned long long*>(d_cnt);
  if (M.S >= 4096) {   // 16-bit LDS records cannot hold the successor: records from L2
    a.lds_hist = 0;
    hipLaunchKernelGGL(n == 2 ? count_transitions_global_kernel<2> : count_transitions_global_kernel<3>,
                       dim3((unsigned)((nseq + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    HIP_CHECK(hipGetLastError());
    return CVD_OK;
  }
  const size_t SR = (size_t)M.S * R;
  a.lds_hist = SR * 6 <= 160 * 1024;
  const size_t lds = SR * 2 + (a.lds_hist ? SR * 4 : 0);
  void (*kern)(CountArgs) = n == 2 ? count_transitions_kernel<2> : count_transitions_kernel<3>;
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const unsigned grid = (unsigned)((nseq + kCountBlock - 1) / kCountBlock);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kCountBlock), lds, (hipStream_t)stream, a);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}

extern "C" int cvd_chernoff_build(int32_t K, int32_t R, const double* d_cnt1, const double* d_cnt2, double laplace,
                                  const double* d_u, int32_t U, double* d_a, double* d_vals, void* stream) {
  if (K < 1 || R < 1 || U < 0 || !(laplace > 0.0) || !d_cnt1 || !d_cnt2 || (U > 0 && (!d_u || !d_a || !d_vals))) {
    cvd::set_error("bad chernoff_build arguments (laplace must be > 0: the structured M(u) needs P > 0)");
    return CVD_E_INVALID;
  }
  if (U == 0) return CVD_OK;
  BuildArgs b{K, R, U, d_cnt1, d_cnt2, laplace, d_u, d_a, d_vals};
  const int64_t tot = (int64_t)U * K;
  hipLaunchKernelGGL(chernoff_build_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, b);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}

extern "C" int cvd_chernoff_build_dense(int32_t K, int32_t R, const double* d_P1, const double* d_P2,
                                        const double* d_u, int32_t U, double* d_vals, void* stream) {
  if (K < 1 || R < 1 || U < 0 || !d_P1 || !d_P2 || (U > 0 && (!d_u || !d_vals))) {
    cvd::set_error("bad chernoff_build_dense arguments");
    return CVD_E_INVALID;
  }
  if (U == 0) return CVD_OK;
  DenseArgs d{K, R, U, d_P1, d_P2, d_u, d_vals};
  const int64_t tot = (int64_t)U * K * K;
  hipLaunchKernelGGL(dense_build_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}

extern "C" int cvd_spectral_radius(int32_t K, int32_t E, const double* d_a, const double* d_vals,
                                   const int32_t* d_cols, int32_t U, double tol, int32_t max_iter, double* d_rho,
                                   int32_t* d_iters, void* stream) {
  if (K < 1 || E < 1 || U < 0 || !(tol >= 0.0) || max_iter < 1 || (U > 0 && (!d_vals || !d_rho || !d_iters)) ||
      (!d_cols && E != K)) {
    cvd::set_error("bad spectral_radius arguments");
    return CVD_E_INVALID;
  }
  const size_t lds = (size_t)2 * K * sizeof(double) + 16 * sizeof(double);
  const char* force = std::getenv("CVD_RHO_GLOBAL");   // tests: the HBM path at small K
  if (lds > 160 * 1024 || (force && force[0] == '1')) {
    if (!d_cols) { cvd::set_error("spectral_radius: K > 10000 needs the structured (cols) form"); return CVD_E_UNSUPPORTED; }
    if (U == 0) return CVD_OK;
    return spectral_radius_global(K, E, d_a, d_vals, d_cols, U, tol, max_iter, d_rho, d_iters, (hipStream_t)stream);
  }
  if (U == 0) return CVD_OK;
  RhoArgs p{K, E, d_a, d_vals, d_cols, tol, max_iter, d_rho, d_iters};
  if (lds > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute((const void*)spectral_radius_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
  hipLaunchKernelGGL(spectral_radius_kernel, dim3((unsigned)U), dim3(kRhoBlock), lds, (hipStream_t)stream, p);
  HIP_CHECK(hipGetLastError());
  return CVD_OK;
}
