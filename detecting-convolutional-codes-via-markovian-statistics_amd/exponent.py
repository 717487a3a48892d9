"""Error-exponent engine, MI355X path.

Reference (So-bonkers/Detecting-Convolutional-Codes-Via-Markovian-Statistics):
  alpha_exponent.spectral_radius          alpha_exponent.py:69-76
  alpha_exponent.learn_transition_tensor  alpha_exponent.py:83-156
  alpha_exponent.compute_error_exponent   alpha_exponent.py:159-188   (Eq. 7)
  alpha_exponent.fit_error_exponent       alpha_exponent.py:191-215

Eq. 7:  I_err = min_{u in [0,1]} -log rho(M(u)),
        M(u)[i, j] = sum_r P1(i->j, r)^u P2(i->j, r)^(1-u).

GPU work (libcvd.so, csrc/cvd_exponent.hip):
  * joint counts of (metric state, received word) along trial-spec streams
    (cvd_generate + cvd_count_transitions: LDS-resident automaton, LDS
    histograms);
  * M(u) for the whole u grid (cvd_chernoff_build: O(K 2^n) per u for learned
    tensors, whose only structure beyond Laplace smoothing is C[i, j, r] != 0
    iff j = next(i, r); cvd_chernoff_build_dense for arbitrary tensors);
  * rho(M(u)) for every u at once (cvd_spectral_radius: one workgroup per u,
    power iteration with Collatz-Wielandt bounds to a stated tolerance).

Declared deviations: the reference's learner does not run as
written (enumerate_markov_states_allzero / build_trellis are called with 2 of
their 4 / 3 arguments, alpha_exponent.py:109,116; octal_to_taps is missing,
:57) and its _encoder_step shifts the register the other way from
viterbi_markov (alpha_exponent.py:233 vs viterbi_markov.py:102-104).  Here the
chain is the detector's own: encoder and BSC(p) of the trial spec (D1/D2),
metric states of the decoder's BFS automaton, `chains` independent chains of
burn_in + length/chains steps (chains = 1: one chain, as the reference).
rho is the Perron root (the spectral radius of the nonnegative M(u)); the
reference computes it with np.linalg.eigvals -- agreement is to `tol`.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .codes import as_code
from .detector import _detector, _stream_ptr, enumerate_markov_states_allzero

EXPONENT_TAG = 0xE4B0E470   # stream tag of the transition-learning chains (top bit set: no grid tag)


def _dev(device):
    if not torch.cuda.is_available():
        raise RuntimeError("the error-exponent engine runs on the GPU (HIP); no GPU is visible")
    return torch.device("cuda", torch.cuda.current_device() if device is None else device)


class TransitionTensor:
    """Learned P(i -> j, r) of alpha_exponent.py:152-154 in the form the chain
    produces it: joint counts counts[i, r] of (state i, received word r), the
    decoder automaton next[i, r], and the Laplace constant.  np.asarray(T)
    (or T.dense()) gives the reference's normalised K x K x 2^n tensor."""

    def __init__(self, counts, next_state, laplace):
        self.counts = np.asarray(counts, np.float64)
        self.next = np.asarray(next_state, np.int32)
        self.laplace = float(laplace)
        self.K, self.R = self.counts.shape

    def dense(self):
        C = np.zeros((self.K, self.K, self.R), np.float64)
        i = np.repeat(np.arange(self.K), self.R)
        r = np.tile(np.arange(self.R), self.K)
        np.add.at(C, (i, self.next.reshape(-1), r), self.counts.reshape(-1))
        C += self.laplace
        C /= np.maximum(C.sum(axis=(1, 2), keepdims=True), 1.0)
        return C

    def __array__(self, dtype=None, copy=None):
        d = self.dense()
        return d if dtype is None else d.astype(dtype)


def learn_transition_tensor(encoder_taps, decoder_taps, m, p, length=300_000, burn_in=5_000, laplace=1.0,
                            seed=None, k=1, n=None, chains=1, device=None):
    """(P, states, sidx, all_r) as alpha_exponent.py:83-156; P is a
    TransitionTensor over the decoder's BFS states (dense models only)."""
    n = len(decoder_taps) if n is None else n
    det = _detector(k, n, m, decoder_taps, device)
    model = det.model(float(p), learn_len=0, learn_burn=0, laplace=1.0, seed=0)
    if model.info()["kind"] != 0:
        raise _lib.CvdError("learn_transition_tensor: the decoder's metric states are not enumerable "
                            "(the reference needs the full BFS, alpha_exponent.py:109)")
    states, transitions, all_r = enumerate_markov_states_allzero(decoder_taps, m, k, n)
    K, R = len(states), 1 << n
    nxt = np.zeros((K, R), np.int32)
    for i in range(K):
        for j, rs in transitions[i].items():
            for rt in rs:
                nxt[i, sum(b << q for q, b in enumerate(rt))] = j
    chains = max(1, int(chains))
    per = -(-int(length) // chains)
    steps = int(burn_in) + per
    sd = 0 if seed is None else int(seed)
    enc = as_code(encoder_taps, m, k, n)
    r = det.generate(enc, steps, float(p), sd, EXPONENT_TAG, 0, 1, chains)
    cnt = torch.zeros(K * R, dtype=torch.int64, device=det.device)
    _lib.check(_lib.lib().cvd_count_transitions(model.handle, ctypes.c_void_p(r.data_ptr()), steps, chains,
                                                int(burn_in), ctypes.c_void_p(cnt.data_ptr()), _stream_ptr(None)))
    counts = cnt.view(K, R).cpu().numpy().astype(np.float64)
    sidx = {s: i for i, s in enumerate(states)}
    return TransitionTensor(counts, nxt, laplace), states, sidx, all_r


def _rho_batch(K, E, a, vals, cols, U, tol, max_iter, dev):
    rho = torch.empty(3 * U, dtype=torch.float64, device=dev)
    its = torch.empty(U, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().cvd_spectral_radius(
        int(K), int(E), ctypes.c_void_p(a.data_ptr() if a is not None else 0), ctypes.c_void_p(vals.data_ptr()),
        ctypes.c_void_p(cols.data_ptr() if cols is not None else 0), int(U), float(tol), int(max_iter),
        ctypes.c_void_p(rho.data_ptr()), ctypes.c_void_p(its.data_ptr()), _stream_ptr(None)))
    return rho.view(U, 3).cpu().numpy(), its.cpu().numpy()


def chernoff_rhos(P1, P2, u_vals, tol=1e-13, max_iter=200_000, device=None, return_bounds=False):
    """rho(M(u)) for every u in u_vals (GPU), M(u) as in Eq. 7."""
    dev = _dev(device)
    u = torch.as_tensor(np.asarray(u_vals, np.float64), device=dev)
    U = len(u)
    if isinstance(P1, TransitionTensor) and isinstance(P2, TransitionTensor):
        if (P1.K, P1.R) != (P2.K, P2.R) or not np.array_equal(P1.next, P2.next) or P1.laplace != P2.laplace:
            raise ValueError("P1 and P2 must share the decoder automaton and the Laplace constant")
        K, R = P1.K, P1.R
        c1 = torch.as_tensor(P1.counts, device=dev)
        c2 = torch.as_tensor(P2.counts, device=dev)
        cols = torch.as_tensor(P1.next.reshape(-1), device=dev)
        a = torch.empty(U * K, dtype=torch.float64, device=dev)
        vals = torch.empty(U * K * R, dtype=torch.float64, device=dev)
        _lib.check(_lib.lib().cvd_chernoff_build(K, R, ctypes.c_void_p(c1.data_ptr()), ctypes.c_void_p(c2.data_ptr()),
                                                 P1.laplace, ctypes.c_void_p(u.data_ptr()), U,
                                                 ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(vals.data_ptr()),
                                                 _stream_ptr(None)))
        out, its = _rho_batch(K, R, a, vals, cols, U, tol, max_iter, dev)
    else:
        A1, A2 = np.asarray(P1, np.float64), np.asarray(P2, np.float64)
        if A1.shape != A2.shape or A1.ndim != 3 or A1.shape[0] != A1.shape[1]:
            raise ValueError("P1, P2 must be K x K x R tensors of one shape")
        K, R = A1.shape[0], A1.shape[2]
        d1 = torch.as_tensor(np.ascontiguousarray(A1), device=dev)
        d2 = torch.as_tensor(np.ascontiguousarray(A2), device=dev)
        chunk = max(1, min(U, (1 << 28) // (K * K)))   # <= 2 GiB of M(u) at a time
        outs, itss = [], []
        for lo in range(0, U, chunk):
            hi = min(U, lo + chunk)
            vals = torch.empty((hi - lo) * K * K, dtype=torch.float64, device=dev)
            us = u[lo:hi].contiguous()
            _lib.check(_lib.lib().cvd_chernoff_build_dense(K, R, ctypes.c_void_p(d1.data_ptr()),
                                                           ctypes.c_void_p(d2.data_ptr()), ctypes.c_void_p(us.data_ptr()),
                                                           hi - lo, ctypes.c_void_p(vals.data_ptr()), _stream_ptr(None)))
            o, it = _rho_batch(K, K, None, vals, None, hi - lo, tol, max_iter, dev)
            outs.append(o)
            itss.append(it)
        out, its = np.concatenate(outs), np.concatenate(itss)
    return (out, its) if return_bounds else out[:, 0]


def compute_error_exponent(P1_ijr, P2_ijr, u_grid=401, tol=1e-13, max_iter=200_000, device=None):
    """(I_err, u*) of Eq. 7 (alpha_exponent.py:159-188): the first u of
    linspace(0, 1, u_grid) with the smallest rho(M(u)), I_err = -log rho."""
    u_vals = np.linspace(0.0, 1.0, int(u_grid))
    rhos = chernoff_rhos(P1_ijr, P2_ijr, u_vals, tol, max_iter, device)
    best_rho, best_u = None, None
    for u, rho in zip(u_vals, rhos):
        rho = max(float(rho), 1e-300)
        if best_rho is None or rho < best_rho:
            best_rho, best_u = rho, u
    return float(-np.log(best_rho)), float(best_u)


def spectral_radius(A, tol=1e-13, max_iter=200_000, device=None):
    """rho(A) for a nonnegative square matrix (alpha_exponent.py:69-76): the
    Perron root, on the GPU.  Matrices with negative entries are rejected (the
    reference's general eigvals has no GPU counterpart here)."""
    A = np.asarray(A, np.float64)
    if A.ndim != 2 or A.shape[0] != A.shape[1]:
        raise ValueError("spectral_radius: square matrix expected")
    if np.any(A < 0):
        raise ValueError("spectral_radius: the GPU path computes the Perron root of a nonnegative matrix")
    dev = _dev(device)
    K = A.shape[0]
    vals = torch.as_tensor(np.ascontiguousarray(A).reshape(-1), device=dev)
    out, _ = _rho_batch(K, K, None, vals, None, 1, tol, max_iter, dev)
    return float(out[0, 0])


def fit_error_exponent(N_vals, P_e_vals, tail_cap=0.2):
    """Least-squares fit of P_e(N) ~ A exp(-I N) on the tail 0 < P_e <= tail_cap
    (alpha_exponent.py:191-215); host numpy, (I_emp, A) or (0.0, nan)."""
    N = np.asarray(N_vals, dtype=float)
    P_e = np.asarray(P_e_vals, dtype=float)
    mask = (P_e > 0) & (P_e <= tail_cap)
    if np.sum(mask) < 3:
        return 0.0, float("nan")
    y = np.log(P_e[mask])
    X = np.vstack([np.ones_like(N[mask]), -N[mask]]).T
    beta, *_ = np.linalg.lstsq(X, y, rcond=None)
    return float(beta[1]), float(np.exp(beta[0]))
