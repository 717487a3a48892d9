"""Parity-template baseline detector, MI355X path.

Reference (So-bonkers/Detecting-Convolutional-Codes-Via-Markovian-Statistics):
  parity_eqn_check.parse_poly_token          parity_eqn_check.py:60-86
  parity_eqn_check.nullspace_mod2            parity_eqn_check.py:93-141
  parity_eqn_check.build_parity_system       parity_eqn_check.py:148-181
  parity_eqn_check.parity_vector_to_equation parity_eqn_check.py:188-201
  comp_parity.parity_satisfaction_fraction   comp_parity.py:90-117
  comp_parity.parity_detector                comp_parity.py:120-128
  comp_parity.__main__ (template choice, MC) comp_parity.py:135-181

The template algebra (GF(2) nullspace of a small system) is host work, done
here with bit-packed Python ints.  The per-trial scan runs on the GPU through
libcvd.so (cvd_parity_detect) over the same received streams the Markov
detector reads (cvd_generate), so `parity_experiment` yields the baseline's
{N, p, Pd, Pc} table on exactly the trials `run_experiment` uses -- the CSV
pair plots_compare.py:70-134 compares.  No CPU fallback.
"""
import ctypes
import re

import numpy as np
import torch

from . import _lib
from .codes import as_code
from .detector import _detector, _stream_ptr, grid_tag, N_SPECTRUM_BY_M


def parse_poly_token(token):
    """Octal ("133"), binary MSB-first ("1011") or comma list ("1,0,1") ->
    LSB-first coefficients (parity_eqn_check.py:60-86)."""
    token = token.strip()
    if "," in token:
        return [int(x) for x in token.split(",")]
    if re.fullmatch(r"[01]+", token):
        return [int(b) for b in reversed(token)]
    if re.fullmatch(r"[0-7]+", token):
        v = int(token, 8)
        return [(v >> i) & 1 for i in range(v.bit_length())]
    raise ValueError(f"Cannot parse polynomial token: {token}")


def build_parity_system(generators, deg_h):
    """GF(2) system A h = 0 whose solutions are the parity-check vectors
    h(D) = (h_1, ..., h_n), deg h_j <= deg_h, with sum_j h_j g_{j,i} = 0 for every
    input i (parity_eqn_check.py:148-181).  Rows i*(Kmax+1) + t, columns
    j*(deg_h+1) + s; uint8 array."""
    n, k = len(generators), len(generators[0])
    deg_g = max(len(g) - 1 for out in generators for g in out)
    kmax = deg_g + deg_h
    A = np.zeros((k * (kmax + 1), n * (deg_h + 1)), np.uint8)
    for i in range(k):
        for j in range(n):
            for u, bit in enumerate(generators[j][i]):
                if not bit:
                    continue
                for s in range(deg_h + 1):          # coefficient of D^(s+u) in h_j g_{j,i}
                    A[i * (kmax + 1) + s + u, j * (deg_h + 1) + s] ^= 1
    return A


def nullspace_mod2(A):
    """Basis of {x : A x = 0 over GF(2)}, one vector per free column of the
    reduced row echelon form, in column order (parity_eqn_check.py:93-141).
    Rows are Python ints (bit c = column c) during elimination."""
    A = np.asarray(A, np.uint8)
    nrow, ncol = A.shape
    rows = [int("".join(str(int(b)) for b in A[r, ::-1]), 2) if ncol else 0 for r in range(nrow)]
    pivots = []
    top = 0
    for c in range(ncol):
        if top >= nrow:
            break
        bit = 1 << c
        sel = next((r for r in range(top, nrow) if rows[r] & bit), None)
        if sel is None:
            continue
        rows[top], rows[sel] = rows[sel], rows[top]
        for r in range(nrow):
            if r != top and rows[r] & bit:
                rows[r] ^= rows[top]
        pivots.append(c)
        top += 1
    free = [c for c in range(ncol) if c not in set(pivots)]
    basis = np.zeros((len(free), ncol), np.uint8)
    for b, f in enumerate(free):
        basis[b, f] = 1
        for r, pc in enumerate(pivots):
            if (rows[r] >> f) & 1:
                basis[b, pc] = 1
    return basis


def parity_vector_to_equation(h_vec):
    """"v0[t-0] ⊕ v1[t-2] ⊕ ... = 0" (parity_eqn_check.py:188-201)."""
    terms = [f"v{j}[t-{s}]" for j, poly in enumerate(h_vec) for s, bit in enumerate(poly) if bit]
    return " ⊕ ".join(terms) + " = 0"


def parity_vectors(generators, deg_h):
    """Every basis parity-check vector as h_vec[j] = coefficient list (length deg_h+1)."""
    n = len(generators)
    basis = nullspace_mod2(build_parity_system(generators, deg_h))
    return [[row[j * (deg_h + 1):(j + 1) * (deg_h + 1)].tolist() for j in range(n)] for row in basis]


def template_of(h_vec):
    """(output j, delay s) for every set coefficient (comp_parity.py:160-165)."""
    return [(j, s) for j, poly in enumerate(h_vec) for s, bit in enumerate(poly) if bit]


def default_template(generators, m, deg_h=None, index=0):
    """The reference's choice: basis vector `index` (0) of the system with
    deg_h = m + 3 (comp_parity.py:143-165)."""
    deg_h = m + 3 if deg_h is None else int(deg_h)
    vecs = parity_vectors(generators, deg_h)
    if not vecs:
        raise ValueError(f"no parity-check vector of degree <= {deg_h}")
    return template_of(vecs[index])


def _terms(template):
    t = np.array([[int(j), int(s)] for (j, s) in template], np.int32).reshape(-1, 2)
    if len(t) == 0:
        raise ValueError("empty parity template")
    return t


def parity_detect(r, n, N, nseq, n_h1, template, gamma, sat=None, counts=None, device=None, stream=None):
    """cvd_parity_detect over a received-word buffer [W/4, nseq, 4] (include/cvd.h
    layout): accumulates (H1 successes, H2 successes) into `counts`."""
    dev = r.device
    if counts is None:
        counts = torch.zeros(2, dtype=torch.int64, device=dev)
    t = _terms(template)
    _lib.check(_lib.lib().cvd_parity_detect(
        ctypes.c_void_p(r.data_ptr()), int(n), int(N), int(nseq), int(n_h1), t.ctypes.data, len(t),
        float(gamma), ctypes.c_void_p(sat.data_ptr() if sat is not None else 0),
        ctypes.c_void_p(counts.data_ptr()), _stream_ptr(stream)))
    return counts


def parity_satisfaction_fraction(y, template, device=None):
    """P̂(N) of one received sequence y[j][t] (comp_parity.py:90-117), on the GPU."""
    n, T = len(y), len(y[0])
    if not torch.cuda.is_available():
        raise RuntimeError("the parity detector runs on the GPU (HIP); no GPU is visible")
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    spw = 32 // n
    W = ((T + spw - 1) // spw + 3) // 4 * 4
    words = np.zeros(max(W, 4), np.uint64)
    yy = np.asarray(y, np.uint64).reshape(n, T)
    for j in range(n):
        t = np.arange(T)
        np.bitwise_or.at(words, t // spw, yy[j] << ((t % spw) * n + j).astype(np.uint64))
    buf = torch.from_numpy(words.astype(np.uint32).view(np.int32).reshape(-1, 1, 4)).to(dev)
    sat = torch.zeros(1, dtype=torch.int32, device=dev)
    parity_detect(buf, n, T, 1, 1, template, 0.0, sat=sat)
    first = max(s for (_, s) in template)
    total = T - first if T > first else 0
    return int(sat.item()) / total if total > 0 else 0.0


def parity_detector(y, template, gamma, device=None):
    """(P̂ >= gamma, P̂) (comp_parity.py:120-128)."""
    ph = parity_satisfaction_fraction(y, template, device)
    return ph >= gamma, ph


def parity_experiment(k, n, m, gen1, gen2, num_iter, p_vec, gamma, seed, N_list=None, template=None,
                      deg_h=None, device=None, batch=None):
    """The baseline's {N, p, Pd, Pc} table on the trials run_experiment uses:
    trial t of grid point (N, p) = H1 stream (gen1, seq 2t) + H2 stream (gen2,
    seq 2t+1), both tested against the template of gen1 (default: the
    reference's basis vector 0 at deg_h = m + 3).  Pd = P(P̂ >= gamma | H1),
    Pc = (H1 correct + H2 correct) / (2 num_iter).  Sharded over ranks and
    reduced with one all_reduce like run_experiment."""
    import pandas as pd
    from .distributed import run_sharded, pd_rows

    det = _detector(k, n, m, gen1, device)
    g1, g2 = as_code(gen1, m, k, n), as_code(gen2, m, k, n)
    if template is None:
        template = default_template(gen1, m, deg_h)
    N_spectrum = list(N_SPECTRUM_BY_M.get(m, [50, 100, 200]) if N_list is None else N_list)

    def count_fn(iN, N, ip, p, lo, hi, out):
        T = hi - lo
        if T <= 0:
            return
        B = det.default_batch(N, T) if batch is None else int(batch)
        tag = grid_tag(N, p)
        for b in range(lo, hi, B):
            Tb = min(B, hi - b)
            r = det.stream_buffer(N, 2 * Tb)
            det.generate(g1, N, p, seed, tag, 2 * b, 2, Tb, out=r, q0=0, pitch=2 * Tb)
            det.generate(g2, N, p, seed, tag, 2 * b + 1, 2, Tb, out=r, q0=Tb, pitch=2 * Tb)
            parity_detect(r, n, N, 2 * Tb, Tb, template, gamma, counts=out)

    counts = run_sharded(count_fn, N_spectrum, list(p_vec), num_iter, det.device)
    return pd.DataFrame(pd_rows(counts, N_spectrum, list(p_vec), num_iter))
