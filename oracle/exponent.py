"""Error-exponent engine, restated for checking (TEST INFRASTRUCTURE ONLY).

Only tests/ may use this module.  Restates alpha_exponent.py's arithmetic
(counts -> normalised tensor :152-154, Eq. 7 via np.linalg.eigvals :69-76,
:159-188, the tail fit :191-215), pinned to the reference's own outputs by
tests/golden/exponent.{npz,json} (tests/golden/make_golden_exponent.py).
"""
import numpy as np


def automaton_counts(r_stream, nxt, burn_in, R):
    """Joint counts [K, R] of (state, received word) along one stream walked on
    the automaton nxt[i, r] from state 0, steps t >= burn_in."""
    K = nxt.shape[0]
    cnt = np.zeros((K, R), np.int64)
    s = 0
    for t, rv in enumerate(r_stream):
        if t >= burn_in:
            cnt[s, rv] += 1
        s = nxt[s, rv]
    return cnt


def dense_tensor(counts, nxt, laplace):
    """alpha_exponent.py:152-154 on C[i, next(i, r), r] = counts[i, r]."""
    K, R = counts.shape
    C = np.zeros((K, K, R), np.float64)
    for i in range(K):
        for r in range(R):
            C[i, nxt[i, r], r] += counts[i, r]
    C += laplace
    C /= np.maximum(C.sum(axis=(1, 2), keepdims=True), 1.0)
    return C


def compute_error_exponent(P1, P2, u_grid=401):
    """alpha_exponent.py:159-188 (numpy eigvals)."""
    P1 = np.clip(P1, 1e-300, 1.0)
    P2 = np.clip(P2, 1e-300, 1.0)
    best_rho = best_u = None
    for u in np.linspace(0.0, 1.0, u_grid):
        M = np.sum((P1 ** u) * (P2 ** (1.0 - u)), axis=2)
        rho = max(float(np.max(np.abs(np.linalg.eigvals(M)))), 1e-300)
        if best_rho is None or rho < best_rho:
            best_rho, best_u = rho, u
    return float(-np.log(best_rho)), float(best_u)
