#!/usr/bin/env python3
"""Golden fixtures for the error-exponent engine (tests/golden/exponent.npz +
exponent.json), computed by the REFERENCE's own, unmodified functions:

  alpha_exponent.spectral_radius        (alpha_exponent.py:69-76)
  alpha_exponent.compute_error_exponent (alpha_exponent.py:159-188)
  alpha_exponent.fit_error_exponent     (alpha_exponent.py:191-215)

alpha_exponent.py imports `octal_to_taps` and `simulate_markov_sequence` from
viterbi_markov, which defines neither; stubs are injected
into viterbi_markov only so the module imports -- none of the three functions
above calls them.  The
inputs are fixed random matrices / tensors (seeded numpy), including tensors of
the learned structure C[i, next(i, r), r] + Laplace over the (7,5) decoder's
BFS automaton (viterbi_markov.enumerate_markov_states_allzero).

Runs only in the build container, where /root/reference is importable
(SURVEY.md §8(c)); only inputs/outputs are committed.

Usage:  python tests/golden/make_golden_exponent.py   (≈ 10 s)
"""
import json
import os
import sys

os.environ.setdefault("MPLBACKEND", "Agg")
sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

import viterbi_markov as vm  # noqa: E402  (reference)

for _name in ("octal_to_taps", "simulate_markov_sequence"):
    if not hasattr(vm, _name):   # import-time stubs only (never called below)
        setattr(vm, _name, lambda *a, **k: None)
import alpha_exponent as ae  # noqa: E402  (reference)


def learned_structure(taps, m, k, n, rng, scale):
    """Counts C[i, r] on the decoder's BFS automaton and the normalised tensor
    (alpha_exponent.py:152-154 applied to C[i, next(i, r), r] = counts)."""
    states, transitions, all_r = vm.enumerate_markov_states_allzero(taps, m, k, n)
    K, R = len(states), len(all_r)
    nxt = np.zeros((K, R), np.int64)
    for i in range(K):
        for j, rs in transitions[i].items():
            for rt in rs:
                nxt[i, sum(b << q for q, b in enumerate(rt))] = j
    counts = rng.integers(0, scale, size=(K, R)).astype(np.float64)
    C = np.zeros((K, K, R))
    for i in range(K):
        for r in range(R):
            C[i, nxt[i, r], r] += counts[i, r]
    C += 1.0
    C /= np.maximum(C.sum(axis=(1, 2), keepdims=True), 1.0)
    return counts, nxt, C


def main():
    rng = np.random.default_rng(2026)
    arrays, meta = {}, {"generated_by": "tests/golden/make_golden_exponent.py", "rho": [], "exp": [], "fit": []}
    # spectral radii of nonnegative matrices
    for i, K in enumerate([2, 5, 17, 40]):
        A = rng.random((K, K)) * (rng.random((K, K)) < 0.6) + np.eye(K) * 0.01
        arrays[f"rho{i}/A"] = A
        meta["rho"].append(ae.spectral_radius(A))
    # Eq. 7 on dense random tensors (rows normalised over (j, r))
    for i, (K, R, ug) in enumerate([(3, 4, 11), (6, 4, 401), (9, 8, 51)]):
        P1 = rng.random((K, K, R)) + 0.01
        P2 = rng.random((K, K, R)) ** 3 + 0.01
        P1 /= P1.sum(axis=(1, 2), keepdims=True)
        P2 /= P2.sum(axis=(1, 2), keepdims=True)
        arrays[f"exp{i}/P1"], arrays[f"exp{i}/P2"] = P1, P2
        I, u = ae.compute_error_exponent(P1, P2, u_grid=ug)
        meta["exp"].append({"u_grid": ug, "I_err": I, "u": u})
    # Eq. 7 on tensors of the learned structure (m = 2 (7,5) decoder, 31 states)
    taps = [[[1, 1, 1]], [[1, 0, 1]]]
    c1, nxt, P1 = learned_structure(taps, 2, 1, 2, rng, 5000)
    c2, _, P2 = learned_structure(taps, 2, 1, 2, rng, 50)
    arrays["learned/counts1"], arrays["learned/counts2"], arrays["learned/next"] = c1, c2, nxt
    I, u = ae.compute_error_exponent(P1, P2, u_grid=401)
    meta["learned"] = {"I_err": I, "u": u, "laplace": 1.0, "taps": taps}
    # tail fits
    for i in range(3):
        N = np.array([50, 100, 200, 300, 500, 700, 1000], float)
        Pe = 0.8 * np.exp(-0.01 * (i + 1) * N) * np.exp(rng.normal(0, 0.05, N.size))
        Pe[0] = 0.5   # above the tail cap
        arrays[f"fit{i}/N"], arrays[f"fit{i}/Pe"] = N, Pe
        I_emp, A = ae.fit_error_exponent(N, Pe)
        meta["fit"].append({"I_emp": I_emp, "A": A})
    N = np.array([10, 20, 30.0])
    meta["fit_short"] = list(ae.fit_error_exponent(N, np.array([0.5, 0.4, 0.3])))
    np.savez_compressed(os.path.join(HERE, "exponent.npz"), **arrays)
    with open(os.path.join(HERE, "exponent.json"), "w") as f:
        json.dump(meta, f, indent=1, default=float)
    print("wrote exponent.npz / exponent.json:", len(arrays), "arrays")


if __name__ == "__main__":
    main()
