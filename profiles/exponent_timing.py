#!/usr/bin/env python3
"""Wall-clock timing of the error-exponent engine (alpha_exponent.py, Eq. 7) on
one GPU, with the reference's own numpy algorithm for Eq. 7 timed beside it on
the host (dense M(u) + np.linalg.eigvals, alpha_exponent.py:159-188) where it
finishes in reasonable time.  Prints one JSON line per case.

  python profiles/exponent_timing.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

CASES = {
    "m2": (1, 2, 2, [[[1, 1, 1]], [[1, 0, 1]]], [[[1, 0, 1]], [[1, 1, 1]]]),
    "m3": (1, 2, 3, [[[1, 1, 1, 1]], [[1, 0, 1, 1]]], [[[1, 0, 1, 1]], [[1, 1, 1, 1]]]),
    "r23_m4": (2, 3, 4, [[[1, 0, 0, 0, 1], [0, 1, 1, 1, 1]], [[1, 1, 1, 0, 1], [0, 1, 0, 1, 0]],
                         [[0, 1, 1, 0, 0], [1, 1, 0, 1, 0]]],
               [[[1, 1, 1, 0, 1], [0, 1, 0, 1, 0]], [[0, 1, 1, 0, 0], [1, 1, 0, 1, 0]],
                [[1, 0, 0, 0, 1], [0, 1, 1, 1, 1]]]),
    # K = 150,743: the HBM power iteration (above the LDS limit)
    "m4": (1, 2, 4, [[[1, 0, 0, 1, 1]], [[1, 1, 1, 0, 1]]], [[[1, 1, 1, 0, 1]], [[1, 0, 0, 1, 1]]]),
}


def numpy_eq7(P1, P2, u_grid):
    """alpha_exponent.py:159-188 restated (host baseline; not the product)."""
    P1 = np.clip(P1, 1e-300, 1.0)
    P2 = np.clip(P2, 1e-300, 1.0)
    best = None
    for u in np.linspace(0.0, 1.0, u_grid):
        M = np.sum((P1 ** u) * (P2 ** (1.0 - u)), axis=2)
        rho = max(float(np.max(np.abs(np.linalg.eigvals(M)))), 1e-300)
        if best is None or rho < best[0]:
            best = (rho, u)
    return -np.log(best[0]), best[1]


def main():
    pkg = load_package()
    torch.cuda.init()
    for name, (k, n, m, g1, g2) in CASES.items():
        length, chains, p = 1_000_000, 256, 0.05
        t0 = time.perf_counter()
        P1, *_ = pkg.learn_transition_tensor(g1, g1, m, p, length=length, burn_in=5000, seed=1, k=k, n=n, chains=chains)
        P2, *_ = pkg.learn_transition_tensor(g2, g1, m, p, length=length, burn_in=5000, seed=2, k=k, n=n, chains=chains)
        torch.cuda.synchronize()
        t_learn = time.perf_counter() - t0
        t0 = time.perf_counter()
        I, u = pkg.compute_error_exponent(P1, P2, u_grid=401)
        t_eq7 = time.perf_counter() - t0
        out = {"case": name, "K": P1.K, "R": P1.R, "learn_steps_per_tensor": length, "chains": chains,
               "learn_s_two_tensors": t_learn, "eq7_s_401u_gpu": t_eq7, "I_err": I, "u": u}
        if P1.K <= 500:
            ug = 401 if P1.K <= 64 else 21
            t0 = time.perf_counter()
            I_np, u_np = numpy_eq7(np.asarray(P1), np.asarray(P2), ug)
            out.update({"numpy_eq7_s": time.perf_counter() - t0, "numpy_u_grid": ug, "numpy_I_err": I_np,
                        "numpy_cores": 1 if os.environ.get("OMP_NUM_THREADS") == "1" else "BLAS default"})
            if ug == 401:
                out["abs_diff_I"] = abs(I - I_np)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
