"""Parity-template baseline, restated for checking (TEST INFRASTRUCTURE ONLY).

Only tests/ may use this module.  Plain restatements of the reference's
parity_eqn_check.py / comp_parity.py functions, pinned to the reference's own
outputs by tests/golden/parity.{npz,json} (tests/golden/make_golden_parity.py).
"""
import numpy as np


def build_parity_system(generators, deg_h):
    """parity_eqn_check.py:148-181."""
    n, k = len(generators), len(generators[0])
    deg_g = max(len(g) - 1 for out in generators for g in out)
    kmax = deg_g + deg_h
    A = np.zeros((k * (kmax + 1), n * (deg_h + 1)), np.uint8)
    for i in range(k):
        for t in range(kmax + 1):
            for j in range(n):
                for u, bit in enumerate(generators[j][i]):
                    if bit and 0 <= t - u <= deg_h:
                        A[i * (kmax + 1) + t, j * (deg_h + 1) + t - u] ^= 1
    return A


def nullspace_mod2(A):
    """parity_eqn_check.py:93-141 (Gauss-Jordan over GF(2), free columns in order)."""
    R = np.array(A, np.uint8) % 2
    m, n = R.shape
    piv, row = [], 0
    for col in range(n):
        if row >= m:
            break
        nz = np.nonzero(R[row:, col])[0]
        if len(nz) == 0:
            continue
        sel = row + nz[0]
        R[[row, sel]] = R[[sel, row]]
        for r in np.nonzero(R[:, col])[0]:
            if r != row:
                R[r] ^= R[row]
        piv.append(col)
        row += 1
    free = [c for c in range(n) if c not in piv]
    out = np.zeros((len(free), n), np.uint8)
    for b, f in enumerate(free):
        out[b, f] = 1
        for r, pc in enumerate(piv):
            if R[r, f]:
                out[b, pc] = 1
    return out


def satisfied_count(y, template):
    """(satisfied anchors, anchors) of comp_parity.py:90-117: anchors
    t in [max delay, T), satisfied iff XOR_{(j,s)} y[j][t-s] == 0."""
    y = np.asarray(y, np.uint8)
    T = y.shape[1]
    first = max(s for (_, s) in template)
    if T <= first:
        return 0, 0
    x = np.zeros(T - first, np.uint8)
    for (j, s) in template:
        x ^= y[j, first - s:T - s]
    return int(np.sum(x == 0)), T - first


def parity_satisfaction_fraction(y, template):
    sat, tot = satisfied_count(y, template)
    return sat / tot if tot > 0 else 0.0


def streams_from_words(r, n):
    """received words r[t] (bit j = output j) -> y[j][t]."""
    r = np.asarray(r, np.int64)
    return np.stack([(r >> j) & 1 for j in range(n)]).astype(np.uint8)
