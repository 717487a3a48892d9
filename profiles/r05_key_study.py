#!/usr/bin/env python3
"""Key-layout study for the bit-sliced m = 6 detector core.

The bit-sliced step keeps the 64 metrics in a layout that rotates with the step (period
6): at phase f the metric of state s sits at location ror6(s, f).  The row tables must
therefore be found from any of six images of one metric vector.  Storing six images per
row in the Bloom filter multiplies its keys by six (the filter must stay L2-resident, so
that is not affordable), and canonicalising the planes before hashing costs a bit
permutation network per step.  The alternative measured here: hash a ROTATION-INVARIANT
function of the vector -- popcounts of plane combinations over unions of the necklace
orbits of the 6-bit state index (an orbit-union mask is the same set of locations in
every phase) -- so one filter entry per row serves every phase, and compare the exact
key only on filter positives.

For a candidate invariant this script reports, on the learned rows of the headline
decoder (C oracle's D4 model, learn_len 1e6) and on D_t of H1 and H2 sequences at the
same p (the detector's queries): the share of non-row query states whose invariant
equals some row's (these would pass any filter on the invariant: extra directory reads),
and the number of rows sharing an invariant value (directory probe chains).

  python profiles/r05_key_study.py [p ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import c_oracle as C  # noqa: E402  (design study, not product code)
from oracle import restatement as R  # noqa: E402

G1 = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]
G2 = [[[1, 1, 1, 1, 0, 0, 1]], [[1, 0, 1, 1, 0, 1, 1]]]


def rot6(s, k):
    return ((s << k) | (s >> (6 - k))) & 63


def orbits():
    seen, out = set(), []
    for s in range(64):
        if s in seen:
            continue
        o = sorted({rot6(s, k) for k in range(6)})
        seen.update(o)
        out.append(o)
    return out


ORB = orbits()
ORB_ID = np.zeros(64, np.int64)
for i, o in enumerate(ORB):
    ORB_ID[o] = i


def d_states(enc, p, nseq, N, seed=7, tag=12345):
    """D_1..D_N of nseq sequences (canonical state order), vectorised over sequences."""
    out_sym, nxt = R.encoder_tables(G1, 6, 1, 2)
    r = np.stack([C.stream(C.Code(enc, 6, 1, 2), N, p, seed, tag, 2 * q + (0 if enc is G1 else 1))
                  for q in range(nseq)])
    # predecessor table: new state ns has predecessors (s, u) with nxt[s, u] == ns
    pred = [[] for _ in range(64)]
    for s in range(64):
        for u in range(2):
            pred[nxt[s, u]].append((s, out_sym[s, u]))
    ps = np.array([[a for a, _ in pred[ns]] for ns in range(64)])       # [64, 2]
    po = np.array([[o for _, o in pred[ns]] for ns in range(64)])
    pc = np.array([bin(v).count("1") for v in range(4)])
    D = np.zeros((nseq, 64), np.int64)
    outs = np.empty((N, nseq, 64), np.uint8)
    for t in range(N):
        y = r[:, t][:, None, None]
        cand = D[:, ps] + pc[po[None] ^ y]
        Dn = cand.min(axis=2)
        D = Dn - Dn.min(axis=1, keepdims=True)
        outs[t] = D
    return outs.reshape(-1, 64)


def planes(D):
    return [((D >> i) & 1).astype(np.int64) for i in range(4)]


# ─────────── candidate invariants (each: [n, 64] uint8 -> [n, F] int64) ───────────

def inv_orbit_multiset(D):
    """upper bound for orbit-popcount features: per orbit, the histogram of values"""
    H = np.zeros((D.shape[0], len(ORB), 16), np.int64)
    for i in range(len(ORB)):
        for v in range(16):
            H[:, i, v] = (D[:, ORB[i]] == v).sum(axis=1)
    return H.reshape(D.shape[0], -1)


def inv_orbit_sums(D):
    return np.stack([D[:, o].sum(axis=1) for o in ORB], axis=1)


def inv_plane_orbit(D, masks, funcs):
    """popcount over orbit-union mask of elementwise plane functions"""
    P = planes(D.astype(np.int64))
    cols = []
    for f in funcs:
        x = f(P)
        for M in masks:
            cols.append((x * M[None]).sum(axis=1))
    return np.stack(cols, axis=1)


def mask_of(orbit_ids):
    M = np.zeros(64, np.int64)
    for i in orbit_ids:
        M[ORB[i]] = 1
    return M


def study(p, nseq, N, invs):
    t0 = time.time()
    M = C.Model(C.Code(G1, 6, 1, 2), p)
    _, keys = M.rows()
    keys = keys.astype(np.int64)
    rowset = {k.tobytes() for k in keys.astype(np.uint8)}
    print(f"p={p}: rows {keys.shape[0]}  ({time.time() - t0:.1f}s)", flush=True)
    Q = {}
    for name, enc in (("H1", G1), ("H2", G2)):
        Q[name] = d_states(enc, p, nseq, N)
    for iname, fn in invs:
        rk = fn(keys)
        rv = {tuple(v) for v in rk}
        # rows per invariant value
        _, cnt = np.unique(rk, axis=0, return_counts=True)
        line = [f"  {iname:28s} distinct {len(rv):8d}  rows/value mean {keys.shape[0] / len(rv):6.2f} max {cnt.max():6d}"]
        for name in ("H1", "H2"):
            D = Q[name]
            isrow = np.fromiter((d.tobytes() in rowset for d in D), bool, D.shape[0])
            qv = fn(D.astype(np.int64))
            hit = np.fromiter((tuple(v) in rv for v in qv), bool, D.shape[0])
            nr = ~isrow
            line.append(f"{name}: rows {isrow.mean():.3f} false-match {hit[nr].mean():.2e}")
        print("  ".join(line), flush=True)


def main():
    ps = [float(a) for a in sys.argv[1:]] or [0.05, 0.2]
    nseq, N = int(os.environ.get("NSEQ", "64")), int(os.environ.get("NSTEP", "2000"))
    sizes = [len(o) for o in ORB]
    print(f"{len(ORB)} necklace orbits, sizes {sizes}")
    big = [i for i, o in enumerate(ORB) if len(o) == 6]
    small = [i for i, o in enumerate(ORB) if len(o) < 6]
    # orbit-union masks: halves / thirds of the size-6 orbits
    m_all = mask_of(range(len(ORB)))
    m_a = mask_of(big[0::2] + small[0::2])
    m_b = mask_of(big[1::2] + small[1::2])
    m_c = mask_of(big[0::3] + small[0::3])
    m_d = mask_of(big[1::3] + small[1::3])
    m_e = mask_of([big[i] for i in (0, 3, 4, 7)] + small[1::2])
    pl = [lambda P, i=i: P[i] for i in range(4)]
    x01 = [lambda P: P[0] ^ P[1], lambda P: P[1] ^ P[2], lambda P: P[0] & P[1]]
    dig = lambda f: (lambda D: np.stack([f(D.astype(np.int64))[:, :32] @ (1 << np.arange(32)),
                                          f(D.astype(np.int64))[:, 32:] @ (1 << np.arange(32))], axis=1))
    invs = [
        ("digest P0", dig(lambda D: D & 1)),
        ("digest D==0", dig(lambda D: (D == 0).astype(np.int64))),
        ("digest P0^P1", dig(lambda D: (D ^ (D >> 1)) & 1)),
        ("digest D<=1", dig(lambda D: (D <= 1).astype(np.int64))),
        ("digest P0,P1", lambda D: np.concatenate([dig(lambda D: D & 1)(D), dig(lambda D: (D >> 1) & 1)(D)], axis=1)),
        ("digest P0^P2,P1^P3", lambda D: np.concatenate([dig(lambda D: (D ^ (D >> 2)) & 1)(D), dig(lambda D: ((D >> 1) ^ (D >> 3)) & 1)(D)], axis=1)),
        ("orbit multiset (bound)", inv_orbit_multiset),
        ("orbit sums", inv_orbit_sums),
        ("planes x all", lambda D: inv_plane_orbit(D, [m_all], pl)),
        ("planes x {a,b}", lambda D: inv_plane_orbit(D, [m_a, m_b], pl)),
        ("planes x {a,c,d}", lambda D: inv_plane_orbit(D, [m_all, m_a, m_c, m_d], pl)),
        ("planes x {a,c,d,e}+x01", lambda D: np.concatenate(
            [inv_plane_orbit(D, [m_all, m_a, m_c, m_d, m_e], pl), inv_plane_orbit(D, [m_a, m_c], x01)], axis=1)),
    ]
    for p in ps:
        study(p, nseq, N, invs)


if __name__ == "__main__":
    main()
