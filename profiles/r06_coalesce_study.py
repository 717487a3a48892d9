#!/usr/bin/env python3
"""Round 6: how fast the relative-metric recursion forgets its start (CPU study; the C oracle's
streams, TEST / STUDY infrastructure only).

The chunked detector starts a time chunk W steps early from D = 0 and keeps the
chunk only if its D at the chunk start equals the previous chunk's final D.  For the m = 6 pair at
each p this walks the recursion (viterbi_markov.py:139-159) of 64 H1 and 64 H2 sequences from
D_0 = 0, restarts a second copy from D = 0 at step s0, and records the steps until both vectors are
equal (they stay equal afterwards: the step is a function of D and r).  Prints the quantiles and
the share of restarts not yet coalesced after W steps for a few W.

  python profiles/r06_coalesce_study.py [--p 0.01,0.05,0.1,0.2,0.3,0.5] [--starts 8]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import c_oracle as C  # noqa: E402
from r05_lookup_mix import G1, G2, step_tables  # noqa: E402

WS = [64, 128, 192, 384, 768, 1536]


def step(D, rt, pa, pb, bma, bmb):
    Dn = np.minimum(D[:, pa] + bma[rt], D[:, pb] + bmb[rt])
    return Dn - Dn.min(axis=1, keepdims=True)


def run(p, seqs, starts, span, seed=12345):
    dec = C.Code(G1, 6, 1, 2)
    enc2 = C.Code(G2, 6, 1, 2)
    N = starts * span + 4096
    tag = C.lib().oc_grid_tag(100_000, p)
    pa, pb, bma, bmb = step_tables()
    out = {}
    for h, enc in (("H1", dec), ("H2", enc2)):
        r = np.stack([C.stream(enc, N, p, seed, tag, 2 * q + (h == "H2")) for q in range(seqs)])
        # one pass over the true recursion; restarts at s0_k, each tracked until it coalesces
        D = np.zeros((seqs, 64), np.int16)
        act = []          # [s0, restarted D, steps to coalesce per sequence (-1: not yet)]
        s0s = [k * span + 512 for k in range(starts)]
        res = []
        for t in range(N):
            for s0 in s0s:
                if t == s0:
                    act.append([s0, np.zeros((seqs, 64), np.int16), np.full(seqs, -1)])
            rt = r[:, t]
            D = step(D, rt, pa, pb, bma, bmb)
            keep = []
            for e in act:
                e[1] = step(e[1], rt, pa, pb, bma, bmb)
                eq = (e[1] == D).all(axis=1)
                newly = eq & (e[2] < 0)
                e[2][newly] = t + 1 - e[0]
                if (e[2] >= 0).all() or t + 1 - e[0] >= 4096:
                    res.append(e[2].copy())
                else:
                    keep.append(e)
            act = keep
        L = np.concatenate(res)
        miss = L < 0
        Lf = np.where(miss, 10 ** 9, L)
        out[h] = {"restarts": int(L.size), "median": float(np.median(Lf)), "p99": float(np.quantile(Lf, 0.99)),
                  "max": int(Lf.max()) if not miss.any() else "> 4096",
                  "not_coalesced_after_W": {W: float((Lf > W).mean()) for W in WS}}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", default="0.01,0.05,0.1,0.2,0.3,0.5")
    ap.add_argument("--seqs", type=int, default=64)
    ap.add_argument("--starts", type=int, default=8)
    ap.add_argument("--span", type=int, default=1000)
    a = ap.parse_args()
    for p in [float(x) for x in a.p.split(",")]:
        out = run(p, a.seqs, a.starts, a.span)
        print(f"p={p}")
        for h, e in out.items():
            print("  ", h, e, flush=True)


if __name__ == "__main__":
    main()
