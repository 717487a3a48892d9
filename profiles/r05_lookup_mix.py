#!/usr/bin/env python3
"""Where the m = 6 detector's row-table requests come from, per lane-step, on the headline
workload's own streams (CPU study; the C oracle's learned rows and streams, TEST/STUDY
infrastructure only).

For H1 and H2 sequences of C2 (N steps each, p from the sweep) it walks the reference
recursion (viterbi_markov.py:139-159) vectorised over sequences and classifies every step
t the way k1s's cursor (csrc/cvd_k1s.h BsCursor) handles D_t:
  * known  -- D_{t-1} is a row, so D_t's status comes from D_{t-1}'s record (no lookup);
  * lookup -- D_{t-1} is not a row: D_t is hashed and its pre-filter bit tested; a set bit
    costs the L2 filter read (all rows, and a share `pf_fp` of non-rows: 1 - exp(-rows /
    2^20) for the 2^20-bit pre-filter), a row (filter positive) the candidate loads (2
    image + 1 record);
  * and every step whose D_t is a row loads D_t's record for the next word (1 request).
Prints the per-lane-step request mix per hypothesis and p.

  python profiles/r05_lookup_mix.py [--N 20000] [--seqs 64] [--p 0.05,0.1,0.2]
"""
import argparse
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import c_oracle as C  # noqa: E402
from oracle import restatement as R  # noqa: E402

G1 = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]
G2 = [[[1, 1, 1, 1, 0, 0, 1]], [[1, 0, 1, 1, 0, 1, 1]]]


def step_tables():
    out_sym, nxt = R.encoder_tables(G1, 6, 1, 2)
    M = 64
    preds = [[] for _ in range(M)]
    for s in range(M):
        for u in range(2):
            preds[nxt[s, u]].append((s, u))
    pa = np.array([preds[t][0][0] for t in range(M)])
    ua = np.array([preds[t][0][1] for t in range(M)])
    pb = np.array([preds[t][1][0] for t in range(M)])
    ub = np.array([preds[t][1][1] for t in range(M)])
    pc = np.array([bin(v).count("1") for v in range(4)])
    bma = np.array([[pc[out_sym[pa[t], ua[t]] ^ r] for t in range(M)] for r in range(4)])
    bmb = np.array([[pc[out_sym[pb[t], ub[t]] ^ r] for t in range(M)] for r in range(4)])
    return pa, pb, bma, bmb


def run(p, N, seqs, seed=12345):
    dec = C.Code(G1, 6, 1, 2)
    enc2 = C.Code(G2, 6, 1, 2)
    model = C.Model(dec, p, 1_000_000, 200, 1.0, seed)
    _, keys = model.rows()
    rows = {bytes(k) for k in keys}
    pf_fp = 1.0 - math.exp(-len(rows) / float(1 << 20))
    tag = C.lib().oc_grid_tag(N, p)
    pa, pb, bma, bmb = step_tables()
    out = {}
    for h, enc in (("H1", dec), ("H2", enc2)):
        r = np.stack([C.stream(enc, N, p, seed, tag, 2 * q + (h == "H2")) for q in range(seqs)])
        D = np.zeros((seqs, 64), np.int16)
        prev_row = np.ones(seqs, bool)          # D_0 = 0 is a row
        cnt = dict(known=0, lookup=0, filt=0.0, cand=0, rec=0, steps=0)
        for t in range(N):
            rt = r[:, t]
            a = D[:, pa] + bma[rt]
            b = D[:, pb] + bmb[rt]
            Dn = np.minimum(a, b)
            Dn -= Dn.min(axis=1, keepdims=True)
            isrow = np.fromiter((bytes(x) in rows for x in Dn.astype(np.uint8)), bool, seqs)
            known = prev_row
            look = ~known
            cnt["known"] += int(known.sum())
            cnt["lookup"] += int(look.sum())
            cnt["filt"] += float((look & isrow).sum()) + pf_fp * float((look & ~isrow).sum())
            cnt["cand"] += int((look & isrow).sum())
            cnt["rec"] += int(isrow.sum())
            cnt["steps"] += seqs
            D, prev_row = Dn, isrow
        s = cnt["steps"]
        out[h] = {"rows_share": cnt["rec"] / s, "known": cnt["known"] / s, "lookup": cnt["lookup"] / s,
                  "l2_filter_reads": cnt["filt"] / s, "cand_steps": cnt["cand"] / s,
                  "record_loads": cnt["rec"] / s,
                  "requests_per_lane_step": (cnt["filt"] + 3 * cnt["cand"] + cnt["rec"]) / s}
    return len(rows), pf_fp, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=20000)
    ap.add_argument("--seqs", type=int, default=64)
    ap.add_argument("--p", default="0.02,0.05,0.1,0.2")
    a = ap.parse_args()
    for p in [float(x) for x in a.p.split(",")]:
        nrows, fp, out = run(p, a.N, a.seqs)
        print(f"p={p} rows={nrows} pf_fp={fp:.3f}")
        for h, e in out.items():
            print("  ", h, {k: round(v, 4) for k, v in e.items()}, flush=True)


if __name__ == "__main__":
    main()
