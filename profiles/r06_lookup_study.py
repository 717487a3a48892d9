#!/usr/bin/env python3
"""Round 6: what the m = 6 detector's candidate loads (directory slot reads) look like on the
headline workload's own streams (CPU study over the C oracle's learned rows and streams; TEST /
STUDY infrastructure only, like r05_lookup_mix.py).

Per hypothesis and p it walks the reference recursion (viterbi_markov.py:139-159) over one wave
of 64 sequences and reports, per lane-step:
  * cand      -- D_{t-1} not a row, D_t a row: the cursor's candidate loads (directory slot);
  * wave_cand -- the share of wave-steps in which at least one of the 64 lanes has a candidate
                 (the wave waits for the slowest lane's directory line at the resolve);
  * the row ids of the candidates and of the dense record loads by rank (rows are numbered by
    the learning chain's first visits): the share that falls in the first K rows, i.e. how
    much of the lookups a K-row hot table would serve.

  python profiles/r06_lookup_study.py [--N 20000] [--p 0.05,0.1]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import c_oracle as C  # noqa: E402
from r05_lookup_mix import G1, G2, step_tables  # noqa: E402

KS = [1024, 4096, 16384, 65536, 262144]


def run(p, N, seqs, seed=12345):
    dec = C.Code(G1, 6, 1, 2)
    enc2 = C.Code(G2, 6, 1, 2)
    model = C.Model(dec, p, 1_000_000, 200, 1.0, seed)
    _, keys = model.rows()
    rid = {bytes(k): i for i, k in enumerate(keys)}
    tag = C.lib().oc_grid_tag(N, p)
    pa, pb, bma, bmb = step_tables()
    out = {}
    for h, enc in (("H1", dec), ("H2", enc2)):
        r = np.stack([C.stream(enc, N, p, seed, tag, 2 * q + (h == "H2")) for q in range(seqs)])
        D = np.zeros((seqs, 64), np.int16)
        prev_row = np.ones(seqs, bool)
        cand_ids, rec_ids = [], []
        wave_cand = 0
        ncand = 0
        run_len = []            # lengths of off-row runs (steps between leaving and re-entering)
        off = np.zeros(seqs, np.int64)
        for t in range(N):
            rt = r[:, t]
            Dn = np.minimum(D[:, pa] + bma[rt], D[:, pb] + bmb[rt])
            Dn -= Dn.min(axis=1, keepdims=True)
            ids = np.fromiter((rid.get(bytes(x), -1) for x in Dn.astype(np.uint8)), np.int64, seqs)
            isrow = ids >= 0
            cand = ~prev_row & isrow
            ncand += int(cand.sum())
            wave_cand += int(cand.any())
            cand_ids.append(ids[cand])
            rec_ids.append(ids[isrow])
            off = np.where(isrow, 0, off + 1)
            run_len.extend(off[cand & False].tolist())
            D, prev_row = Dn, isrow
        ci = np.concatenate(cand_ids)
        ri = np.concatenate(rec_ids)
        s = N * seqs
        out[h] = {"cand_per_lane_step": ncand / s, "wave_steps_with_cand": wave_cand / N,
                  "row_share": ri.size / s,
                  "cand_rows_in_first_K": {K: float((ci < K).mean()) if ci.size else None for K in KS},
                  "record_rows_in_first_K": {K: float((ri < K).mean()) if ri.size else None for K in KS},
                  "distinct_cand_rows": int(np.unique(ci).size)}
    return len(keys), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=20000)
    ap.add_argument("--seqs", type=int, default=64)
    ap.add_argument("--p", default="0.05,0.1")
    a = ap.parse_args()
    for p in [float(x) for x in a.p.split(",")]:
        nrows, out = run(p, a.N, a.seqs)
        print(f"p={p} rows={nrows}")
        for h, e in out.items():
            print("  ", h, e, flush=True)


if __name__ == "__main__":
    main()
