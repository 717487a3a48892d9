"""Would a cheap feature of D_t reject the H2 waves' certain-miss row lookups?

VERDICT r03 "next" item 2: before the key hash and the Bloom-filter read of a lane
whose metric state D_t is not a learned row (98.5% of H2 steps), test a feature of
D_t computable in a few VALU from the packed key against the range the learned rows
span.  A lane-level reject only saves that lane's filter load (the VALU of the hash
is issued for the whole wave while any lane needs it); the VALU is saved only when
EVERY lane of a wave rejects.  This scan measures both on the C oracle's own streams
(CPU only, test infrastructure): per p of the sweep, per feature, the share of
non-row states outside the rows' feature range (lane reject) and the share of
(wave, step) pairs where all 64 lanes of a wave reject (wave skip).

Usage: python profiles/h2_feature_scan.py [--seqs 256] [--N 20000] [--out file.json]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import c_oracle as C  # noqa: E402  (test infrastructure: the checker's model rows and streams)

G1 = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]   # (133,171), delay-ordered taps
G2 = [[[1, 1, 1, 1, 0, 0, 1]], [[1, 0, 1, 1, 0, 1, 1]]]   # (171,133)
M_MEM = 6


def trellis(gen, m):
    """Predecessors and branch outputs of viterbi_markov.py:82-132 for k = 1:
    new state s' = ((s << 1) | u) & (2^m - 1), out_j = parity(gmask_j & ((s << 1) | u))."""
    M = 1 << m
    gm = [sum(int(b) << d for d, b in enumerate(gen[j][0])) for j in range(len(gen))]
    pred = np.zeros((M, 2), np.int64)
    outp = np.zeros((M, 2), np.int64)
    for sp in range(M):
        u = sp & 1
        for i, s in enumerate((sp >> 1, (sp >> 1) | (M >> 1))):
            reg = (s << 1) | u
            o = 0
            for j, g in enumerate(gm):
                o |= (bin(g & reg).count("1") & 1) << j
            pred[sp, i] = s
            outp[sp, i] = o
    return pred, outp


def run_D(pred, outp, words, burn):
    """Eq. 4-5 (viterbi_markov.py:139-159) over sequences in parallel: yields D_t [nseq, M]."""
    nseq, N = words.shape
    M = pred.shape[0]
    pc = np.array([bin(x).count("1") for x in range(8)])
    bm = np.stack([pc[outp ^ y] for y in range(4)])            # [4, M, 2]
    D = np.zeros((nseq, M), np.int64)
    for t in range(N):
        b = bm[words[:, t]]                                      # [nseq, M, 2]
        c0 = D[:, pred[:, 0]] + b[:, :, 0]
        c1 = D[:, pred[:, 1]] + b[:, :, 1]
        Dn = np.minimum(c0, c1)
        D = Dn - Dn.min(axis=1, keepdims=True)
        if t + 1 >= burn:
            yield D


# device key layout (cvd_keys.h key_nibble): state s sits in nibble bitrev3(s & 7) of word
# s >> 3; a v_sad_u8 over the word's bytes weighs the high nibble of each byte by 16
WEIGHT = np.array([16 if ((((s & 7) & 1) << 2) | ((s & 7) & 2) | (((s & 7) >> 2) & 1)) & 1 else 1
                   for s in range(1 << M_MEM)])
SET_FEATURES = ("bin_pop_sad",)


def features(D):
    """Candidate features of D (canonical state order), each cheap on the packed key."""
    nib1 = D + 1                                                  # the lazy key's nibbles (offset 1)
    pop = np.array([bin(x).count("1") for x in range(32)])
    return {
        "max": D.max(axis=1),                                     # OR of (key & 0x8888..) style tests
        "sum": D.sum(axis=1),
        "popsum_off1": pop[nib1].sum(axis=1),                     # sum of v_bcnt over the 8 key words
        "zeros": (D == 0).sum(axis=1),
        "ge4": (D >= 4).sum(axis=1),
        "sum_lo32": D[:, :32].sum(axis=1),
        # joint bin of two 8-VALU features of the lazy key words (sum of v_bcnt, sum of
        # v_sad_u8 bytes): membership in the rows' set of bins, not a range
        "bin_pop_sad": pop[nib1].sum(axis=1) * 4096 + (nib1 * WEIGHT).sum(axis=1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=256)
    ap.add_argument("--N", type=int, default=20000)
    ap.add_argument("--burn", type=int, default=200)
    ap.add_argument("--learn-len", type=int, default=1_000_000)
    ap.add_argument("--p", default="0.01,0.02,0.05,0.1,0.15,0.2")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    c1, c2 = C.Code(G1, M_MEM, 1, 2), C.Code(G2, M_MEM, 1, 2)
    pred, outp = trellis(G1, M_MEM)
    seed, N = 12345, 100_000
    res = {}
    for p in [float(x) for x in a.p.split(",")]:
        mod = C.Model(c1, p, a.learn_len, 200, 1.0, seed)
        _, keys = mod.rows()
        rowset = {k.tobytes() for k in keys.astype(np.uint8)}
        rf = features(keys.astype(np.int64))
        rng = {f: (int(v.min()), int(v.max())) for f, v in rf.items()}
        bins = {f: set(rf[f].tolist()) for f in SET_FEATURES}
        tag = C.lib().oc_grid_tag(N, p)
        out = {"rows": int(keys.shape[0]), "row_feature_range": {f: rng[f] for f in rng if f not in SET_FEATURES},
               "row_bins": {f: len(bins[f]) for f in SET_FEATURES}}
        for hyp, enc in (("H1", c1), ("H2", c2)):
            words = np.stack([C.stream(enc, a.N, p, seed, tag, 2 * q + (hyp == "H2")) for q in range(a.seqs)])
            nwave = a.seqs // 64
            tot = 0
            inrow = 0
            lane_rej = {f: 0 for f in rf}
            nonrow = 0
            wave_skip = {f: 0 for f in rf}
            wave_steps = 0
            for D in run_D(pred, outp, words, a.burn):
                isrow = np.array([d.astype(np.uint8).tobytes() in rowset for d in D])
                ft = features(D)
                tot += D.shape[0]
                inrow += int(isrow.sum())
                nonrow += int((~isrow).sum())
                for f, v in ft.items():
                    if f in SET_FEATURES:
                        rej = ~np.isin(v, list(bins[f]))
                    else:
                        lo, hi = rng[f]
                        rej = (v < lo) | (v > hi)
                    assert not np.any(rej & isrow)
                    lane_rej[f] += int((rej & ~isrow).sum())
                    wave_skip[f] += int(rej[: nwave * 64].reshape(nwave, 64).all(axis=1).sum())
                wave_steps += nwave
            out[hyp] = {"steps": tot, "in_row": inrow / tot,
                        "lane_reject_of_nonrow": {f: lane_rej[f] / max(nonrow, 1) for f in rf},
                        "wave_skip": {f: wave_skip[f] / max(wave_steps, 1) for f in rf}}
        res[str(p)] = out
        print(json.dumps({str(p): out}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
