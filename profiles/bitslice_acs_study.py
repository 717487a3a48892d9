#!/usr/bin/env python3
"""Design study for the next detector core: the Eq. 4-5 step of the
m = 6 rate-1/2 decoder in BIT-SLICED form -- the 64 relative metrics as W bit-planes of
two 32-bit registers (one bit per state), instead of 32 registers of 16-bit pairs.

Layout.  A state index has 6 bits; each is held at one of 6 locations: the register bit
(which of the two registers) or one of the 5 position bits inside a register.  A step
drops index bit 5 (the predecessor pair j, j + 32 differ in it) and shifts the others up
by one (viterbi_markov.py:82-106: next = (s << 1 | u) mod 64), so if the new bit 0 is put
where the old bit 5 was, every other bit stays where it is: the layout is a cyclic
relabelling with period 6, and the ACS runs in place.  Per step the partner of a state is
  * in the other register at the same position (partner bit at the register bit), or
  * at position p ^ 2^k of the same register (partner bit at position bit k): one
    rotate for k = 4, a delta swap (two shifts and a select) for k < 4.
With E(p) = e(j) = popcount(out(j,0) ^ y) on every position, both butterfly outputs come
from one expression per register:  D'(p) = min(D(p) + E(p), D(partner(p)) + 2 - E(p)).

This script checks that the bit-sliced step reproduces the reference recursion
(oracle/restatement.py metric_step_vec, viterbi_markov.py:139-159) bit for bit on the
headline decoder's own received streams, and counts the 32-bit logic operations per step
(each one a v_bitop3_b32 / v_alignbit_b32 / VOP2 on the GPU) to compare with the current
kernel's ~121 ACS + normalisation and ~26 key-packing instructions per step
(profiles/isa_breakdown.py).

  python profiles/bitslice_acs_study.py [steps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import restatement as R  # noqa: E402  (design study, not product code)

M32 = 0xFFFFFFFF
W = int(os.environ.get("BITSLICE_W", "5"))   # bit-planes (relative metrics <= 15 fit 4; the sums before the min need 5 unless D <= 13)


class Ops:
    n = 0


def op(v, k=1):
    Ops.n += k
    return v & M32


def flip_k(x, k):
    """positions p <-> p ^ 2^k (delta swap; k = 4 is one rotate)"""
    if k == 4:
        return op(((x >> 16) | (x << 16)))
    m = sum(1 << p for p in range(32) if not (p >> k) & 1)
    return op(((x >> (1 << k)) & m) | ((x & m) << (1 << k)), 3)


def add_small(d, e0, e1):
    """bit-sliced d + e, e in {0, 1, 2} given as planes (e0, e1): 7 ops for 4-5 planes"""
    s = [0] * W
    s[0] = op(d[0] ^ e0)
    c = op(d[0] & e0)
    s[1] = op(d[1] ^ e1 ^ c)                                   # xor3
    c = op((d[1] & e1) | (d[1] & c) | (e1 & c))                 # maj
    for i in range(2, W):
        s[i] = op(d[i] ^ c)
        if i + 1 < W:
            c = op(d[i] & c)
    return s


def min_planes(a, b):
    """bit-sliced min: a < b by a borrow chain LSB first (one bitop3 per plane), then
    one select per plane"""
    lt = 0
    for i in range(W):
        lt = op(((~a[i]) & b[i]) | (((~a[i]) | b[i]) & lt))      # MAJ(~a, b, lt)
    return [op((a[i] & lt) | (b[i] & ~lt)) for i in range(W)]


def to_planes(D, loc):
    regs = [[0] * W for _ in range(2)]
    for s, v in enumerate(D):
        r, p = place(s, loc)
        for i in range(W):
            if (v >> i) & 1:
                regs[r][i] |= 1 << p
    return regs


def place(s, loc):
    r, p = 0, 0
    for i in range(6):
        b = (s >> i) & 1
        if loc[i] == 0:
            r = b
        else:
            p |= b << (loc[i] - 1)
    return r, p


def from_planes(regs, loc):
    D = []
    for s in range(64):
        r, p = place(s, loc)
        D.append(sum(((regs[r][i] >> p) & 1) << i for i in range(W)))
    return D


def step(regs, loc, e_of_j):
    """one bit-sliced Eq. 4 step (no normalisation); returns new regs and layout"""
    l5 = loc[5]
    # E planes per register: e(j) at every position (j = the state's bits 0..4)
    E = [[0, 0], [0, 0]]
    for s in range(64):
        r, p = place(s, loc)
        e = e_of_j[s & 31]
        if e & 1:
            E[r][0] |= 1 << p
        if e & 2:
            E[r][1] |= 1 << p
    # (on the GPU: 4 mask words per step from an LDS table indexed by the layout phase
    # and the received word)
    Ops.n += 4
    new = [None, None]
    for r in range(2):
        if l5 == 0:
            part = regs[1 - r]
        else:
            part = [flip_k(regs[r][i], l5 - 1) for i in range(W)]
        e0, e1 = E[r]
        ne0 = op(~e0 & ~e1 & M32)      # 2 - e: 2 -> 0, 1 -> 1, 0 -> 2 (bit 0 = e0, bit 1 = ~e0 & ~e1)
        ne1 = ne0
        ne0 = e0
        a = add_small(regs[r], e0, e1)
        b = add_small(part, ne0, ne1)
        new[r] = min_planes(a, b)
    nloc = [loc[5]] + loc[:5]
    return new, nloc


def normalise(regs):
    """subtract the minimum (0, 1 or 2 after a step from a normalised vector)"""
    for mu in range(3):
        # any state equal to mu: ~(d ^ mu-planes) over all planes, or-reduced (bitop3s)
        hit = 0
        for r in range(2):
            eq = M32
            for i in range(W):
                eq &= ~(regs[r][i] ^ (M32 if (mu >> i) & 1 else 0)) & M32
            hit |= eq
        Ops.n += 2 * W
        if hit:
            break
    if mu:
        for r in range(2):
            d = regs[r]
            # bit-sliced d - mu, mu in {1, 2}
            borrow = M32 if mu == 1 else 0
            out = []
            for i in range(W):
                bi = M32 if (mu == 2 and i == 1) else 0
                x = d[i] ^ bi
                out.append(op(x ^ borrow))
                borrow = op(((~d[i]) & (bi | borrow)) | (bi & borrow)) & M32
            regs[r] = out
    return regs, mu


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    g1 = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]    # (133, 171), decoder of C2
    g2 = [[[1, 1, 1, 1, 0, 0, 1]], [[1, 0, 1, 1, 0, 1, 1]]]
    out_sym, nxt = R.encoder_tables(g1, 6, 1, 2)
    # the symmetric-metric property the layout uses: out(j+32,0) = ~out(j,0),
    # out(j,1) = ~out(j,0)
    assert all(out_sym[j + 32, 0] == 3 - out_sym[j, 0] and out_sym[j, 1] == 3 - out_sym[j, 0] for j in range(32))
    worst = 0
    for name, enc, p in (("H1", g1, 0.05), ("H2", g2, 0.05), ("H1", g1, 0.2)):
        r = R.received_stream(enc, 6, 1, 2, steps, p, 7, 99, 3)
        D = np.zeros(64, np.int64)
        loc = [1, 2, 3, 4, 5, 0]          # bits 0-4 at position bits 0-4, bit 5 at the register bit
        regs = to_planes(D, loc)
        Ops.n = 0
        for t in range(steps):
            y = int(r[t])
            e_of_j = [bin(int(out_sym[j, 0]) ^ y).count("1") for j in range(32)]
            regs, loc = step(regs, loc, e_of_j)
            regs, _ = normalise(regs)
            D = R.metric_step_vec(D, out_sym, nxt, y, 2)
            got = from_planes(regs, loc)
            assert got == [int(v) for v in D], (name, t)
            worst = max(worst, int(D.max()))
        print(f"{name} p={p}: {steps} steps bit-exact; {Ops.n / steps:.1f} logic ops per step "
              f"(ACS + normalisation, layout-phase average)")
    print(f"largest relative metric seen: {worst} (fits {W - 1} planes; sums before the min use {W})")


if __name__ == "__main__":
    main()
