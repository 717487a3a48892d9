#!/usr/bin/env python3
"""Runs profiles/bitslice_acs_bench.hip (design study of DESIGN.md §11) on the GPU: checks
lanes against the reference recursion (oracle/restatement.py metric_step_vec) and times
the bit-sliced m = 6 step alone.  Build (CPU, in-tree):
  hipcc -O3 --offload-arch=gfx950 -fPIC -shared profiles/bitslice_acs_bench.hip -o profiles/libbitslice_acs.so
  python profiles/bitslice_acs_run.py [steps_per_lane/6] [lanes]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from oracle import restatement as R  # noqa: E402  (design study)

LOC0 = [1, 2, 3, 4, 5, 0]   # index bit i -> location (0 = register bit, 1 + k = position bit k)


def place(s, loc):
    r, p = 0, 0
    for i in range(6):
        b = (s >> i) & 1
        if loc[i] == 0:
            r = b
        else:
            p |= b << (loc[i] - 1)
    return r, p


def masks(out_sym):
    o = np.zeros(24, np.uint32)
    loc = list(LOC0)
    for ph in range(6):
        for s in range(64):
            r, p = place(s, loc)
            oj = int(out_sym[s & 31, 0])
            if oj & 1:
                o[ph * 2 + r] |= np.uint32(1 << p)
            if oj & 2:
                o[12 + ph * 2 + r] |= np.uint32(1 << p)
        loc = [loc[5]] + loc[:5]
    return o


def xs(s):
    s ^= (s << 13) & 0xFFFFFFFF
    s ^= s >> 17
    s ^= (s << 5) & 0xFFFFFFFF
    return s


def reference_lane(q, seed, nsix, out_sym, nxt):
    s = (seed ^ ((q * 0x9E3779B9) & 0xFFFFFFFF)) & 0xFFFFFFFF or 1
    D = np.zeros(64, np.int64)
    mus = 0
    for _ in range(nsix):
        s = xs(s)
        for k in range(6):
            y = (s >> (2 * k)) & 3
            bm = np.array([bin(int(o) ^ y).count("1") for o in out_sym.reshape(-1)]).reshape(out_sym.shape)
            cand = D[:, None] + bm
            Dn = np.full(64, 1 << 40, np.int64)
            np.minimum.at(Dn, nxt.reshape(-1), cand.reshape(-1))
            mus += int(Dn.min())
            D = Dn - Dn.min()
    return D, mus


def main():
    nsix = int(sys.argv[1]) if len(sys.argv) > 1 else 16_667          # ~10^5 steps
    lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 262_144
    lib = ctypes.CDLL(os.path.join(ROOT, "profiles", "libbitslice_acs.so"))
    g1 = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]
    out_sym, nxt = R.encoder_tables(g1, 6, 1, 2)
    mk = masks(out_sym)
    res = {}
    for variant, vname in ((0, "compiler"), (1, "bitop3_asm"), (2, "mu_first")):
        for tag, ns, nl in (("check", 50, 256), ("warm", nsix, lanes), ("time", nsix, lanes)):
            out = torch.zeros(nl * 9, dtype=torch.int32, device="cuda")
            ms = ctypes.c_float(0.0)
            rc = lib.bitslice_run(mk.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(ns), ctypes.c_uint32(12345),
                                  ctypes.c_void_p(out.data_ptr()), ctypes.c_int64(nl), ctypes.byref(ms),
                                  ctypes.c_int(variant))
            assert rc == 0, rc
            if tag == "check":
                o = out.cpu().numpy().view(np.uint32).reshape(nl, 9)
                for q in (0, 1, 77, 255):
                    D, mus = reference_lane(q, 12345, ns, out_sym, nxt)
                    got = [0] * 64
                    for s in range(64):
                        r, p = place(s, LOC0)
                        got[s] = sum(((int(o[q, r * 4 + i]) >> p) & 1) << i for i in range(4))
                    assert got == [int(v) for v in D] and int(o[q, 8]) == mus, (vname, q)
                print(vname, ": lanes 0, 1, 77, 255 equal the reference recursion after", ns * 6, "steps", flush=True)
            elif tag == "time":
                steps = nl * ns * 6
                res[vname] = {"lanes": nl, "steps_per_lane": ns * 6, "ms": ms.value,
                              "lane_steps_per_s": steps / (ms.value / 1e3),
                              "cycles_per_wave_step_per_simd": ms.value * 1e-3 * 2.4e9 / (steps / 64 / 1024)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
