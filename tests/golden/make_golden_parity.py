#!/usr/bin/env python3
"""Golden fixtures for the parity-template baseline (tests/golden/parity.npz +
parity.json), computed by the REFERENCE's own, unmodified functions:

  parity_eqn_check.parse_poly_token / build_parity_system / nullspace_mod2 /
  parity_vector_to_equation                         (parity_eqn_check.py:60-201)
  comp_parity.encode_convolutional / parity_satisfaction_fraction /
  parity_detector                                   (comp_parity.py:65-128)

Runs only in the build container, where /root/reference is importable
(SURVEY.md §8(c)); only inputs/outputs are committed.

Usage:  python tests/golden/make_golden_parity.py   (a few seconds)
"""
import json
import os
import random
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

import parity_eqn_check as pe  # noqa: E402  (reference)
import comp_parity as cp  # noqa: E402  (reference)

# generator tokens per code (octal, as the reference's parse_poly_token takes them)
# plus delay-ordered tap lists for codes given as taps (k = 2)
CODES = {
    "m2_75": {"tokens": [["7"], ["5"]]},                  # comp_parity.py:140-141
    "m2_57": {"tokens": [["5"], ["7"]]},
    "m3_demo": {"tokens": [["17"], ["13"]]},             # demo_script.py:45-50 (1111, 1011)
    "m6_133_171": {"tokens": [["1,0,1,1,0,1,1"], ["1,1,1,1,0,0,1"]]},
    "m6_171_133": {"tokens": [["1,1,1,1,0,0,1"], ["1,0,1,1,0,1,1"]]},
    "r23_m4": {"gens": [[[1, 0, 0, 0, 1], [0, 1, 1, 1, 1]],
                        [[1, 1, 1, 0, 1], [0, 1, 0, 1, 0]],
                        [[0, 1, 1, 0, 0], [1, 1, 0, 1, 0]]]},
}


def gens_of(spec):
    if "gens" in spec:
        return spec["gens"]
    return [[pe.parse_poly_token(t) for t in out] for out in spec["tokens"]]


def template_of(h_vec):
    """comp_parity.py:160-165: (output j, delay s) for every set coefficient."""
    return [(j, s) for j, poly in enumerate(h_vec) for s, bit in enumerate(poly) if bit]


def main():
    meta = {"generated_by": "tests/golden/make_golden_parity.py", "codes": {}, "tokens": {}}
    arrays = {}
    # parse_poly_token on every accepted format (parity_eqn_check.py:60-86)
    for tok in ["7", "5", "13", "17", "133", "171", "111", "1011", "1,0,1", "0,1,1,0"]:
        meta["tokens"][tok] = pe.parse_poly_token(tok)
    for name, spec in CODES.items():
        gens = gens_of(spec)
        n, k = len(gens), len(gens[0])
        m = max(len(g) - 1 for out in gens for g in out)
        entry = {"gens": gens, "n": n, "k": k, "m": m, "deg_h": {}}
        for deg_h in sorted({m, m + 1, m + 3}):
            A = pe.build_parity_system(gens, deg_h)
            basis = pe.nullspace_mod2(A)
            arrays[f"{name}/d{deg_h}/A"] = A
            arrays[f"{name}/d{deg_h}/basis"] = basis
            eqs, tpls = [], []
            for row in basis[:4]:
                h = [row[j * (deg_h + 1):(j + 1) * (deg_h + 1)].tolist() for j in range(n)]
                eqs.append(pe.parity_vector_to_equation(h))
                tpls.append(template_of(h))
            entry["deg_h"][str(deg_h)] = {"equations": eqs, "templates": tpls, "n_basis": int(len(basis))}
        meta["codes"][name] = entry

        # satisfaction fractions on fixed streams (k = 1 codes: the reference's
        # encoder reads generators[j][0] only, comp_parity.py:65-84)
        if k == 1:
            rng = random.Random(1000 + len(name))
            deg_h = m + 3
            tpl = entry["deg_h"][str(deg_h)]["templates"][0]
            cases = []
            for (N, p) in [(50, 0.0), (200, 0.05), (333, 0.2), (7, 0.1), (deg_h, 0.1)]:
                u = [rng.randint(0, 1) for _ in range(N)]
                v = cp.encode_convolutional(u, gens, m)
                y = [[bit ^ (rng.random() < p) for bit in stream] for stream in v]
                frac = cp.parity_satisfaction_fraction(y, tpl)
                dec, ph = cp.parity_detector(y, tpl, 0.6)
                cases.append({"N": N, "p": p, "frac": frac, "decision_0.6": bool(dec), "P_hat": ph})
                arrays[f"{name}/frac{len(cases) - 1}/y"] = np.array(y, np.uint8)
            entry["fractions"] = cases
            # encoder output (with the m-step tail) for one input
            u = [rng.randint(0, 1) for _ in range(40)]
            arrays[f"{name}/enc_u"] = np.array(u, np.uint8)
            arrays[f"{name}/enc_v"] = np.array(cp.encode_convolutional(u, gens, m), np.uint8)
    np.savez_compressed(os.path.join(HERE, "parity.npz"), **arrays)
    with open(os.path.join(HERE, "parity.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote parity.npz / parity.json:", len(arrays), "arrays")


if __name__ == "__main__":
    main()
