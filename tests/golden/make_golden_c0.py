#!/usr/bin/env python3
"""Golden fixtures for BASELINE configuration C0 at its OWN size, from the reference itself
(tests/golden/golden_c0.{json,npz}).

C0 is the demo preset: rate-1/2 m = 2 at N = 1e3 with 1e3 trials.  The reference's own
run_experiment (Pd_plotter.py:176-235) runs unmodified, with the demo's p grid and seed
(demo_script.py:113-131: p_vec = [0.01, 0.05, 0.1, 0.2, 0.3], learn_len None, learn_burn
200, laplace 1, seed 123); the only change is N_SPECTRUM_BY_M (Pd_plotter.py:78), patched
to {2: [1000]} so that the m = 2 presets run at C0's N.  Cases: (7,5) vs (5,7) (BASELINE
C0's pair), the demo's preset 1 (7,5) vs (6,5) (demo_script.py:35-42), and preset 2, m = 3
(15,13) vs (13,15) (demo_script.py:43-50), at its default N = 500 with 500 trials.  The
missing simulator is the shim of make_golden.py (build's Philox streams, reference encoder
and Eq. 4-5).  Per trial the four log-likelihood sums are recorded in the reference's call
order, with the DataFrame.

Usage:  python tests/golden/make_golden_c0.py   (pure-Python reference: ≈ 10 minutes)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402  (imports the reference from /root/reference)

pdp, vm = mg.pdp, mg.vm

P_DEMO = [0.01, 0.05, 0.1, 0.2, 0.3]
CASES = [
    # name, g1, g2, num_iter, p_vec, seed, N_SPECTRUM_BY_M patch
    ("c0_m2_75_57", "m2_75", "m2_57", 1000, P_DEMO, 123, {2: [1000]}),
    ("c0_m2_75_65", "m2_75", "m2_65", 1000, P_DEMO, 123, {2: [1000]}),
    ("c0_m3_demo", "m3_demo", "m3_demo2", 500, P_DEMO, 123, None),
]


def main():
    t0 = time.time()
    meta = {"generated_by": "tests/golden/make_golden_c0.py", "reference": "/root/reference",
            "codes": {n: {"k": c[0], "n": c[1], "m": c[2], "taps": c[3]} for n, c in mg.CODES.items()}}
    arrays = {}
    orig_lps = pdp.log_prob_sequence
    orig_spec = dict(pdp.N_SPECTRUM_BY_M)
    for ename, g1, g2, iters, pv, seed, spec in CASES:
        k, n, m, taps1 = mg.CODES[g1]
        taps2 = mg.CODES[g2][3]
        pdp.N_SPECTRUM_BY_M.clear()
        pdp.N_SPECTRUM_BY_M.update(orig_spec)
        if spec:
            pdp.N_SPECTRUM_BY_M.update(spec)
        rec = []

        def recording(metrics, state_index, T, _rec=rec):
            v = orig_lps(metrics, state_index, T)
            _rec.append(v)
            return v
        pdp.log_prob_sequence = recording
        vm.simulate_markov_sequence = mg.make_shim(taps1, seed)
        pdp.learn_P1_empirical.cache_clear()
        df = pdp.run_experiment(k, n, m, taps1, taps2, iters, pv, None, 200, 1.0, seed)
        pdp.log_prob_sequence = orig_lps
        meta[ename] = {"g1": g1, "g2": g2, "num_iter": iters, "p_vec": pv, "seed": seed,
                       "N_list": list(pdp.N_SPECTRUM_BY_M[m]), "learn_burn": 200, "laplace": 1.0,
                       "rows": df.to_dict(orient="records")}
        arrays[f"{ename}/sums"] = np.array(rec, np.float64).reshape(-1, 4)
        print("run_experiment", ename, df.to_dict(orient="records"), round(time.time() - t0, 1), flush=True)
    pdp.N_SPECTRUM_BY_M.clear()
    pdp.N_SPECTRUM_BY_M.update(orig_spec)
    np.savez_compressed(os.path.join(HERE, "golden_c0.npz"), **arrays)
    with open(os.path.join(HERE, "golden_c0.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("done", round(time.time() - t0, 1))


if __name__ == "__main__":
    main()
