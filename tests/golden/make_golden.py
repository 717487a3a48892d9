#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs only in the build container, where /root/reference is importable
(SURVEY.md §8(c)).  The reference never travels: only the inputs/outputs below
are committed.  Everything is computed by the reference's own, unmodified
functions:

  viterbi_markov.branch_output_and_next_state / build_trellis      (vm:82-132)
  viterbi_markov.viterbi_metric_step                                (vm:139-159)
  viterbi_markov.enumerate_markov_states_allzero                    (vm:166-195)
  viterbi_markov.build_symbolic_T + Pd_plotter.evaluate_symbolic_T  (vm:202-230, Pd:89-99)
  Pd_plotter.log_prob_sequence / learn_P1_empirical / run_experiment (Pd:106-235)

The reference's missing `viterbi_markov.simulate_markov_sequence`
is injected as a shim that draws encoder inputs and BSC flips from the build's
Philox stream (oracle/philox.py) and otherwise uses ONLY reference functions
(branch_output_and_next_state for the encoder, build_trellis +
viterbi_metric_step for the metrics, decoder = G1 per Pd_plotter.py:188).

Usage:  python tests/golden/make_golden.py   (≈ 2-3 minutes)
"""
import json
import os
import sys
import time

os.environ.setdefault("MPLBACKEND", "Agg")
sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

import viterbi_markov as vm  # noqa: E402  (reference)
import Pd_plotter as pdp  # noqa: E402  (reference)
from oracle import philox  # noqa: E402

CODES = {
    # name: (k, n, m, taps)   taps[j][i] delay-ordered (reference convention)
    "m2_75": (1, 2, 2, [[[1, 1, 1]], [[1, 0, 1]]]),            # Pd_plotter.py:247 / demo preset 1
    "m2_57": (1, 2, 2, [[[1, 0, 1]], [[1, 1, 1]]]),            # BASELINE config 0 G2
    "m2_65": (1, 2, 2, [[[1, 1, 0]], [[1, 0, 1]]]),            # Pd_plotter.py:248 / demo preset 1 G2
    "m3_demo": (1, 2, 3, [[[1, 1, 1, 1]], [[1, 0, 1, 1]]]),    # demo_script.py:45-50
    "m3_demo2": (1, 2, 3, [[[1, 0, 1, 1]], [[1, 1, 1, 1]]]),
    "r23_m4": (2, 3, 4, [[[1, 0, 0, 0, 1], [0, 1, 1, 1, 1]],   # SURVEY §8 rate-2/3 example
                         [[1, 1, 1, 0, 1], [0, 1, 0, 1, 0]],
                         [[0, 1, 1, 0, 0], [1, 1, 0, 1, 0]]]),
    "r23_m4_b": (2, 3, 4, [[[1, 1, 1, 0, 1], [0, 1, 0, 1, 0]],  # rows permuted (G2)
                           [[0, 1, 1, 0, 0], [1, 1, 0, 1, 0]],
                           [[1, 0, 0, 0, 1], [0, 1, 1, 1, 1]]]),
    "m6_133_171": (1, 2, 6, [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]),
    "m6_171_133": (1, 2, 6, [[[1, 1, 1, 1, 0, 0, 1]], [[1, 0, 1, 1, 0, 1, 1]]]),
}


def enc_tables(taps, k, n, m):
    S, K = 1 << m, 1 << k
    out = np.zeros((S, K), np.int64)
    nxt = np.zeros((S, K), np.int64)
    for s in range(S):
        for U in range(K):
            u = tuple((U >> i) & 1 for i in range(k))
            o, ns = vm.branch_output_and_next_state(s, u, taps, m, k)
            out[s, U] = sum(b << j for j, b in enumerate(o))
            nxt[s, U] = ns
    return out, nxt


def trellis_arrays(taps, k, m):
    """build_trellis as arrays: for each next state, its incoming (ps, U, out) in list order."""
    tr = vm.build_trellis(taps, m, k)
    rows = []
    for ns in range(1 << m):
        for (ps, u, out) in tr[ns]:
            rows.append([ns, ps, sum(b << i for i, b in enumerate(u)),
                         sum(b << j for j, b in enumerate(out))])
    return np.array(rows, np.int64)


def make_shim(gen1, trial_seed):
    """Inject the missing simulator; counts calls per (N, p) to recover
    (trial, hypothesis) from the reference's call order (Pd_plotter.py:210-223)."""
    counters = {}
    trellis1 = vm.build_trellis(gen1, len(gen1[0][0]) - 1, len(gen1[0]))

    def shim(generator_matrix, m, k, n, N, p_val, random_input=True, seed=None):
        if seed is not None:            # learning call, Pd_plotter.py:149-155
            sd, tag, sid = int(seed), philox.LEARN_TAG, 0
        else:                           # trial calls, Pd_plotter.py:212/219
            key = (N, float(p_val))
            c = counters.get(key, 0)
            counters[key] = c + 1
            sd, tag, sid = trial_seed, philox.grid_tag(N, p_val), c
            if c % 2 == 0:
                assert generator_matrix == gen1
        if random_input:
            ub = philox.input_bits(sd, tag, sid, N, k)
        else:
            ub = np.zeros((N, k), np.uint8)
        nb = philox.noise_bits(sd, tag, sid, N, n, p_val)
        s = 0
        D = tuple([0] * (1 << m))
        metrics = [D]
        for t in range(N):
            out, s = vm.branch_output_and_next_state(s, tuple(int(b) for b in ub[t]),
                                                     generator_matrix, m, k)
            r = tuple(int(o) ^ int(e) for o, e in zip(out, nb[t]))
            D = vm.viterbi_metric_step(list(D), trellis1, r)
            metrics.append(D)
        return {"metrics": metrics}
    return shim


def main():
    t0 = time.time()
    meta = {"codes": {}, "generated_by": "tests/golden/make_golden.py", "reference": "/root/reference"}
    arrays = {}

    # 1. encoder / trellis tables (A1, A3)
    for name, (k, n, m, taps) in CODES.items():
        meta["codes"][name] = {"k": k, "n": n, "m": m, "taps": taps}
        out, nxt = enc_tables(taps, k, n, m)
        arrays[f"{name}/out_sym"] = out
        arrays[f"{name}/next_state"] = nxt
        arrays[f"{name}/trellis"] = trellis_arrays(taps, k, m)
    print("tables", time.time() - t0, flush=True)

    # 2. BFS state enumeration (A6)
    bfs = {}
    for name in ["m2_75", "m2_57", "m2_65", "m3_demo", "r23_m4"]:
        k, n, m, taps = CODES[name]
        states, transitions, all_r = vm.enumerate_markov_states_allzero(taps, m, k, n)
        bfs[name] = (states, transitions, all_r)
        arrays[f"{name}/states"] = np.array(states, np.uint8)
        trip = []
        for i in range(len(states)):
            for j, rl in transitions[i].items():
                for r in rl:
                    trip.append([i, j, sum(b << q for q, b in enumerate(r))])
        arrays[f"{name}/transitions"] = np.array(trip, np.int64)
        meta["codes"][name]["S"] = len(states)
        print("bfs", name, len(states), time.time() - t0, flush=True)

    # 3. T(p) from the reference's sympy path (A7)
    for name, plist in [("m2_75", [0.5, 0.1, 0.3]), ("m2_65", [0.5]), ("m3_demo", [0.5])]:
        states, transitions, all_r = bfs[name]
        p_sym, T_sym = vm.build_symbolic_T(states, transitions, all_r)
        for p in plist:
            arrays[f"{name}/T_{p}"] = pdp.evaluate_symbolic_T(T_sym, p_sym, p)
        print("sympy T", name, time.time() - t0, flush=True)

    # 4. D sequences for fixed received streams (A4)
    rng = np.random.default_rng(20261015)
    for name, N in [("m2_75", 2000), ("m3_demo", 2000), ("r23_m4", 1500), ("m6_133_171", 1200)]:
        k, n, m, taps = CODES[name]
        trellis = vm.build_trellis(taps, m, k)
        r = rng.integers(0, 1 << n, size=N)
        D = tuple([0] * (1 << m))
        Ds = [D]
        for rv in r:
            D = vm.viterbi_metric_step(list(D), trellis, tuple((int(rv) >> j) & 1 for j in range(n)))
            Ds.append(D)
        arrays[f"{name}/trace_r"] = r.astype(np.int64)
        arrays[f"{name}/trace_D"] = np.array(Ds, np.uint8)
        print("trace", name, time.time() - t0, flush=True)

    # 5+6. learned P̂1 through the injected simulator (A8), log-likelihoods (A9)
    learn_cases = [("m2_75", p, 123) for p in [0.01, 0.05, 0.1, 0.2, 0.3]]
    learn_cases += [("m2_75", 0.05, 12345), ("m3_demo", 0.05, 123), ("r23_m4", 0.05, 123)]
    for name, p, seed in learn_cases:
        k, n, m, taps = CODES[name]
        vm.simulate_markov_sequence = make_shim(taps, 0)
        pdp.learn_P1_empirical.cache_clear()
        states_L, sidx, P = pdp.learn_P1_empirical(
            tuple(tuple(tuple(x) for x in row) for row in taps), k, n, m, p, None, 200, 1.0, seed)
        if name == "r23_m4":
            # store only the (sparse) count-derived rows actually visited to keep the fixture small
            nz = np.argwhere(P > P.min(axis=1, keepdims=True))
            arrays[f"{name}/P1_{p}_{seed}_rowmin"] = P.min(axis=1)
            arrays[f"{name}/P1_{p}_{seed}_nz_idx"] = nz.astype(np.int64)
            arrays[f"{name}/P1_{p}_{seed}_nz_val"] = P[nz[:, 0], nz[:, 1]]
        else:
            arrays[f"{name}/P1_{p}_{seed}"] = P
        print("learn", name, p, seed, time.time() - t0, flush=True)

    # log-likelihoods of the trace sequences under T_ref and a learned P̂1
    for name in ["m2_75", "m3_demo"]:
        states, _, _ = bfs[name]
        sidx = {s: i for i, s in enumerate(states)}
        Ds = [tuple(int(v) for v in row) for row in arrays[f"{name}/trace_D"]]
        T = arrays[f"{name}/T_0.5"]
        P = arrays[f"{name}/P1_0.05_123"]
        arrays[f"{name}/trace_logp"] = np.array([pdp.log_prob_sequence(Ds, sidx, P),
                                                 pdp.log_prob_sequence(Ds, sidx, T)])

    # 7. run_experiment end to end (A10), with a recording log_prob_sequence
    exp_cases = [
        ("exp_m2_75_57", "m2_75", "m2_57", 200, [0.01, 0.05, 0.1, 0.2, 0.3], 123),
        ("exp_m2_75_65", "m2_75", "m2_65", 100, [0.01, 0.1, 0.3], 12345),
        ("exp_m3_demo", "m3_demo", "m3_demo2", 40, [0.01, 0.05, 0.2], 123),
    ]
    orig_lps = pdp.log_prob_sequence
    for ename, g1, g2, iters, pv, seed in exp_cases:
        k, n, m, taps1 = CODES[g1]
        taps2 = CODES[g2][3]
        rec = []

        def recording(metrics, state_index, T, _rec=rec):
            v = orig_lps(metrics, state_index, T)
            _rec.append(v)
            return v
        pdp.log_prob_sequence = recording
        vm.simulate_markov_sequence = make_shim(taps1, seed)
        pdp.learn_P1_empirical.cache_clear()
        df = pdp.run_experiment(k, n, m, taps1, taps2, iters, pv, None, 200, 1.0, seed)
        pdp.log_prob_sequence = orig_lps
        meta[ename] = {"g1": g1, "g2": g2, "num_iter": iters, "p_vec": pv, "seed": seed,
                       "N_list": pdp.N_SPECTRUM_BY_M[m], "learn_burn": 200, "laplace": 1.0,
                       "rows": df.to_dict(orient="records")}
        # per trial: (logp1, logp1_ref, logp2, logp2_ref) in the reference's call order
        arrays[f"{ename}/sums"] = np.array(rec, np.float64).reshape(-1, 4)
        print("run_experiment", ename, df.to_dict(orient="records"), time.time() - t0, flush=True)

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("done", time.time() - t0)


if __name__ == "__main__":
    main()
