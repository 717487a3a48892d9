#!/usr/bin/env python3
"""The headline workload at the reference's own call shape (Pd_plotter.py:176-235, 242-264:
run_experiment with num_iter = 10,000 trials per p over the C2 p grid at N = 1e5), through the
product's drop-in, chunked and not (CVD_CHUNK=0), full run and early decision.
Each configuration is called twice; the second call (models, tables and JIT cached) is timed.

  python profiles/r06_refcall.py [--num-iter 10000] [--reps 2] > out.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-iter", type=int, default=10_000)
    ap.add_argument("--N", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--modes", default="0,-1")
    ap.add_argument("--early", default="0,1", help="early_decision values to run (0, 1)")
    a = ap.parse_args()
    import torch
    from __graft_entry__ import load_package
    pkg = load_package()
    cc = pkg.CONFIG_CODES["m6"]
    p_grid = [0.01, 0.02, 0.05, 0.1, 0.15, 0.2]
    args = (1, 2, 6, cc["gen1"], cc["gen2"], a.num_iter, p_grid, 1_000_000, 200, 1.0, 12345)
    out = {"call": f"run_experiment(num_iter={a.num_iter}, p_vec={p_grid}, N_list=[{a.N}])", "runs": []}
    dfs = {}
    for early in [bool(int(x)) for x in a.early.split(",")]:
        for mode in a.modes.split(","):
            os.environ["CVD_CHUNK"] = mode
            times = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                df = pkg.run_experiment(*args, N_list=[a.N], early_decision=early)
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t0)
            dfs[(early, mode)] = df
            st = pkg._lib.chunk_last()
            out["runs"].append({"early_decision": early, "CVD_CHUNK": mode, "seconds": times,
                                "trials_per_s_last": 6 * a.num_iter / times[-1], "chunk_last": st})
            print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    base = next(iter(dfs.values()))
    out["dataframes_equal"] = {f"early={e},chunk={m}": bool(df.equals(base)) for (e, m), df in dfs.items()}
    out["rows"] = base.to_dict(orient="records")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
