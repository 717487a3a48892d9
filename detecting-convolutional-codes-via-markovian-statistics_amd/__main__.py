"""Command line: the reference's script entry points on the MI355X engine.

  python -m detecting-convolutional-codes-via-markovian-statistics_amd experiment ...
      Pd_plotter.py:242-264 -- run_experiment over (N, p), writes
      <save-dir>/Pd_hybrid_results.csv (columns N, p, Pd, Pc)
  ... parity ...
      comp_parity.py:135-181 -- the parity-template baseline (template of G1,
      basis vector 0 of deg_h = m + 3) on the same trial streams, writes
      <save-dir>/Pd_parity_results.csv: the --baseline CSV of plots_compare.py
  ... exponent ...
      alpha_exponent.py -- learned transition tensors of G1 and G2 streams on
      G1's metric automaton, Eq. 7 per p, writes <save-dir>/error_exponent.csv
  ... compare --hybrid H.csv --baseline B.csv [--outdir plots]
      plots_compare.py:70-148 -- P_err = 1 - Pc of both detectors against p
      (per N) and against N (per p), one PNG each (host only, matplotlib)

Codes: the BASELINE configurations (m2, m6, r23_m4) or the demo presets
(example:1, example:2, demo_script.py:35-52).  Every subcommand but compare
runs on the GPU through libcvd.so.  Under torchrun (one process per GPU) the trials are
sharded over the ranks, the counts reduced with one all_reduce, and rank 0
writes the CSV.
"""
import argparse
import os
import sys

from . import (CONFIG_CODES, DEFAULTS, EXAMPLE_CODES, compute_error_exponent, default_template,
               learn_transition_tensor, parity_experiment, parity_vector_to_equation, parity_vectors,
               run_experiment)

PROG = "python -m detecting-convolutional-codes-via-markovian-statistics_amd"


def code_of(name):
    """(k, n, m, gen1, gen2) of a configuration or demo preset name."""
    if name.startswith("example:"):
        key = name.split(":", 1)[1]
        if key not in EXAMPLE_CODES:
            raise SystemExit(f"unknown preset {name!r} (example:{' | example:'.join(EXAMPLE_CODES)})")
        c = EXAMPLE_CODES[key]
    elif name in CONFIG_CODES:
        c = CONFIG_CODES[name]
    else:
        raise SystemExit(f"unknown code {name!r}: {', '.join(CONFIG_CODES)} or example:<preset>")
    return c["k"], c["n"], c["m"], c["gen1"], c["gen2"]


def _floats(s):
    return [float(x) for x in s.split(",") if x.strip()]


def _ints(s):
    return [int(x) for x in s.split(",") if x.strip()]


def parser():
    ap = argparse.ArgumentParser(prog=PROG, description="MI355X relative-Viterbi-metric detector")
    sub = ap.add_subparsers(dest="cmd", required=True)
    common = argparse.ArgumentParser(add_help=False)
    common.add_argument("--code", default="example:1",
                        help="m2 | m6 | r23_m4 (BASELINE configs) or example:1 | example:2 (demo presets)")
    common.add_argument("--p", type=_floats, default=None,
                        help="comma list of BSC crossover probabilities (default: Pd_plotter.py DEFAULTS p_vec)")
    common.add_argument("--seed", type=int, default=DEFAULTS["seed"])
    common.add_argument("--save-dir", default=DEFAULTS["save_dir"])
    common.add_argument("--out", default=None, help="CSV path (default: <save-dir>/<subcommand file>)")

    e = sub.add_parser("experiment", parents=[common], help="Pd/Pc of the Markov detector (Pd_plotter.py)")
    e.add_argument("--num-iter", type=int, default=DEFAULTS["num_iter"])
    e.add_argument("--N", type=_ints, default=None, help="blocklengths (default: N_SPECTRUM_BY_M[m])")
    e.add_argument("--learn-len", type=int, default=DEFAULTS["learn_len"])
    e.add_argument("--learn-burn", type=int, default=DEFAULTS["learn_burn"])
    e.add_argument("--laplace", type=float, default=DEFAULTS["laplace"])

    pa = sub.add_parser("parity", parents=[common], help="parity-template baseline (comp_parity.py)")
    pa.add_argument("--num-iter", type=int, default=DEFAULTS["num_iter"])
    pa.add_argument("--N", type=_ints, default=None, help="blocklengths (default: N_SPECTRUM_BY_M[m])")
    pa.add_argument("--gamma", type=float, default=0.6, help="decision threshold (comp_parity.py:166)")
    pa.add_argument("--deg-h", type=int, default=None, help="parity polynomial degree (default m + 3)")

    x = sub.add_parser("exponent", parents=[common], help="Eq. 7 error exponent (alpha_exponent.py)")
    x.add_argument("--length", type=int, default=300_000, help="learning chain steps per tensor")
    x.add_argument("--burn-in", type=int, default=5_000)
    x.add_argument("--laplace", type=float, default=1.0)
    x.add_argument("--chains", type=int, default=1, help="independent chains (1: the reference's one chain)")
    x.add_argument("--u-grid", type=int, default=401)

    c = sub.add_parser("compare", help="P_err figures of both detectors (plots_compare.py)")
    c.add_argument("--hybrid", required=True, help="CSV of the experiment subcommand")
    c.add_argument("--baseline", required=True, help="CSV of the parity subcommand")
    c.add_argument("--outdir", default="plots")
    return ap


def _init_dist():
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return dist


def cmd_experiment(a):
    k, n, m, g1, g2 = code_of(a.code)
    df = run_experiment(k, n, m, g1, g2, a.num_iter, a.p or DEFAULTS["p_vec"], a.learn_len, a.learn_burn,
                        a.laplace, a.seed, N_list=a.N)
    return df, "Pd_hybrid_results.csv", "Hybrid Markov-based detector"


def cmd_parity(a):
    k, n, m, g1, g2 = code_of(a.code)
    deg_h = m + 3 if a.deg_h is None else a.deg_h
    eq = parity_vector_to_equation(parity_vectors(g1, deg_h)[0])
    df = parity_experiment(k, n, m, g1, g2, a.num_iter, a.p or DEFAULTS["p_vec"], a.gamma, a.seed,
                           N_list=a.N, template=default_template(g1, m, deg_h))
    return df, "Pd_parity_results.csv", f"Parity-template baseline, equation {eq}"


def cmd_exponent(a):
    import pandas as pd
    k, n, m, g1, g2 = code_of(a.code)
    rows = []
    for p in a.p or DEFAULTS["p_vec"]:
        P1 = learn_transition_tensor(g1, g1, m, p, a.length, a.burn_in, a.laplace, a.seed, k=k, n=n,
                                     chains=a.chains)[0]
        P2 = learn_transition_tensor(g2, g1, m, p, a.length, a.burn_in, a.laplace, a.seed + 1, k=k, n=n,
                                     chains=a.chains)[0]
        I_err, u = compute_error_exponent(P1, P2, u_grid=a.u_grid)
        rows.append({"p": p, "I_err": I_err, "u_star": u, "states": P1.K})
    return pd.DataFrame(rows), "error_exponent.csv", "Error exponent (Eq. 7)"


def main(argv=None):
    a = parser().parse_args(argv)
    if a.cmd == "compare":
        from .compare import compare_figures
        for path in compare_figures(a.hybrid, a.baseline, a.outdir):
            print("Saved", path)
        return 0
    dist = _init_dist()
    run = {"experiment": cmd_experiment, "parity": cmd_parity, "exponent": cmd_exponent}[a.cmd]
    df, name, title = run(a)
    if dist is None or dist.get_rank() == 0:
        out = a.out or os.path.join(a.save_dir, name)
        os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
        df.to_csv(out, index=False)
        print(title)
        print(df.to_string(index=False))
        print("Saved results to", out)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
