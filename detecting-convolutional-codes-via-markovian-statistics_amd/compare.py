"""Comparison figures of the two detectors (plots_compare.py:35-134), host only.

Reads the CSVs the command line writes (experiment -> Pd_hybrid_results.csv,
parity -> Pd_parity_results.csv), converts Pc to the probability of error
P_err = clip(1 - Pc, 0, 1) (plots_compare.py:35-41; a table with only Pd uses
Pd in place of Pc, :77-81) and draws P_err against p for every N and against N
for every p, one PNG per curve pair (:90-134).  matplotlib is needed only for
the drawing; `curves()` gives the same data without it.
"""
import os

import numpy as np


def p_error(Pc):
    """P_err = 1 - P_c clipped to [0, 1]."""
    return np.clip(1.0 - np.asarray(Pc, dtype=float), 0.0, 1.0)


def _with_pc(df):
    if "Pc" not in df.columns and "Pd" in df.columns:
        df = df.assign(Pc=df["Pd"])
    return df


def _curve(df, key, value, x):
    """(x values, P_err) of the rows with df[key] == value, sorted by x."""
    sel = np.isclose(df[key].to_numpy(dtype=float), float(value))
    q = df[sel].sort_values(by=x)
    return q[x].to_numpy(), p_error(q["Pc"].to_numpy())


def curves(hybrid, baseline):
    """{("N", N) or ("p", p): {"hybrid": (x, P_err), "baseline": (x, P_err)}} for every
    blocklength and crossover probability present in either table (DataFrames)."""
    h, b = _with_pc(hybrid), _with_pc(baseline)
    out = {}
    for key, x in (("N", "p"), ("p", "N")):
        for v in sorted(set(h[key]).union(b[key])):
            out[(key, v)] = {"hybrid": _curve(h, key, v, x), "baseline": _curve(b, key, v, x)}
    return out


def compare_figures(hybrid_csv, baseline_csv, outdir="plots"):
    """Write Perr_vs_p_N<N>.png and Perr_vs_N_p<p>.png into outdir; returns the paths."""
    import pandas as pd
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    os.makedirs(outdir, exist_ok=True)
    paths = []
    for (key, v), cv in curves(pd.read_csv(hybrid_csv), pd.read_csv(baseline_csv)).items():
        x_label = "BSC crossover probability p" if key == "N" else "Blocklength N"
        v_txt = int(v) if key == "N" else v
        fig, ax = plt.subplots(figsize=(6, 5))
        for name, style, label in (("hybrid", dict(marker="o"), "Hybrid"),
                                   ("baseline", dict(marker="s", linestyle="--"), "Parity baseline")):
            xs, ys = cv[name]
            if len(xs):
                ax.plot(xs, ys, label=f"{label} ({key}={v_txt})", **style)
        ax.set_xlabel(x_label)
        ax.set_ylabel("Probability of error $P_{\\mathrm{err}}$")
        ax.set_title(f"$P_{{\\mathrm{{err}}}}$ vs ${'p' if key == 'N' else 'N'}$ ({key}={v_txt})")
        ax.grid(True)
        ax.legend()
        path = os.path.join(outdir, f"Perr_vs_{'p' if key == 'N' else 'N'}_{key}{v_txt}.png")
        fig.savefig(path, dpi=200, bbox_inches="tight")
        plt.close(fig)
        paths.append(path)
    return paths
