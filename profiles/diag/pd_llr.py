"""Windowed mean log-likelihood ratio (log P1 - log Tref) of H1 trials by trial id,
seed 12345 (= the learning seed) vs seed 1, at the m6 Pd-match point."""
import sys
import numpy as np
sys.path.insert(0, '/root/repo')
from __graft_entry__ import load_package
pkg = load_package()
cc = pkg.CONFIG_CODES["m6"]
N, p, ll = 100_000, 0.0033, 10_000_000
det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
model = det.model(p, ll, 200, 1.0, 12345)
T = 1 << 15
for seed in (12345, 1):
    s = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, 0, T, return_sums=True)["sums"]
    llr = s[:, 0] - s[:, 1]
    print(f"seed {seed}: mean llr {llr.mean():.3f} std {llr.std():.3f}")
    w = 256
    m = llr.reshape(-1, w).mean(axis=1)
    print("  window means (256):", " ".join(f"{x:.2f}" for x in m[:12]), "... overall", f"{m.mean():.2f}", "std", f"{m.std():.3f}")
    print("  h2 llr mean", (s[:, 2] - s[:, 3]).mean(), "first 256", (s[:256, 2] - s[:256, 3]).mean())
    print("  lp1 first256", s[:256, 0].mean(), "rest", s[256:, 0].mean(), " lref first256", s[:256, 1].mean(), "rest", s[256:, 1].mean())
