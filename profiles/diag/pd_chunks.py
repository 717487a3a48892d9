"""Dispersion of per-trial H1 decisions at the m6 Pd-match point: Pd of consecutive
848-trial chunks vs the binomial spread, and the lag-1 correlation of decisions."""
import sys
import numpy as np
sys.path.insert(0, '/root/repo')
from __graft_entry__ import load_package
pkg = load_package()
cc = pkg.CONFIG_CODES["m6"]
N, p, ll, seed = 100_000, 0.0033, 10_000_000, 12345
det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
model = det.model(p, ll, 200, 1.0, seed)
T = 131072
s = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, 0, T, return_sums=True)["sums"]
d = (s[:, 0] > s[:, 1]).astype(np.float64)
pd = d.mean()
ch = d[: (T // 848) * 848].reshape(-1, 848).mean(axis=1)
print("Pd", pd, "first848", d[:848].mean(), "chunk std", ch.std(), "binomial std", np.sqrt(pd * (1 - pd) / 848))
print("chunk min/max", ch.min(), ch.max(), "rank of first chunk", (ch < ch[0]).sum(), "of", len(ch))
x = d - pd
print("lag-1 corr", (x[1:] * x[:-1]).mean() / x.var(), "lag-2", (x[2:] * x[:-2]).mean() / x.var())
for a, b in ((0, 64), (64, 128), (0, 256), (256, 512), (512, 848)):
    print("range", a, b, d[a:b].mean())
