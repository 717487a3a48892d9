"""Is the low Pd of trial ids [0, 848) at the m6 Pd-match point systematic?  Same
model, trial streams of other seeds: Pd of the first 848 trials vs 131,072 trials."""
import sys
import numpy as np
sys.path.insert(0, '/root/repo')
from __graft_entry__ import load_package
pkg = load_package()
cc = pkg.CONFIG_CODES["m6"]
N, p, ll = 100_000, 0.0033, 10_000_000
det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
model = det.model(p, ll, 200, 1.0, 12345)
T = 131072
for seed in (12345, 1, 2, 3, 4, 5, 6, 7):
    s = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, 0, T, return_sums=True)["sums"]
    d = (s[:, 0] > s[:, 1]).astype(np.float64)
    ch = d[: (T // 848) * 848].reshape(-1, 848).mean(axis=1)
    z = (ch[0] - d.mean()) / np.sqrt(d.mean() * (1 - d.mean()) / 848)
    print(f"seed {seed}: Pd {d.mean():.4f} first848 {ch[0]:.4f} z {z:+.2f} rank {(ch < ch[0]).sum()}/{len(ch)}", flush=True)
