"""First-chunk Pd at the m6 Pd-match point for (model learning seed, trial seed) pairs:
does the deficit follow the trial streams or the learning/trial seed coincidence?"""
import sys
import numpy as np
sys.path.insert(0, '/root/repo')
from __graft_entry__ import load_package
pkg = load_package()
cc = pkg.CONFIG_CODES["m6"]
N, p, ll = 100_000, 0.0033, 10_000_000
det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
T = 1 << 15
for mseed, tseed in ((12345, 12345), (99, 12345), (1, 1), (2, 2), (3, 3), (99, 99), (12345, 99)):
    model = det.model(p, ll, 200, 1.0, mseed)
    s = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, tseed, 0, T, return_sums=True)["sums"]
    d = (s[:, 0] > s[:, 1]).astype(np.float64)
    llr = s[:, 0] - s[:, 1]
    z = (llr[:768].mean() - llr.mean()) / (llr.std() / np.sqrt(768))
    print(f"model seed {mseed:5d} trial seed {tseed:5d}: Pd {d.mean():.4f} first768 {d[:768].mean():.4f} "
          f"llr z(first768) {z:+.2f}", flush=True)
