import sys, time
sys.path.insert(0, '/root/repo')
from __graft_entry__ import load_package
from oracle import c_oracle as C
pkg = load_package()
cc = pkg.CONFIG_CODES["m6"]
N, p, ll, seed = 100_000, 0.0033, 10_000_000, 12345
det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
model = det.model(p, ll, 200, 1.0, seed)
for t0 in (0, 1 << 20, 1 << 31, 1 << 32, 1 << 40):
    T = 131072
    c = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, t0, t0 + T)["counts"].cpu().tolist()
    print("gpu", t0, c, c[0] / T, flush=True)
c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
cm = C.Model(c1, p, ll, 200, 1.0, seed)
for t0 in (1 << 32, 1 << 40):
    want, _ = cm.run_trials(c1, c2, N, p, seed, t0, t0 + 256)
    got = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, t0, t0 + 256)["counts"].cpu().tolist()
    print("exact", t0, list(want), got, flush=True)
