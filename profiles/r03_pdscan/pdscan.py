import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import c_oracle as C
import __graft_entry__ as g
pkg = g.load_package()
cc = pkg.CONFIG_CODES["m6"]
c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
for p, ll in [(0.01, 10_000_000), (0.01, 30_000_000), (0.005, 10_000_000), (0.0066, 10_000_000)]:
    t0 = time.time()
    m = C.Model(c1, p, ll, 200, 1.0, 12345)
    t1 = time.time()
    cnt, _ = m.run_trials(c1, c2, 100_000, p, 12345, 0, 48, nthreads=8)
    print(p, ll, "S", m.S, "learn %.1fs" % (t1 - t0), "counts", list(cnt), "Pd", cnt[0] / 48, "%.1fs" % (time.time() - t1), flush=True)
