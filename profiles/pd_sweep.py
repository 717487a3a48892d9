import sys, time, itertools
sys.path.insert(0, '/root/repo')
from oracle import c_oracle as C
from __graft_entry__ import load_package
pkg = load_package()
cfg = sys.argv[1]
cc = pkg.CONFIG_CODES[cfg]
k, n, m = cc["k"], cc["n"], cc["m"]
c1, c2 = C.Code(cc["gen1"], m, k, n), C.Code(cc["gen2"], m, k, n)
Ns = [int(x) for x in sys.argv[2].split(',')]
ps = [float(x) for x in sys.argv[3].split(',')]
lls = [None if x == 'None' else int(float(x)) for x in sys.argv[4].split(',')]
T = int(sys.argv[5])
for ll, p in itertools.product(lls, ps):
    t0 = time.time()
    mod = C.Model(c1, p, ll, 200, 1.0, 12345)
    tl = time.time() - t0
    for N in Ns:
        t0 = time.time()
        cnt, _ = mod.run_trials(c1, c2, N, p, 12345, 0, T, nthreads=8)
        print(f"{cfg} learn={ll} S={mod.S} p={p} N={N} T={T} Pd={cnt[0]/T:.4f} Pc={(cnt[0]+cnt[1])/(2*T):.4f} learn_s={tl:.1f} run_s={time.time()-t0:.1f}", flush=True)
