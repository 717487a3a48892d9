"""Pin the C oracle (oracle/cvd_oracle.c) to the Python restatement and the
reference's golden vectors; check the product's native sparse (m = 6) model
against the C oracle's independent restatement of the same policy.  CPU only."""
import math

import numpy as np
import pytest

from conftest import code_of
from oracle import c_oracle as C
from oracle import philox
from oracle import restatement as R


@pytest.mark.parametrize("name,N,p", [("m2_75", 500, 0.05), ("r23_m4", 301, 0.2), ("m6_133_171", 777, 0.01)])
def test_c_stream_matches_spec(golden, name, N, p):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    tag = philox.grid_tag(N, p)
    assert C.lib().oc_grid_tag(N, p) == tag
    for sid in (0, 5, 2**33 + 7):
        np.testing.assert_array_equal(C.stream(C.Code(taps, m, k, n), N, p, 77, tag, sid),
                                      R.received_stream(taps, m, k, n, N, p, 77, tag, sid))


@pytest.mark.parametrize("p", [0.0, 1.0, 0.5, 2.0 ** -32, 0.25 + 2.0 ** -32, 1 - 2.0 ** -32, 0.0033, 0.2])
@pytest.mark.parametrize("n", [1, 2, 3])
def test_noise_spec_edges(n, p):
    """Bit-sliced noise: the C oracle's early-exit plane comparison equals the
    numpy spec (all 32 planes composed into uniforms) at threshold edge cases
    (thr = 0, 2^32, powers of two, a single low bit, all ones)."""
    taps = {1: [[[1, 1, 1]]], 2: [[[1, 1, 1]], [[1, 0, 1]]], 3: [[[1, 1, 1]], [[1, 0, 1]], [[0, 1, 1]]]}[n]
    N = 701
    tag = philox.grid_tag(N, p)
    for sid in (0, 3):
        np.testing.assert_array_equal(C.stream(C.Code(taps, 2, 1, n), N, p, 99, tag, sid),
                                      R.received_stream(taps, 2, 1, n, N, p, 99, tag, sid))


def test_noise_spec_definition():
    """noise_bits against the spec's definition written out bit by bit with Python ints."""
    seed, tag, sid, n, N, p = 5, 17, 9, 2, 40, 0.3
    thr = philox.threshold(p)
    got = philox.noise_bits(seed, tag, sid, N, n, p)
    for w in range(N // 16 + 1):
        planes = []
        for j in range(8):
            x = philox.philox4x32_10([8 * w + j], [sid], [philox._ctr_hi(sid, philox.KIND_NOISE)], [tag],
                                     seed, 0)
            planes += [int(v[0]) for v in x]
        for b in range(32):
            t, jb = divmod(w * 32 + b, n)
            if t >= N:
                continue
            u = sum(((planes[i] >> b) & 1) << (31 - i) for i in range(32))
            assert got[t, jb] == (u < thr)


@pytest.mark.parametrize("ename", ["exp_m2_75_57", "exp_m3_demo"])
def test_c_oracle_sums_vs_reference(golden, ename):
    z, meta = golden
    e = meta[ename]
    k, n, m, t1 = code_of(meta, e["g1"])
    t2 = code_of(meta, e["g2"])[3]
    c1, c2 = C.Code(t1, m, k, n), C.Code(t2, m, k, n)
    iters = e["num_iter"]
    sums = z[f"{ename}/sums"]
    for N in e["N_list"]:
        for ip, p in enumerate(e["p_vec"]):
            mod = C.Model(c1, p, None, e["learn_burn"], e["laplace"], e["seed"])
            assert mod.kind == 0
            counts, got = mod.run_trials(c1, c2, N, p, e["seed"], 0, iters, sums=True, nthreads=4)
            assert np.array_equal(got, sums[ip * iters:(ip + 1) * iters])
            row = e["rows"][ip]
            assert counts[0] / iters == row["Pd"] and (counts[0] + counts[1]) / (2 * iters) == row["Pc"]


def test_native_sparse_model_equals_c_oracle(pkg):
    """Product host learning (libcvd) == C oracle for the m = 6 sparse policy."""
    cc = pkg.CONFIG_CODES["m6"]
    for p in (0.01, 0.1):
        mod = pkg.Model(pkg.Code(cc["gen1"], 6, 1, 2), p, 50000, 200, 1.0, 12345, enum_cap=1000)
        lp, keys = mod.rows()
        om = C.Model(C.Code(cc["gen1"], 6, 1, 2), p, 50000, 200, 1.0, 12345, enum_cap=1000)
        olp, okeys = om.rows()
        assert om.kind == 1 and mod.info()["kind"] == 1
        np.testing.assert_array_equal(keys, okeys)
        assert np.array_equal(lp, olp)
        assert mod.info()["logp1_unseen"] == math.log(1.0 / om.S)


# certified lower bound on the m = 6 (133,171) state count from the GPU BFS
# (cvd_enumerate_device, profiles/r03b/bfs_m6.json)
S_M6_LOWER = 3_192_590_107


@pytest.mark.parametrize("S_lap", [S_M6_LOWER, 5_000_000_000_123])
def test_laplace_states_model_equals_c_oracle(pkg, S_lap):
    """The reference's estimator with a measured / bounded S in the Laplace denominator
    (Pd_plotter.py:166-167; laplace_states): product host learning == C oracle given the
    same S, row for row, bit for bit (numpy's pairwise row sum over S entries vs the
    closed form R_i + S*laplace, equal for integral laplace)."""
    cc = pkg.CONFIG_CODES["m6"]
    mod = pkg.Model(pkg.Code(cc["gen1"], 6, 1, 2), 0.05, 50000, 200, 1.0, 12345, enum_cap=1000,
                    laplace_states=S_lap)
    om = C.Model(C.Code(cc["gen1"], 6, 1, 2), 0.05, 50000, 200, 1.0, 12345, enum_cap=1000, laplace_states=S_lap)
    lp, keys = mod.rows()
    olp, okeys = om.rows()
    np.testing.assert_array_equal(keys, okeys)
    assert np.array_equal(lp, olp)
    inf = mod.info()
    assert inf["S"] == S_lap and inf["n_rows"] == om.S == len(keys)
    assert inf["logp1_unseen"] == math.log(1.0 / S_lap)


def test_laplace_states_rejected_when_inconsistent(pkg):
    cc = pkg.CONFIG_CODES["m6"]
    with pytest.raises(pkg.CvdError, match="below the number of visited"):
        pkg.Model(pkg.Code(cc["gen1"], 6, 1, 2), 0.05, 50000, 200, 1.0, 1, enum_cap=1000, laplace_states=10)
    m2 = pkg.CONFIG_CODES["m2"]
    with pytest.raises(pkg.CvdError, match="enumerable"):
        pkg.Model(pkg.Code(m2["gen1"], 2, 1, 2), 0.05, None, 200, 1.0, 1, laplace_states=32)
    assert pkg.Model(pkg.Code(m2["gen1"], 2, 1, 2), 0.05, None, 200, 1.0, 1, laplace_states=31).info()["S"] == 31


def test_c_oracle_sparse_sums_vs_python(pkg):
    """C oracle m = 6 sums == Python recursion over the same rows (T_ref by
    comparing all 2^n successors)."""
    cc = pkg.CONFIG_CODES["m6"]
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    p, N = 0.05, 150
    om = C.Model(c1, p, 20000, 200, 1.0, 3, enum_cap=1000)
    counts, sums = om.run_trials(c1, c2, N, p, 3, 10, 14, sums=True, nthreads=2)
    lp_tab, keys = om.rows()
    index = {bytes(row): i for i, row in enumerate(keys)}
    out, nxt = R.encoder_tables(cc["gen1"], 6, 1, 2)
    tag = philox.grid_tag(N, p)
    for t in range(10, 14):
        for hyp, g in ((0, cc["gen1"]), (1, cc["gen2"])):
            r = R.received_stream(g, 6, 1, 2, N, p, 3, tag, 2 * t + hyp)
            D = np.zeros(64, np.int64)
            lp = lr = 0.0
            for rv in r:
                i = index.get(bytes(D.astype(np.uint8)))
                succ = [R.metric_step_vec(D, out, nxt, q, 2) for q in range(4)]
                c = sum(np.array_equal(succ[q], succ[rv]) for q in range(4))
                lp += lp_tab[i, rv] if i is not None else math.log(1.0 / om.S)
                lr += math.log(c / 4)
                D = succ[rv]
            assert sums[t - 10, 2 * hyp] == lp and sums[t - 10, 2 * hyp + 1] == lr


def test_models_learned_in_parallel_equal_sequential(pkg):
    """Models of a p sweep learned on concurrent host threads (Detector.prepare_models)
    are identical to sequentially learned ones (host only, no upload)."""
    from concurrent.futures import ThreadPoolExecutor
    cc = pkg.CONFIG_CODES["m6"]
    dec = pkg.Code(cc["gen1"], 6, 1, 2)
    ps = [0.02, 0.1, 0.2]
    seq = [pkg.Model(dec, p, 20000, 200, 1.0, 7) for p in ps]
    with ThreadPoolExecutor(3) as ex:
        par = list(ex.map(lambda p: pkg.Model(dec, p, 20000, 200, 1.0, 7), ps))
    for a, b in zip(seq, par):
        la, ka = a.rows()
        lb, kb = b.rows()
        assert np.array_equal(la, lb) and np.array_equal(ka, kb)
