"""CPU tests of libcvd.so: it loads, exports every symbol of include/cvd.h, and
its host-side setup (code algebra, Eq. 4-5 step, BFS, P̂1 learning, T_ref) is
bit-identical to the reference's golden vectors and to the oracle.  No GPU."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

from conftest import ROOT, code_of
from oracle import restatement as R


def header_functions():
    src = open(os.path.join(ROOT, "include", "cvd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cvd_[a-z0-9_]+)\s*\(", src)))


def test_lib_exports_every_header_symbol(pkg):
    lib = pkg.lib()
    names = header_functions()
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), f"libcvd.so does not export {name}"
    assert lib.cvd_version() == pkg._lib.ABI_VERSION == 11
    assert set(names) <= set(pkg._lib.EXPORTS), "python binding misses a header function"


@pytest.mark.parametrize("name", ["m2_75", "m3_demo", "r23_m4", "m6_133_171"])
def test_code_tables(pkg, golden, name):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    out, nxt = pkg.Code(taps, m, k, n).tables()
    np.testing.assert_array_equal(out, z[f"{name}/out_sym"])
    np.testing.assert_array_equal(nxt, z[f"{name}/next_state"])
    tr = pkg.build_trellis(taps, m, k)
    rows = [[ns, ps, sum(b << i for i, b in enumerate(u)), sum(b << j for j, b in enumerate(o))]
            for ns in range(1 << m) for (ps, u, o) in tr[ns]]
    np.testing.assert_array_equal(np.array(rows), z[f"{name}/trellis"])


@pytest.mark.parametrize("name", ["m2_75", "m3_demo", "r23_m4", "m6_133_171"])
def test_host_metric_step(pkg, golden, name):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    tr = pkg.build_trellis(taps, m, k)
    r = z[f"{name}/trace_r"]
    D = z[f"{name}/trace_D"]
    for t in range(0, len(r), 3):
        y = tuple((int(r[t]) >> j) & 1 for j in range(n))
        assert pkg.viterbi_metric_step(tuple(D[t]), tr, y) == tuple(int(v) for v in D[t + 1])


@pytest.mark.parametrize("name", ["m2_75", "m2_57", "m2_65", "m3_demo", "r23_m4"])
def test_native_bfs(pkg, golden, name):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    states, transitions, all_r = pkg.enumerate_markov_states_allzero(taps, m, k, n)
    np.testing.assert_array_equal(np.array(states, np.uint8), z[f"{name}/states"])
    trip = [[i, j, sum(b << q for q, b in enumerate(r))]
            for i in range(len(states)) for j, rl in transitions[i].items() for r in rl]
    np.testing.assert_array_equal(np.array(trip), z[f"{name}/transitions"])


def test_bfs_cap(pkg):
    taps = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]
    with pytest.raises(pkg.CvdError):
        pkg.enumerate_markov_states_allzero(taps, 6, 1, 2, cap=10000)


@pytest.mark.parametrize("p,seed", [(0.01, 123), (0.05, 123), (0.1, 123), (0.2, 123), (0.3, 123),
                                    (0.05, 12345)])
def test_native_learned_P1_bit_exact_m2(pkg, golden, p, seed):
    z, meta = golden
    k, n, m, taps = code_of(meta, "m2_75")
    gens = tuple(tuple(tuple(x) for x in row) for row in taps)
    states, sidx, P = pkg.learn_P1_empirical(gens, k, n, m, p, None, 200, 1.0, seed)
    assert np.array_equal(P, z[f"m2_75/P1_{p}_{seed}"])


def test_native_learned_P1_bit_exact_m3(pkg, golden):
    z, meta = golden
    k, n, m, taps = code_of(meta, "m3_demo")
    gens = tuple(tuple(tuple(x) for x in row) for row in taps)
    _, _, P = pkg.learn_P1_empirical(gens, k, n, m, 0.05, None, 200, 1.0, 123)
    assert np.array_equal(P, z["m3_demo/P1_0.05_123"])


def test_native_learned_P1_bit_exact_rate23(pkg, golden):
    z, meta = golden
    k, n, m, taps = code_of(meta, "r23_m4")
    mod = pkg.Model(pkg.Code(taps, m, k, n), 0.05, None, 200, 1.0, 123)
    assert mod.info()["kind"] == 0 and mod.info()["S"] == 1807
    P = mod.dense_P1()
    np.testing.assert_array_equal(P.min(axis=1), z["r23_m4/P1_0.05_123_rowmin"])
    idx = z["r23_m4/P1_0.05_123_nz_idx"]
    assert np.array_equal(P[idx[:, 0], idx[:, 1]], z["r23_m4/P1_0.05_123_nz_val"])
    assert int((P > P.min(axis=1, keepdims=True)).sum()) == len(idx)


@pytest.mark.parametrize("laplace,burn,learn_len", [(0.3, 200, None), (2.5, 0, 7000), (1.0, 50, 300)])
def test_native_P1_matches_oracle_numpy(pkg, laplace, burn, learn_len):
    """Non-integer Laplace terms exercise the emulated numpy pairwise row sums."""
    taps = [[[1, 1, 1]], [[1, 0, 1]]]
    _, _, Pn = pkg.learn_P1_empirical(tuple(tuple(tuple(x) for x in r) for r in taps), 1, 2, 2, 0.07,
                                      learn_len, burn, laplace, 99)
    _, _, Po = R.learn_P1_empirical(taps, 1, 2, 2, 0.07, learn_len, burn, laplace, 99)
    assert np.array_equal(Pn, Po)


def test_model_rows_and_tref(pkg, golden):
    """log P̂1 per (row, received word) = log(max(P[i, next(i,r)], 1e-300))."""
    z, meta = golden
    k, n, m, taps = code_of(meta, "m2_75")
    mod = pkg.Model(pkg.Code(taps, m, k, n), 0.05, None, 200, 1.0, 123)
    lp, keys = mod.rows()
    np.testing.assert_array_equal(keys, z["m2_75/states"])
    P = z["m2_75/P1_0.05_123"]
    trans = z["m2_75/transitions"]
    for i, j, r in trans:
        assert lp[i, r] == math.log(max(P[i, j], 1e-300))
    inf = mod.info()
    assert inf["S"] == 31 and inf["kind"] == 0 and inf["learn_len_eff"] == max(5000, 200 * 31)


def test_sparse_model_m6(pkg):
    """m = 6 is not enumerable: the model holds the learning chain's visited states."""
    taps = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]
    mod = pkg.Model(pkg.Code(taps, 6, 1, 2), 0.05, 20000, 200, 1.0, 7, enum_cap=20000)
    inf = mod.info()
    assert inf["kind"] == 1 and inf["learn_len_eff"] == 20000
    assert inf["S"] == inf["n_rows"] and 100 < inf["S"] <= 20001
    assert inf["hash_capacity"] >= 2 * inf["S"]
    lp, keys = mod.rows()
    assert (keys[0] == 0).all()
    assert np.all(lp <= 0.0) and np.all(np.isfinite(lp))
    # a visited row's entries are (C + 1) / (R_i + S), an unvisited row's 1 / S
    assert np.all(lp >= math.log(1.0 / (20000 + inf["S"])))
    assert inf["logp1_unseen"] == math.log(1.0 / inf["S"])


def test_directory_sizing(pkg, monkeypatch):
    """Explicit-path directory (csrc/cvd_host.cpp build_hash): a power of two at load
    <= 1/16 by default; CVD_DIR_LOAD_LOG2=s sets load <= 2^-s (read at model build)."""
    taps = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]
    code = pkg.Code(taps, 6, 1, 2)
    inf = pkg.Model(code, 0.05, 20000, 200, 1.0, 7, enum_cap=20000).info()
    cap, rows = inf["hash_capacity"], inf["n_rows"]
    assert cap & (cap - 1) == 0 and 16 * rows <= cap < 32 * rows
    monkeypatch.setenv("CVD_DIR_LOAD_LOG2", "1")
    inf2 = pkg.Model(code, 0.05, 20000, 200, 1.0, 7, enum_cap=20000).info()
    assert inf2["n_rows"] == rows and 2 * rows <= inf2["hash_capacity"] < 4 * rows
    assert inf2["max_probe"] >= inf["max_probe"]


def test_walk_and_lds_filter_flags(pkg, monkeypatch):
    """cvd_model_info.walk / lds_filter before upload (cvd_kernels.hip walk_preferred,
    ldsf_wanted, ldsf_preferred): the bit-sliced kernel does not walk by default (round 6:
    lockstep with the LDS filter is faster at p = 0.01), and a model of <= 98,304 rows keeps its
    whole Bloom filter in LDS (CVD_LDSF_LOCKSTEP, default on for the bit-sliced kernel);
    CVD_NO_LDSF=1 (read at build) turns the LDS filter off, CVD_LDSF_LOCKSTEP=0 too unless the
    model walks, and CVD_WALK=1 forces walk mode (with the LDS filter)."""
    taps = [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]]
    code = pkg.Code(taps, 6, 1, 2)
    for v in ("CVD_WALK", "CVD_NO_LDSF", "CVD_LDSF_LOCKSTEP"):
        monkeypatch.delenv(v, raising=False)
    inf = pkg.Model(code, 0.01, 300_000, 200, 1.0, 7).info()
    assert 20 * inf["n_rows"] < inf["learn_len_eff"] and inf["n_rows"] <= 32768
    assert inf["walk"] == 0 and inf["lds_filter"] == 1
    hi = pkg.Model(code, 0.2, 120_000, 200, 1.0, 7).info()   # > 98,304 rows: the filter stays in L2
    assert hi["n_rows"] > 98304 and hi["walk"] == 0 and hi["lds_filter"] == 0
    monkeypatch.setenv("CVD_NO_LDSF", "1")
    assert pkg.Model(code, 0.01, 300_000, 200, 1.0, 7).info()["lds_filter"] == 0
    monkeypatch.delenv("CVD_NO_LDSF")
    monkeypatch.setenv("CVD_LDSF_LOCKSTEP", "0")
    off = pkg.Model(code, 0.01, 200_000, 200, 1.0, 7).info()
    assert off["walk"] == 0 and off["lds_filter"] == 0
    monkeypatch.setenv("CVD_WALK", "1")
    on = pkg.Model(code, 0.01, 200_000, 200, 1.0, 7).info()
    assert on["walk"] == 1 and on["lds_filter"] == 1


@pytest.mark.parametrize("name,kernel", [("m6_133_171", 3), ("m3_demo", 3), ("m2_75", 2), ("r23_m4", 1)])
def test_explicit_kernel_selection(pkg, golden, name, kernel):
    """The explicit path's kernel: butterfly (k = 1, n = 2, standard butterflies,
    m >= 3), else orbit (k = 1), else generic."""
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    mod = pkg.Model(pkg.Code(taps, m, k, n), 0.05, 5000, 200, 1.0, 7, enum_cap=100)
    assert mod.info()["explicit_kernel"] == kernel
    assert kernel in pkg.KERNEL_NAMES


def test_explicit_grid_batch_is_clamped_to_the_budget(pkg):
    """run_grid's `batch` is per grid point and the p row holds one stream slot per point
    (ADVICE r04): an explicit batch is clamped so that the whole row's workspace fits the
    budget, and a batch that fits is kept."""
    from dccvm_amd.detector import clamp_grid_batch, grid_workspace_bytes
    cc = pkg.CONFIG_CODES["m6"]
    g1 = pkg.Code(cc["gen1"], 6, 1, 2)
    models = [pkg.Model(g1, p, 5000, 200, 1.0, 7) for p in (0.05, 0.1, 0.2)]
    N_list = [100_000]
    one = grid_workspace_bytes(models[:1], g1, N_list, 1000, 0)
    row = grid_workspace_bytes(models, g1, N_list, 1000, 0)
    assert row == 3 * one > 0
    b = clamp_grid_batch(models, g1, N_list, 1000, 0, row // 2)
    assert 1 <= b < 1000 and grid_workspace_bytes(models, g1, N_list, b, 0) <= row // 2
    assert clamp_grid_batch(models, g1, N_list, 1000, 0, row) == 1000


def test_multi_groups_follow_variant_and_persistence(pkg, monkeypatch):
    """Detector.multi_groups (bench.py's per-launch timing) mirrors cvd_detect_multi's merge
    rule: runs of one nonzero variant, at most 8, a model whose batch is past its
    persist_seqs alone (ABI 10), CVD_NO_MULTI=1 every model alone."""
    class M:
        def __init__(self, v, cap):
            self.inf = {"multi_variant": v, "persist_seqs": cap}

        def info(self):
            return self.inf

    monkeypatch.delenv("CVD_NO_MULTI", raising=False)
    g = pkg.Detector.multi_groups
    ms = [M(7, 0), M(7, 0), M(9, 0), M(9, 0), M(0, 0), M(9, 0)]
    assert g(ms) == [[0, 1], [2, 3], [4], [5]]
    assert g([M(7, 0)] * 10) == [list(range(8)), [8, 9]]
    cap = [M(7, 1000)] * 4
    assert g(cap, [500, 500, 500, 500]) == [[0, 1, 2, 3]]
    assert g(cap, [500, 2000, 500, 500]) == [[0], [1], [2, 3]]
    assert g(cap) == [[0, 1, 2, 3]]          # no batch sizes: variant only
    monkeypatch.setenv("CVD_NO_MULTI", "1")
    assert g(ms[:2]) == [[0], [1]]


def test_jit_prebuild_only_for_bit_sliced_codes(pkg):
    """cvd_jit_prebuild compiles nothing for a code without the bit-sliced kernel (m = 2) and
    reports the m = 6 code's variants when build() has put them in the prebuilt cache"""
    import ctypes
    import os
    lib = pkg.lib()
    cc = pkg.CONFIG_CODES["m2"]
    n = ctypes.c_int32(-1)
    assert lib.cvd_jit_prebuild(pkg.Code(cc["gen1"], cc["m"], cc["k"], cc["n"]).c, b"gfx950", b"/nonexistent/x",
                                ctypes.byref(n)) == 0
    assert n.value == 0
    jit = os.path.join(os.path.dirname(pkg.__file__), "lib", "jit")
    if os.path.isdir(jit) and len(os.listdir(jit)) >= 3:
        c6 = pkg.CONFIG_CODES["m6"]
        n6 = ctypes.c_int32(-1)
        assert lib.cvd_jit_prebuild(pkg.Code(c6["gen1"], 6, 1, 2).c, b"gfx950", jit.encode(), ctypes.byref(n6)) == 0
        assert n6.value == 3   # (found, not recompiled: each is already there)
