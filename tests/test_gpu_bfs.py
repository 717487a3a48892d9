"""State enumeration on the GPU (viterbi_markov.py:166-195):
cvd_enumerate_device gives the reference's BFS -- the same states in the same
discovery order and the same successor table -- as the reference's own goldens
(tests/golden: m2, m3, rate 2/3 S = 1,807) and the host BFS (cvd_enumerate) on
(23,35), S = 150,743; also with candidate chunks far smaller than a level and with
the hash narrowed to a few bits, which forces the 64-bit-collision path (a hash
shared by different states is never merged).  At m = 6 the search stops at its
capacity and reports a lower bound with per-level sizes."""
import numpy as np
import pytest

from conftest import code_of

pytestmark = pytest.mark.gpu

M4_2335 = [[[1, 0, 0, 1, 1]], [[1, 1, 1, 0, 1]]]


def _check_golden(pkg, z, meta, name):
    k, n, m, taps = code_of(meta, name)
    out = pkg.enumerate_states_device(taps, m, k, n, device=0, with_tables=True)
    assert out["complete"]
    np.testing.assert_array_equal(out["states"], z[f"{name}/states"])
    tr = z[f"{name}/transitions"]
    np.testing.assert_array_equal(out["next"][tr[:, 0], tr[:, 2]], tr[:, 1])
    assert sum(out["level_sizes"]) == out["S"] == len(z[f"{name}/states"])
    return out


@pytest.mark.parametrize("name", ["m2_75", "m2_65", "m3_demo", "r23_m4"])
def test_gpu_bfs_equals_reference_goldens(pkg, golden, name):
    z, meta = golden
    _check_golden(pkg, z, meta, name)


@pytest.mark.parametrize("chunk,bits", [("1024", "64"), ("64", "6"), ("100000", "3")])
def test_gpu_bfs_small_chunks_and_forced_collisions(pkg, golden, monkeypatch, chunk, bits):
    """Chunks smaller than a level (new states met again from a later chunk) and hashes
    cut to `bits` bits (most states share a hash: each must still be kept apart)."""
    monkeypatch.setenv("CVD_BFS_CHUNK", chunk)
    monkeypatch.setenv("CVD_BFS_HASH_BITS", bits)
    z, meta = golden
    for name in ("m3_demo", "r23_m4"):
        _check_golden(pkg, z, meta, name)


def test_gpu_bfs_equals_host_bfs_m4_2335(pkg):
    """(23,35): 150,743 states, states and successors as cvd_enumerate."""
    S_host = 150_743
    st_h, tr_h, _ = pkg.enumerate_markov_states_allzero(M4_2335, 4, 1, 2, cap=200_000)
    assert len(st_h) == S_host
    out = pkg.enumerate_states_device(M4_2335, 4, 1, 2, device=0, with_tables=True)
    assert out["complete"] and out["S"] == S_host
    np.testing.assert_array_equal(out["states"], np.array(st_h, np.uint8))
    nx = np.full((S_host, 4), -1, np.int64)
    for i, d in tr_h.items():
        for j, rl in d.items():
            for r in rl:
                nx[i, sum(b << q for q, b in enumerate(r))] = j
    np.testing.assert_array_equal(out["next"], nx)


def test_gpu_bfs_capacity_gives_lower_bound(pkg):
    """cap below S: CVD_E_CAPACITY with S a lower bound (distinct states found) and the
    level sizes of the levels reached; the m = 6 headline code past 10^6 states."""
    out = pkg.enumerate_states_device(M4_2335, 4, 1, 2, device=0, cap=50_000)
    assert not out["complete"] and 50_000 < out["S"] <= 150_743
    m6 = pkg.CONFIG_CODES["m6"]
    out = pkg.enumerate_states_device(m6["gen1"], 6, 1, 2, device=0, cap=2_000_000)
    assert not out["complete"] and out["S"] > 2_000_000
    assert out["level_sizes"][0] == 1 and sum(out["level_sizes"]) == out["S"]


def test_m6_detector_with_bfs_lower_bound_as_laplace_S(pkg):
    """The reference's own estimator at the headline code with S = the GPU BFS's certified
    lower bound in the Laplace denominator (laplace_states): the GPU detector's per-trial
    fp64 sums and counts equal the C oracle's given the same S."""
    from oracle import c_oracle as C
    S_lap = 3_192_590_107
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    mod = det.model(0.02, 200_000, 200, 1.0, 12345, laplace_states=S_lap)
    assert mod.info()["S"] == S_lap
    N, T = 2000, 128
    got = det.run_trials(mod, cc["gen1"], cc["gen2"], N, 0.02, 12345, 0, T, return_sums=True)
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    om = C.Model(c1, 0.02, 200_000, 200, 1.0, 12345, enum_cap=1000, laplace_states=S_lap)
    cnt, sums = om.run_trials(c1, c2, N, 0.02, 12345, 0, T, sums=True, nthreads=8)
    assert np.array_equal(got["sums"], sums)
    assert got["counts"].cpu().tolist() == [int(x) for x in cnt]
