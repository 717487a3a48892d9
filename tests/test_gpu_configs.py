"""GPU parity at every BASELINE.json configuration's own size, and at an
informative grid point of each code (Pd neither 0 nor 1), against the pinned C
oracle (oracle/cvd_oracle.c, itself pinned to the reference's golden vectors by
tests/test_c_oracle.py): success counts equal and per-trial fp64 sums bit-exact
on the same trial ids.  Plus the Monte-Carlo tolerance of the "Pd match vs CPU"
clause: Pd of a large independent GPU sample within 3 binomial standard
deviations of the oracle's Pd (stated in each test)."""
import math

import numpy as np
import pytest
import torch

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

SEED = 12345


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda", 0)


def _codes(pkg, cfg):
    cc = pkg.CONFIG_CODES[cfg]
    k, n, m = cc["k"], cc["n"], cc["m"]
    return cc, k, n, m, C.Code(cc["gen1"], m, k, n), C.Code(cc["gen2"], m, k, n)


def _check(pkg, cfg, N, p, learn_len, t0, t1, paths, nsums=None, seed=SEED):
    """GPU counts over trials [t0, t1) on every path == C oracle counts; sums of the
    first `nsums` trials bit-exact.  Returns the oracle counts."""
    cc, k, n, m, c1, c2 = _codes(pkg, cfg)
    det = pkg.Detector(k, n, m, cc["gen1"], device=0)
    model = det.model(p, learn_len, 200, 1.0, seed)
    cm = C.Model(c1, p, learn_len, 200, 1.0, seed)
    want, _ = cm.run_trials(c1, c2, N, p, seed, t0, t1)
    ns = (t1 - t0) if nsums is None else nsums
    _, want_sums = cm.run_trials(c1, c2, N, p, seed, t0, t0 + ns, sums=True)
    for path in paths:
        got = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, t0, t1, path=path)
        assert tuple(got["counts"].cpu().tolist()) == tuple(int(x) for x in want), (path, want)
        s = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, t0, t0 + ns, path=path, return_sums=True)
        assert np.array_equal(s["sums"], want_sums), path
    return [int(x) for x in want]


def _binomial_3sigma(x1, t1, x2, t2):
    """|x1/t1 - x2/t2| <= 3 sigma of the difference (pooled proportion)."""
    pool = (x1 + x2) / (t1 + t2)
    sd = math.sqrt(max(pool * (1 - pool), 1e-12) * (1 / t1 + 1 / t2))
    return abs(x1 / t1 - x2 / t2) <= 3 * sd


# ───────────── C1: m = 2 pair, N = 1e4, p = 0.05 (1 GPU) ─────────────

def test_c1_m2_config_size(pkg, dev):
    """C1 at its size: 2,000 trials, table (LDS automaton) and explicit paths."""
    _check(pkg, "m2", 10_000, 0.05, None, 0, 2000, (pkg.PATH_TABLE, pkg.PATH_EXPLICIT), nsums=256)


def test_c1_m2_informative_point_and_tolerance(pkg, dev):
    """m = 2 at N = 1e4, p = 0.092 (Pd ~ 0.57): exact counts on 4,096 shared trial ids;
    tolerance: Pd and Pc of 2^20 further GPU trials within 3 sigma of the oracle's."""
    cc, k, n, m, c1, c2 = _codes(pkg, "m2")
    want = _check(pkg, "m2", 10_000, 0.092, None, 0, 4096, (pkg.PATH_TABLE,), nsums=64)
    assert 0.05 < want[0] / 4096 < 0.95, want
    det = pkg.Detector(k, n, m, cc["gen1"], device=0)
    model = det.model(0.092, None, 200, 1.0, SEED)
    big = 1 << 20
    g = det.run_trials(model, cc["gen1"], cc["gen2"], 10_000, 0.092, SEED, 1 << 30, (1 << 30) + big)
    g = g["counts"].cpu().tolist()
    assert _binomial_3sigma(want[0], 4096, g[0], big)
    assert _binomial_3sigma(want[0] + want[1], 8192, g[0] + g[1], 2 * big)


# ───────────── C3: rate-2/3 m = 4 pair, N = 1e5 (1 GPU) ─────────────

def test_c3_r23_config_size(pkg, dev):
    """C3 at its size: N = 1e5, 48 trials, table and explicit paths, all sums bit-exact."""
    _check(pkg, "r23_m4", 100_000, 0.05, None, 0, 48, (pkg.PATH_TABLE, pkg.PATH_EXPLICIT))


def test_c3_r23_informative_point(pkg, dev):
    """rate-2/3 m = 4 at N = 1e5, p = 0.0135 (Pd ~ 0.33): exact counts on 320 trials;
    tolerance: Pd of 2^17 further GPU trials within 3 sigma of the oracle's."""
    cc, k, n, m, c1, c2 = _codes(pkg, "r23_m4")
    want = _check(pkg, "r23_m4", 100_000, 0.0135, None, 0, 320, (pkg.PATH_TABLE,), nsums=32)
    assert 0.05 < want[0] / 320 < 0.95, want
    det = pkg.Detector(k, n, m, cc["gen1"], device=0)
    model = det.model(0.0135, None, 200, 1.0, SEED)
    big = 1 << 17
    g = det.run_trials(model, cc["gen1"], cc["gen2"], 100_000, 0.0135, SEED, 1 << 30, (1 << 30) + big)
    g = g["counts"].cpu().tolist()
    assert _binomial_3sigma(want[0], 320, g[0], big)


# ───────────── C2/C4: m = 6 pair (the single-GPU leg of the N sweep) ─────────────

@pytest.mark.parametrize("N,trials,p", [(1000, 2048, 0.05), (10_000, 256, 0.2), (1_000_000, 8, 0.02)])
def test_c4_m6_n_sweep_leg(pkg, dev, N, trials, p):
    """C4's N grid on one GPU (N = 1e3 .. 1e6), default 10^6-step sparse model."""
    _check(pkg, "m6", N, p, None, 0, trials, (pkg.PATH_EXPLICIT,), nsums=min(trials, 64))


def test_m6_informative_point_small_n(pkg, dev):
    """m = 6 at N = 3,000, p = 0.002 (default 10^6-step model; Pd ~ 0.48): exact
    counts on 2,048 trial ids, plus the 3-sigma Pd tolerance on 2^17 further trials."""
    cc, k, n, m, c1, c2 = _codes(pkg, "m6")
    want = _check(pkg, "m6", 3000, 0.002, None, 0, 2048, (pkg.PATH_EXPLICIT,), nsums=64)
    assert 0.05 < want[0] / 2048 < 0.95, want
    det = pkg.Detector(k, n, m, cc["gen1"], device=0)
    model = det.model(0.002, None, 200, 1.0, SEED)
    big = 1 << 17
    g = det.run_trials(model, cc["gen1"], cc["gen2"], 3000, 0.002, SEED, 1 << 30, (1 << 30) + big)
    g = g["counts"].cpu().tolist()
    assert _binomial_3sigma(want[0], 2048, g[0], big)


def test_m6_informative_point_headline_n(pkg, dev):
    """The bench's Pd-match point: m = 6 at the headline N = 1e5, p = 0.0033, a 10^7-step
    learning chain (Pd ~ 0.27): counts and sums equal the oracle's on 96 trial ids."""
    want = _check(pkg, "m6", 100_000, 0.0033, 10_000_000, 0, 96, (pkg.PATH_EXPLICIT,), nsums=16)
    assert 0.02 < want[0] / 96 < 0.98, want
