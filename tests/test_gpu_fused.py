"""The fused trial kernel (cvd_mc_fused; Pd_plotter.py:210-223 in one launch): every
lane generates its own sequence's received words (the generator's encoder and
bit-sliced noise) and runs the LDS-resident table automaton on them, with no stream
in HBM.  Its per-trial fp64 sums and counts must equal the two-kernel path
(cvd_generate + cvd_detect) bit for bit -- and the C oracle's -- for every dense
config code, trial counts that are not whole waves, offset trial ranges, the
noise extremes (p = 0: no draws; p = 1: every bit flips), the multi-round noise
exchange and early decision."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CODES = {
    "m2": ("m2", None),
    "demo1": ("example", "1"),
    "demo2": ("example", "2"),
    "r23_m4": ("r23_m4", None),
}


def _code(pkg, name):
    kind, key = CODES[name]
    c = pkg.EXAMPLE_CODES[key] if kind == "example" else pkg.CONFIG_CODES[kind]
    return c["k"], c["n"], c["m"], c["gen1"], c["gen2"]


def _unfused(det, model, g1, g2, N, p, seed, lo, hi):
    return det.run_trials(model, g1, g2, N, p, seed, lo, hi, return_sums=True)


@pytest.mark.parametrize("name", list(CODES))
@pytest.mark.parametrize("p", [0.0, 0.05, 0.3, 1.0])
def test_fused_sums_equal_two_kernel_path(pkg, name, p):
    k, n, m, g1, g2 = _code(pkg, name)
    det = pkg.Detector(k, n, m, g1, device=0)
    model = det.model(p, None, 200, 1.0, 777)
    N, lo, hi = 1237, 3_000_000_011, 3_000_000_011 + 1000   # not whole waves, offset ids
    ref = _unfused(det, model, g1, g2, N, p, 777, lo, hi)
    got = det.run_trials(model, g1, g2, N, p, 777, lo, hi, return_sums=True, fused=True)
    assert np.array_equal(got["sums"], ref["sums"])
    assert got["counts"].cpu().tolist() == ref["counts"].cpu().tolist()


def test_fused_equals_c_oracle_m2(pkg):
    from oracle import c_oracle as C
    k, n, m, g1, g2 = _code(pkg, "m2")
    det = pkg.Detector(k, n, m, g1, device=0)
    p, N, T = 0.092, 10_000, 256
    model = det.model(p, None, 200, 1.0, 12345)
    got = det.run_trials(model, g1, g2, N, p, 12345, 0, T, return_sums=True, fused=True)
    c1, c2 = C.Code(g1, m, k, n), C.Code(g2, m, k, n)
    cnt, sums = C.Model(c1, p, None, 200, 1.0, 12345).run_trials(c1, c2, N, p, 12345, 0, T, sums=True, nthreads=8)
    assert np.array_equal(got["sums"], sums)
    assert got["counts"].cpu().tolist() == [int(x) for x in cnt]


def test_fused_exchange_rounds_and_early_decision(pkg, monkeypatch):
    """CVD_GEN_SLOTS=3: the noise exchange runs many rounds per chunk; early decision
    (counts only) gives the full run's counts; cvd_mc_run (PATH_AUTO -> fused) equals
    the two-kernel path (PATH_TABLE)."""
    k, n, m, g1, g2 = _code(pkg, "r23_m4")
    det = pkg.Detector(k, n, m, g1, device=0)
    p, N = 0.0135, 20_000
    model = det.model(p, None, 200, 1.0, 5)
    ref = _unfused(det, model, g1, g2, N, p, 5, 0, 600)
    monkeypatch.setenv("CVD_GEN_SLOTS", "3")
    got = det.run_trials(model, g1, g2, N, p, 5, 0, 600, return_sums=True, fused=True)
    monkeypatch.delenv("CVD_GEN_SLOTS")
    assert np.array_equal(got["sums"], ref["sums"])
    early = det.run_trials(model, g1, g2, N, p, 5, 0, 600, fused=True, early_decision=True)
    assert early["counts"].cpu().tolist() == ref["counts"].cpu().tolist()
    auto = det.run_trials(model, g1, g2, N, p, 5, 0, 600)
    table = det.run_trials(model, g1, g2, N, p, 5, 0, 600, path=pkg.PATH_TABLE)
    assert auto["counts"].cpu().tolist() == table["counts"].cpu().tolist() == ref["counts"].cpu().tolist()


def test_fused_refuses_sparse_models(pkg):
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    model = det.model(0.05, 20_000, 200, 1.0, 1)
    with pytest.raises(pkg.CvdError, match="fused"):
        det.run_trials(model, cc["gen1"], cc["gen2"], 100, 0.05, 1, 0, 64, fused=True)
    # the counts path falls back to generator + explicit detector on its own
    c = det.run_trials(model, cc["gen1"], cc["gen2"], 100, 0.05, 1, 0, 64)["counts"]
    assert int(c.sum()) >= 0
    torch.cuda.synchronize()
