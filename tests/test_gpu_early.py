"""Early decision (CVD_DETECT_EARLY_DECISION): a trial stops once its decision is
certain (rigorous IEEE bounds on the remaining log-likelihood increments), and a
wavefront stops when all its lanes have decided.  The success counts must be
identical to the full recursion's on every detector kernel, at informative grid
points (Pd strictly between 0 and 1) and at the headline sweep's points."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
SEED = 12345


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda", 0)


def _both(pkg, cfg, N, p, learn_len, T, path=0, t0=0, taps=None):
    cc = pkg.CONFIG_CODES[cfg]
    det = pkg.Detector(cc["k"], cc["n"], cc["m"], cc["gen1"], device=0)
    model = det.model(p, learn_len, 200, 1.0, SEED)
    out = []
    for early in (False, True):
        torch.cuda.synchronize()
        t = time.perf_counter()
        c = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, t0, t0 + T, path=path,
                           early_decision=early)["counts"].cpu().tolist()
        torch.cuda.synchronize()
        out.append((c, time.perf_counter() - t))
    (full, tf), (early, te) = out
    print(f"\n  {cfg} N={N} p={p} path={path}: counts {full}, full {tf:.3f} s, early {te:.3f} s")
    assert early == full
    return full


@pytest.mark.parametrize("p,learn_len", [(0.01, None), (0.05, None), (0.2, None), (0.0033, 10_000_000)])
def test_m6_headline_kernel(pkg, dev, p, learn_len):
    _both(pkg, "m6", 100_000, p, learn_len, 8192)


def test_m6_informative_small_n(pkg, dev):
    full = _both(pkg, "m6", 3000, 0.002, None, 32768, t0=1_000_000)
    assert 0.05 < full[0] / 32768 < 0.95


@pytest.mark.parametrize("path", [3, 4, 5])   # generic, orbit, table-driven butterfly explicit kernels
def test_m6_other_explicit_kernels(pkg, dev, path):
    _both(pkg, "m6", 5000, 0.05, 30000, 4096, path=path)


@pytest.mark.parametrize("p", [0.05, 0.092])
def test_m2_table_kernels(pkg, dev, p, monkeypatch):
    full = _both(pkg, "m2", 10_000, p, None, 65536)
    monkeypatch.setenv("CVD_TABLE_WIDE", "1")
    assert _both(pkg, "m2", 10_000, p, None, 65536) == full


def test_r23_table_kernel(pkg, dev):
    full = _both(pkg, "r23_m4", 100_000, 0.0135, None, 4096)
    assert 0.05 < full[0] / 4096 < 0.95


def test_sums_refused_with_early_decision(pkg, dev):
    cc = pkg.CONFIG_CODES["m2"]
    det = pkg.Detector(1, 2, 2, cc["gen1"], device=0)
    model = det.model(0.05, None, 200, 1.0, SEED)
    with pytest.raises(ValueError):
        det.run_trials(model, cc["gen1"], cc["gen2"], 100, 0.05, SEED, 0, 10, return_sums=True, early_decision=True)
    r = det.generate(cc["gen1"], 100, 0.05, SEED, 1, 0, 1, 2)
    sums = torch.zeros((2, 2), dtype=torch.float64, device=dev)
    with pytest.raises(pkg.CvdError):
        det.detect(model, r, 100, 2, 1, sums=sums, early_decision=True)


def test_run_experiment_default_equals_full(pkg, dev):
    cc = pkg.CONFIG_CODES["m2"]
    a = pkg.run_experiment(1, 2, 2, cc["gen1"], cc["gen2"], 3000, [0.05, 0.1], None, 200, 1.0, 7, N_list=[500, 2000])
    b = pkg.run_experiment(1, 2, 2, cc["gen1"], cc["gen2"], 3000, [0.05, 0.1], None, 200, 1.0, 7, N_list=[500, 2000],
                           early_decision=False)
    assert a.to_dict(orient="records") == b.to_dict(orient="records")
