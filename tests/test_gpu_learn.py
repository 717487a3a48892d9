"""P̂1 learning on the GPU (Pd_plotter.py:143-167):
cvd_model_create_device (speculative parallel-in-time chain, verified block
boundaries, first visits by a sort of key hashes) builds the SAME model as the
sequential host chain of cvd_model_create -- rows in the same first-visit order,
the same counts and the same log P̂1 bit for bit -- for the m = 6 headline code at
10^6 and 10^7 steps, the enumerable m = 4 (23,35) code at 200*S steps, and the
dense BASELINE codes; also when the speculation is forced to fail (no warm-up,
tiny blocks), which exercises the re-run passes."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

M4_2335 = [[[1, 0, 0, 1, 1]], [[1, 1, 1, 0, 1]]]


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda", 0)


def _pair(pkg, taps, m, k, n, p, learn_len, enum_cap=500_000, seed=12345, dense_P1=True):
    code = pkg.Code(taps, m, k, n)
    t0 = time.perf_counter()
    host = pkg.Model(code, p, learn_len, 200, 1.0, seed, enum_cap)
    th = time.perf_counter() - t0
    t0 = time.perf_counter()
    gpu = pkg.Model(code, p, learn_len, 200, 1.0, seed, enum_cap, learn_device=0)
    tg = time.perf_counter() - t0
    ih, ig = host.info(), gpu.info()
    for f in ("kind", "S", "n_rows", "learn_len_eff", "hash_capacity", "max_probe", "logp1_unseen"):
        assert ih[f] == ig[f], (f, ih[f], ig[f])
    lh, kh = host.rows()
    lg, kg = gpu.rows()
    assert np.array_equal(kh, kg), "row order (first visit) differs"
    assert np.array_equal(lh, lg), "log P1 differs"
    if dense_P1 and ih["kind"] == 0:
        assert np.array_equal(host.dense_P1(), gpu.dense_P1())
    print(f"\n  S={ig['S']} kind={ig['kind']} host {th:.2f} s, gpu {tg:.2f} s, stats {gpu.learn_stats}")
    return host, gpu


@pytest.mark.parametrize("p,learn_len", [(0.01, 1_000_000), (0.2, 1_000_000), (0.0033, 10_000_000)])
def test_m6_sparse_model_identical(pkg, dev, p, learn_len):
    cc = pkg.CONFIG_CODES["m6"]
    _pair(pkg, cc["gen1"], 6, 1, 2, p, learn_len)


def test_m4_2335_dense_model_identical(pkg, dev):
    """(23,35), S = 150,743: the reference's own chain length max(5000, 200*S) = 30.1M steps."""
    host, gpu = _pair(pkg, M4_2335, 4, 1, 2, 0.05, None, dense_P1=False)
    assert host.info()["S"] == 150_743 and host.info()["learn_len_eff"] == 200 * 150_743


@pytest.mark.parametrize("cfg,p", [("m2", 0.05), ("r23_m4", 0.1)])
def test_dense_config_models_identical(pkg, dev, cfg, p):
    cc = pkg.CONFIG_CODES[cfg]
    _pair(pkg, cc["gen1"], cc["m"], cc["k"], cc["n"], p, None)


@pytest.mark.parametrize("cfg,p", [("m2", 0.1), ("r23_m4", 0.05)])
def test_forced_sparse_small_codes_identical(pkg, dev, cfg, p):
    """enum_cap below S: the sparse (first-visit) policy on the small codes."""
    cc = pkg.CONFIG_CODES[cfg]
    _pair(pkg, cc["gen1"], cc["m"], cc["k"], cc["n"], p, 200_000, enum_cap=8)


@pytest.mark.parametrize("block,warm", [("0", "0"), ("64", "0"), ("300", "3")])
def test_speculation_failures_are_repaired(pkg, dev, monkeypatch, block, warm):
    """No or almost no warm-up: many speculative blocks start wrong; the verified re-run
    passes (and the sequential tail) must still give the host chain's model."""
    monkeypatch.setenv("CVD_LEARN_WARM", warm)
    if block != "0":
        monkeypatch.setenv("CVD_LEARN_BLOCK", block)
    cc = pkg.CONFIG_CODES["m6"]
    _, gpu = _pair(pkg, cc["gen1"], 6, 1, 2, 0.05, 60_000)
    assert gpu.learn_stats["mismatched_blocks"] > 0
    _, gpu = _pair(pkg, pkg.CONFIG_CODES["m2"]["gen1"], 2, 1, 2, 0.05, None)


def test_detector_learns_on_gpu_by_default(pkg, dev):
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    mod = det.model(0.05, 200_000, 200, 1.0, 3)
    assert mod.learn_stats is not None and mod.learn_stats["hash_attempts"] >= 1


def test_sequential_tail_is_one_bounded_launch(pkg, dev, monkeypatch):
    """CVD_LEARN_MAX_PASSES=0: the first failing block and everything after it re-run in
    ONE launch, one lane walking the blocks in order (no per-block launches); the model
    is still the host chain's and the tail's time is reported."""
    monkeypatch.setenv("CVD_LEARN_WARM", "0")
    monkeypatch.setenv("CVD_LEARN_BLOCK", "256")
    monkeypatch.setenv("CVD_LEARN_MAX_PASSES", "0")
    cc = pkg.CONFIG_CODES["m6"]
    _, gpu = _pair(pkg, cc["gen1"], 6, 1, 2, 0.05, 60_000)
    st = gpu.learn_stats
    assert st["mismatched_blocks"] > 0 and st["sequential_blocks"] > 0 and st["sequential_seconds"] > 0.0
    _, gpu = _pair(pkg, pkg.CONFIG_CODES["m2"]["gen1"], 2, 1, 2, 0.05, None)


def test_gpu_learning_falls_back_to_host_chain(pkg, dev):
    """A dense code the GPU chain does not take (n = 4 > 3) still builds through the
    device path: the host chain runs (host_fallback = 1), same model as cvd_model_create."""
    taps = [[[1, 1, 1]], [[1, 0, 1]], [[1, 1, 0]], [[0, 1, 1]]]   # rate 1/4, m = 2
    host, gpu = _pair(pkg, taps, 2, 1, 4, 0.05, None)
    assert gpu.learn_stats["host_fallback"] == 1.0
    det = pkg.Detector(1, 4, 2, taps, device=0)   # the default (GPU-learning) Detector path
    assert det.model(0.05).learn_stats["host_fallback"] == 1.0
    _, gpu = _pair(pkg, pkg.CONFIG_CODES["m2"]["gen1"], 2, 1, 2, 0.05, None)
    assert gpu.learn_stats["host_fallback"] == 0.0
