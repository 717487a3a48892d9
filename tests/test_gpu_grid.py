"""The (N, p) grid in one library call (cvd_mc_run_grid; the loop of
Pd_plotter.py:196-233: N outer, p inner, num_iter trials per point) and the fused
kernel's launch slicing (cvd_mc_run / cvd_mc_fused cut a trial range into launches of
at most 2^28 trials; CVD_MC_FUSED_SLICE lowers the slice so small ranges run the
multi-slice path).  Counts must equal the per-point calls exactly, and the sliced
fused kernel's sums the one-launch sums bit for bit."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SEED = 12345


def _points(det, models, cc, p_list, N_list, lo, hi, **kw):
    out = np.zeros((len(N_list), len(p_list), 2), np.int64)
    for j, N in enumerate(N_list):
        for i, p in enumerate(p_list):
            out[j, i] = det.run_trials(models[i], cc["gen1"], cc["gen2"], N, p, SEED, lo, hi,
                                       **kw)["counts"].cpu().numpy()
    return out


@pytest.mark.parametrize("config,path", [("m2", 0), ("m2", 1), ("m6", 0), ("r23_m4", 0)])
def test_grid_equals_per_point_calls(pkg, config, path):
    """path 0 = PATH_AUTO (m2: the fused kernel; m6: generator + one multi-model detect per
    batch of the p row), 1 = PATH_TABLE (two kernels, one detect per point)"""
    cc = pkg.CONFIG_CODES[config]
    det = pkg.Detector(cc["k"], cc["n"], cc["m"], cc["gen1"], device=0)
    p_list, N_list = [0.02, 0.1, 0.2], [300, 1237]
    ll = 200_000 if config == "m6" else None
    models = [det.model(p, ll, 200, 1.0, SEED) for p in p_list]
    lo, hi = 1_000_003, 1_000_003 + 700          # not whole waves, offset ids
    ref = _points(det, models, cc, p_list, N_list, lo, hi, batch=256, path=path)
    got = det.run_grid(models, cc["gen1"], cc["gen2"], p_list, N_list, SEED, lo, hi, batch=256, path=path)
    assert np.array_equal(got.cpu().numpy(), ref)
    # early decision: the same counts
    early = det.run_grid(models, cc["gen1"], cc["gen2"], p_list, N_list, SEED, lo, hi, batch=256,
                         early_decision=True, path=path)
    assert np.array_equal(early.cpu().numpy(), ref)
    # accumulates into the caller's tensor like cvd_mc_run
    got2 = det.run_grid(models, cc["gen1"], cc["gen2"], p_list, N_list, SEED, lo, hi, batch=256, counts=got,
                        path=path)
    assert np.array_equal(got2.cpu().numpy(), 2 * ref)
    for mdl in models:
        assert mdl.device_error() == 0


def test_grid_workspace_and_null_workspace(pkg):
    """The grid workspace is the largest N's stream buffer, and 0 when every point runs
    the fused kernel (no workspace pointer needed); a two-kernel point without one fails."""
    lib = pkg.lib()
    cc = pkg.CONFIG_CODES["m2"]
    det = pkg.Detector(1, 2, 2, cc["gen1"], device=0)
    g1 = pkg.Code(cc["gen1"], 2, 1, 2)
    mods = [det.model(p, None, 200, 1.0, SEED) for p in (0.05, 0.1)]
    assert all(m.info()["mc_fused"] == 1 for m in mods)
    hs = (ctypes.c_void_p * 2)(*[m.handle.value for m in mods])
    Nv = (ctypes.c_int64 * 2)(100, 10_000)
    assert lib.cvd_mc_grid_workspace_bytes(hs, 2, g1.c, Nv, 2, 4096, pkg.PATH_AUTO) == 0
    assert lib.cvd_mc_grid_workspace_bytes(hs, 2, g1.c, Nv, 2, 4096, pkg.PATH_TABLE) == 2 * \
        lib.cvd_mc_workspace_bytes(g1.c, 10_000, 4096)
    m6 = pkg.CONFIG_CODES["m6"]
    d6 = pkg.Detector(1, 2, 6, m6["gen1"], device=0)
    mod6 = d6.model(0.05, 20_000, 200, 1.0, SEED)
    c6 = pkg.Code(m6["gen1"], 6, 1, 2)
    c62 = pkg.Code(m6["gen2"], 6, 1, 2)
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda:0")
    rc = lib.cvd_mc_run(mod6.handle, c6.c, c62.c, 0.05, 100, SEED, 0, 64, 64, None,
                        ctypes.c_void_p(cnt.data_ptr()), pkg.PATH_AUTO, None)
    assert rc == -1 and b"workspace" in lib.cvd_last_error()


def test_fused_slices_equal_one_launch(pkg, monkeypatch):
    """the fused path is cut into launches of at most 2^28 trials; with the
    slice lowered to 1,000 trials a 5,000-trial range (from id 3e9) runs five launches
    with the one-launch sums and the two-kernel counts."""
    cc = pkg.CONFIG_CODES["m2"]
    det = pkg.Detector(1, 2, 2, cc["gen1"], device=0)
    p, N, lo, hi = 0.092, 2_000, 3_000_000_000, 3_000_005_000
    model = det.model(p, None, 200, 1.0, SEED)
    monkeypatch.delenv("CVD_MC_FUSED_SLICE", raising=False)
    one = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, lo, hi, return_sums=True, fused=True)
    table = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, lo, hi, path=pkg.PATH_TABLE)
    monkeypatch.setenv("CVD_MC_FUSED_SLICE", "1000")
    sl = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, lo, hi, return_sums=True, fused=True)
    auto = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, lo, hi)     # cvd_mc_run, AUTO -> fused
    assert np.array_equal(sl["sums"], one["sums"])
    assert sl["counts"].cpu().tolist() == one["counts"].cpu().tolist() == table["counts"].cpu().tolist() \
        == auto["counts"].cpu().tolist()
