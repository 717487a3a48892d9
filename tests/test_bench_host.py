"""bench.py's sweep weighting (CPU, no GPU): the headline weighs the six p of the sweep
equally whatever --steps is (Pd_plotter.py:199-233 runs num_iter trials
at every p)."""
import importlib.util
import os

import pytest

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


PER_P_MS = [1974.0, 2348.0, 2629.0, 2737.0, 2672.0, 2632.0]   # profiles/r04d/perp6.json (detector only)


def test_per_p_value_independent_of_step_count():
    b = _bench()
    B = 2_621_440
    ref = B / (sum(PER_P_MS) / 6 * 1e-3)
    for steps in (6, 8, 12, 20, 25):
        ms = [PER_P_MS[s % 6] for s in range(steps)]
        v, cov = b.sweep_value(ms, 6, B, 1)
        assert v == pytest.approx(ref, rel=1e-12) and cov == list(range(6)), steps
        # the unweighted wall rate over-weights the p that get an extra step
        wall = steps * B / (sum(ms) * 1e-3)
        assert (steps % 6 == 0) == (wall == pytest.approx(ref, rel=1e-12))


def test_per_p_value_scales_with_ranks_and_reports_coverage():
    b = _bench()
    v1, _ = b.sweep_value(PER_P_MS, 6, 1000, 1)
    v8, _ = b.sweep_value(PER_P_MS, 6, 1000, 8)
    assert v8 == pytest.approx(8 * v1)
    v, cov = b.sweep_value(PER_P_MS[:4], 6, 1000, 1)     # fewer steps than p: the covered p only
    assert cov == [0, 1, 2, 3] and v == pytest.approx(1000 / (sum(PER_P_MS[:4]) / 4 * 1e-3))


def test_sweep_all_value_is_trials_over_time():
    b = _bench()
    v, cov = b.sweep_value([4000.0, 4100.0], 6, 655_360, 2, sweep_all=True)
    assert v == pytest.approx(2 * 6 * 655_360 / (4050.0 * 1e-3)) and cov == list(range(6))
    with pytest.raises(ValueError):
        b.sweep_value([], 6, 1, 1)


def test_box_record_parsing(monkeypatch):
    """The box record (bench.py box_identity / ClockSampler): the visible cards follow the
    HIP visibility list, and the medians under load parse rocm-smi's clock / power strings."""
    b = _bench()
    d = {"card0": {}, "card1": {}, "card2": {}, "system": {}}
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2")
    assert b._visible_cards(d) == ["card2"]
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    assert b._visible_cards(d) == ["card0", "card1", "card2"]
    s = b.ClockSampler(period=1.0)
    s.samples = [{"card0": {"sclk clock speed:": "(2383Mhz)", "Current Socket Graphics Package Power (W)": "1344.0",
                            "Temperature (Sensor junction) (C)": "58.0", "Card SKU": "N/A"}},
                 {"card0": {"sclk clock speed:": "(2100Mhz)", "Current Socket Graphics Package Power (W)": "1300.0",
                            "Temperature (Sensor junction) (C)": "57.0"}},
                 {"card0": {"sclk clock speed:": "(2390Mhz)", "Current Socket Graphics Package Power (W)": "1350.0",
                            "Temperature (Sensor junction) (C)": "59.0"}}]
    med = s.summary()["median_under_load"]["card0"]
    assert med["sclk clock speed:"] == 2383.0
    assert med["Current Socket Graphics Package Power (W)"] == 1344.0
    assert med["Temperature (Sensor junction) (C)"] == 58.0
    assert "Card SKU" not in med
