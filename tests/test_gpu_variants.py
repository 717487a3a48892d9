"""The dense-table timing variants of VERDICT r04 items 5 and 6 compute the same sums as the
default kernels and the C oracle, bit for bit (their A/B timings: profiles/r05m_c1/,
profiles/r05n_c3/):
  * C1's fused kernel with kCp interleaved copies of its LDS image (CVD_C1_COPIES,
    cvd_kernels.hip LdsModel kCp);
  * C3's table detector with the records in LDS and log P̂1 gathered from global memory
    (CVD_T16_LPG=1, LdsModel kLpG)."""
import numpy as np
import pytest

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu
SEED = 12345


def _codes(pkg, cfg):
    cc = pkg.CONFIG_CODES[cfg]
    k, n, m = cc["k"], cc["n"], cc["m"]
    return cc, k, n, m, C.Code(cc["gen1"], m, k, n), C.Code(cc["gen2"], m, k, n)


@pytest.mark.parametrize("copies", ["4", "8", "16"])
def test_c1_fused_image_copies_equal_oracle(pkg, monkeypatch, copies):
    cc, k, n, m, c1, c2 = _codes(pkg, "m2")
    N, p, t0, t1 = 10_000, 0.05, 5, 5 + 300
    det = pkg.Detector(k, n, m, cc["gen1"], device=0)
    model = det.model(p, None, 200, 1.0, SEED)
    _, want = C.Model(c1, p, None, 200, 1.0, SEED).run_trials(c1, c2, N, p, SEED, t0, t1, sums=True)
    monkeypatch.setenv("CVD_C1_COPIES", copies)
    got = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, t0, t1, return_sums=True, fused=True)
    assert np.array_equal(got["sums"], want)


def test_c3_log_p1_from_global_equals_oracle(pkg, monkeypatch):
    cc, k, n, m, c1, c2 = _codes(pkg, "r23_m4")
    N, p, t0, t1 = 100_000, 0.05, 0, 48
    det = pkg.Detector(k, n, m, cc["gen1"], device=0)
    model = det.model(p, None, 200, 1.0, SEED)
    cm = C.Model(c1, p, None, 200, 1.0, SEED)
    counts, want = cm.run_trials(c1, c2, N, p, SEED, t0, t1, sums=True)
    monkeypatch.setenv("CVD_T16_LPG", "1")
    got = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, t0, t1, path=pkg.PATH_TABLE, return_sums=True)
    assert np.array_equal(got["sums"], want)
    assert tuple(got["counts"].cpu().tolist()) == tuple(int(x) for x in counts)
