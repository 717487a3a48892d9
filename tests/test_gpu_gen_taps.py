"""The bit-parallel encoder's unrolled tap lists (ChunkEncoder kT > 0: per output a fixed
list of window shifts padded with shifts onto empty lanes, instead of the scalar loop over
the tap mask) must give the same received streams as the loop form (CVD_GEN_TAP_LOOP=1),
the per-step generic kernel and the oracle, for every list length the host picks
(3, 4, 5, 6, 8 and the loop beyond 8 taps), for rate 1/2, 1/3 and 2/3 encoders; and the
fused trial kernel (C1's rate 1/2 variants kT = 3, 5) the same sums as its loop form."""
import numpy as np
import pytest
import torch

from oracle import philox
from oracle import restatement as R
from test_gpu_parity import unpack_words

pytestmark = pytest.mark.gpu

SEED = 2024


def _random_code(rng, k, n, m, ntap_target=None):
    """taps[j][i][d] (reference layout); at least one tap per output"""
    taps = np.zeros((n, k, m + 1), np.int64)
    for j in range(n):
        while taps[j].sum() == 0:
            taps[j] = rng.integers(0, 2, size=(k, m + 1))
    if ntap_target is not None:   # output 0 with exactly ntap_target taps
        flat = np.zeros(k * (m + 1), np.int64)
        flat[rng.choice(k * (m + 1), size=ntap_target, replace=False)] = 1
        taps[0] = flat.reshape(k, m + 1)
    return taps.tolist()


CASES = []
_rng = np.random.default_rng(7)
for (k, n, m, nt) in [(1, 2, 2, 3), (1, 2, 3, 4), (1, 2, 6, 5), (1, 2, 7, 6), (1, 2, 8, 8), (1, 2, 8, 9),
                      (1, 3, 4, 3), (1, 3, 6, 6), (1, 3, 8, 9),
                      (2, 3, 4, 6), (2, 3, 5, 4), (2, 3, 7, 8), (2, 3, 8, 10)]:
    CASES.append((k, n, m, nt, _random_code(_rng, k, n, m, nt)))


@pytest.mark.parametrize("k,n,m,nt,taps", CASES, ids=[f"k{c[0]}n{c[1]}m{c[2]}t{c[3]}" for c in CASES])
def test_tap_lists_equal_loop_generic_oracle(pkg, k, n, m, nt, taps, monkeypatch):
    det = pkg.Detector(k, n, m, taps, device=0)
    N, p, count = 4_099, 0.09, 200
    tag = philox.grid_tag(N, p)
    monkeypatch.delenv("CVD_GEN_TAP_LOOP", raising=False)
    lists = det.generate(taps, N, p, SEED, tag, 11, 3, count)
    monkeypatch.setenv("CVD_GEN_TAP_LOOP", "1")
    loop = det.generate(taps, N, p, SEED, tag, 11, 3, count)
    monkeypatch.delenv("CVD_GEN_TAP_LOOP")
    monkeypatch.setenv("CVD_GEN_GENERIC", "1")
    generic = det.generate(taps, N, p, SEED, tag, 11, 3, count)
    monkeypatch.delenv("CVD_GEN_GENERIC")
    assert torch.equal(lists, loop)
    assert torch.equal(lists, generic)
    got = unpack_words(lists, n, N)
    for q in (0, 97, count - 1):
        np.testing.assert_array_equal(got[:, q], R.received_stream(taps, m, k, n, N, p, SEED, tag, 11 + 3 * q))


@pytest.mark.parametrize("gen1,gen2", [
    ([[[1, 1, 1]], [[1, 0, 1]]], [[[1, 0, 1]], [[1, 1, 1]]]),                       # m2: 3 taps -> kT 3
    ([[[1, 1, 0, 1]], [[1, 1, 1, 1]]], [[[1, 1, 1, 1]], [[1, 1, 0, 1]]]),             # (15, 17): 4 -> kT 5
])
def test_fused_tap_lists_equal_loop(pkg, gen1, gen2, monkeypatch):
    m = len(gen1[0][0]) - 1
    det = pkg.Detector(1, 2, m, gen1, device=0)
    p, N, lo, hi = 0.06, 3_001, 5_000, 5_000 + 900
    model = det.model(p, None, 200, 1.0, SEED)
    if not model.info()["mc_fused"]:
        pytest.skip("model not LDS-resident for the fused kernel")
    monkeypatch.delenv("CVD_GEN_TAP_LOOP", raising=False)
    a = det.run_trials(model, gen1, gen2, N, p, SEED, lo, hi, return_sums=True, fused=True)
    monkeypatch.setenv("CVD_GEN_TAP_LOOP", "1")
    b = det.run_trials(model, gen1, gen2, N, p, SEED, lo, hi, return_sums=True, fused=True)
    monkeypatch.delenv("CVD_GEN_TAP_LOOP")
    t = det.run_trials(model, gen1, gen2, N, p, SEED, lo, hi, path=pkg.PATH_TABLE)
    assert np.array_equal(a["sums"], b["sums"])
    assert a["counts"].cpu().tolist() == b["counts"].cpu().tolist() == t["counts"].cpu().tolist()
