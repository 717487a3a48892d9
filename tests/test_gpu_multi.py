"""Several models in one launch (cvd_detect_multi; cvd_device.h k1b_multi): the p sweep's
batches, one learned P̂1 per p (Pd_plotter.py:123-169, 199-233), detected with the models
that share the specialised kernel variant in ONE launch.  Per-trial sums and counts must
equal separate cvd_detect calls bit for bit -- for walking and lockstep models, the
LDS-filter variant (which cannot share a launch with the others and runs on its own),
batches that are not whole blocks, per-model sequence counts that differ, early
decision -- and the C oracle's."""
import numpy as np
import pytest
import torch

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

SEED = 12345


def _setup(pkg, ps, N, T, lo=0, ll=300_000):
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    models = [det.model(p, ll, 200, 1.0, SEED) for p in ps]
    g1, g2 = pkg.Code(cc["gen1"], 6, 1, 2), pkg.Code(cc["gen2"], 6, 1, 2)
    bufs = []
    for p, t in zip(ps, T):
        tag = pkg.grid_tag(N, p)
        r = det.stream_buffer(N, 2 * t)
        det.generate(g1, N, p, SEED, tag, 2 * lo, 2, t, out=r, q0=0, pitch=2 * t)
        det.generate(g2, N, p, SEED, tag, 2 * lo + 1, 2, t, out=r, q0=t, pitch=2 * t)
        bufs.append(r)
    return cc, det, models, bufs


def test_multi_equals_separate_launches(pkg):
    ps = [0.01, 0.02, 0.05, 0.1, 0.2]
    T = [333, 700, 129, 64, 1000]                 # not whole blocks, different per model
    N = 3001
    cc, det, models, bufs = _setup(pkg, ps, N, T)
    inf = [m.info() for m in models]
    assert inf[0]["lds_filter"] == 1 and inf[-1]["lds_filter"] == 0
    groups = det.multi_groups(models)
    # runs of one variant, in order; the LDS-filter models apart from the others
    assert sum(groups, []) == list(range(len(ps))) and max(len(g) for g in groups) >= 3, groups
    for g in groups:
        assert len({inf[i]["lds_filter"] for i in g}) == 1
    ref_s, ref_c = [], []
    for m, r, t in zip(models, bufs, T):
        s = torch.full((2 * t, 2), float("nan"), dtype=torch.float64, device=det.device)
        c = det.detect(m, r, N, 2 * t, t, sums=s)
        ref_s.append(s.cpu().numpy())
        ref_c.append(c.cpu().tolist())
    sums = [torch.full((2 * t, 2), float("nan"), dtype=torch.float64, device=det.device) for t in T]
    cnts = [torch.zeros(2, dtype=torch.int64, device=det.device) for _ in T]
    det.detect_multi(models, bufs, N, [2 * t for t in T], T, cnts, sums=sums)
    for i in range(len(ps)):
        assert np.array_equal(sums[i].cpu().numpy(), ref_s[i]), ps[i]
        assert cnts[i].cpu().tolist() == ref_c[i], ps[i]
    early = [torch.zeros(2, dtype=torch.int64, device=det.device) for _ in T]
    det.detect_multi(models, bufs, N, [2 * t for t in T], T, early, early_decision=True)
    assert [c.cpu().tolist() for c in early] == ref_c
    for m in models:
        assert m.device_error() == 0


def test_multi_equals_c_oracle(pkg):
    """The merged launch of four lockstep and walking models against the C oracle's
    independent restatement (learning chain, rows, recursion, fp64 sums)."""
    ps = [0.02, 0.05, 0.1, 0.15]
    N, T, lo = 2000, [96] * 4, 1_000_000
    cc, det, models, bufs = _setup(pkg, ps, N, T, lo=lo, ll=200_000)
    sums = [torch.full((2 * t, 2), float("nan"), dtype=torch.float64, device=det.device) for t in T]
    cnts = [torch.zeros(2, dtype=torch.int64, device=det.device) for _ in T]
    det.detect_multi(models, bufs, N, [2 * t for t in T], T, cnts, sums=sums)
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    for i, p in enumerate(ps):
        cnt, s = C.Model(c1, p, 200_000, 200, 1.0, SEED).run_trials(c1, c2, N, p, SEED, lo, lo + T[i], sums=True,
                                                                    nthreads=8)
        got = sums[i].cpu().numpy()
        got4 = np.concatenate([got[:T[i]], got[T[i]:]], axis=1)
        assert np.array_equal(got4, s), p
        assert cnts[i].cpu().tolist() == [int(x) for x in cnt], p


def test_multi_disabled_and_single_model(pkg, monkeypatch):
    """CVD_NO_MULTI=1 and one-model calls take the separate-launch path: same counts."""
    ps = [0.05, 0.1]
    N, T = 1500, [200, 300]
    cc, det, models, bufs = _setup(pkg, ps, N, T)
    a = [torch.zeros(2, dtype=torch.int64, device=det.device) for _ in T]
    det.detect_multi(models, bufs, N, [2 * t for t in T], T, a)
    monkeypatch.setenv("CVD_NO_MULTI", "1")
    assert det.multi_groups(models) == [[0], [1]]
    b = [torch.zeros(2, dtype=torch.int64, device=det.device) for _ in T]
    det.detect_multi(models, bufs, N, [2 * t for t in T], T, b)
    c = det.detect_multi(models[:1], bufs[:1], N, [2 * T[0]], T[:1],
                         [torch.zeros(2, dtype=torch.int64, device=det.device)])
    assert [x.cpu().tolist() for x in a] == [x.cpu().tolist() for x in b]
    assert c[0].cpu().tolist() == a[0].cpu().tolist()


def test_multi_runs_persistent_batches_alone(pkg, monkeypatch):
    """A model whose batch is past the persistent launch's capacity (cvd_model_info.
    persist_seqs; capped at 2 blocks here so that small batches cross it) is launched alone
    and persistently, the rest merged; sums and counts equal the all-merged block launch, and
    multi_groups (bench.py's per-launch timing) gives the same split."""
    ps = [0.02, 0.05, 0.1, 0.2]
    T = [1500, 300, 2100, 700]
    N = 2001
    # (one kernel variant for all four: p = 0.02's rows would otherwise take the LDS filter)
    monkeypatch.setenv("CVD_LDSF_LOCKSTEP", "0")
    cc, det, models, bufs = _setup(pkg, ps, N, T)
    nseq = [2 * t for t in T]

    def run():
        sums = [torch.full((2 * t, 2), float("nan"), dtype=torch.float64, device=det.device) for t in T]
        cnts = [torch.zeros(2, dtype=torch.int64, device=det.device) for _ in T]
        det.detect_multi(models, bufs, N, nseq, T, cnts, sums=sums)
        return [s.cpu().numpy() for s in sums], [c.cpu().tolist() for c in cnts]

    monkeypatch.setenv("CVD_K1S_PERSIST", "0")
    assert all(m.info()["persist_seqs"] == 0 for m in models)
    assert det.multi_groups(models, nseq) == [[0, 1, 2, 3]]
    ref_s, ref_c = run()
    monkeypatch.setenv("CVD_K1S_PERSIST", "1")
    monkeypatch.setenv("CVD_K1S_PERSIST_BLOCKS", "2")
    cap = models[0].info()["persist_seqs"]
    assert cap == 2 * 1024
    alone = [i for i, s in enumerate(nseq) if s > cap]
    assert alone == [0, 2]
    assert det.multi_groups(models, nseq) == [[0], [1], [2], [3]]
    got_s, got_c = run()
    for i in range(len(ps)):
        assert not np.isnan(got_s[i]).any()
        assert np.array_equal(got_s[i], ref_s[i]), ps[i]
    assert got_c == ref_c
