"""Walk mode of the specialised m = 6 kernel (cvd_device.h k1b_walk): H1 lanes that sit
in learned rows take their steps from the row records (log P̂1, successor, T_ref count
c) without the ACS, and rebuild the metric vector from the row key when they leave.
Per-trial fp64 sums and counts must equal the lockstep kernel's (CVD_WALK=0) bit for
bit -- and the C oracle's -- at every p of the sweep, for trial counts that are not
whole waves (one wave mixes H1 and H2 lanes), N not a multiple of the 16-step word,
and every schedule extreme (burst of one step, always / never preferring walks)."""
import warnings

import numpy as np
import pytest

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

SEED = 12345


def _m6(pkg):
    cc = pkg.CONFIG_CODES["m6"]
    return cc, pkg.Detector(1, 2, 6, cc["gen1"], device=0)


def _sums(det, model, cc, N, p, t0, t1):
    s = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, t0, t1, return_sums=True)
    return s["sums"], s["counts"].cpu().tolist()


@pytest.mark.parametrize("p", [0.01, 0.02, 0.05, 0.1, 0.2])
def test_walk_equals_lockstep(pkg, monkeypatch, p):
    cc, det = _m6(pkg)
    model = det.model(p, 200_000, 200, 1.0, SEED)
    for N, t0, t1 in [(1237, 0, 300), (4096, 1_000_003, 1_000_003 + 128)]:
        monkeypatch.setenv("CVD_WALK", "0")
        ref, rc = _sums(det, model, cc, N, p, t0, t1)
        monkeypatch.setenv("CVD_WALK", "1")
        got, gc = _sums(det, model, cc, N, p, t0, t1)
        assert np.array_equal(got, ref), (p, N)
        assert gc == rc
    assert model.device_error() == 0      # no walk wave left its loop by the guard


def test_compact_walk_records_equal_full_records(pkg, monkeypatch):
    """The walk's compact 8-B two-step records (log P̂1 as indices into a value table the block
    keeps in LDS beside the filter; cvd_model_info.walk_compact) give the 32-B records' sums
    and counts -- and the lockstep kernel's -- bit for bit, at the headline's p = 0.01 model
    (10^6-step chain: 29,626 rows, 2,110 distinct values)."""
    cc, det = _m6(pkg)
    p = 0.01
    monkeypatch.setenv("CVD_WALK", "1")
    monkeypatch.setenv("CVD_WALK_T2C", "1")
    m1 = pkg.Model(det.dec, p, 1_000_000, 200, 1.0, SEED).upload(0)
    monkeypatch.delenv("CVD_WALK_T2C")
    i1 = m1.info()
    assert i1["walk_compact"] == 1 and i1["lds_filter"] == 1 and i1["walk"] == 1, i1
    m0 = pkg.Model(det.dec, p, 1_000_000, 200, 1.0, SEED).upload(0)
    assert m0.info()["walk_compact"] == 0
    for N, t0, t1 in [(4093, 5, 5 + 900), (20_000, 2_000_001, 2_000_001 + 256)]:
        got, gc = _sums(det, m1, cc, N, p, t0, t1)
        ref, rc = _sums(det, m0, cc, N, p, t0, t1)
        assert not np.isnan(got).any()
        assert np.array_equal(got, ref), N
        assert gc == rc
        monkeypatch.setenv("CVD_WALK", "0")
        lock, lc = _sums(det, m1, cc, N, p, t0, t1)
        monkeypatch.setenv("CVD_WALK", "1")
        assert np.array_equal(got, lock), N
    assert m1.device_error() == 0 and m0.device_error() == 0


@pytest.mark.parametrize("wmin,amin,burst", [("1", "64", "1"), ("64", "1", "3"), ("8", "16", "64")])
def test_walk_schedules(pkg, monkeypatch, wmin, amin, burst):
    """Schedule knobs change only the order of work, never a sum."""
    cc, det = _m6(pkg)
    p = 0.03
    model = det.model(p, 200_000, 200, 1.0, SEED)
    monkeypatch.setenv("CVD_WALK", "0")
    ref, rc = _sums(det, model, cc, 3000, p, 0, 200)
    monkeypatch.setenv("CVD_WALK", "1")
    monkeypatch.setenv("CVD_WALK_WMIN", wmin)
    monkeypatch.setenv("CVD_WALK_AMIN", amin)
    monkeypatch.setenv("CVD_WALK_BURST", burst)
    got, gc = _sums(det, model, cc, 3000, p, 0, 200)
    assert np.array_equal(got, ref)
    assert gc == rc


def test_walk_equals_c_oracle(pkg, monkeypatch):
    cc, det = _m6(pkg)
    p, N, T = 0.02, 5000, 192
    monkeypatch.setenv("CVD_WALK", "1")
    model = det.model(p, 300_000, 200, 1.0, SEED)
    got, gc = _sums(det, model, cc, N, p, 0, T)
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    cnt, sums = C.Model(c1, p, 300_000, 200, 1.0, SEED).run_trials(c1, c2, N, p, SEED, 0, T, sums=True,
                                                                    nthreads=8)
    assert np.array_equal(got, sums)
    assert gc == [int(x) for x in cnt]


@pytest.mark.parametrize("p", [0.01, 0.05])
def test_walk_early_decision_counts(pkg, monkeypatch, p):
    """Early decision in walk mode (each lane stops once certain, checked every 128 of its
    own steps): the full run's counts."""
    cc, det = _m6(pkg)
    model = det.model(p, 200_000, 200, 1.0, SEED)
    monkeypatch.setenv("CVD_WALK", "1")
    full = det.run_trials(model, cc["gen1"], cc["gen2"], 20_000, p, SEED, 0, 640)["counts"].cpu().tolist()
    early = det.run_trials(model, cc["gen1"], cc["gen2"], 20_000, p, SEED, 0, 640,
                           early_decision=True)["counts"].cpu().tolist()
    monkeypatch.setenv("CVD_WALK", "0")
    lock = det.run_trials(model, cc["gen1"], cc["gen2"], 20_000, p, SEED, 0, 640,
                          early_decision=True)["counts"].cpu().tolist()
    assert early == full == lock


def test_walk_flag_follows_row_share(pkg, monkeypatch):
    """cvd_model_info.walk: the bit-sliced kernel runs lockstep at every p by default (round 6:
    p = 0.01 lockstep with the LDS filter 1,300 against 1,472 ms walking), with the whole filter
    in LDS where the rows fit (p = 0.01, 0.02); off for dense models; CVD_WALK forces it."""
    cc, det = _m6(pkg)
    monkeypatch.delenv("CVD_WALK", raising=False)
    monkeypatch.delenv("CVD_LDSF_LOCKSTEP", raising=False)
    lo = det.model(0.01, 1_000_000, 200, 1.0, SEED).info()
    hi = det.model(0.1, 1_000_000, 200, 1.0, SEED).info()
    assert lo["walk"] == 0 and lo["lds_filter"] == 1 and lo["n_rows"] <= 32768
    assert hi["walk"] == 0 and hi["lds_filter"] == 0
    mid = det.model(0.02, 1_000_000, 200, 1.0, SEED).info()   # 70,134 rows: the LDS filter too
    assert mid["walk"] == 0 and mid["lds_filter"] == 1
    monkeypatch.setenv("CVD_WALK", "1")
    assert det.model(0.1, 1_000_000, 200, 1.0, SEED).info()["walk"] == 1
    m2 = pkg.CONFIG_CODES["m2"]
    d2 = pkg.Detector(1, 2, 2, m2["gen1"], device=0)
    monkeypatch.delenv("CVD_WALK")
    assert d2.model(0.05, None, 200, 1.0, SEED).info()["walk"] == 0


def test_lds_filter_equals_global_filter(pkg, monkeypatch):
    """cvd_model_info.lds_filter: models of <= 98,304 rows keep their whole Bloom filter in
    LDS (the lockstep default, and walk mode); the sums equal the global-filter kernel's
    (CVD_NO_LDSF=1: the pre-filter and the L2 filter) and the walking run's."""
    cc, det = _m6(pkg)
    p, N, t0, t1 = 0.01, 3001, 17, 17 + 700
    for v in ("CVD_WALK", "CVD_NO_LDSF", "CVD_LDSF_LOCKSTEP"):
        monkeypatch.delenv(v, raising=False)
    # fresh models (Detector.model keeps one per key): the filter is sized at build, the
    # kernel variant chosen at upload
    lds = pkg.Model(det.dec, p, 300_000, 200, 1.0, SEED).upload(0)
    assert lds.info()["walk"] == 0 and lds.info()["lds_filter"] == 1
    got, gc = _sums(det, lds, cc, N, p, t0, t1)
    monkeypatch.setenv("CVD_NO_LDSF", "1")
    glob = pkg.Model(det.dec, p, 300_000, 200, 1.0, SEED).upload(0)
    assert glob.info()["lds_filter"] == 0
    ref, rc = _sums(det, glob, cc, N, p, t0, t1)
    monkeypatch.delenv("CVD_NO_LDSF")
    monkeypatch.setenv("CVD_WALK", "1")
    walk = pkg.Model(det.dec, p, 300_000, 200, 1.0, SEED).upload(0)
    assert walk.info()["walk"] == 1 and walk.info()["lds_filter"] == 1
    wk, wc = _sums(det, walk, cc, N, p, t0, t1)
    assert np.array_equal(got, ref) and np.array_equal(wk, ref)
    assert gc == rc == wc
    assert pkg.Model(det.dec, 0.1, 300_000, 200, 1.0, SEED).upload(0).info()["lds_filter"] == 0


@pytest.mark.parametrize("how", ["hiprtc", "nojit"])
def test_lds_filter_model_under_jit_fallbacks(pkg, monkeypatch, how):
    """A model built for the LDS-filter kernel (walking, <= 32,768 rows) stays exact when the
    kernel comes from the hipRTC fallback (the variant's -D defines become #define lines) or
    when there is no specialised kernel at all (the library's table-driven butterfly kernel
    reads the global filter copy with the 4,096-pattern table)."""
    cc, det = _m6(pkg)
    p, N, t0, t1 = 0.01, 2500, 5, 5 + 320
    for v in ("CVD_WALK", "CVD_NO_LDSF", "CVD_JIT_VIA", "CVD_NO_JIT"):
        monkeypatch.delenv(v, raising=False)
    ref_model = pkg.Model(det.dec, p, 300_000, 200, 1.0, SEED).upload(0)
    assert ref_model.info()["lds_filter"] == 1
    ref, rc = _sums(det, ref_model, cc, N, p, t0, t1)
    if how == "hiprtc":
        monkeypatch.setenv("CVD_JIT_VIA", "hiprtc")
    else:
        monkeypatch.setenv("CVD_NO_JIT", "1")
    with warnings.catch_warnings():   # (no JIT: upload warns that the table-driven kernel runs)
        warnings.simplefilter("ignore", RuntimeWarning)
        alt = pkg.Model(det.dec, p, 300_000, 200, 1.0, SEED).upload(0)
    inf = alt.info()
    # info.walk reports what runs: walk mode needs the specialised kernel
    if how == "hiprtc":
        # (the bit-sliced form k1s if the hipRTC compiler takes it, else the butterfly kernel)
        # (walk mode only where the butterfly kernel is what runs: the bit-sliced one stays lockstep)
        assert inf["explicit_kernel"] in (4, 5) and inf["lds_filter"] == 1
        assert inf["walk"] == (1 if inf["explicit_kernel"] == 4 else 0)
    else:
        assert inf["explicit_kernel"] == 3 and inf["lds_filter"] == 0 and inf["walk"] == 0
    got, gc = _sums(det, alt, cc, N, p, t0, t1)
    assert np.array_equal(got, ref)
    assert gc == rc


def test_walk_guard_flag_is_reported(pkg, monkeypatch):
    """The walk loop's guard (never reached in a correct schedule) sets the model's error
    flag; a kernel built with a zero guard bound trips it at once, and run_trials (sums)
    raises instead of returning void counts."""
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    monkeypatch.setenv("CVD_JIT_DEFINES", "-DCVD_WALK_GUARD=0")
    monkeypatch.setenv("CVD_WALK", "1")
    model = pkg.Model(det.dec, 0.01, 300_000, 200, 1.0, 7).upload(0)
    assert model.info()["walk"] == 1
    with pytest.raises(pkg.CvdError, match="scheduler guard"):
        det.run_trials(model, cc["gen1"], cc["gen2"], 2000, 0.01, 7, 0, 256, return_sums=True)
    assert model.device_error() == 0          # the flag was read and cleared


@pytest.mark.parametrize("p,walk", [(0.01, "1"), (0.02, "1"), (0.05, "0"), (0.2, "0")])
def test_persistent_launch_equals_block_launch(pkg, monkeypatch, p, walk):
    """The k1s work-queue launch (cvd_k1s.h k1s_body: one block per resident slot, waves
    taking 64 sequences at a time) gives the block launch's sums and counts, lockstep and walk
    mode, trial counts that leave a partial last unit and an odd number of units.  Capping it
    at 2 blocks (CVD_K1S_PERSIST_BLOCKS) makes these small launches go through the queue."""
    cc, det = _m6(pkg)
    model = det.model(p, 200_000, 200, 1.0, SEED)
    monkeypatch.setenv("CVD_WALK", walk)
    for N, t0, t1 in [(1237, 0, 1500), (2000, 77, 77 + 2111)]:
        monkeypatch.setenv("CVD_K1S_PERSIST", "0")
        ref, rc = _sums(det, model, cc, N, p, t0, t1)
        monkeypatch.setenv("CVD_K1S_PERSIST", "1")
        monkeypatch.setenv("CVD_K1S_PERSIST_BLOCKS", "2")
        got, gc = _sums(det, model, cc, N, p, t0, t1)
        monkeypatch.delenv("CVD_K1S_PERSIST_BLOCKS")
        assert not np.isnan(got).any()
        assert np.array_equal(got, ref), (p, N)
        assert gc == rc
    assert model.device_error() == 0


@pytest.mark.parametrize("p", [0.05, 0.2])
def test_mixed_unit_order_equals_in_order(pkg, monkeypatch, p):
    """Lockstep units alternating H1 and H2 waves (ExpArgs.mix, CVD_K1S_MIX; the default where
    rows < learn_len / 2) give the in-order launch's sums and counts, persistent and block
    launches, a partial last unit and an odd number of units."""
    cc, det = _m6(pkg)
    model = det.model(p, 200_000, 200, 1.0, SEED)
    monkeypatch.setenv("CVD_WALK", "0")
    for N, t0, t1, blocks in [(1237, 0, 1500, "2"), (2000, 77, 77 + 2111, "0")]:
        monkeypatch.setenv("CVD_K1S_MIX", "0")
        monkeypatch.setenv("CVD_K1S_PERSIST_BLOCKS", blocks)
        ref, rc = _sums(det, model, cc, N, p, t0, t1)
        monkeypatch.setenv("CVD_K1S_MIX", "1")
        got, gc = _sums(det, model, cc, N, p, t0, t1)
        assert not np.isnan(got).any()
        assert np.array_equal(got, ref), (p, N)
        assert gc == rc
    assert model.device_error() == 0


@pytest.mark.parametrize("p,walk", [(0.01, "1"), (0.1, "0")])
def test_persistent_launch_early_decision_counts(pkg, monkeypatch, p, walk):
    """Counts-only early decision under the work-queue launch (a wave that has decided its
    64 trials takes the next unit): the block launch's counts, which equal the full run's."""
    cc, det = _m6(pkg)
    model = det.model(p, 200_000, 200, 1.0, SEED)
    monkeypatch.setenv("CVD_WALK", walk)
    args = (model, cc["gen1"], cc["gen2"], 20_000, p, SEED, 3, 3 + 2500)
    monkeypatch.setenv("CVD_K1S_PERSIST", "0")
    full = det.run_trials(*args)["counts"].cpu().tolist()
    block = det.run_trials(*args, early_decision=True)["counts"].cpu().tolist()
    monkeypatch.setenv("CVD_K1S_PERSIST", "1")
    monkeypatch.setenv("CVD_K1S_PERSIST_BLOCKS", "2")
    pers = det.run_trials(*args, early_decision=True)["counts"].cpu().tolist()
    assert pers == block == full
    assert model.device_error() == 0
