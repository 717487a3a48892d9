"""Chunked detection (csrc/cvd_kernels.hip ck_submit / ck_combine_kernel,
csrc/cvd_k1s.h k1s_wave<XM, true>): a batch too small to fill the device -- the reference's
own call shape, run_experiment with num_iter = 10,000 (Pd_plotter.py:67-75, 199-233) -- has
every sequence's N steps cut into time chunks that start warm-up steps early from D = 0 on
lanes of their own.  A sequence's chunks count only where they join (D at a chunk's start =
the previous chunk's D at its end: the recursion of viterbi_markov.py:139-159 is a function of
D and the word) and its decision (Pd_plotter.py:215, :222) is certain under the rounding
bounds of both summation orders; every other sequence is rerun sequentially.  So the counts
must equal the sequential launch's and the C oracle's EXACTLY -- with chunks that mostly do
not join (no warm-up), with every sequence rerun, ragged N and batches, multi-model launches,
the persistent launch, and at the headline's N = 1e5."""
import numpy as np
import pytest
import torch

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu

SEED = 12345


def _buf(pkg, det, g1, g2, N, p, T, lo=0):
    tag = pkg.grid_tag(N, p)
    r = det.stream_buffer(N, 2 * T)
    det.generate(g1, N, p, SEED, tag, 2 * lo, 2, T, out=r, q0=0, pitch=2 * T)
    det.generate(g2, N, p, SEED, tag, 2 * lo + 1, 2, T, out=r, q0=T, pitch=2 * T)
    return r


@pytest.fixture(scope="module")
def m6(pkg):
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    g1, g2 = pkg.Code(cc["gen1"], 6, 1, 2), pkg.Code(cc["gen2"], 6, 1, 2)
    models = {p: det.model(p, 300_000, 200, 1.0, SEED) for p in (0.01, 0.05, 0.2)}
    return cc, det, g1, g2, models


def _counts(pkg, det, model, r, N, T, **env):
    c = det.detect(model, r, N, 2 * T, T)
    torch.cuda.synchronize()
    return c.cpu().tolist(), pkg._lib.chunk_last()


def _seq_counts(det, model, r, N, T):
    """the unchunked launch's counts (per-sequence sums: sums force the sequential path)"""
    s = torch.empty((2 * T, 2), dtype=torch.float64, device=det.device)
    c = det.detect(model, r, N, 2 * T, T, sums=s)
    s = s.cpu().numpy()
    assert c.cpu().tolist() == [int((s[:T, 0] > s[:T, 1]).sum()), int((s[T:, 0] <= s[T:, 1]).sum())]
    return c.cpu().tolist()


@pytest.mark.parametrize("p,N,T,warm", [(0.05, 20_000, 333, 1152), (0.2, 10_007, 200, 384), (0.01, 20_000, 129, 768),
                                        (0.2, 4_000, 64, 192)])
def test_chunked_counts_equal_sequential(pkg, m6, monkeypatch, p, N, T, warm):
    cc, det, g1, g2, models = m6
    r = _buf(pkg, det, g1, g2, N, p, T)
    ref = _seq_counts(det, models[p], r, N, T)
    monkeypatch.setenv("CVD_CHUNK", "1")
    monkeypatch.setenv("CVD_CHUNK_WARM", str(warm))
    got, st = _counts(pkg, det, models[p], r, N, T)
    assert st["groups"] == 1 and st["C"] >= 2, st
    assert got == ref, (got, ref, st)
    assert models[p].device_error() == 0


def test_chunks_that_do_not_join_are_rerun(pkg, m6, monkeypatch):
    """no warm-up: chunk j starts from D = 0 at its first summed step, so most chunks do not
    join their predecessor; the reruns must restore the exact counts"""
    cc, det, g1, g2, models = m6
    N, T, p = 9_000, 100, 0.2
    r = _buf(pkg, det, g1, g2, N, p, T, lo=5_000)
    ref = _seq_counts(det, models[p], r, N, T)
    monkeypatch.setenv("CVD_CHUNK", "1")
    monkeypatch.setenv("CVD_CHUNK_WARM", "0")
    got, st = _counts(pkg, det, models[p], r, N, T)
    assert st["groups"] == 1 and st["reruns"] > T, st
    assert got == ref


def test_every_sequence_rerun(pkg, m6, monkeypatch):
    cc, det, g1, g2, models = m6
    N, T, p = 6_000, 77, 0.05
    r = _buf(pkg, det, g1, g2, N, p, T, lo=9_000)
    ref = _seq_counts(det, models[p], r, N, T)
    monkeypatch.setenv("CVD_CHUNK", "1")
    monkeypatch.setenv("CVD_CHUNK_WARM", "384")
    monkeypatch.setenv("CVD_CHUNK_REDO_ALL", "1")
    got, st = _counts(pkg, det, models[p], r, N, T)
    assert st["reruns"] == 2 * T, st
    assert got == ref


def test_chunked_persistent_launch(pkg, m6, monkeypatch):
    """more chunk units than resident slots: the single-model chunked launch is persistent"""
    cc, det, g1, g2, models = m6
    N, T, p = 12_000, 300, 0.05
    r = _buf(pkg, det, g1, g2, N, p, T, lo=20_000)
    ref = _seq_counts(det, models[p], r, N, T)
    monkeypatch.setenv("CVD_CHUNK", "1")
    monkeypatch.setenv("CVD_CHUNK_WARM", "192")
    monkeypatch.setenv("CVD_K1S_PERSIST_BLOCKS", "3")   # a tiny persistent grid: the queue drains every unit
    got, st = _counts(pkg, det, models[p], r, N, T)
    assert st["C"] >= 2
    assert got == ref


def test_chunked_multi_model_launch(pkg, m6, monkeypatch):
    """a p row in cvd_detect_multi: the LDS-filter model (p = 0.01) and the others in chunked
    groups; every model's counts equal its sequential launch"""
    cc, det, g1, g2, models = m6
    N = 15_000
    ps, T = [0.01, 0.05, 0.2], [129, 200, 64]
    bufs = [_buf(pkg, det, g1, g2, N, p, t, lo=30_000) for p, t in zip(ps, T)]
    ref = [_seq_counts(det, models[p], r, N, t) for p, r, t in zip(ps, bufs, T)]
    monkeypatch.setenv("CVD_CHUNK", "1")
    monkeypatch.setenv("CVD_CHUNK_WARM", "768")
    cnts = [torch.zeros(2, dtype=torch.int64, device=det.device) for _ in ps]
    det.detect_multi([models[p] for p in ps], bufs, N, [2 * t for t in T], T, cnts)
    st = pkg._lib.chunk_last()
    assert st["groups"] >= 2, st     # the LDS-filter variant apart from the others
    assert [c.cpu().tolist() for c in cnts] == ref


def test_chunked_headline_N_equals_c_oracle(pkg, m6):
    """the default (automatic) chunking at the headline's N = 1e5: counts = the C oracle's"""
    cc, det, g1, g2, models = m6
    N, T, p, lo = 100_000, 256, 0.05, 3_000_000
    res = det.run_trials(models[p], cc["gen1"], cc["gen2"], N, p, SEED, lo, lo + T)
    torch.cuda.synchronize()
    st = pkg._lib.chunk_last()
    assert st["groups"] == 1 and st["C"] >= 2, st
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    cnt, _ = C.Model(c1, p, 300_000, 200, 1.0, SEED).run_trials(c1, c2, N, p, SEED, lo, lo + T, nthreads=16)
    assert res["counts"].cpu().tolist() == [int(x) for x in cnt]


def test_run_experiment_chunked_equals_unchunked(pkg, monkeypatch):
    """the reference's call shape through the drop-in (cvd_mc_run_grid -> cvd_detect_multi):
    the DataFrame with chunking equals the one without"""
    cc = pkg.CONFIG_CODES["m6"]
    args = (1, 2, 6, cc["gen1"], cc["gen2"], 300, [0.02, 0.1], 200_000, 200, 1.0, SEED)
    monkeypatch.setenv("CVD_CHUNK", "0")
    df0 = pkg.run_experiment(*args, N_list=[30_000], early_decision=False)
    monkeypatch.setenv("CVD_CHUNK", "-1")
    df1 = pkg.run_experiment(*args, N_list=[30_000], early_decision=False)
    assert pkg._lib.chunk_last()["groups"] >= 1
    assert df0.equals(df1), (df0, df1)
