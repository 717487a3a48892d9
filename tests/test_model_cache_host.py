"""On-disk model cache (SURVEY.md §5 "Checkpoint": the reference memoises P̂1 per
learning key with @lru_cache, Pd_plotter.py:123-127).  Host-only: a model written
by cvd_model_save and read back by cvd_model_load has the same rows, log P̂1,
dense P̂1 and row-table geometry as the freshly learned one.  No GPU."""
import os

import numpy as np
import pytest

from conftest import code_of


def _same(a, b):
    ia, ib = a.info(), b.info()
    for f in ("kind", "k", "n", "m", "S", "n_rows", "learn_len_eff", "hash_capacity", "max_probe",
              "logp1_unseen", "explicit_kernel"):
        assert ia[f] == ib[f], f
    la, ka = a.rows()
    lb, kb = b.rows()
    assert np.array_equal(la, lb) and np.array_equal(ka, kb)
    if ia["kind"] == 0:
        assert np.array_equal(a.dense_P1(), b.dense_P1())


@pytest.mark.parametrize("name,p,learn_len", [("m2_75", 0.05, None), ("r23_m4", 0.1, None),
                                              ("m6_133_171", 0.05, 30000)])
def test_save_load_roundtrip(pkg, golden, tmp_path, name, p, learn_len):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    code = pkg.Code(taps, m, k, n)
    a = pkg.Model(code, p, learn_len, 200, 1.0, 77)
    path = tmp_path / "model.bin"
    a.save(path)
    b = pkg.Model.load(code, path)
    _same(a, b)


def test_cache_dir_reuses_learned_model(pkg, golden, tmp_path, monkeypatch):
    z, meta = golden
    k, n, m, taps = code_of(meta, "m6_133_171")
    code = pkg.Code(taps, m, k, n)
    monkeypatch.setenv("CVD_MODEL_CACHE", str(tmp_path))
    a = pkg.Model(code, 0.02, 20000, 200, 1.0, 5)
    assert not a.from_cache and len(os.listdir(tmp_path)) == 1
    b = pkg.Model(code, 0.02, 20000, 200, 1.0, 5)
    assert b.from_cache
    _same(a, b)
    c = pkg.Model(code, 0.02, 20000, 200, 1.0, 6)          # another seed: another key
    assert not c.from_cache and len(os.listdir(tmp_path)) == 2
    monkeypatch.setenv("CVD_MODEL_CACHE", "off")
    assert not pkg.Model(code, 0.02, 20000, 200, 1.0, 5).from_cache


def test_load_rejects_foreign_file(pkg, tmp_path):
    bad = tmp_path / "x.bin"
    bad.write_bytes(b"CVDMnot a model")
    code = pkg.Code([[[1, 1, 1]], [[1, 0, 1]]], 2, 1, 2)
    with pytest.raises(pkg.CvdError):
        pkg.Model.load(code, bad)


def test_concurrent_saves_of_one_key(pkg, golden, tmp_path):
    """Ranks sharing a cache directory save the same model at once: every save
    succeeds (unique tmp names, atomic rename) and the file loads."""
    import threading
    z, meta = golden
    k, n, m, taps = code_of(meta, "m2_75")
    code = pkg.Code(taps, m, k, n)
    a = pkg.Model(code, 0.05, None, 200, 1.0, 9)
    path = tmp_path / "same.bin"
    errs = []

    def save():
        try:
            for _ in range(20):
                a.save(path)
        except Exception as e:   # pragma: no cover - the failure being tested for
            errs.append(e)

    th = [threading.Thread(target=save) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    assert [f for f in os.listdir(tmp_path)] == ["same.bin"]   # no tmp files left behind
    _same(a, pkg.Model.load(code, path))


def test_unwritable_cache_warns_instead_of_failing(pkg, golden, tmp_path, monkeypatch):
    z, meta = golden
    k, n, m, taps = code_of(meta, "m2_75")
    code = pkg.Code(taps, m, k, n)
    monkeypatch.setenv("CVD_MODEL_CACHE", str(tmp_path))
    key = pkg.detector.model_cache_key(code, 0.05, None, 200, 1.0, 4, pkg.detector.DEFAULT_ENUM_CAP,
                                       pkg.detector.DEFAULT_SPARSE_LEARN_LEN)
    (tmp_path / key).mkdir()          # the cache file's name is taken by a directory
    with pytest.warns(RuntimeWarning, match="model cache not written"):
        mod = pkg.Model(code, 0.05, None, 200, 1.0, 4)
    assert not mod.from_cache and mod.info()["S"] == 31


def test_load_rejects_corrupt_successor_and_foreign_code(pkg, golden, tmp_path):
    z, meta = golden
    k, n, m, taps = code_of(meta, "m6_133_171")
    code = pkg.Code(taps, m, k, n)
    a = pkg.Model(code, 0.05, 20000, 200, 1.0, 3)
    path = tmp_path / "m.bin"
    a.save(path)
    raw = bytearray(path.read_bytes())
    n = a.info()["n_rows"]
    o = len(raw) - 8 * n - 8 - 8       # the last successor entry (the visits vector follows it)
    raw[o:o + 8] = np.int64(n + 5).tobytes()   # out of range
    bad = tmp_path / "bad.bin"
    bad.write_bytes(bytes(raw))
    with pytest.raises(pkg.CvdError, match="corrupt"):
        pkg.Model.load(code, bad)
    other = pkg.Code([[[1, 1, 1, 1, 0, 0, 1]], [[1, 0, 1, 1, 0, 1, 1]]], 6, 1, 2)
    with pytest.raises(pkg.CvdError, match="another code"):
        pkg.Model.load(other, path)
