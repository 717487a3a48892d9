"""Build-time variants of the code-specialised m = 6 detector kernel (CVD_JIT_DEFINES,
csrc/cvd_rtc.cpp) must give per-trial fp64 sums bit-identical to the default kernel
and to the C oracle: the eager key normalisation (CVD_K1B_LAZYKEY=0; the default
keeps the key offset by the step minimum and folds the offset into the hash), and the
lookup-load placement knob."""
import numpy as np
import pytest
import torch

from oracle import c_oracle as C

pytestmark = pytest.mark.gpu
SEED = 12345


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda", 0)


def _sums(pkg, det, cc, p, N, T, t0, defines, monkeypatch):
    monkeypatch.setenv("CVD_JIT_DEFINES", defines)
    model = pkg.Model(det.dec, p, None, 200, 1.0, SEED).upload(0)
    monkeypatch.delenv("CVD_JIT_DEFINES")
    assert model.jit_status()[0] == 1, model.jit_status()
    return det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, t0, t0 + T, return_sums=True)["sums"]


@pytest.mark.parametrize("p", [0.01, 0.1])
def test_lazy_key_variants_bit_identical(pkg, dev, p, monkeypatch):
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    N, T, t0 = 20_000, 2048, 777
    ref = _sums(pkg, det, cc, p, N, T, t0, "", monkeypatch)
    for v in ("-DCVD_K1B_LAZYKEY=0", "-DCVD_K1B_LAZYKEY=1", "-DCVD_K1B_MID=1"):
        got = _sums(pkg, det, cc, p, N, T, t0, v, monkeypatch)
        assert np.array_equal(got, ref), v
    # and the C oracle (independent restatement of the sparse-model policy) on a few trials
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    cm = C.Model(c1, p, None, 200, 1.0, SEED)
    _, s_cpu = cm.run_trials(c1, c2, N, p, SEED, t0, t0 + 16, sums=True)
    assert np.array_equal(ref[:16], s_cpu)


def _dir_sums(pkg, det, cc, p, N, T, t0, env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    model = pkg.Model(det.dec, p, None, 200, 1.0, SEED).upload(0)
    for k in env:
        monkeypatch.delenv(k)
    return model, det.run_trials(model, cc["gen1"], cc["gen2"], N, p, SEED, t0, t0 + T, return_sums=True)["sums"]


@pytest.mark.parametrize("p", [0.02, 0.1])
def test_directory_layouts_bit_identical(pkg, dev, p, monkeypatch):
    """Directory layouts (csrc/cvd_host.cpp build_hash): key and record in one slot
    (default) or in two arrays (CVD_SLOT_IL=0), at load 1/16 (default) and 1/2
    (CVD_DIR_LOAD_LOG2=1: most hits probe past the home slot)."""
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    N, T, t0 = 20_000, 2048, 4242
    m0, ref = _dir_sums(pkg, det, cc, p, N, T, t0, {}, monkeypatch)
    assert m0.info()["hash_capacity"] >= 16 * m0.info()["n_rows"]
    for env in ({"CVD_SLOT_IL": "0"}, {"CVD_DIR_LOAD_LOG2": "1"}, {"CVD_SLOT_IL": "0", "CVD_DIR_LOAD_LOG2": "1"}):
        mv, got = _dir_sums(pkg, det, cc, p, N, T, t0, env, monkeypatch)
        if "CVD_DIR_LOAD_LOG2" in env:
            assert mv.info()["hash_capacity"] < 4 * mv.info()["n_rows"] and mv.info()["max_probe"] > 1
        assert np.array_equal(got, ref), env
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    cm = C.Model(c1, p, None, 200, 1.0, SEED)
    _, s_cpu = cm.run_trials(c1, c2, N, p, SEED, t0, t0 + 16, sums=True)
    assert np.array_equal(ref[:16], s_cpu)


def test_prebuilt_jit_objects_are_loaded(pkg, dev, tmp_path):
    """__graft_entry__.build() compiles the m = 6 code's default variants into the library's
    prebuilt cache (cvd_jit_prebuild -> <package>/lib/jit); a fresh process with an EMPTY user
    JIT cache must load them at model upload -- the lockstep (pre-filter) and walking (LDS
    filter) variants -- and compile nothing (the user cache stays empty)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    jit = os.path.join(root, "detecting-convolutional-codes-via-markovian-statistics_amd", "lib", "jit")
    if not os.path.isdir(jit) or not os.listdir(jit):
        pytest.skip("no prebuilt JIT objects (build() not run)")
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from __graft_entry__ import load_package\n"
            "pkg = load_package(); cc = pkg.CONFIG_CODES['m6']\n"
            "det = pkg.Detector(1, 2, 6, cc['gen1'], device=0)\n"
            "for p in (0.01, 0.05):\n"
            "    m = det.model(p, 1000000, 200, 1.0, 12345); s = m.jit_status()\n"
            "    assert s[0] == 1, s\n"
            "    print(p, m.info()['lds_filter'], pkg.KERNEL_NAMES[m.info()['explicit_kernel']])\n") % root
    env = dict(os.environ, CVD_JIT_CACHE=str(tmp_path))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bit-sliced" in out.stdout and " 1 " in out.stdout, out.stdout
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".co")], os.listdir(tmp_path)
