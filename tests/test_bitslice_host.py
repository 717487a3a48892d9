"""The bit-sliced m = 6 step of the specialised kernel (csrc/cvd_bitslice.h, the core of
k1s) on the host, against the plain Eq. 4-5 recursion (viterbi_markov.py:139-159): the new
planes, the step minimum, the T_ref count (Pd_plotter.py:89-99) and the canonical digest
hash, at every layout phase, over 80,000 steps of random and encoded streams.  The header is
compiled with g++ (its host emulation of v_bitop3 / v_perm / v_alignbit); the GPU tests run
the same functions inside the kernel."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "bs_host_check.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_bitslice_step_matches_reference_recursion(tmp_path):
    exe = str(tmp_path / "bs_host_check")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-o", exe, SRC])
    out = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok steps=80000")
