"""The product's Philox4x32-10 forms (csrc/cvd_common.h: philox, philox_blocks under the
launch key pair and under VGPR round keys, philox_round) on the host against the Random123
known-answer vectors and each other (tests/philox_host_check.cpp, compiled with g++).  The
device forms are checked through the streams in the GPU tests."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "philox_host_check.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_philox_forms_known_answers(tmp_path):
    exe = str(tmp_path / "philox_host_check")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-Wno-unknown-pragmas", "-o", exe, SRC])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip() == "ok philox forms"
