"""The drop-in boundary from plain C (VERDICT / SURVEY §8(b)): tests/c_abi/host_calls.c -- a C99
program over include/cvd.h -- compiles with gcc, links libcvd.so and runs the host-only calls
(version, code tables of (7,5) per viterbi_markov.py:82-106, the dense model's host build per
Pd_plotter.py:123-169 with S = 31, the chunk diagnostic, a status-code error).  No GPU."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

LIBDIR = os.path.join(ROOT, "detecting-convolutional-codes-via-markovian-statistics_amd", "lib")


@pytest.mark.skipif(not shutil.which("gcc"), reason="gcc not present")
def test_c_program_over_the_abi(tmp_path):
    exe = str(tmp_path / "host_calls")
    src = os.path.join(ROOT, "tests", "c_abi", "host_calls.c")
    cc = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                         "-L", LIBDIR, "-lcvd", "-Wl,-rpath," + LIBDIR], capture_output=True, text=True, timeout=120)
    assert cc.returncode == 0, cc.stdout + cc.stderr
    run = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert run.returncode == 0, run.stdout + run.stderr
    lines = run.stdout.splitlines()
    # state 0: input 0 -> word 0, input 1 -> word 3 (1 + D + D^2 and 1 + D^2 both 1), next 0 / 1;
    # state 1 (D = 1): input 0 -> word 1 (only 1 + D + D^2), input 1 -> word 2 (only 1 + D^2)
    assert lines[0] == "out 0 3 1 2 next 0 1", lines
    assert lines[1] == "kind 0 S 31 rows 31", lines      # the reference's BFS of (7,5): 31 states
    assert lines[2] == "chunk 0", lines
    assert lines[3] == "bad -1 ok", lines
