import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    z = np.load(os.path.join(GOLDEN_DIR, "golden.npz"))
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        meta = json.load(f)
    return z, meta


@pytest.fixture(scope="session")
def pkg():
    """The product package (directory name has hyphens; loaded via importlib)."""
    from __graft_entry__ import load_package
    return load_package()


def code_of(meta, name):
    c = meta["codes"][name]
    return c["k"], c["n"], c["m"], c["taps"]
