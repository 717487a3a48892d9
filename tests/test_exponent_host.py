"""Error-exponent engine, host side (no GPU): the oracle's restatement of
Eq. 7 and the package's host pieces against the reference's own outputs
(tests/golden/exponent.*, made by make_golden_exponent.py from
alpha_exponent.py)."""
import json
import math
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import exponent as OE

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def egold():
    z = np.load(os.path.join(GOLD, "exponent.npz"))
    with open(os.path.join(GOLD, "exponent.json")) as f:
        meta = json.load(f)
    return z, meta


def test_oracle_eq7_vs_reference(egold):
    z, meta = egold
    for i, e in enumerate(meta["exp"]):
        assert OE.compute_error_exponent(z[f"exp{i}/P1"], z[f"exp{i}/P2"], e["u_grid"]) == (e["I_err"], e["u"])


def test_oracle_learned_tensor_vs_reference(pkg, egold):
    """counts -> normalised tensor (alpha_exponent.py:152-154) -> Eq. 7 equals the
    reference's value; the package's TransitionTensor builds the same tensor."""
    z, meta = egold
    nxt = z["learned/next"]
    P1 = OE.dense_tensor(z["learned/counts1"], nxt, 1.0)
    P2 = OE.dense_tensor(z["learned/counts2"], nxt, 1.0)
    assert OE.compute_error_exponent(P1, P2, 401) == (meta["learned"]["I_err"], meta["learned"]["u"])
    T1 = pkg.TransitionTensor(z["learned/counts1"], nxt, 1.0)
    np.testing.assert_array_equal(np.asarray(T1), P1)


def test_fit_error_exponent_vs_reference(pkg, egold):
    z, meta = egold
    for i, f in enumerate(meta["fit"]):
        assert pkg.fit_error_exponent(z[f"fit{i}/N"], z[f"fit{i}/Pe"]) == (f["I_emp"], f["A"])
    I, A = pkg.fit_error_exponent([10, 20, 30], [0.5, 0.4, 0.3])
    assert I == meta["fit_short"][0] and math.isnan(A) and math.isnan(meta["fit_short"][1])
