"""Parity-template baseline, host side (no GPU): the package's GF(2) template
algebra and the oracle's scan against the reference's own outputs
(tests/golden/parity.*, made by make_golden_parity.py from
parity_eqn_check.py / comp_parity.py)."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import parity as OP

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def pgold():
    z = np.load(os.path.join(GOLD, "parity.npz"))
    with open(os.path.join(GOLD, "parity.json")) as f:
        meta = json.load(f)
    return z, meta


def test_parse_poly_token(pkg, pgold):
    z, meta = pgold
    for tok, want in meta["tokens"].items():
        assert pkg.parse_poly_token(tok) == want
    with pytest.raises(ValueError):
        pkg.parse_poly_token("9x")


@pytest.mark.parametrize("name", ["m2_75", "m2_57", "m3_demo", "m6_133_171", "m6_171_133", "r23_m4"])
def test_system_nullspace_equations(pkg, pgold, name):
    z, meta = pgold
    c = meta["codes"][name]
    for dh, e in c["deg_h"].items():
        d = int(dh)
        A = pkg.build_parity_system(c["gens"], d)
        np.testing.assert_array_equal(A, z[f"{name}/d{d}/A"])
        np.testing.assert_array_equal(OP.build_parity_system(c["gens"], d), A)
        B = pkg.nullspace_mod2(A)
        np.testing.assert_array_equal(B.reshape(-1, A.shape[1]), z[f"{name}/d{d}/basis"].reshape(-1, A.shape[1]))
        np.testing.assert_array_equal(OP.nullspace_mod2(A).reshape(-1, A.shape[1]), B.reshape(-1, A.shape[1]))
        assert len(B) == e["n_basis"]
        vecs = pkg.parity_vectors(c["gens"], d)
        for i, (eq, tpl) in enumerate(zip(e["equations"], e["templates"])):
            assert pkg.parity_vector_to_equation(vecs[i]) == eq
            assert pkg.template_of(vecs[i]) == [tuple(t) for t in tpl]
        # every basis vector annihilates the code: A h = 0
        for row in B:
            assert not np.any((A.astype(int) @ row.astype(int)) % 2)


@pytest.mark.parametrize("name", ["m2_75", "m2_57", "m3_demo", "m6_133_171"])
def test_oracle_scan_vs_reference(pkg, pgold, name):
    z, meta = pgold
    c = meta["codes"][name]
    tpl = [tuple(t) for t in c["deg_h"][str(c["m"] + 3)]["templates"][0]]
    assert pkg.default_template(c["gens"], c["m"]) == tpl
    for i, case in enumerate(c["fractions"]):
        y = z[f"{name}/frac{i}/y"]
        assert OP.parity_satisfaction_fraction(y, tpl) == case["frac"]
