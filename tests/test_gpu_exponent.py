"""GPU parity of the error-exponent engine (csrc/cvd_exponent.hip) against the
reference's own Eq. 7 values (tests/golden/exponent.*) and the oracle.

Tolerances: transition counts are integers (bit-exact).  rho is the Perron
root by power iteration stopped when the Collatz-Wielandt bounds agree to
tol = 1e-13 relative; the reference uses np.linalg.eigvals.  The tests accept
|rho - rho_ref| <= 1e-11 rho_ref and |I_err - I_ref| <= 1e-10 |I_ref|, and the
same argmin u unless the two u's rho differ by less than that tolerance."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT, code_of
from oracle import exponent as OE
from oracle import restatement as R

pytestmark = pytest.mark.gpu

GOLD = os.path.join(ROOT, "tests", "golden")
RTOL_RHO, RTOL_I = 1e-11, 1e-10


@pytest.fixture(scope="module")
def egold():
    z = np.load(os.path.join(GOLD, "exponent.npz"))
    with open(os.path.join(GOLD, "exponent.json")) as f:
        meta = json.load(f)
    return z, meta


def test_spectral_radius_vs_reference(pkg, egold):
    z, meta = egold
    for i, want in enumerate(meta["rho"]):
        got = pkg.spectral_radius(z[f"rho{i}/A"])
        assert abs(got - want) <= RTOL_RHO * want, (i, got, want)
    with pytest.raises(ValueError):
        pkg.spectral_radius(-np.eye(3))


def _check_exponent(pkg, P1, P2, u_grid, want_I, want_u):
    I, u = pkg.compute_error_exponent(P1, P2, u_grid=u_grid)
    assert abs(I - want_I) <= RTOL_I * abs(want_I), (I, want_I)
    if u != want_u:   # a near-tie between two grid points
        rh = pkg.chernoff_rhos(P1, P2, [u, want_u])
        assert abs(rh[0] - rh[1]) <= RTOL_RHO * rh[1]


def test_eq7_dense_vs_reference(pkg, egold):
    z, meta = egold
    for i, e in enumerate(meta["exp"]):
        _check_exponent(pkg, z[f"exp{i}/P1"], z[f"exp{i}/P2"], e["u_grid"], e["I_err"], e["u"])


def test_eq7_structured_vs_reference(pkg, egold):
    """The O(K 2^n) structured M(u) of learned tensors == the reference's dense sum."""
    z, meta = egold
    nxt = z["learned/next"]
    T1 = pkg.TransitionTensor(z["learned/counts1"], nxt, 1.0)
    T2 = pkg.TransitionTensor(z["learned/counts2"], nxt, 1.0)
    _check_exponent(pkg, T1, T2, 401, meta["learned"]["I_err"], meta["learned"]["u"])
    # and the dense GPU path on the same tensors
    u = np.linspace(0, 1, 21)
    a = pkg.chernoff_rhos(T1, T2, u)
    b = pkg.chernoff_rhos(np.asarray(T1), np.asarray(T2), u)
    np.testing.assert_allclose(a, b, rtol=RTOL_RHO)


@pytest.mark.parametrize("name,enc,p,length,chains", [("m2_75", "m2_57", 0.05, 20_000, 1),
                                                      ("m3_demo", "m3_demo", 0.1, 30_000, 7),
                                                      ("r23_m4", "r23_m4_b", 0.02, 9_000, 3)])
def test_learn_transition_counts_vs_oracle(pkg, golden, name, enc, p, length, chains):
    """GPU joint counts == the oracle's automaton walk over the same streams."""
    zg, meta = golden
    k, n, m, dec = code_of(meta, name)
    etaps = code_of(meta, enc)[3]
    burn = 500
    T, states, sidx, all_r = pkg.learn_transition_tensor(etaps, dec, m, p, length=length, burn_in=burn,
                                                         seed=31, k=k, n=n, chains=chains)
    assert T.counts.sum() == chains * (-(-length // chains))
    steps = burn + (-(-length // chains))
    want = np.zeros_like(T.counts)
    for c in range(chains):
        r = R.received_stream(etaps, m, k, n, steps, p, 31, pkg.EXPONENT_TAG, c)
        want += OE.automaton_counts(r, T.next, burn, 1 << n)
    np.testing.assert_array_equal(T.counts, want)


def test_rate23_exponent_end_to_end(pkg, golden):
    """Rate-2/3 m = 4 (K = 1807 states, 8 words): learned P1 (H1 encoder) and P2
    (H2 encoder) on the GPU, Eq. 7 over 401 u by the structured path."""
    zg, meta = golden
    k, n, m, g1 = code_of(meta, "r23_m4")
    g2 = code_of(meta, "r23_m4_b")[3]
    P1, *_ = pkg.learn_transition_tensor(g1, g1, m, 0.05, length=400_000, burn_in=2_000, seed=3, k=k, n=n,
                                         chains=64)
    P2, *_ = pkg.learn_transition_tensor(g2, g1, m, 0.05, length=400_000, burn_in=2_000, seed=4, k=k, n=n,
                                         chains=64)
    assert P1.K == 1807
    I, u = pkg.compute_error_exponent(P1, P2, u_grid=401)
    assert I > 0 and 0.0 <= u <= 1.0
    # self-certifying: every rho comes with Collatz-Wielandt bounds that met the tolerance
    out, its = pkg.chernoff_rhos(P1, P2, np.linspace(0, 1, 401), return_bounds=True)
    assert np.all(out[:, 2] - out[:, 1] <= 1e-13 * out[:, 2]) and np.all(its < 200_000)
    # rho(M(0)) = rho(M(1)) = 1: the rows of P2 (u = 0) and P1 (u = 1) are stochastic over (j, r)
    np.testing.assert_allclose(out[[0, -1], 0], 1.0, rtol=1e-12)
