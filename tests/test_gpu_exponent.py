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


def test_rho_hbm_path_equals_lds_path(pkg, golden, monkeypatch):
    """The HBM power iteration (K above the LDS limit) forced at K = 1807: same
    Perron roots as the LDS kernel to 1e-12, bounds met."""
    zg, meta = golden
    k, n, m, g1 = code_of(meta, "r23_m4")
    g2 = code_of(meta, "r23_m4_b")[3]
    P1 = pkg.learn_transition_tensor(g1, g1, m, 0.05, length=100_000, burn_in=1_000, seed=3, k=k, n=n, chains=32)[0]
    P2 = pkg.learn_transition_tensor(g2, g1, m, 0.05, length=100_000, burn_in=1_000, seed=4, k=k, n=n, chains=32)[0]
    u = np.linspace(0, 1, 41)
    a, ia = pkg.chernoff_rhos(P1, P2, u, return_bounds=True)
    monkeypatch.setenv("CVD_RHO_GLOBAL", "1")
    b, ib = pkg.chernoff_rhos(P1, P2, u, return_bounds=True)
    monkeypatch.delenv("CVD_RHO_GLOBAL")
    np.testing.assert_allclose(b[:, 0], a[:, 0], rtol=1e-12)
    assert np.all(b[:, 2] - b[:, 1] <= 1e-13 * b[:, 2])
    assert np.all(np.abs(ib - ia) <= 1)


# (23,35) vs (35,23), m = 4, rate 1/2: K = 150,743 metric states (above the LDS limit)
_M4 = ([[[1, 0, 0, 1, 1]], [[1, 1, 1, 0, 1]]], [[[1, 1, 1, 0, 1]], [[1, 0, 0, 1, 1]]])


def test_m4_counts_global_kernel_vs_oracle(pkg):
    """S = 150,743 >= 4096: joint counts from the global-record kernel equal the
    oracle's automaton walk."""
    g1, g2 = _M4
    T, states, sidx, all_r = pkg.learn_transition_tensor(g2, g1, 4, 0.1, length=40_000, burn_in=300, seed=5,
                                                         k=1, n=2, chains=4)
    assert T.K == 150_743
    steps = 300 + 10_000
    want = np.zeros_like(T.counts)
    for c in range(4):
        r = R.received_stream(g2, 4, 1, 2, steps, 0.1, 5, pkg.EXPONENT_TAG, c)
        want += OE.automaton_counts(r, T.next, 300, 4)
    np.testing.assert_array_equal(T.counts, want)


def _structured_host(T1, T2, u):
    """a(u), V(u) of M(u) = a 1^T + V (cvd_exponent.hip header) restated in numpy."""
    lam = T1.laplace
    K, R = T1.counts.shape
    rs1 = np.maximum(T1.counts.sum(1) + K * R * lam, 1.0)
    rs2 = np.maximum(T2.counts.sum(1) + K * R * lam, 1.0)

    def term(c1, c2):
        p1 = np.clip((c1 + lam) / rs1[:, None], 1e-300, 1.0)
        p2 = np.clip((c2 + lam) / rs2[:, None], 1e-300, 1.0)
        return p1 ** u * p2 ** (1.0 - u)

    t0 = term(np.zeros((K, 1)), np.zeros((K, 1)))
    vals = term(T1.counts, T2.counts) - t0
    return R * t0[:, 0], vals


def test_m4_perron_roots_vs_arpack(pkg):
    """K = 150,743: the HBM iteration's Perron roots against ARPACK (scipy) on the
    same structured M(u), rebuilt on the host; rho(M(0)) = rho(M(1)) = 1."""
    import scipy.sparse as sp
    from scipy.sparse.linalg import LinearOperator, eigs
    g1, g2 = _M4
    P1 = pkg.learn_transition_tensor(g1, g1, 4, 0.05, length=2_000_000, burn_in=1_000, seed=1, k=1, n=2,
                                     chains=256)[0]
    P2 = pkg.learn_transition_tensor(g2, g1, 4, 0.05, length=2_000_000, burn_in=1_000, seed=2, k=1, n=2,
                                     chains=256)[0]
    us = np.array([0.0, 0.35, 0.6, 1.0])
    out, its = pkg.chernoff_rhos(P1, P2, us, return_bounds=True)
    assert np.all(out[:, 2] - out[:, 1] <= 1e-13 * out[:, 2])
    np.testing.assert_allclose(out[[0, -1], 0], 1.0, rtol=1e-12)
    K = P1.K
    rows = np.repeat(np.arange(K), 4)
    for j in (1, 2):
        a, vals = _structured_host(P1, P2, us[j])
        V = sp.csr_matrix((vals.reshape(-1), (rows, P1.next.reshape(-1))), shape=(K, K))
        op = LinearOperator((K, K), matvec=lambda x, a=a, V=V: a * x.sum() + V @ x, dtype=np.float64)
        lam = eigs(op, k=1, which="LM", tol=1e-13, maxiter=20_000, return_eigenvectors=False)
        assert abs(abs(lam[0]) - out[j, 0]) <= 1e-10 * out[j, 0]
