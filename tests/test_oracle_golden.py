"""Pin the oracle (oracle/restatement.py) against vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import philox
from oracle import restatement as R
from conftest import code_of

ALL_CODES = ["m2_75", "m2_57", "m2_65", "m3_demo", "m3_demo2", "r23_m4", "r23_m4_b",
             "m6_133_171", "m6_171_133"]
BFS_CODES = ["m2_75", "m2_57", "m2_65", "m3_demo", "r23_m4"]


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = philox.philox4x32_10(*[np.array([c], np.uint64) for c in ctr], *key)
        assert tuple(int(g[0]) for g in got) == want


def test_threshold_and_tags():
    assert philox.threshold(0.5) == 1 << 31
    assert philox.threshold(1.0) == 1 << 32
    assert philox.threshold(0.0) == 0
    assert philox.grid_tag(500, 0.05) != philox.grid_tag(500, 0.1)
    assert philox.grid_tag(500, 0.05) < (1 << 31)
    with pytest.raises(ValueError):
        philox.threshold(1.5)


@pytest.mark.parametrize("name", ALL_CODES)
def test_encoder_tables(golden, name):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    out, nxt = R.encoder_tables(taps, m, k, n)
    np.testing.assert_array_equal(out, z[f"{name}/out_sym"])
    np.testing.assert_array_equal(nxt, z[f"{name}/next_state"])
    tr = R.build_trellis(taps, m, k)
    rows = [[ns, ps, sum(b << i for i, b in enumerate(u)), sum(b << j for j, b in enumerate(o))]
            for ns in range(1 << m) for (ps, u, o) in tr[ns]]
    np.testing.assert_array_equal(np.array(rows), z[f"{name}/trellis"])


@pytest.mark.parametrize("name", ["m2_75", "m3_demo", "r23_m4", "m6_133_171"])
def test_metric_trace(golden, name):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    r = z[f"{name}/trace_r"]
    D = R.metrics_from_stream(taps, m, k, n, r)
    np.testing.assert_array_equal(np.array(D, np.uint8), z[f"{name}/trace_D"])
    out, nxt = R.encoder_tables(taps, m, k, n)
    Dv = np.zeros(1 << m, np.int64)
    for t in range(0, len(r), 7):
        Dv = R.metric_step_vec(z[f"{name}/trace_D"][t].astype(np.int64), out, nxt, r[t], n)
        np.testing.assert_array_equal(Dv, z[f"{name}/trace_D"][t + 1])


@pytest.mark.parametrize("name", BFS_CODES)
def test_bfs(golden, name):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    states, transitions, all_r = R.enumerate_markov_states_allzero(taps, m, k, n)
    np.testing.assert_array_equal(np.array(states, np.uint8), z[f"{name}/states"])
    trip = [[i, j, sum(b << q for q, b in enumerate(r))]
            for i in range(len(states)) for j, rl in transitions[i].items() for r in rl]
    np.testing.assert_array_equal(np.array(trip), z[f"{name}/transitions"])


@pytest.mark.parametrize("name", ["m2_75", "m2_65", "m3_demo"])
def test_T_half_bit_exact_vs_sympy(golden, name):
    """T(1/2) = |Y(i,j)|/2^n, bit-identical to the reference's sympy path."""
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    T = R.T_half(*R.enumerate_markov_states_allzero(taps, m, k, n))
    assert np.array_equal(T, z[f"{name}/T_0.5"])


def test_T_p_weights_m2(golden):
    """Eq. 6 weights at p != 1/2 (pins the restated p^w (1-p)^(n-w) reading)."""
    z, meta = golden
    k, n, m, taps = code_of(meta, "m2_75")
    states, transitions, all_r = R.enumerate_markov_states_allzero(taps, m, k, n)
    for p in (0.1, 0.3):
        S = len(states)
        T = np.zeros((S, S))
        for i in range(S):
            for j, rl in transitions[i].items():
                T[i, j] = sum(p ** sum(r) * (1 - p) ** (n - sum(r)) for r in rl)
        T /= T.sum(axis=1, keepdims=True)
        np.testing.assert_allclose(T, z[f"m2_75/T_{p}"], rtol=1e-14, atol=1e-15)


@pytest.mark.parametrize("p,seed", [(0.01, 123), (0.05, 123), (0.1, 123), (0.2, 123), (0.3, 123),
                                    (0.05, 12345)])
def test_learn_P1_m2(golden, p, seed):
    z, meta = golden
    k, n, m, taps = code_of(meta, "m2_75")
    _, _, P = R.learn_P1_empirical(taps, k, n, m, p, None, 200, 1.0, seed)
    assert np.array_equal(P, z[f"m2_75/P1_{p}_{seed}"])


def test_learn_P1_m3(golden):
    z, meta = golden
    k, n, m, taps = code_of(meta, "m3_demo")
    _, _, P = R.learn_P1_empirical(taps, k, n, m, 0.05, None, 200, 1.0, 123)
    assert np.array_equal(P, z["m3_demo/P1_0.05_123"])


@pytest.mark.parametrize("name", ["m2_75", "m3_demo"])
def test_log_prob_sequence(golden, name):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    states = [tuple(int(v) for v in s) for s in z[f"{name}/states"]]
    sidx = {s: i for i, s in enumerate(states)}
    Ds = [tuple(int(v) for v in row) for row in z[f"{name}/trace_D"]]
    lp = R.log_prob_sequence(Ds, sidx, z[f"{name}/P1_0.05_123"])
    lr = R.log_prob_sequence(Ds, sidx, z[f"{name}/T_0.5"])
    assert lp == z[f"{name}/trace_logp"][0] and lr == z[f"{name}/trace_logp"][1]


@pytest.mark.parametrize("ename", ["exp_m2_75_57", "exp_m2_75_65", "exp_m3_demo"])
def test_run_experiment_bit_exact(golden, ename):
    """Per-trial log-likelihood sums and Pd/Pc identical to the reference's own
    run_experiment driven by the spec'd simulator."""
    z, meta = golden
    e = meta[ename]
    k, n, m, t1 = code_of(meta, e["g1"])
    t2 = code_of(meta, e["g2"])[3]
    states, transitions, all_r = R.enumerate_markov_states_allzero(t1, m, k, n)
    Tref = R.T_half(states, transitions, all_r)
    sums = z[f"{ename}/sums"]
    row = 0
    iters = e["num_iter"]
    for N in e["N_list"]:
        for ip, p in enumerate(e["p_vec"]):
            _, sidx, P1 = R.learn_P1_empirical(t1, k, n, m, p, None, e["learn_burn"],
                                               e["laplace"], e["seed"], states, transitions)
            ntr = min(iters, 25)   # keep the CPU suite fast; the GPU tests cover all trials
            s1, s2, got = R.run_trials(t1, t2, k, n, m, N, p, e["seed"], 0, ntr, sidx, P1, Tref,
                                       return_sums=True)
            want = sums[ip * iters: ip * iters + ntr]
            got = np.array(got).reshape(ntr, 4)
            assert np.array_equal(got, want)
            row += 1
    # Pd/Pc of the full grid follow from the recorded sums with the reference's rule
    for ip, rowd in enumerate(e["rows"]):
        blk = sums[ip * iters:(ip + 1) * iters]
        s1 = int(np.sum(blk[:, 0] > blk[:, 1]))
        s2 = int(np.sum(blk[:, 2] <= blk[:, 3]))
        assert rowd["Pd"] == s1 / iters
        assert rowd["Pc"] == (s1 + s2) / (2 * iters)
