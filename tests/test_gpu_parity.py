"""GPU parity: the HIP path (through the C-ABI) against the oracle and the
reference's golden vectors.  Integer work (received streams, metric vectors,
counts) is bit-exact; the fp64 log-likelihood sums are bit-exact as well,
because both sides add the same log values in the same t order."""
import math

import os

import numpy as np
import pytest
import torch

from conftest import code_of
from oracle import philox
from oracle import restatement as R

pytestmark = pytest.mark.gpu


def pack_words(r_list, n):
    """[nseq] arrays of received words -> device buffer [W/4, nseq, 4] (include/cvd.h layout)."""
    spw = 32 // n
    N = len(r_list[0])
    W = ((N + spw - 1) // spw + 3) // 4 * 4
    out = np.zeros((W, len(r_list)), np.uint64)
    for q, r in enumerate(r_list):
        for t, v in enumerate(r):
            out[t // spw, q] |= np.uint64(int(v) << (n * (t % spw)))
    lay = out.astype(np.uint32).reshape(W // 4, 4, len(r_list)).transpose(0, 2, 1).copy()
    return torch.from_numpy(lay.view(np.int32)).cuda()


def unpack_words(words, n, N):
    """device buffer [W/4, nseq, 4] -> received words [N, nseq]."""
    b = words.cpu().numpy().view(np.uint32).astype(np.int64)
    w = b.transpose(0, 2, 1).reshape(-1, b.shape[1])   # [W, nseq]
    spw = 32 // n
    t = np.arange(N)
    return (w[t // spw, :] >> ((t % spw) * n)[:, None]) & ((1 << n) - 1)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda", 0)


# ───────────────────────────── generator ────────────────────────────────────

@pytest.mark.parametrize("name,N,p,ri", [("m2_75", 1000, 0.05, True), ("m2_75", 37, 0.5, True),
                                          ("m3_demo", 333, 0.2, True), ("r23_m4", 1001, 0.1, True),
                                          ("r23_m4", 23, 0.0, True), ("m6_133_171", 517, 0.03, True),
                                          ("m6_133_171", 64, 1.0, False), ("m2_57", 1, 0.3, True)])
def test_generator_bit_exact(pkg, golden, dev, name, N, p, ri):
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    det = pkg.Detector(k, n, m, taps, device=0)
    seed, tag, base, stride, count = 0x1234_5678_9ABC, philox.grid_tag(N, p), 7, 3, 130
    r = det.generate(taps, N, p, seed, tag, base, stride, count, random_input=ri)
    got = unpack_words(r, n, N)
    for q in range(0, count, 11):
        want = R.received_stream(taps, m, k, n, N, p, seed, tag, base + q * stride, random_input=ri)
        np.testing.assert_array_equal(got[:, q], want)


@pytest.mark.parametrize("name", ["m6_133_171", "r23_m4", "k1n3"])
def test_fast_generator_equals_generic_long(pkg, golden, dev, name, monkeypatch):
    """The bit-parallel generator (gen_fast_kernel) against the per-step generic
    kernel at a long ragged N, and against the oracle on a few sequences."""
    if name == "k1n3":
        k, n, m, taps = 1, 3, 4, [[[1, 0, 1, 1, 1]], [[1, 1, 0, 1, 1]], [[1, 1, 1, 1, 1]]]
    else:
        z, meta = golden
        k, n, m, taps = code_of(meta, name)
    det = pkg.Detector(k, n, m, taps, device=0)
    N, p, seed, count = 100_003, 0.07, 99, 300
    tag = philox.grid_tag(N, p)
    fast = det.generate(taps, N, p, seed, tag, 5, 2, count)
    monkeypatch.setenv("CVD_GEN_GENERIC", "1")
    generic = det.generate(taps, N, p, seed, tag, 5, 2, count)
    monkeypatch.delenv("CVD_GEN_GENERIC")
    assert torch.equal(fast, generic)
    got = unpack_words(fast, n, N)
    for q in (0, 131, count - 1):
        want = R.received_stream(taps, m, k, n, N, p, seed, tag, 5 + 2 * q)
        np.testing.assert_array_equal(got[:, q], want)


@pytest.mark.parametrize("slots", [1, 5, 17])
def test_fast_generator_noise_exchange_rounds(pkg, golden, dev, slots, monkeypatch):
    """The wave's undecided (sequence, word) pairs are finished by slot lanes in
    rounds of 64 (noise_chunk_wave); with ~30 pairs per chunk a second round almost
    never runs.  CVD_GEN_SLOTS shrinks the round so that the multi-round path runs,
    on a ragged wave count, and must give the same stream."""
    z, meta = golden
    k, n, m, taps = code_of(meta, "m2_75")
    det = pkg.Detector(k, n, m, taps, device=0)
    N, p, seed, count = 20_011, 0.2, 7, 200
    tag = philox.grid_tag(N, p)
    ref = det.generate(taps, N, p, seed, tag, 3, 1, count)
    monkeypatch.setenv("CVD_GEN_SLOTS", str(slots))
    got = det.generate(taps, N, p, seed, tag, 3, 1, count)
    monkeypatch.delenv("CVD_GEN_SLOTS")
    assert torch.equal(got, ref)
    words = unpack_words(got, n, N)
    for q in (0, 77, count - 1):
        np.testing.assert_array_equal(words[:, q], R.received_stream(taps, m, k, n, N, p, seed, tag, 3 + q))


# ───────────────────────────── metric trace ─────────────────────────────────

@pytest.mark.parametrize("name", ["m2_75", "m3_demo", "r23_m4", "m6_133_171"])
def test_trace_vs_reference_golden(pkg, golden, dev, name):
    """D_0..D_N of the explicit kernel == the reference's viterbi_metric_step."""
    z, meta = golden
    k, n, m, taps = code_of(meta, name)
    r = z[f"{name}/trace_r"]
    D = z[f"{name}/trace_D"]
    det = pkg.Detector(k, n, m, taps, device=0)
    model = det.model(0.05, learn_len=0, learn_burn=0, laplace=1.0, seed=0)
    N = len(r)
    # three copies, the middle one shifted by a random stream, to exercise lanes
    rng = np.random.default_rng(5)
    r2 = rng.integers(0, 1 << n, size=N)
    words = pack_words([r, r2, r], n)
    T = det.trace(model, words, N, 3).cpu().numpy()
    np.testing.assert_array_equal(T[:, 0, :], D)
    np.testing.assert_array_equal(T[:, 2, :], D)
    want2 = np.array(R.metrics_from_stream(taps, m, k, n, r2[:300]), np.uint8)
    np.testing.assert_array_equal(T[:301, 1, :], want2)


def test_simulate_markov_sequence_spec(pkg, golden, dev):
    z, meta = golden
    k, n, m, taps = code_of(meta, "m3_demo")
    g1 = code_of(meta, "m3_demo2")[3]
    sim = pkg.simulate_markov_sequence(g1, m, k, n, 400, 0.1, True, seed=99, decoder=taps)
    want = R.simulate_markov_sequence(g1, m, k, n, 400, 0.1, True, seed=99, decoder=taps)
    assert sim["metrics"] == want["metrics"]
    np.testing.assert_array_equal(sim["received"], want["received"])


# ───────────────────── detector vs reference run_experiment ────────────────

@pytest.mark.parametrize("ename", ["exp_m2_75_57", "exp_m2_75_65", "exp_m3_demo"])
@pytest.mark.parametrize("path", [1, 2])
def test_trial_sums_bit_exact_vs_reference(pkg, golden, dev, ename, path):
    """Every per-trial (logp1, logp1_ref, logp2, logp2_ref) equals the value the
    reference's own run_experiment produced (table AND explicit path)."""
    z, meta = golden
    e = meta[ename]
    k, n, m, t1 = code_of(meta, e["g1"])
    t2 = code_of(meta, e["g2"])[3]
    det = pkg.Detector(k, n, m, t1, device=0)
    sums = z[f"{ename}/sums"]
    iters = e["num_iter"]
    for N in e["N_list"]:
        for ip, p in enumerate(e["p_vec"]):
            model = det.model(p, None, e["learn_burn"], e["laplace"], e["seed"])
            res = det.run_trials(model, t1, t2, N, p, e["seed"], 0, iters, batch=77, path=path,
                                 return_sums=True)
            assert np.array_equal(res["sums"], sums[ip * iters:(ip + 1) * iters])
            s1 = int(np.sum(sums[ip * iters:(ip + 1) * iters, 0] > sums[ip * iters:(ip + 1) * iters, 1]))
            s2 = int(np.sum(sums[ip * iters:(ip + 1) * iters, 2] <= sums[ip * iters:(ip + 1) * iters, 3]))
            assert tuple(res["counts"].cpu().tolist()) == (s1, s2)


@pytest.mark.parametrize("ename", ["exp_m2_75_57", "exp_m3_demo"])
def test_run_experiment_dataframe(pkg, golden, dev, ename):
    z, meta = golden
    e = meta[ename]
    k, n, m, t1 = code_of(meta, e["g1"])
    t2 = code_of(meta, e["g2"])[3]
    df = pkg.run_experiment(k, n, m, t1, t2, e["num_iter"], e["p_vec"], None, e["learn_burn"],
                            e["laplace"], e["seed"])
    assert df.to_dict(orient="records") == e["rows"]


def test_mc_run_counts_batch_and_shard_invariant(pkg, dev):
    cc = pkg.CONFIG_CODES["m2"]
    det = pkg.Detector(1, 2, 2, cc["gen1"], device=0)
    model = det.model(0.08, None, 200, 1.0, 5)
    ref = det.run_trials(model, cc["gen1"], cc["gen2"], 300, 0.08, 5, 0, 5000, return_sums=True)
    want = tuple(ref["counts"].cpu().tolist())
    for batch in (5000, 999, 64):
        got = det.run_trials(model, cc["gen1"], cc["gen2"], 300, 0.08, 5, 0, 5000, batch=batch)
        assert tuple(got["counts"].cpu().tolist()) == want
    c = torch.zeros(2, dtype=torch.int64, device=dev)
    for lo, hi in [(0, 1234), (1234, 1235), (1235, 5000)]:
        det.run_trials(model, cc["gen1"], cc["gen2"], 300, 0.08, 5, lo, hi, counts=c)
    assert tuple(c.cpu().tolist()) == want


def test_edge_cases(pkg, dev):
    cc = pkg.CONFIG_CODES["m2"]
    det = pkg.Detector(1, 2, 2, cc["gen1"], device=0)
    model = det.model(0.1, None, 200, 1.0, 1)
    # N = 0: empty metric sequences, log-likelihoods 0.0 == 0.0 -> H1 fails, H2 succeeds
    res = det.run_trials(model, cc["gen1"], cc["gen2"], 0, 0.1, 1, 0, 10, return_sums=True)
    assert tuple(res["counts"].cpu().tolist()) == (0, 10)
    # empty trial range
    res = det.run_trials(model, cc["gen1"], cc["gen2"], 50, 0.1, 1, 3, 3)
    assert tuple(res["counts"].cpu().tolist()) == (0, 0)
    # ragged sizes (not a multiple of the 256-lane block) and p = 0 / 1
    for p in (0.0, 1.0):
        mod = det.model(p, None, 200, 1.0, 1)
        a = det.run_trials(mod, cc["gen1"], cc["gen2"], 77, p, 1, 0, 301, return_sums=True)
        states, transitions, all_r = R.enumerate_markov_states_allzero(cc["gen1"], 2, 1, 2)
        Tref = R.T_half(states, transitions, all_r)
        _, sidx, P1 = R.learn_P1_empirical(cc["gen1"], 1, 2, 2, p, None, 200, 1.0, 1, states, transitions)
        _, _, want = R.run_trials(cc["gen1"], cc["gen2"], 1, 2, 2, 77, p, 1, 290, 301, sidx, P1, Tref,
                                  return_sums=True)
        assert np.array_equal(a["sums"][290:], np.array(want).reshape(-1, 4))


def test_explicit_path_equals_table_path_rate23(pkg, golden, dev):
    z, meta = golden
    k, n, m, t1 = code_of(meta, "r23_m4")
    t2 = code_of(meta, "r23_m4_b")[3]
    det = pkg.Detector(k, n, m, t1, device=0)
    model = det.model(0.05, None, 200, 1.0, 123)
    a = det.run_trials(model, t1, t2, 2000, 0.05, 123, 0, 700, path=1, return_sums=True)
    b = det.run_trials(model, t1, t2, 2000, 0.05, 123, 0, 700, path=2, return_sums=True)
    assert np.array_equal(a["sums"], b["sums"])
    # and the first trials against the oracle
    states, transitions, all_r = R.enumerate_markov_states_allzero(t1, m, k, n)
    Tref = R.T_half(states, transitions, all_r)
    _, sidx, P1 = R.learn_P1_empirical(t1, k, n, m, 0.05, None, 200, 1.0, 123, states, transitions)
    _, _, want = R.run_trials(t1, t2, k, n, m, 2000, 0.05, 123, 0, 3, sidx, P1, Tref, return_sums=True)
    assert np.array_equal(a["sums"][:3], np.array(want).reshape(-1, 4))


@pytest.mark.parametrize("name,g2name,N", [("r23_m4", "r23_m4_b", 4003), ("m2_75", "m2_57", 1291),
                                           ("m3_demo", "m3_demo2", 640)])
def test_lds_table_kernel_equals_global_table_kernel(pkg, golden, dev, name, g2name, N, monkeypatch):
    """The LDS-resident 16-bit-record table kernel against the 32-bit-record
    kernel (L2 gathers) on the same streams: bit-identical sums, ragged N and
    a trial count that is not a multiple of the block."""
    z, meta = golden
    k, n, m, t1 = code_of(meta, name)
    t2 = code_of(meta, g2name)[3]
    det = pkg.Detector(k, n, m, t1, device=0)
    model = det.model(0.07, None, 200, 1.0, 9)
    a = det.run_trials(model, t1, t2, N, 0.07, 9, 0, 1500, path=1, return_sums=True)
    monkeypatch.setenv("CVD_TABLE_WIDE", "1")
    b = det.run_trials(model, t1, t2, N, 0.07, 9, 0, 1500, path=1, return_sums=True)
    monkeypatch.delenv("CVD_TABLE_WIDE")
    assert np.array_equal(a["sums"], b["sums"])
    assert tuple(a["counts"].cpu().tolist()) == tuple(b["counts"].cpu().tolist())


# ─────────────────────────── m = 6 sparse model ─────────────────────────────

def oracle_sums_sparse(model_rows, taps, m, k, n, r_stream, lp_unseen):
    """Oracle recursion for a sparse model: row lookup by metric vector, unseen
    rows -> log(1/S); T_ref count from all 2^n successors."""
    lp_tab, keys = model_rows
    index = {bytes(row): i for i, row in enumerate(keys)}
    out, nxt = R.encoder_tables(taps, m, k, n)
    D = np.zeros(1 << m, np.int64)
    lp = lr = 0.0
    for rv in r_stream:
        i = index.get(bytes(D.astype(np.uint8)))
        succ = [R.metric_step_vec(D, out, nxt, q, n) for q in range(1 << n)]
        c = sum(np.array_equal(succ[q], succ[rv]) for q in range(1 << n))
        lp += lp_tab[i, rv] if i is not None else lp_unseen
        lr += math.log(max(c / (1 << n), 1e-300))
        D = succ[rv]
    return lp, lr


@pytest.mark.parametrize("p", [0.02, 0.15])
def test_m6_sparse_sums_vs_oracle(pkg, dev, p):
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    model = det.model(p, 30000, 200, 1.0, 12345)
    inf = model.info()
    assert inf["kind"] == 1
    N = 400
    res = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, 12345, 0, 200, return_sums=True)
    rows = model.rows()
    tag = philox.grid_tag(N, p)
    for t in (0, 1, 57, 199):
        for hyp, g in ((0, cc["gen1"]), (1, cc["gen2"])):
            r = R.received_stream(g, 6, 1, 2, N, p, 12345, tag, 2 * t + hyp)
            lp, lr = oracle_sums_sparse(rows, cc["gen1"], 6, 1, 2, r, inf["logp1_unseen"])
            assert res["sums"][t, 2 * hyp] == lp and res["sums"][t, 2 * hyp + 1] == lr


def test_m6_full_size_properties(pkg, dev):
    """BASELINE size N = 1e5: counts independent of batching and sharding; the
    trace of one full-length sequence matches the host step at sampled t."""
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    model = det.model(0.01, 200000, 200, 1.0, 12345)
    N, T = 100000, 512
    a = det.run_trials(model, cc["gen1"], cc["gen2"], N, 0.01, 12345, 0, T, batch=T)
    b = torch.zeros(2, dtype=torch.int64, device=dev)
    det.run_trials(model, cc["gen1"], cc["gen2"], N, 0.01, 12345, 0, 200, batch=100, counts=b)
    det.run_trials(model, cc["gen1"], cc["gen2"], N, 0.01, 12345, 200, T, batch=157, counts=b)
    assert a["counts"].cpu().tolist() == b.cpu().tolist()
    words = det.generate(cc["gen1"], N, 0.01, 12345, 17, 0, 1, 1)
    D = det.trace(model, words, N, 1)[:, 0, :].cpu().numpy()
    r = unpack_words(words, 2, N)[:, 0]
    tr = pkg.build_trellis(cc["gen1"], 6, 1)
    for t in range(0, N, 997):
        y = ((int(r[t]) >> 0) & 1, (int(r[t]) >> 1) & 1)
        assert pkg.viterbi_metric_step(tuple(D[t]), tr, y) == tuple(int(v) for v in D[t + 1])
    assert D.max() <= 12


@pytest.mark.parametrize("name,g2name,N,p", [("m2_75", "m2_57", 700, 0.1), ("m3_demo", "m3_demo2", 900, 0.05),
                                             ("m6_133_171", "m6_171_133", 1500, 0.05),
                                             ("m6_133_171", "m6_171_133", 333, 0.2)])
def test_orbit_kernel_equals_generic_explicit(pkg, golden, dev, name, g2name, N, p):
    """k = 1 butterfly kernel (default explicit path) == k = 1 orbit kernel (ACS
    only for r < r ^ g0) == generic explicit kernel (ACS for every received
    word) == table automaton (dense codes)."""
    z, meta = golden
    k, n, m, t1 = code_of(meta, name)
    t2 = code_of(meta, g2name)[3]
    _three_explicit_paths_agree(pkg, k, n, m, t1, t2, N, p)


# (23,35) m = 4 and (53,75) m = 5, delay-ordered taps: standard butterflies, the
# k = 1 kernels at the intermediate memories
_EXTRA_K1 = {4: ([[[1, 0, 0, 1, 1]], [[1, 1, 1, 0, 1]]], [[[1, 1, 1, 0, 1]], [[1, 0, 0, 1, 1]]]),
             5: ([[[1, 0, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 1]]], [[[1, 1, 1, 1, 0, 1]], [[1, 0, 1, 0, 1, 1]]])}


@pytest.mark.parametrize("m,N,p", [(4, 800, 0.05), (4, 300, 0.3), (5, 1100, 0.02), (5, 500, 0.12)])
def test_k1_kernels_intermediate_memory(pkg, dev, m, N, p):
    t1, t2 = _EXTRA_K1[m]
    _three_explicit_paths_agree(pkg, 1, 2, m, t1, t2, N, p, learn_len=20000)


def _three_explicit_paths_agree(pkg, k, n, m, t1, t2, N, p, learn_len=None):
    det = pkg.Detector(k, n, m, t1, device=0)
    model = det.model(p, 20000 if m == 6 else learn_len, 200, 1.0, 77)
    paths = (pkg.PATH_EXPLICIT, pkg.PATH_EXPLICIT_BUTTERFLY, pkg.PATH_EXPLICIT_ORBIT, pkg.PATH_EXPLICIT_GENERIC)
    runs = {path: det.run_trials(model, t1, t2, N, p, 77, 0, 300, path=path, return_sums=True) for path in paths}
    if k == 1 and n == 2 and m >= 3:
        # standard butterflies: the default explicit kernel is the specialised one, for m = 6
        # its bit-sliced form (k1s) on the bit-sliced tables (unless CVD_BITSLICE=0)
        bs = m == 6 and os.environ.get("CVD_BITSLICE", "1") != "0"
        assert model.info()["explicit_kernel"] == (5 if bs else 4), pkg.lib().cvd_last_error()
    a = runs[pkg.PATH_EXPLICIT]
    for path in paths[1:]:
        assert np.array_equal(a["sums"], runs[path]["sums"]), path
        assert a["counts"].cpu().tolist() == runs[path]["counts"].cpu().tolist(), path
    if m < 6 and model.info()["kind"] == 0:
        c = det.run_trials(model, t1, t2, N, p, 77, 0, 300, path=pkg.PATH_TABLE, return_sums=True)
        assert np.array_equal(a["sums"], c["sums"])


@pytest.mark.parametrize("p", [0.01, 0.1])
def test_m6_headline_config_sums_vs_c_oracle(pkg, dev, p):
    """The bench workload itself (m = 6 pair, N = 1e5, the default 10^6-step
    sparse model): per-trial fp64 sums of the code-specialised kernel equal the C
    oracle's bit for bit, for the first trials and for trial ids past 10^6."""
    from oracle import c_oracle as C
    cc = pkg.CONFIG_CODES["m6"]
    N, seed = 100_000, 12345
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    model = det.model(p, None, 200, 1.0, seed)
    assert model.info()["kind"] == 1 and "spec" in pkg.KERNEL_NAMES[model.info()["explicit_kernel"]]
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    cm = C.Model(c1, p, None, 200, 1.0, seed)
    for t0, t1 in ((0, 12), (1_000_003, 1_000_011)):
        got = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, t0, t1, return_sums=True)
        cnt, want = cm.run_trials(c1, c2, N, p, seed, t0, t1, sums=True)
        assert np.array_equal(got["sums"], want)
        assert tuple(got["counts"].cpu().tolist()) == tuple(int(x) for x in cnt)


def test_m6_batch_beyond_32bit_offsets(pkg, dev):
    """One launch over a 35 GB stream buffer (dword offsets past 2^32): the sums of
    the last trials, whose words sit at the highest offsets, equal the C oracle's."""
    from oracle import c_oracle as C
    cc = pkg.CONFIG_CODES["m6"]
    N, p, seed, B = 100_000, 0.05, 12345, 700_000
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    model = det.model(p, 200_000, 200, 1.0, seed)
    assert det.words_per_seq(N) * 2 * B > (1 << 32)
    tag = pkg.grid_tag(N, p)
    r = det.stream_buffer(N, 2 * B)
    det.generate(cc["gen1"], N, p, seed, tag, 0, 2, B, out=r, q0=0, pitch=2 * B)
    det.generate(cc["gen2"], N, p, seed, tag, 1, 2, B, out=r, q0=B, pitch=2 * B)
    sums = torch.full((2 * B, 2), float("nan"), dtype=torch.float64, device=r.device)
    det.detect(model, r, N, 2 * B, B, sums=sums)
    s = sums[torch.tensor([B - 2, B - 1, 2 * B - 2, 2 * B - 1], device=r.device)].cpu().numpy()
    del r, sums
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    _, want = C.Model(c1, p, 200_000, 200, 1.0, seed).run_trials(c1, c2, N, p, seed, B - 2, B, sums=True)
    assert np.array_equal(s[:2], want[:, :2]) and np.array_equal(s[2:], want[:, 2:])


@pytest.mark.parametrize("walk", ["0", "1"])
def test_m6_bitslice_small_and_ragged_N_vs_c_oracle(pkg, dev, monkeypatch, walk):
    """The bit-sliced kernel's step loop runs six steps per iteration (one per layout phase)
    and then the last 1-5; its stream chunks are four words (64 steps).  Every N around
    those boundaries -- and N = 0, 1 -- gives the C oracle's per-trial sums, lockstep and in
    walk mode, on a persistent launch (2 blocks) and a block launch."""
    from oracle import c_oracle as C
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    p = 0.02
    model = det.model(p, 100_000, 200, 1.0, 12345)
    c1, c2 = C.Code(cc["gen1"], 6, 1, 2), C.Code(cc["gen2"], 6, 1, 2)
    cm = C.Model(c1, p, 100_000, 200, 1.0, 12345)
    monkeypatch.setenv("CVD_WALK", walk)
    for N in (0, 1, 5, 6, 7, 11, 12, 13, 15, 16, 17, 63, 64, 65, 127, 129):
        want_c, want = cm.run_trials(c1, c2, N, p, 12345, 40, 40 + 2100, sums=True, nthreads=8)
        for persist in ("0", "1"):
            monkeypatch.setenv("CVD_K1S_PERSIST", persist)
            monkeypatch.setenv("CVD_K1S_PERSIST_BLOCKS", "2")
            got = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, 12345, 40, 40 + 2100, return_sums=True)
            assert np.array_equal(got["sums"], want), (N, persist)
            assert tuple(got["counts"].cpu().tolist()) == tuple(int(x) for x in want_c), (N, persist)
    assert model.device_error() == 0
