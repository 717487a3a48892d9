"""GPU parity of the parity-template baseline (cvd_parity_detect) against the
reference's own fractions (tests/golden/parity.*) and the oracle's scan on the
build's trial streams.  Satisfied counts are integers (bit-exact); P̂ and the
threshold test are the same IEEE double division and compare on both sides."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, code_of
from oracle import parity as OP
from oracle import philox
from oracle import restatement as R

pytestmark = pytest.mark.gpu

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def pgold():
    z = np.load(os.path.join(GOLD, "parity.npz"))
    with open(os.path.join(GOLD, "parity.json")) as f:
        meta = json.load(f)
    return z, meta


@pytest.mark.parametrize("name", ["m2_75", "m2_57", "m3_demo", "m6_133_171"])
def test_fraction_vs_reference_golden(pkg, pgold, name):
    z, meta = pgold
    c = meta["codes"][name]
    tpl = [tuple(t) for t in c["deg_h"][str(c["m"] + 3)]["templates"][0]]
    for i, case in enumerate(c["fractions"]):
        y = z[f"{name}/frac{i}/y"].tolist()
        assert pkg.parity_satisfaction_fraction(y, tpl) == case["frac"]
        dec, ph = pkg.parity_detector(y, tpl, 0.6)
        assert (bool(dec), ph) == (case["decision_0.6"], case["P_hat"])


@pytest.mark.parametrize("name,g2,N,p,gamma", [("m2_75", "m2_57", 1001, 0.05, 0.7),
                                               ("m6_133_171", "m6_171_133", 777, 0.02, 0.8),
                                               ("m3_demo", "m3_demo2", 9, 0.1, 0.5),
                                               ("r23_m4", "r23_m4_b", 503, 0.01, 0.6)])
def test_counts_vs_oracle_on_trial_streams(pkg, golden, name, g2, N, p, gamma):
    """Generated H1/H2 streams (ragged count, not a multiple of the block):
    per-sequence satisfied counts and the decision counts equal the oracle's."""
    z, meta = golden
    k, n, m, t1 = code_of(meta, name)
    t2 = code_of(meta, g2)[3]
    det = pkg.Detector(k, n, m, t1, device=0)
    deg_h = m + 3
    tpl = pkg.default_template(t1, m, deg_h)
    T, seed = 301, 42
    tag = philox.grid_tag(N, p)
    r = det.stream_buffer(N, 2 * T)
    det.generate(t1, N, p, seed, tag, 0, 2, T, out=r, q0=0, pitch=2 * T)
    det.generate(t2, N, p, seed, tag, 1, 2, T, out=r, q0=T, pitch=2 * T)
    sat = torch.zeros(2 * T, dtype=torch.int32, device=r.device)
    counts = pkg.parity_detect(r, n, N, 2 * T, T, tpl, gamma, sat=sat)
    sat = sat.cpu().numpy()
    want_s1 = want_s2 = 0
    for q in list(range(0, 2 * T, 37)) + [T - 1, T, 2 * T - 1]:
        h = q >= T
        sid = 2 * (q - T) + 1 if h else 2 * q
        recv = R.received_stream(t2 if h else t1, m, k, n, N, p, seed, tag, sid)
        s, tot = OP.satisfied_count(OP.streams_from_words(recv, n), tpl)
        assert sat[q] == s, (q, sat[q], s)
    first = max(s for (_, s) in tpl)
    tot = max(0, N - first)
    ph = sat / tot if tot > 0 else np.zeros_like(sat, dtype=float)
    want_s1 = int(np.sum(ph[:T] >= gamma))
    want_s2 = int(np.sum(~(ph[T:] >= gamma)))
    assert tuple(counts.cpu().tolist()) == (want_s1, want_s2)


def test_noiseless_full_size_property(pkg):
    """p = 0, N = 1e5 (BASELINE size): every H1 stream satisfies the template at
    every anchor (h annihilates the code), so sat = N - max delay exactly."""
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    N, T = 100_000, 4096
    tpl = pkg.default_template(cc["gen1"], 6)
    r = det.generate(cc["gen1"], N, 0.0, 7, 11, 0, 1, T)
    sat = torch.zeros(T, dtype=torch.int32, device=r.device)
    counts = pkg.parity_detect(r, 2, N, T, T, tpl, 1.0, sat=sat)
    first = max(s for (_, s) in tpl)
    assert torch.all(sat == N - first)
    assert tuple(counts.cpu().tolist()) == (T, 0)


def test_edge_cases(pkg):
    cc = pkg.CONFIG_CODES["m2"]
    det = pkg.Detector(1, 2, 2, cc["gen1"], device=0)
    tpl = pkg.default_template(cc["gen1"], 2)
    first = max(s for (_, s) in tpl)
    # N <= max delay: no anchor, P̂ = 0.0 -> H1 fails unless gamma <= 0, H2 succeeds
    for N in (0, 1, first):
        r = det.stream_buffer(max(N, 1), 6)
        r.zero_()
        c = pkg.parity_detect(r, 2, N, 6, 3, tpl, 0.5)
        assert tuple(c.cpu().tolist()) == (0, 3)
        c = pkg.parity_detect(r, 2, N, 6, 3, tpl, 0.0)
        assert tuple(c.cpu().tolist()) == (3, 0)
    # bad template terms are rejected
    r = det.stream_buffer(64, 1)
    with pytest.raises(pkg.CvdError):
        pkg.parity_detect(r, 2, 64, 1, 1, [(2, 0)], 0.5)
    with pytest.raises(pkg.CvdError):
        pkg.parity_detect(r, 2, 64, 1, 1, [(0, 49)], 0.5)


def test_parity_experiment_table(pkg):
    """parity_experiment rows equal the oracle's decisions on the same trials."""
    cc = pkg.CONFIG_CODES["m2"]
    g1, g2 = cc["gen1"], cc["gen2"]
    iters, N_list, p_vec, gamma, seed = 40, [60, 200], [0.02, 0.2], 0.75, 9
    df = pkg.parity_experiment(1, 2, 2, g1, g2, iters, p_vec, gamma, seed, N_list=N_list, batch=17)
    tpl = pkg.default_template(g1, 2)
    rows = []
    for N in N_list:
        for p in p_vec:
            tag = philox.grid_tag(N, p)
            s1 = s2 = 0
            for t in range(iters):
                for h, g in ((0, g1), (1, g2)):
                    recv = R.received_stream(g, 2, 1, 2, N, p, seed, tag, 2 * t + h)
                    ph = OP.parity_satisfaction_fraction(OP.streams_from_words(recv, 2), tpl)
                    if h == 0:
                        s1 += ph >= gamma
                    else:
                        s2 += not (ph >= gamma)
            rows.append({"N": N, "p": p, "Pd": s1 / iters, "Pc": (s1 + s2) / (2 * iters)})
    assert df.to_dict(orient="records") == rows
