"""BASELINE configuration C0 at its own size against the reference itself (VERDICT r04 item
2): the demo preset, rate-1/2 m = 2 at N = 1e3 with 1e3 trials over the demo's p grid and
seed (demo_script.py:113-131), both the BASELINE pair (7,5) vs (5,7) and the demo's (7,5) vs
(6,5), and preset 2 (m = 3) at N = 500 with 500 trials.  tests/golden/make_golden_c0.py ran
the reference's unmodified run_experiment (Pd_plotter.py:176-235; only N_SPECTRUM_BY_M
patched to {2: [1000]}) and recorded its DataFrame and every trial's four log-likelihood
sums.  Here the product's run_experiment must give the same DataFrame and the detector the
same sums bit for bit, on the table path and on the explicit path."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR, code_of

pytestmark = pytest.mark.gpu
CASES = ["c0_m2_75_57", "c0_m2_75_65", "c0_m3_demo"]


@pytest.fixture(scope="module")
def golden_c0():
    z = np.load(os.path.join(GOLDEN_DIR, "golden_c0.npz"))
    with open(os.path.join(GOLDEN_DIR, "golden_c0.json")) as f:
        meta = json.load(f)
    return z, meta


@pytest.mark.parametrize("ename", CASES)
def test_c0_dataframe_equals_reference(pkg, golden_c0, ename):
    z, meta = golden_c0
    e = meta[ename]
    k, n, m, t1 = code_of(meta, e["g1"])
    t2 = code_of(meta, e["g2"])[3]
    df = pkg.run_experiment(k, n, m, t1, t2, e["num_iter"], e["p_vec"], None, e["learn_burn"], e["laplace"],
                            e["seed"], N_list=e["N_list"])
    assert df.to_dict(orient="records") == e["rows"]


@pytest.mark.parametrize("ename", CASES)
@pytest.mark.parametrize("path", [1, 2])
def test_c0_trial_sums_bit_exact(pkg, golden_c0, ename, path):
    """Every trial's (logp1, logp1_ref, logp2, logp2_ref) = the reference's own, at C0's N and
    trial count (path 1 table automaton, 2 explicit)."""
    z, meta = golden_c0
    e = meta[ename]
    k, n, m, t1 = code_of(meta, e["g1"])
    t2 = code_of(meta, e["g2"])[3]
    det = pkg.Detector(k, n, m, t1, device=0)
    sums = z[f"{ename}/sums"]
    it = e["num_iter"]
    (N,) = e["N_list"]
    for ip, p in enumerate(e["p_vec"]):
        model = det.model(p, None, e["learn_burn"], e["laplace"], e["seed"])
        res = det.run_trials(model, t1, t2, N, p, e["seed"], 0, it, path=path, return_sums=True)
        want = sums[ip * it:(ip + 1) * it]
        assert np.array_equal(res["sums"], want), (ename, p)
        s1 = int(np.sum(want[:, 0] > want[:, 1]))
        s2 = int(np.sum(want[:, 2] <= want[:, 3]))
        assert tuple(res["counts"].cpu().tolist()) == (s1, s2)
