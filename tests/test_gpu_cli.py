"""The command line's CSVs equal the library calls they wrap (same trials,
same seeds): experiment = run_experiment (Pd_plotter.py:242-264), parity =
parity_experiment (comp_parity.py:135-181), exponent = Eq. 7 per p."""
import importlib

import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cli(pkg):
    return importlib.import_module(pkg.__name__ + ".__main__")


def test_experiment_csv(cli, pkg, tmp_path):
    out = tmp_path / "hybrid.csv"
    cli.main(["experiment", "--code", "m2", "--num-iter", "300", "--p", "0.05,0.2", "--N", "60,200",
              "--out", str(out)])
    cc = pkg.CONFIG_CODES["m2"]
    want = pkg.run_experiment(1, 2, 2, cc["gen1"], cc["gen2"], 300, [0.05, 0.2], None, 200, 1.0, 12345,
                              N_list=[60, 200])
    assert pd.read_csv(out, float_precision="round_trip").to_dict(orient="records") == want.to_dict(orient="records")


def test_parity_csv(cli, pkg, tmp_path):
    out = tmp_path / "parity.csv"
    cli.main(["parity", "--code", "m2", "--num-iter", "200", "--p", "0.02,0.1", "--N", "80",
              "--gamma", "0.7", "--out", str(out)])
    cc = pkg.CONFIG_CODES["m2"]
    want = pkg.parity_experiment(1, 2, 2, cc["gen1"], cc["gen2"], 200, [0.02, 0.1], 0.7, 12345, N_list=[80])
    assert pd.read_csv(out, float_precision="round_trip").to_dict(orient="records") == want.to_dict(orient="records")


def test_exponent_csv(cli, pkg, tmp_path):
    out = tmp_path / "exp.csv"
    cli.main(["exponent", "--code", "example:1", "--p", "0.05", "--length", "20000", "--burn-in", "500",
              "--u-grid", "41", "--out", str(out)])
    c = pkg.EXAMPLE_CODES["1"]
    P1 = pkg.learn_transition_tensor(c["gen1"], c["gen1"], 2, 0.05, 20000, 500, 1.0, 12345)[0]
    P2 = pkg.learn_transition_tensor(c["gen2"], c["gen1"], 2, 0.05, 20000, 500, 1.0, 12346)[0]
    I_err, u = pkg.compute_error_exponent(P1, P2, u_grid=41)
    row = pd.read_csv(out, float_precision="round_trip").to_dict(orient="records")[0]
    assert (row["I_err"], row["u_star"], row["states"]) == (I_err, u, 31)
