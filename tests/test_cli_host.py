"""Command-line front end (package __main__): argument parsing and code
selection, no GPU (the subcommands themselves: tests/test_gpu_cli.py)."""
import importlib
import os

import pytest


@pytest.fixture(scope="module")
def cli(pkg):
    return importlib.import_module(pkg.__name__ + ".__main__")


def test_parse_experiment(cli):
    a = cli.parser().parse_args(["experiment", "--code", "m2", "--p", "0.01,0.05", "--N", "100,200",
                                 "--num-iter", "64"])
    assert (a.cmd, a.p, a.N, a.num_iter, a.learn_len, a.learn_burn, a.laplace, a.seed) == \
        ("experiment", [0.01, 0.05], [100, 200], 64, None, 200, 1.0, 12345)


def test_parse_parity_and_exponent(cli):
    a = cli.parser().parse_args(["parity", "--gamma", "0.7", "--deg-h", "6"])
    assert (a.gamma, a.deg_h, a.code) == (0.7, 6, "example:1")
    a = cli.parser().parse_args(["exponent", "--length", "1000", "--u-grid", "11", "--chains", "4"])
    assert (a.length, a.u_grid, a.chains, a.burn_in) == (1000, 11, 4, 5000)


def test_code_names(cli, pkg):
    assert cli.code_of("example:1")[:3] == (1, 2, 2)
    assert cli.code_of("example:2")[:3] == (1, 2, 3)
    assert cli.code_of("r23_m4")[:3] == (2, 3, 4)
    assert cli.code_of("m6")[3] == pkg.CONFIG_CODES["m6"]["gen1"]
    for bad in ("m7", "example:9"):
        with pytest.raises(SystemExit):
            cli.code_of(bad)
    with pytest.raises(SystemExit):
        cli.parser().parse_args(["bogus"])


def test_compare_figures(cli, pkg, tmp_path):
    """compare: P_err = clip(1 - Pc) curves per N and per p (plots_compare.py:35-134)."""
    import pandas as pd
    from importlib import import_module
    cmp = import_module(pkg.__name__ + ".compare")
    h = pd.DataFrame({"N": [100, 100, 500, 500], "p": [0.01, 0.1, 0.01, 0.1],
                      "Pd": [1.0, 0.8, 1.0, 0.9], "Pc": [1.0, 0.85, 1.0, 0.95]})
    b = pd.DataFrame({"N": [100, 100], "p": [0.01, 0.1], "Pd": [0.7, 0.55]})   # Pd only: used as Pc
    cv = cmp.curves(h, b)
    assert set(cv) == {("N", 100), ("N", 500), ("p", 0.01), ("p", 0.1)}
    x, y = cv[("N", 100)]["hybrid"]
    assert list(x) == [0.01, 0.1] and list(y) == [0.0, 1.0 - 0.85]
    x, y = cv[("p", 0.1)]["baseline"]
    assert list(x) == [100] and list(y) == [1.0 - 0.55]
    assert len(cv[("N", 500)]["baseline"][0]) == 0
    hp, bp = tmp_path / "h.csv", tmp_path / "b.csv"
    h.to_csv(hp, index=False)
    b.to_csv(bp, index=False)
    assert cli.main(["compare", "--hybrid", str(hp), "--baseline", str(bp), "--outdir", str(tmp_path / "plots")]) == 0
    assert sorted(os.listdir(tmp_path / "plots")) == ["Perr_vs_N_p0.01.png", "Perr_vs_N_p0.1.png",
                                                      "Perr_vs_p_N100.png", "Perr_vs_p_N500.png"]
