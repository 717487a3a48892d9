"""Command-line front end (package __main__): argument parsing and code
selection, no GPU (the subcommands themselves: tests/test_gpu_cli.py)."""
import importlib

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
