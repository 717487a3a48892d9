"""Oracle: CPU restatement of the reference's hot path — TEST INFRASTRUCTURE.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import, call, link or execute anything under `oracle/`, and only as the
checker, never as the thing measured or shipped.

* `philox.py`       — the build's trial-stream randomness spec (Philox4x32-10)
* `restatement.py`  — Python/numpy restatement of viterbi_markov.py and
                      Pd_plotter.py, function by function (file:line cited)
* `cvd_oracle.c`    — the same path in plain C, for large-size parity checks and
                      the CPU baseline of bench.py (built by `make -C oracle`)

Pinned against fixtures generated from the reference itself
(tests/golden/make_golden.py) — see tests/test_oracle_golden.py.
"""
