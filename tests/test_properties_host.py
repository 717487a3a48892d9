"""Property tests (hypothesis) of the native host path against the oracle's
restatement on random codes and received streams (SURVEY.md §4 layer 1):
encoder tables (viterbi_markov.py:82-106), the Eq. 4-5 step (:139-159) and
the BFS state enumeration (:166-195), for rate-1/2, 1/3 and 2/3 shapes.
No GPU."""
import numpy as np
from hypothesis import given, settings, strategies as st

from oracle import restatement as R


@st.composite
def codes(draw, shapes=((1, 2), (1, 3), (2, 3)), mmax=4):
    k, n = draw(st.sampled_from(shapes))
    m = draw(st.integers(max(2, k), mmax))
    taps = [[[draw(st.integers(0, 1)) for _ in range(m + 1)] for _ in range(k)] for _ in range(n)]
    return k, n, m, taps


@settings(max_examples=40, deadline=None)
@given(code=codes())
def test_code_tables_random(pkg, code):
    k, n, m, taps = code
    out, nxt = pkg.Code(taps, m, k, n).tables()
    want_out, want_nxt = R.encoder_tables(taps, m, k, n)
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(nxt, want_nxt)


@settings(max_examples=40, deadline=None)
@given(code=codes(), data=st.data())
def test_metric_step_random_streams(pkg, code, data):
    k, n, m, taps = code
    rs = data.draw(st.lists(st.integers(0, (1 << n) - 1), min_size=1, max_size=40))
    tr_native = pkg.build_trellis(taps, m, k, n)
    tr_oracle = R.build_trellis(taps, m, k)
    D = tuple([0] * (1 << m))
    for rv in rs:
        y = R.r_tuple(rv, n)
        got = pkg.viterbi_metric_step(D, tr_native, y)
        want = R.viterbi_metric_step(list(D), tr_oracle, y)
        assert tuple(got) == tuple(want)
        assert min(got) == 0
        D = got


@settings(max_examples=15, deadline=None)
@given(code=codes(shapes=((1, 2), (1, 3)), mmax=3))
def test_bfs_random(pkg, code):
    k, n, m, taps = code
    s1, t1, r1 = pkg.enumerate_markov_states_allzero(taps, m, k, n)
    s2, t2, r2 = R.enumerate_markov_states_allzero(taps, m, k, n)
    assert s1 == [tuple(s) for s in s2]
    assert list(r1) == [tuple(r) for r in r2]
    for i in range(len(s1)):
        assert {j: sorted(map(tuple, v)) for j, v in t1[i].items()} == \
               {j: sorted(map(tuple, v)) for j, v in t2[i].items()}
