"""CPU restatement of the reference's hot path (pure Python / numpy).

TEST INFRASTRUCTURE ONLY — the oracle.  Only `tests/`, `__graft_entry__.smoke()`
and `bench.py`'s cpu_baseline leg may import this module, and only as the
checker.  The product (the package's HIP kernels + native host setup) never
calls it.

Every function restates one reference function; the reference file:line it
follows is cited in its docstring.  The reference is
So-bonkers/Detecting-Convolutional-Codes-Via-Markovian-Statistics (pure Python).
Pinned against golden vectors produced by the reference itself
(tests/golden/make_golden.py, tests/test_oracle_golden.py).

Conventions restated from the reference (SURVEY.md §2 "Inventory notes"):
* generator_matrix[j][i] is the tap list of output j for input i, delay
  ordered: taps[0] multiplies the current input bit, taps[d] (d >= 1) the
  state bit d-1 (viterbi_markov.py:92-99); taps longer than m+1 are truncated
  (viterbi_markov.py:97).
* every input of a rate-k/n code sees the same m-bit register in its tap
  window while the register advances by k (viterbi_markov.py:94-104).
* states are ints, bit i = register cell i (viterbi_markov.py:60-75).
"""
import itertools
import math
from collections import defaultdict, deque

import numpy as np

from . import philox


# ─────────────────────────── trellis (L0) ────────────────────────────────

def branch_output_and_next_state(state_int, input_bits, generator_matrix, m, k):
    """Restates viterbi_markov.py:82-106 (one encoder branch)."""
    x_state = [(state_int >> i) & 1 for i in range(m)]
    out = []
    for gen in generator_matrix:
        b = 0
        for i in range(k):
            x = [int(input_bits[i])] + x_state
            taps = gen[i]
            for j in range(min(len(taps), len(x))):
                b ^= int(taps[j]) & x[j]
        out.append(b)
    regs = (list(input_bits) + x_state[:max(0, m - k)])[:m] if m > 0 else []
    ns = 0
    for i, bit in enumerate(regs):
        ns |= (int(bit) & 1) << i
    return tuple(out), ns


def build_trellis(generator_matrix, m, k):
    """Restates viterbi_markov.py:118-132: incoming branches per next state,
    predecessors listed in ascending (state, input) order."""
    incoming = {s: [] for s in range(1 << m)}
    for s in range(1 << m):
        for u in itertools.product([0, 1], repeat=k):
            out, ns = branch_output_and_next_state(s, u, generator_matrix, m, k)
            incoming[ns].append((s, u, out))
    return incoming


def encoder_tables(generator_matrix, m, k, n):
    """Dense encoder tables: out_sym[s][U] (bit j = output j) and
    next_state[s][U], U = sum_i u_i << i (the reference's input tuple u with
    u[i] = bit i of U, viterbi_markov.py:128)."""
    S, K = 1 << m, 1 << k
    out_sym = np.zeros((S, K), dtype=np.int64)
    nxt = np.zeros((S, K), dtype=np.int64)
    for s in range(S):
        for U in range(K):
            u = tuple((U >> i) & 1 for i in range(k))
            out, ns = branch_output_and_next_state(s, u, generator_matrix, m, k)
            out_sym[s, U] = sum(b << j for j, b in enumerate(out))
            nxt[s, U] = ns
    return out_sym, nxt


# ─────────────────────── Eq. 4-5 recursion (L1) ─────────────────────────

def viterbi_metric_step(D_prev, trellis, y_t):
    """Restates viterbi_markov.py:139-159.
    Eq. 4: D'(i) = min_s D(s) + d_H(y, V(s));  Eq. 5: D = D' - min D'."""
    num_states = len(D_prev)
    nxt = [math.inf] * num_states
    for ns in range(num_states):
        best = math.inf
        for (ps, _, out) in trellis[ns]:
            v = D_prev[ps] + sum(a != b for a, b in zip(out, y_t))
            if v < best:
                best = v
        nxt[ns] = best
    mn = min(nxt)
    return tuple(int(v - mn) for v in nxt)


def metric_step_vec(D_prev, out_sym, nxt, r, n):
    """The same step on numpy tables (vectorised over states).  r is the
    received word as an int (bit j = output j)."""
    S = len(D_prev)
    bm = np.array([bin(int(o) ^ int(r)).count("1") for o in out_sym.reshape(-1)],
                  dtype=np.int64).reshape(out_sym.shape)
    cand = np.asarray(D_prev, dtype=np.int64)[:, None] + bm
    Dn = np.full(S, np.iinfo(np.int64).max, dtype=np.int64)
    np.minimum.at(Dn, nxt.reshape(-1), cand.reshape(-1))
    return Dn - Dn.min()


# ───────────────── Markov state enumeration (Sec. III-B) ─────────────────

def enumerate_markov_states_allzero(generator_matrix, m, k, n):
    """Restates viterbi_markov.py:166-195: BFS from D_0 = 0 over all 2^n
    received words; index = discovery order; Y(i,j) lists received words."""
    trellis = build_trellis(generator_matrix, m, k)
    all_r = list(itertools.product([0, 1], repeat=n))
    start = tuple([0] * (1 << m))
    queue = deque([start])
    visited = {start: 0}
    states = [start]
    transitions = defaultdict(lambda: defaultdict(list))
    while queue:
        cur = queue.popleft()
        ci = visited[cur]
        for r in all_r:
            nx = viterbi_metric_step(list(cur), trellis, r)
            if nx not in visited:
                visited[nx] = len(states)
                states.append(nx)
                queue.append(nx)
            transitions[ci][visited[nx]].append(r)
    return states, transitions, all_r


def T_half(states, transitions, all_r):
    """T(p) of Eq. 6 (viterbi_markov.py:202-230) evaluated at p = 1/2 and
    row-renormalised (Pd_plotter.py:89-99).  At p = 1/2 every received word
    has weight 2^-n, so T[i,j] = |Y(i,j)| / 2^n exactly (SURVEY.md §0.4;
    pinned by the golden T matrices from the reference's sympy path)."""
    S = len(states)
    R = len(all_r)
    T = np.zeros((S, S))
    for i in range(S):
        for j, rl in transitions[i].items():
            T[i, j] = len(rl) / R
    rs = T.sum(axis=1, keepdims=True)
    rs[rs == 0] = 1.0
    return T / rs


# ───────────────────── missing simulator, spec'd (A5) ─────────────────────

def r_tuple(rint, n):
    return tuple((rint >> j) & 1 for j in range(n))


def received_stream(enc_gen, m, k, n, N, p, seed, tag, seq_id, random_input=True):
    """Encoder (G_enc) -> BSC(p) for one sequence of N steps.  Returns an int64
    array of N received words (bit j = output j).  Spec of the missing
    `simulate_markov_sequence`: encoder state starts at
    0, u ~ Bern(1/2)^k per step (zeros if random_input=False), output via
    viterbi_markov.py:82-106, r = out XOR Bern(p)^n."""
    out_sym, nxt = encoder_tables(enc_gen, m, k, n)
    if random_input:
        ub = philox.input_bits(seed, tag, seq_id, N, k).astype(np.int64)
        U = (ub << np.arange(k, dtype=np.int64)).sum(axis=1)
    else:
        U = np.zeros(N, dtype=np.int64)
    nb = philox.noise_bits(seed, tag, seq_id, N, n, p).astype(np.int64)
    noise = (nb << np.arange(n, dtype=np.int64)).sum(axis=1)
    r = np.empty(N, dtype=np.int64)
    s = 0
    for t in range(N):
        r[t] = out_sym[s, U[t]] ^ noise[t]
        s = nxt[s, U[t]]
    return r


def metrics_from_stream(dec_gen, m, k, n, r):
    """D_0..D_N (tuples) for received words r, decoded on trellis(dec_gen);
    D_0 = zeros (viterbi_markov.py:177, Pd_plotter.py:20)."""
    trellis = build_trellis(dec_gen, m, k)
    D = tuple([0] * (1 << m))
    out = [D]
    for rv in r:
        D = viterbi_metric_step(list(D), trellis, r_tuple(int(rv), n))
        out.append(D)
    return out


def simulate_markov_sequence(generator_matrix, m, k, n, N, p_val, random_input=True,
                             seed=None, *, decoder=None, tag=philox.LEARN_TAG, seq_id=0):
    """Spec of the missing viterbi_markov.simulate_markov_sequence (call sites
    Pd_plotter.py:149-155, :212, :219).  Encodes with `generator_matrix`,
    decodes with `decoder` (G1 — the decoder is fixed to H1,
    Pd_plotter.py:188; defaults to the encoder itself).  Returns
    {"metrics": [D_0, ..., D_N]} with hashable tuples (Pd_plotter.py:161)."""
    dec = generator_matrix if decoder is None else decoder
    sd = 0 if seed is None else int(seed)
    r = received_stream(generator_matrix, m, k, n, N, p_val, sd, tag, seq_id, random_input)
    return {"metrics": metrics_from_stream(dec, m, k, n, r), "received": r}


# ───────────────────────── likelihood (A9) ────────────────────────────────

def log_prob_sequence(metrics, state_index, T):
    """Restates Pd_plotter.py:106-116: sequential fp64 sum of
    log(max(T[i,j], 1e-300)) in t order."""
    logp = 0.0
    for t in range(len(metrics) - 1):
        i = state_index[metrics[t]]
        j = state_index[metrics[t + 1]]
        logp += math.log(max(T[i, j], 1e-300))
    return logp


# ─────────────────────── P̂1 learning (A8) ─────────────────────────────────

def learn_len_eff(learn_len, S):
    """Pd_plotter.py:143-146."""
    return max(5000, 200 * S) if learn_len is None else learn_len


def learn_P1_empirical(gen1, k, n, m, p, learn_len, learn_burn, laplace, seed,
                       states=None, transitions=None):
    """Restates Pd_plotter.py:123-169 with the spec'd learning chain
    (seed-keyed Philox stream, LEARN_TAG): counts over t in
    [learn_burn, len(metrics)-1), Laplace smoothing, row normalisation."""
    if states is None:
        states, transitions, _ = enumerate_markov_states_allzero(gen1, m, k, n)
    sidx = {s: i for i, s in enumerate(states)}
    S = len(states)
    L = learn_len_eff(learn_len, S)
    sim = simulate_markov_sequence(gen1, m, k, n, L, p_val=p, random_input=True, seed=seed)
    metrics = sim["metrics"]
    counts = np.zeros((S, S))
    for t in range(learn_burn, len(metrics) - 1):
        counts[sidx[metrics[t]], sidx[metrics[t + 1]]] += 1.0
    P = counts + laplace
    P /= P.sum(axis=1, keepdims=True)
    return states, sidx, P


# ───────────────────────── trial loop (A10) ───────────────────────────────

def run_trials(gen1, gen2, k, n, m, N, p, seed, trial_begin, trial_end, sidx, P1, Tref,
               return_sums=False):
    """Restates the body of Pd_plotter.py:198-223 for one (N, p) grid point
    over global trials [trial_begin, trial_end).  Trial t's H1 stream is
    (tag, seq_id = 2t), its H2 stream (tag, 2t+1)."""
    tag = philox.grid_tag(N, p)
    s1 = s2 = 0
    sums = []
    for t in range(trial_begin, trial_end):
        for hyp, gen in ((0, gen1), (1, gen2)):
            r = received_stream(gen, m, k, n, N, p, seed, tag, 2 * t + hyp)
            met = metrics_from_stream(gen1, m, k, n, r)
            lp = log_prob_sequence(met, sidx, P1)
            lr = log_prob_sequence(met, sidx, Tref)
            sums.append((lp, lr))
            if hyp == 0 and lp > lr:
                s1 += 1
            if hyp == 1 and lp <= lr:
                s2 += 1
    return (s1, s2, sums) if return_sums else (s1, s2)


def run_experiment(k, n, m, gen1, gen2, num_iter, p_vec, learn_len, learn_burn, laplace,
                   seed, N_list):
    """Restates Pd_plotter.py:176-235 (returns a list of dict rows N,p,Pd,Pc)."""
    states, transitions, all_r = enumerate_markov_states_allzero(gen1, m, k, n)
    sidx = {s: i for i, s in enumerate(states)}
    Tref = T_half(states, transitions, all_r)
    rows = []
    for N in N_list:
        for p in p_vec:
            _, sidx_L, P1 = learn_P1_empirical(gen1, k, n, m, p, learn_len, learn_burn,
                                               laplace, seed, states, transitions)
            s1, s2 = run_trials(gen1, gen2, k, n, m, N, p, seed, 0, num_iter, sidx_L, P1, Tref)
            rows.append({"N": N, "p": p, "Pd": s1 / num_iter,
                         "Pc": (s1 + s2) / (2 * num_iter)})
    return rows
