"""Convolutional-code descriptions in the reference's convention.

generator_matrix[j][i] is the tap list of output j for input i, delay-ordered:
taps[0] multiplies the current input bit, taps[d] the register cell d-1
(viterbi_markov.py:92-99).  Taps longer than m+1 are truncated, as the
reference's `min(len(taps), len(x))` does (viterbi_markov.py:97); shorter tap
lists are zero-padded.
"""
import ctypes

import numpy as np

from . import _lib

# demo_script.py:35-52 (preset "2" is labelled (15,13) but its taps are 1111/1011)
EXAMPLE_CODES = {
    "1": {"name": "Rate-1/2, m=2 (7,5) vs (6,5)", "k": 1, "n": 2, "m": 2,
          "gen1": [[[1, 1, 1]], [[1, 0, 1]]], "gen2": [[[1, 1, 0]], [[1, 0, 1]]]},
    "2": {"name": "Rate-1/2, m=3 (15,13) vs (13,15)", "k": 1, "n": 2, "m": 3,
          "gen1": [[[1, 1, 1, 1]], [[1, 0, 1, 1]]], "gen2": [[[1, 0, 1, 1]], [[1, 1, 1, 1]]]},
}

# Code pairs of the BASELINE.json configurations (SURVEY.md §8 "Proposed code pairs").
CONFIG_CODES = {
    "m2": {"k": 1, "n": 2, "m": 2,
           "gen1": [[[1, 1, 1]], [[1, 0, 1]]], "gen2": [[[1, 0, 1]], [[1, 1, 1]]]},
    "m6": {"k": 1, "n": 2, "m": 6,
           "gen1": [[[1, 0, 1, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 0, 1]]],
           "gen2": [[[1, 1, 1, 1, 0, 0, 1]], [[1, 0, 1, 1, 0, 1, 1]]]},
    "r23_m4": {"k": 2, "n": 3, "m": 4,
               "gen1": [[[1, 0, 0, 0, 1], [0, 1, 1, 1, 1]], [[1, 1, 1, 0, 1], [0, 1, 0, 1, 0]],
                        [[0, 1, 1, 0, 0], [1, 1, 0, 1, 0]]],
               "gen2": [[[1, 1, 1, 0, 1], [0, 1, 0, 1, 0]], [[0, 1, 1, 0, 0], [1, 1, 0, 1, 0]],
                        [[1, 0, 0, 0, 1], [0, 1, 1, 1, 1]]]},
}


def octal_to_taps(octal, m):
    """Octal generator (MSB = current input) -> delay-ordered tap list of length m+1.
    e.g. 0o133, m=6 -> [1,0,1,1,0,1,1]."""
    v = int(str(octal), 8) if not isinstance(octal, int) else octal
    return [(v >> (m - d)) & 1 for d in range(m + 1)]


class Code:
    """A (k, n, m) code with flattened taps [n][k][m+1] as uint8 (ABI layout)."""

    def __init__(self, generator_matrix, m, k, n):
        self.k, self.n, self.m = int(k), int(n), int(m)
        g = generator_matrix
        if len(g) != self.n:
            raise ValueError(f"generator matrix has {len(g)} outputs, expected n={self.n}")
        taps = np.zeros((self.n, self.k, self.m + 1), dtype=np.uint8)
        for j in range(self.n):
            if len(g[j]) != self.k:
                raise ValueError(f"output {j} has {len(g[j])} tap lists, expected k={self.k}")
            for i in range(self.k):
                t = [int(b) for b in g[j][i]][: self.m + 1]
                if any(b not in (0, 1) for b in t):
                    raise ValueError("taps must be 0/1")
                taps[j, i, : len(t)] = t
        self.taps = np.ascontiguousarray(taps)
        self._c = _lib.cvd_code(self.k, self.n, self.m,
                                self.taps.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))

    @property
    def c(self):
        return ctypes.byref(self._c)

    @property
    def key(self):
        return (self.k, self.n, self.m, self.taps.tobytes())

    def tables(self):
        """(out_sym[2^m, 2^k], next_state[2^m, 2^k]) — viterbi_markov.py:82-106."""
        M, K = 1 << self.m, 1 << self.k
        out = np.zeros(M * K, np.int32)
        nxt = np.zeros(M * K, np.int32)
        _lib.check(_lib.lib().cvd_code_tables(self.c, out.ctypes.data, nxt.ctypes.data))
        return out.reshape(M, K), nxt.reshape(M, K)

    def __repr__(self):
        return f"Code(k={self.k}, n={self.n}, m={self.m}, taps={self.taps.tolist()})"


def as_code(gen, m, k, n):
    return gen if isinstance(gen, Code) else Code(gen, m, k, n)
