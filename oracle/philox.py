"""Philox4x32-10 and the trial-stream randomness spec (numpy restatement).

TEST INFRASTRUCTURE ONLY.  This module belongs to the oracle: only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may use it.  The
product path (HIP kernels in the package's csrc/) implements the same spec
independently and is checked against this file.

Why a spec at all: the reference never seeds its trial simulations
(Pd_plotter.py:212,219 pass no seed) and the simulator it calls,
`viterbi_markov.simulate_markov_sequence`, does not exist in the repository
(SURVEY.md §0, §8 row A5).  The only seeded draw in the reference is the P̂1
learning chain (Pd_plotter.py:149-155, seed=12345 from Pd_plotter.py:70).
The build therefore defines its own counter-based stream so that every trial
of every grid point is reproducible and independent of how trials are sharded
over lanes, waves, launches or GPUs.

Stream definition (identical in oracle/philox.py, oracle/cvd_oracle.c and
csrc/cvd_common.h):

* key   = (seed & 0xffffffff, seed >> 32)
* a *sequence* is (tag, seq_id).  Trial sequences use seq_id = 2*trial + hyp
  (hyp 0 = H1 stream encoded with G1, hyp 1 = H2 stream encoded with G2) and
  tag = grid_tag(N, p).  The P̂1 learning chain uses seq_id = 0 and
  tag = LEARN_TAG.
* noise (bit-sliced): received word w of a sequence holds steps
  [w*spw, (w+1)*spw), spw = 32 // n, step i of the word in bits [n*i, n*i+n)
  (output bit j of step t is word bit b = (t % spw)*n + j).  The word has 32
  bit-planes P_0..P_31, P_i = word (i % 4) of
  philox(ctr=(8*w + i // 4, seq_lo, seq_hi16 | KIND_NOISE << 16, tag)).  The
  32-bit uniform of word bit b is u_b = sum_i bit_b(P_i) * 2^(31 - i), and the
  bit flips iff u_b < thr(p), thr(p) = floor(p * 2^32) (p == 1.0 -> 2^32, i.e.
  always).  Implementations compare the planes with thr most significant first
  for all bits of the word at once and stop drawing planes once every bit is
  decided (the first plane where u_b and thr differ decides it); the result is
  the same as drawing all 32.
* inputs: input bit i of step t is bit (b % 32) of word ((b // 32) % 4) of
  philox(ctr=(b // 128, seq_lo, seq_hi16 | KIND_INPUT << 16, tag)) with
  b = t*k + i (all zero when random_input=False).
"""
import numpy as np

PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85

KIND_NOISE = 0
KIND_INPUT = 1
LEARN_TAG = 0xC0DE1EA7          # top bit set: never equal to a grid tag
MASK32 = 0xFFFFFFFF


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11).  Arrays of uint32 in,
    tuple of four uint32 arrays out."""
    c0 = np.asarray(c0, dtype=np.uint64) & MASK32
    c1 = np.asarray(c1, dtype=np.uint64) & MASK32
    c2 = np.asarray(c2, dtype=np.uint64) & MASK32
    c3 = np.asarray(c3, dtype=np.uint64) & MASK32
    k0 = int(k0) & MASK32
    k1 = int(k1) & MASK32
    for _ in range(10):
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK32)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK32)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0), lo1,
                          hi0 ^ c3 ^ np.uint64(k1), lo0)
        k0 = (k0 + PHILOX_W0) & MASK32
        k1 = (k1 + PHILOX_W1) & MASK32
    return tuple(x.astype(np.uint32) for x in (c0, c1, c2, c3))


def threshold(p):
    """thr(p) = floor(p * 2^32) as an integer in [0, 2^32]."""
    p = float(p)
    if not (0.0 <= p <= 1.0):
        raise ValueError(f"p must lie in [0, 1], got {p}")
    return int(p * 4294967296.0)


def grid_tag(N, p):
    """32-bit tag of an (N, p) grid point, top bit clear (LEARN_TAG has it set).
    splitmix64 of N and of the IEEE-754 bits of p, folded to 31 bits."""
    bits = int(np.float64(p).view(np.uint64))
    x = (int(N) * 0x9E3779B97F4A7C15 + bits) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 31
    return (x ^ (x >> 32)) & 0x7FFFFFFF


def _ctr_hi(seq_id, kind):
    return ((int(seq_id) >> 32) & 0xFFFF) | (kind << 16)


def noise_word_uniforms(seed, tag, seq_id, w, n):
    """(len(w), 32) uint64 array: the uniforms u_b of word bits b = 0..31 of
    received words `w` (bits b >= spw*n are defined but unused)."""
    w = np.asarray(w, dtype=np.uint64)
    blk = (w[:, None] * np.uint64(8) + np.arange(8, dtype=np.uint64)[None, :]).reshape(-1)
    x = philox4x32_10(blk, np.full_like(blk, int(seq_id) & MASK32),
                      np.full_like(blk, _ctr_hi(seq_id, KIND_NOISE)),
                      np.full_like(blk, tag), seed & MASK32, seed >> 32)
    planes = np.stack(x, axis=1).reshape(len(w), 32).astype(np.uint64)    # plane i = block i//4, word i%4
    bits = (planes[:, :, None] >> np.arange(32, dtype=np.uint64)[None, None, :]) & np.uint64(1)
    weights = (np.uint64(1) << (np.uint64(31) - np.arange(32, dtype=np.uint64)))[None, :, None]
    return (bits * weights).sum(axis=1, dtype=np.uint64)


def noise_bits(seed, tag, seq_id, N, n, p):
    """(N, n) uint8 array of BSC flips for one sequence."""
    spw = 32 // n
    nwords = (N + spw - 1) // spw
    thr = np.uint64(threshold(p))
    out = np.zeros((nwords, spw * n), np.uint8)
    for c0 in range(0, nwords, 4096):                  # bounded memory: (words, 32, 32) per chunk
        ws = np.arange(c0, min(nwords, c0 + 4096))
        u = noise_word_uniforms(seed, tag, seq_id, ws, n)[:, :spw * n]
        out[c0:c0 + len(ws)] = (u < thr).astype(np.uint8)
    return out.reshape(nwords * spw, n)[:N]


def input_bits(seed, tag, seq_id, N, k):
    """(N, k) uint8 array of encoder input bits for one sequence."""
    b = np.arange(N * k, dtype=np.uint64)
    blk = b // 128
    w = ((b // 32) % 4).astype(np.int64)
    x = philox4x32_10(blk, np.full_like(blk, int(seq_id) & MASK32),
                      np.full_like(blk, _ctr_hi(seq_id, KIND_INPUT)),
                      np.full_like(blk, tag), seed & MASK32, seed >> 32)
    word = np.choose(w, x)
    return ((word >> (b % 32).astype(np.uint32)) & 1).astype(np.uint8).reshape(N, k)
