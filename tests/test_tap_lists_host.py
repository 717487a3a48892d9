"""Host check of the generator's unrolled tap lists (ChunkEncoder kT > 0, gen_args in
csrc/cvd_kernels.hip): every tap of output j is one 32-bit funnel shift (v_alignbit) of the
64-bit window of the previous and current word, the lists are padded to a fixed length with
shifts that move only empty window lanes onto lane j, and the lane mask after the XOR
leaves exactly the loop form's word -- for random codes of every bit-parallel shape
(rate 1/2 and 1/3 spread-first windows, rate 2/3 stride-3 window).  This is the
invariant the GPU test (tests/test_gpu_gen_taps.py) checks on the device streams."""
import random

import pytest

M32 = 0xFFFFFFFF


def alignbit(hi, lo, s):
    return (((hi << 32) | lo) >> (s & 31)) & M32


def spread_n(x, n):
    out = 0
    for i in range(32 // n):
        if (x >> i) & 1:
            out |= 1 << (n * i)
    return out


def spread23(x):   # bit 2t + r -> bit 3t + r (t < 10)
    out = 0
    for t in range(10):
        for r in range(2):
            if (x >> (2 * t + r)) & 1:
                out |= 1 << (3 * t + r)
    return out


def window_taps(k, n, m, gmask):
    """per (output j, input phase r) the window tap set (gen_args)"""
    hs = (m + k - 1) // k
    taps = [[0, 0] for _ in range(n)]
    for j in range(n):
        for i in range(k):
            g = gmask[j * k + i]
            if g & 1:
                taps[j][i] ^= 1 << hs
            for b in range(m):
                if (g >> (1 + b)) & 1:
                    taps[j][b % k] ^= 1 << (hs - 1 - b // k)
    return hs, taps


def packed_lists(k, n, hs, taps, slots=10):
    """gen_args: shift per set tap, padded, five bits per slot, six slots per word"""
    stride3 = k == 2
    ntap, packed = 0, []
    for j in range(n):
        sl = [30 - 3 * hs + 3 * sh + r - j if stride3 else n * sh
              for r in range(k) for sh in range(32) if (taps[j][r] >> sh) & 1]
        ntap = max(ntap, len(sl))
        sl += [(5 - j) if stride3 else 1] * (slots - len(sl))
        pk = [0, 0]
        for i, s in enumerate(sl[:slots]):
            pk[i // 6] |= (s & 31) << (5 * (i % 6))
        packed.append(pk)
    return ntap, packed


def slot(pk, i):
    p = pk[i // 6]
    return p >> (5 * (i % 6)) if i % 6 else p


@pytest.mark.parametrize("k,n", [(1, 2), (1, 3), (2, 3)])
def test_padded_tap_lists_equal_loop_form(k, n):
    rng = random.Random(1000 * k + n)
    spw = 32 // n
    checked = 0
    for _ in range(400):
        m = rng.randint(1, 8)
        hs = (m + k - 1) // k
        if hs + spw > 32:
            continue
        gmask = [rng.randrange(1, 1 << (m + 1)) for _ in range(n * k)]
        hs, taps = window_taps(k, n, m, gmask)
        ntap, packed = packed_lists(k, n, hs, taps)
        if ntap > 10:
            continue
        kt = next(t for t in (3, 4, 5, 6, 8, 10) if ntap <= t)
        for _ in range(8):
            loop = lists = 0
            if k == 2:   # stride-3 window X = current << 30 | previous (60 bits)
                prev, cur = spread23(rng.getrandbits(20)), spread23(rng.getrandbits(20))
                lo, hi = ((cur << 30) | prev) & M32, cur >> 2
                for j in range(3):
                    o = 0
                    for r in range(2):
                        for sh in range(32):
                            if (taps[j][r] >> sh) & 1:
                                o ^= alignbit(hi, lo, 30 - 3 * hs + 3 * sh + r - j)
                    loop |= o & (0x09249249 << j)
                    o = 0
                    for i in range(kt):
                        o ^= alignbit(hi, lo, slot(packed[j], i))
                    lists |= o & (0x09249249 << j)
            else:        # spread-first window (hi, lo), data on lane 0 of stride n
                nhs, nrest = n * hs, n * (spw - hs)
                su, sp = spread_n(rng.getrandbits(spw), n), spread_n(rng.getrandbits(spw), n)
                lo, hi = ((su << nhs) | (sp >> nrest)) & M32, su >> (32 - nhs)
                lane0 = 0x55555555 if n == 2 else 0x09249249
                for j in range(n):
                    o = 0
                    for sh in range(32):
                        if (taps[j][0] >> sh) & 1:
                            o ^= alignbit(hi, lo, n * sh)
                    loop |= (o << j) & M32
                    o = 0
                    for i in range(kt):
                        o ^= alignbit(hi, lo, slot(packed[j], i))
                    lists |= ((o & lane0) << j) & M32
                if n == 3:
                    loop &= (1 << 30) - 1
                    lists &= (1 << 30) - 1
            assert lists == loop, (k, n, m, gmask)
            checked += 1
    assert checked > 1000
