#!/usr/bin/env python3
"""Search for the cheapest canonicalisation networks of the bit-sliced m = 6 layout
(csrc/cvd_bitslice.h bs_canon).

The digest plane z is 64 bits held as two 32-bit words: a location address has 6 bits,
0..4 the bit position and 5 the word.  At layout phase f label b of the state index sits
at location kSig0[(b - f) mod 6]; bringing z from phase f to phase 0 moves the bit at
location kSig0[c] to kSig0[c + f] -- a permutation of the address bits.  Primitives and
their VALU cost for the 64-bit plane:
  * any permutation of address bits 3, 4, 5 (the byte address): one v_perm_b32 per word, 2;
  * swap address bit i < 3 with bit 5 (the word): two shifts and two v_bitop3 selects, 4;
  * swap two address bits inside the words: a delta swap (shift, and-xor, shift, xor3) per
    word, 8.
Dijkstra over the 720 permutations gives the cheapest sequence for every target; over the
60 cyclic orders of the six locations this prints the orders with the smallest total over
the five non-trivial phases and the networks of the best one (the kernel uses kSig0 =
(0, 1, 3, 4, 2, 5): 14 / 16 / 16 / 16 / 14 VALU for f = 1..5).

  python profiles/r05_canon_search.py
"""
import heapq
import itertools


def compose(a, b):  # apply a, then b
    return tuple(b[a[i]] for i in range(6))


def primitives():
    ident = tuple(range(6))
    out = []
    for q in itertools.permutations([3, 4, 5]):
        p = list(range(6))
        p[3], p[4], p[5] = q
        if tuple(p) != ident:
            out.append((tuple(p), 2, "bperm" + str(q)))
    for i in range(5):
        for j in range(i + 1, 6):
            p = list(range(6))
            p[i], p[j] = j, i
            cost = 4 if (j == 5 and i < 3) else (2 if i >= 3 else 8)
            out.append((tuple(p), cost, f"swap{i}{j}"))
    return out


def search():
    ident = tuple(range(6))
    prims = primitives()
    dist, prev, pq = {ident: 0}, {ident: None}, [(0, ident)]
    while pq:
        d, u = heapq.heappop(pq)
        if d > dist[u]:
            continue
        for p, c, name in prims:
            v = compose(u, p)
            if d + c < dist.get(v, 1 << 30):
                dist[v], prev[v] = d + c, (u, name)
                heapq.heappush(pq, (d + c, v))
    return dist, prev


def path(prev, v):
    out = []
    while prev[v]:
        u, name = prev[v]
        out.append(name)
        v = u
    return out[::-1]


def rotation(cyc, k):
    p = [0] * 6
    for i in range(6):
        p[cyc[i]] = cyc[(i + k) % 6]
    return tuple(p)


def main():
    dist, prev = search()
    res = []
    for order in itertools.permutations(range(1, 6)):
        cyc = (0,) + order
        costs = [dist[rotation(cyc, k)] for k in range(1, 6)]
        res.append((sum(costs), cyc, costs))
    res.sort()
    for r in res[:6]:
        print("total %d  cycle %s  per phase %s" % r)
    best = (0, 1, 3, 4, 2, 5)
    print("kernel's kSig0", best)
    for k in range(1, 6):
        p = rotation(best, k)
        print(f"  phase {k}: {dist[p]:2d} VALU  {path(prev, p)}")


if __name__ == "__main__":
    main()
