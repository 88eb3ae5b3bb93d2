#!/usr/bin/env python3
"""Search a per-image permutation of the LeNet conv2 output-gradient rows (csrc/lenet_fused.hip DC2, 104
rows per image block) that minimises the modelled LDS bank conflicts of the reads that gather them:
phase F's A-operand rows (16-byte reads, table-driven) and phase E's transposed dC2 reads.  Only a
row's slot matters: 16-byte slot = 2 (stored row mod 8) + column half (F), dword pair slot = stored row
mod 8 and 8-byte chunk (E).  Simulated annealing over swaps; prints the permutation as a Python list.
Usage: python3 scripts/lds_perm_search.py [iterations]"""
import sys

import numpy as np

import lds_sim as S

RS = 104


def f_requests():
    """Phase F: per b128 instruction and lane group, the (logical row t, half) of every lane (one image:
    the groups of every image are the same up to a multiple of 256 bytes)."""
    FT = S.ftab()
    reqs = []
    for mt in range(49):
        for s in range(15):
            lanes = []
            for lane, i, g in S.lanes():
                m = 16 * mt + i
                rem = m % 98
                lanes.append((int(FT[rem, g >> 1, s]) if FT[rem, g >> 1, s] != 255 else 100, g & 1))
            for grp in S.B128_GROUPS:
                reqs.append([lanes[l] for l in grp])
    return reqs


def e_requests():
    """Phase E's dC2 reads: per instruction and half-wave group, the (row t in the image, chunk p)."""
    reqs = []
    for s in range(RS * 8 // 32):
        for half in range(2):
            lanes = []
            for lane, i, g in S.lanes():
                q, p = (lane & 15) >> 2, lane & 3
                mA = 32 * s + 8 * g + q + 4 * half
                lanes.append((mA % RS, p, mA // RS))
            for grp in S.HALF_GROUPS:
                reqs.append([lanes[l] for l in grp])
    return reqs


def cost(perm, F, E):
    tot = 0
    for grp in F:
        slots = {}
        for t, h in grp:
            slots.setdefault(2 * (perm[t] % 8) + h, set()).add(t)
        tot += max(len(v) for v in slots.values())
    for grp in E:
        slots = {}
        for t, p, img in grp:
            slots.setdefault((perm[t] % 8, p), set()).add((img, t))
        tot += max(len(v) for v in slots.values())
    return tot


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    F, E = f_requests(), e_requests()
    rng = np.random.default_rng(1)
    perm = [t ^ ((t >> 3) & 7) for t in range(RS)]  # the current swizzle
    best = cur = cost(perm, F, E)
    print("start", cur, "ideal", len(F) + len(E), flush=True)
    bestp = perm[:]
    T = 2.0
    for it in range(iters):
        a, b = rng.integers(0, RS, 2)
        if a == b:
            continue
        perm[a], perm[b] = perm[b], perm[a]
        c = cost(perm, F, E)
        if c <= cur or rng.random() < np.exp((cur - c) / T):
            cur = c
            if c < best:
                best, bestp = c, perm[:]
        else:
            perm[a], perm[b] = perm[b], perm[a]
        T = max(0.05, T * 0.999)
        if it % 500 == 0:
            print(it, cur, best, flush=True)
    print("best", best, "ideal", len(F) + len(E))
    print("PERM =", bestp)


if __name__ == "__main__":
    main()
