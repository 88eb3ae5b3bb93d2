#!/usr/bin/env python3
"""Search the per-block XOR swizzle of the LeNet conv2 output-gradient rows (csrc/lenet_fused.hip DC2):
row t of an image is stored at t ^ h[t >> 3] (13 blocks of 8 rows, h[b] in 0..7).  Cost = modelled
LDS-array cycles (scripts/lds_sim.py banking rules) of the reads that depend on it: phase F's gathered
A-operand reads and phase E's transposed dC2 reads.  Coordinate descent from h[b] = b & 7 (the previous
t ^ ((t >> 3) & 7)).  Usage: python3 scripts/lds_swizzle_search.py"""
import lds_sim as S


def cost(h):
    swz = lambda t: t ^ h[t >> 3]  # noqa: E731
    S.dc2_swz = swz
    ph_e, ph_f = S.Phase("E"), S.Phase("F")
    S.phase_e(ph_e, S.Phase("E-B"))
    S.phase_f(ph_f)
    return ph_e.cyc + ph_f.cyc, ph_e.cyc, ph_f.cyc


def main():
    h = [b & 7 for b in range(13)]
    best = cost(h)
    print("start", h, best)
    for sweep in range(3):
        improved = False
        for b in range(13):
            for v in range(8):
                if v == h[b]:
                    continue
                h2 = h[:b] + [v] + h[b + 1:]
                c = cost(h2)
                if c[0] < best[0]:
                    h, best, improved = h2, c, True
        print("sweep", sweep, h, best, flush=True)
        if not improved:
            break


if __name__ == "__main__":
    main()
