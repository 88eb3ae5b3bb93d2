#!/usr/bin/env python3
"""LDS bank-conflict model of the fused LeNet-5 train kernel's hot LDS reads (csrc/lenet_fused.hip).

For each phase it replays the byte addresses every lane of every wave issues per LDS instruction over one
workgroup's loop iterations and prices them with the gfx950 banking rules (MI355X_MICROARCH.md, LDS):
an instruction's lanes are serviced in fixed lane groups, one LDS cycle per group when conflict-free;
each extra distinct dword address on a bank within a group costs one more cycle.  Prints, per phase,
LDS-array cycles and the conflict share -- the same ratio as SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
Usage: python3 scripts/lds_sim.py
"""
from collections import defaultdict

import numpy as np

IMG, NT, NW = 8, 512, 8
XS_ELEMS = IMG * 1024 + 32
OFF_XS = 0
OFF_P1 = OFF_XS + XS_ELEMS * 2
OFF_C1 = OFF_P1 + IMG * 196 * 16
OFF_K = OFF_C1 + IMG * 196 * 4
DC2_RS = 104
NM = IMG * DC2_RS
OFF_PX = OFF_K + 32
OFF_FT = OFF_PX + NM * 2
OFF_W = OFF_FT + 98 * 2 * 16
OFF_U = OFF_W + 128 + 32
OFF_XS1 = OFF_U + 32
OFF_DC2 = OFF_U
LD0, LD1, LD2, LD3 = 424, 136, 104, 40
OFF_H0 = OFF_U
OFF_ZR = OFF_U + IMG * LD0 * 2 + IMG * LD1 * 2 + IMG * LD2 * 2 + IMG * LD3 * 2 + IMG * LD2 * 2 + IMG * LD1 * 2
KO = OFF_K
KZ = OFF_W + 128

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]
HALF_GROUPS = [list(range(0, 32)), list(range(32, 64))]


def cycles(kind, addr, active=None):
    """LDS-array cycles of one wave instruction; addr[lane] = byte address (None = inactive lane)."""
    if kind == "b128":
        groups, nd, nb = B128_GROUPS, 4, 64
    elif kind in ("b64", "tr"):
        groups, nd, nb = HALF_GROUPS, 2, 64
    elif kind in ("b32", "b16"):
        groups, nd, nb = HALF_GROUPS, 1, 32
    else:
        raise ValueError(kind)
    total = 0
    for grp in groups:
        banks = defaultdict(set)
        for ln in grp:
            a = addr[ln]
            if a is None:
                continue
            d0 = a // 4
            for k in range(nd):
                banks[(d0 + k) % nb].add(d0 + k)
        total += max([len(v) for v in banks.values()] + [1])
    return total, len(groups)


class Phase:
    def __init__(self, name):
        self.name, self.cyc, self.ideal, self.n = name, 0, 0, 0

    def add(self, kind, addr):
        c, ideal = cycles(kind, addr)
        self.cyc += c
        self.ideal += ideal
        self.n += 1

    def report(self):
        conf = self.cyc - self.ideal
        print(f"{self.name:<28} instr {self.n:6d}  LDS cycles {self.cyc:7d}  conflict {conf:7d} "
              f"({100.0 * conf / max(self.cyc, 1):5.1f} %)")
        return self.cyc, conf


def lanes():
    for lane in range(64):
        yield lane, lane & 15, lane >> 4


def phase_a(ph):
    for w in range(NW):
        for u in range(w, 56, NW):
            mt, x0 = u >> 1, (u & 1) * 16
            for ky in range(5):
                addr = []
                for lane, i, g in lanes():
                    m = 16 * mt + i
                    img, rem = divmod(m, 56)
                    base = (OFF_XS1 if rem & 1 else OFF_XS) + 2 * (img * 1024 + (rem >> 1) * 32 + x0 + 8 * g)
                    addr.append(base + 2 * ky * 32)
                ph.add("b128", addr)


def pxtab():
    px = np.zeros(NM, dtype=np.int64)
    for m in range(NM):
        img, q = divmod(m, DC2_RS)
        if q >= 100:
            px[m] = img * 196
            continue
        win, d = divmod(q, 4)
        py, pxx = divmod(win, 5)
        px[m] = img * 196 + (2 * py + (d >> 1)) * 14 + 2 * pxx + (d & 1)
    return px


def phase_b(ph):
    PX = pxtab()
    for w in range(NW):
        for mt in range(w, NM // 16, NW):
            for s in range(7):
                addr = []
                for lane, i, g in lanes():
                    tap = 4 * s + g
                    toff = ((tap // 5) * 14 + tap % 5) * 8 if tap < 25 else 0
                    addr.append(OFF_P1 + 2 * (int(PX[16 * mt + i]) * 8 + toff))
                ph.add("b128", addr)


def phase_e(ph, ph2=None):
    """A (dC2) reads into ph, the im2col B (P1) reads into ph2 (default: ph too)."""
    PX = pxtab()
    KT = (13 + NW - 1) // NW
    for w in range(NW):
        ntile = (13 - w + NW - 1) // NW
        for s in range(NM // 32):
            # A: two transposed reads of dC2
            for half in range(2):
                addr = []
                for lane, i, g in lanes():
                    q, p = (lane & 15) >> 2, lane & 3
                    mA = 32 * s + 8 * g + q + 4 * half
                    img, t = divmod(mA, DC2_RS)
                    addr.append(OFF_DC2 + 2 * ((img * DC2_RS + dc2_swz(t)) * 16 + 4 * p))
                ph.add("tr", addr)
            for k in range(KT):  # every wave runs KT tiles (taps >= 25 read tap 0's pixel, dropped)
                for half in range(2):
                    addr = []
                    for lane, i, g in lanes():
                        q, p = (lane & 15) >> 2, lane & 3
                        mA = 32 * s + 8 * g + q + 4 * half
                        tap = 2 * (w + NW * k) + (p >> 1)
                        tp = tap if tap < 25 else 0
                        toff = ((tp // 5) * 14 + tp % 5) * 8 + 4 * (p & 1)
                        addr.append(OFF_P1 + 2 * (int(PX[mA]) * 8 + toff))
                    (ph2 if ph2 is not None else ph).add("tr", addr)


def ftab():
    ft = np.full((98, 2, 16), 100, dtype=np.int64)
    for yx in range(98):
        y, X2 = divmod(yx, 7)
        for hf in range(2):
            for s in range(16):
                P = 2 * s + hf
                if P >= 30:
                    continue
                ky, u = divmod(P, 6)
                oy, ox = y - ky, 2 * X2 + 1 - u
                if 0 <= oy < 10 and 0 <= ox < 10:
                    ft[yx, hf, s] = (((oy >> 1) * 5 + (ox >> 1)) << 2) + ((oy & 1) << 1) + (ox & 1)
    return ft


def dc2_swz(t):
    return t ^ ((t >> 3) & 7)


def phase_f(ph):
    FT = ftab()
    for w in range(NW):
        for mt in range(w, 49, NW):
            for s in range(15):
                addr = []
                for lane, i, g in lanes():
                    m = 16 * mt + i
                    img, rem = divmod(m, 98)
                    t = int(FT[rem, g >> 1, s])
                    addr.append(OFF_DC2 + 2 * ((img * DC2_RS + dc2_swz(t)) * 16 + 8 * (g & 1)))
                ph.add("b128", addr)


def phase_g(ph):
    for w in range(NW):
        for rp in range(w, IMG * 14, NW):
            img, py = divmod(rp, 14)
            # pool values: 4 b16 reads per lane
            for wd in range(4):
                addr = []
                for lane, i, g in lanes():
                    ca = i if i < 6 else 5
                    p0 = (img * 14 + py) * 14 + 4 * g
                    ok = 4 * g + wd < 14 and i < 6
                    addr.append(OFF_P1 + 2 * ((p0 + wd) * 8 + ca) if ok else None)
                ph.add("b16", addr)
            for dy in range(2):
                y = 2 * py + dy
                for T in range(2):
                    for h in range(2):  # two ds_read2_b32 (dwords 0, 1 and 2, 3) from a dword-aligned start
                        addr = []
                        for lane, i, g in lanes():
                            tap = 16 * T + i
                            if tap < 25:
                                ky, kx = divmod(tap, 5)
                                base = (OFF_XS1 if kx & 1 else OFF_XS) + 2 * (img * 1024 + y * 32 + ky * 32 + 8 * g)
                                addr.append(base + 4 * (kx >> 1) + 8 * h)
                            else:
                                addr.append((KO if tap == 25 else KZ) + 8 * h)
                        ph.add("b64", addr)


def main():
    tot = conf = 0
    for name, fn in [("A conv1 (A reads)", phase_a), ("B conv2 (A reads)", phase_b),
                     ("E conv2 wgrad (tr reads)", phase_e), ("F conv2 dgrad (A reads)", phase_f),
                     ("G conv1 wgrad", phase_g)]:
        ph = Phase(name)
        if fn is phase_e:
            ph_b = Phase("  of which im2col (P1) reads")
            fn(ph, ph_b)
            ph.cyc += ph_b.cyc
            ph.ideal += ph_b.ideal
            ph.n += ph_b.n
        else:
            fn(ph)
        c, k = ph.report()
        if fn is phase_e:
            ph_b.report()
        tot += c
        conf += k
    print(f"{'modelled total':<28} {'':13} LDS cycles {tot:7d}  conflict {conf:7d} ({100.0 * conf / tot:5.1f} %)")


if __name__ == "__main__":
    main()
