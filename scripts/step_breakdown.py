#!/usr/bin/env python3
"""Steady-state per-step kernel time by kernel name from a rocprofv3 kernel trace (last 10 steps,
step boundary = the SGD launch):  step_breakdown.py <k_kernel_trace.csv> [anchor substring]"""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "sgd_multi"
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
a, b = idx[-11], idx[-1]
acc, cnt = defaultdict(float), defaultdict(int)
for r in rows[a + 1:b + 1]:
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("dfa::", "").replace("(anonymous namespace)::", ""))
    acc[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 10e3
    cnt[k] += 1
tot = sum(acc.values())
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"{v:8.1f} us/step {cnt[k] // 10:4d} calls  {100 * v / tot:5.1f}%  {k[:90]}")
print(f"total {tot:.1f} us/step, {(b - a) // 10} kernels/step")
if "--order" in sys.argv:  # the last step's launches in stream order: start offset, duration, gap
    print("\nlast step in order (us: start offset, duration, idle gap before):")
    t0 = int(rows[idx[-2] + 1]["Start_Timestamp"])
    prev = None
    for r in rows[idx[-2] + 1:idx[-1] + 1]:
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("dfa::", "").replace("(anonymous namespace)::", ""))
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:7.1f}  {k[:90]}")
        prev = e
