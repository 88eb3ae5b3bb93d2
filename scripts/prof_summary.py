#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: per-kernel time per training step."""
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
f = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'us/call':>9} {'calls':>6} {'%':>6} {'us/step':>8}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    n = r["Name"]
    n = n.replace("void dfa::", "").replace("dfa::", "")[:100]
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e3 / int(r['Calls']):9.1f} {r['Calls']:>6} {float(r['Percentage']):6.1f} {t / 1e3 / steps:8.1f}  {n}")
print(f"total kernel time {tot / 1e6:.3f} ms ; per step {tot / 1e3 / steps:.1f} us")
