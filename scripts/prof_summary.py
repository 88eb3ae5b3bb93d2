#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace --stats`` output directory as a per-step kernel table.

    python scripts/prof_summary.py DIR --marker lenet_reduce_kernel<0>

The step count is NOT given by hand (a trace holds warm-up, guard and other engines'
launches, so total / steps over-counted).  ``--marker`` names a kernel launched exactly once per training
step of the engine being measured (e.g. its optimizer / reduce launch).  From the per-dispatch trace every
interval between two consecutive marker starts is one step; the table is the median over the steady-state
intervals (those no longer than 1.5 x the median interval, which drops the warm-up, the correctness guard
and anything another engine ran in between) of each kernel's time inside the interval, and the step total
is the median interval's summed kernel time.  Without a trace file the script falls back to the stats file
and divides by the marker's call count (flagged in the output).
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def _short(n: str) -> str:
    return n.replace("void dfa::", "").replace("dfa::", "").replace("(anonymous namespace)::", "")[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out/prof")
    ap.add_argument("--marker", required=True, help="substring of a kernel launched once per step")
    args = ap.parse_args()
    traces = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not traces:
        stats = glob.glob(os.path.join(args.dir, "**", "*kernel_stats.csv"), recursive=True)
        rows = list(csv.DictReader(open(stats[0])))
        steps = sum(int(r["Calls"]) for r in rows if args.marker in r["Name"])
        print(f"(no kernel trace: stats only, {steps} marker calls; warm-up and guard launches included)")
        for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
            t = float(r["TotalDurationNs"])
            print(f"{t / 1e3 / int(r['Calls']):9.1f} {r['Calls']:>6} {t / 1e3 / max(steps, 1):8.1f}  {_short(r['Name'])}")
        return
    recs = []
    for f in traces:
        for r in csv.DictReader(open(f)):
            recs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    recs.sort()
    marks = [s for s, _, n in recs if args.marker in n]
    if len(marks) < 3:
        raise SystemExit(f"marker {args.marker!r} found {len(marks)} times: need >= 3")
    ivals = list(zip(marks[:-1], marks[1:]))
    med_len = statistics.median(e - s for s, e in ivals)
    steady = [(s, e) for s, e in ivals if e - s <= 1.5 * med_len]
    per = defaultdict(list)  # kernel -> [time in each steady interval]
    calls = defaultdict(list)
    totals = []
    j = 0
    for s, e in steady:
        while j < len(recs) and recs[j][0] < s:
            j += 1
        k = j
        t_in = defaultdict(float)
        c_in = defaultdict(int)
        while k < len(recs) and recs[k][0] < e:
            t_in[recs[k][2]] += (recs[k][1] - recs[k][0]) / 1e3
            c_in[recs[k][2]] += 1
            k += 1
        totals.append(sum(t_in.values()))
        for n in set(t_in) | set(per):
            per[n].append(t_in.get(n, 0.0))
            calls[n].append(c_in.get(n, 0))
    n_st = len(steady)
    print(f"marker {args.marker!r}: {len(marks)} launches, {n_st} steady-state steps "
          f"(median step period {med_len / 1e3:.1f} us)")
    print(f"{'us/step':>8} {'calls/step':>10} {'us/call':>8}  kernel")
    rows = []
    for n, ts in per.items():
        ts = ts + [0.0] * (n_st - len(ts))
        cs = calls[n] + [0] * (n_st - len(calls[n]))
        m = statistics.median(ts)
        c = statistics.median(cs)
        rows.append((m, c, n))
    for m, c, n in sorted(rows, key=lambda r: -r[0]):
        if m <= 0:
            continue
        print(f"{m:8.1f} {c:10.1f} {m / c if c else 0.0:8.1f}  {_short(n)}")
    print(f"kernel time per step (median over steady-state steps): {statistics.median(totals):.1f} us; "
          f"step period {med_len / 1e3:.1f} us")


if __name__ == "__main__":
    main()
