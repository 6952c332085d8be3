#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace (the GPU-side cost of
launching a generation as separate kernels).

  python scripts/kernel_gaps.py gpurun_out/c3k/run_kernel_trace.csv [--last N]

Sorts the dispatches by start time and reports, per (kernel -> next kernel) pair, the count and
the median / mean gap (next start - this end) and the median duration of each kernel, over the
last N dispatches (default: all)."""
import argparse
import csv
import statistics as st
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("mcg::", "")[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=0)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.csv)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows))
    if args.last:
        ks = ks[-args.last:]
    gaps, durs = defaultdict(list), defaultdict(list)
    for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
        gaps[(n0, n1)].append(s1 - e0)
    for s, e, n in ks:
        durs[n].append(e - s)
    print("%-48s %7s %10s" % ("kernel", "count", "med us"))
    for n, d in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        print("%-48s %7d %10.2f" % (n, len(d), st.median(d) / 1e3))
    print()
    print("%-48s -> %-30s %6s %9s %9s" % ("kernel", "next", "count", "med us", "mean us"))
    for (a, b), g in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        print("%-48s -> %-30s %6d %9.2f %9.2f" % (a, b[:30], len(g), st.median(g) / 1e3, st.mean(g) / 1e3))
    span = (ks[-1][1] - ks[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in ks) / 1e3
    print("\nspan %.1f us, kernels busy %.1f us (%.1f %%)" % (span, busy, 100 * busy / span))


if __name__ == "__main__":
    main()
