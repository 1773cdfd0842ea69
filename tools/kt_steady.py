#!/usr/bin/env python3
"""Steady-state per-kernel durations from a rocprofv3 kernel trace (CSV).

    python tools/kt_steady.py DIR [--last 20] [--first KERNEL]

For each kernel: the median duration of its last N dispatches (the stats file's average includes
the first frames, whose births dominate some kernels).  With --first (the frame's first kernel),
also the median frame period, the median summed kernel time per frame and the idle gap between
them (launch / drain overhead of the frame's chain)."""
import argparse
import csv
import glob
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--first", default=None, help="first kernel of a frame (e.g. k_bs_prep)")
    args = ap.parse_args()
    f = glob.glob(args.dir + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    ev = []
    for r in rows:
        m = re.search(r"(k_\w+(<\d+>)?)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:30]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    ev.sort()
    by = {}
    for s, e, n in ev:
        by.setdefault(n, []).append(e - s)
    tot = 0.0
    for n, d in sorted(by.items(), key=lambda kv: -statistics.median(kv[1][-args.last:])):
        med = statistics.median(d[-args.last:]) / 1e3
        print(f"  {n:<24s} n={len(d):4d}  median(last {args.last}) {med:8.2f} us")
    if args.first:
        starts = [i for i, (_, _, n) in enumerate(ev) if n == args.first]
        per, busy = [], []
        for a, b in zip(starts[-args.last - 1:-1], starts[-args.last:]):
            per.append((ev[b][0] - ev[a][0]) / 1e3)
            busy.append(sum(e - s for s, e, _ in ev[a:b]) / 1e3)
        if per:
            p, k = statistics.median(per), statistics.median(busy)
            print(f"  frame period {p:.2f} us, kernels {k:.2f} us, idle {p - k:.2f} us "
                  f"(median of the last {len(per)} frames)")


if __name__ == "__main__":
    main()
