#!/usr/bin/env python3
"""Gaps between consecutive kernels in a rocprofv3 --kernel-trace CSV (one
device): where the GPU sat idle between dispatches, with the kernels on
either side.  Usage: python scripts/kernel_gaps.py run_kernel_trace.csv [min_us]"""
import csv
import sys


def main():
    path = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60])
                 for r in rows), key=lambda t: t[0])
    prev = None
    for s, e, name in ks:
        if prev is not None:
            gap = (s - prev[1]) / 1e3
            if gap >= min_us:
                print("%10.1f us idle  after %-60s before %s  (dur %.3f ms)"
                      % (gap, prev[2], name, (e - s) / 1e6))
        prev = (s, e, name)


if __name__ == "__main__":
    main()
