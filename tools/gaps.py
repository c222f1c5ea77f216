#!/usr/bin/env python3
"""Kernel durations and the idle gaps between consecutive kernels, from a
rocprofv3 --kernel-trace CSV (run_kernel_trace.csv): per kernel name the
median duration, and the median gap before each kernel (end of the previous
kernel on the device to this one's start), over the last N dispatches.
usage: python tools/gaps.py run_kernel_trace.csv [--last 200]
"""
import argparse
import collections
import csv

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=200)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.last:]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][-60:]
        dur[name].append((e - s) / 1e3)
        if prev_end is not None:
            gap[name].append((s - prev_end) / 1e3)
        prev_end = e
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    busy = sum(sum(v) for v in dur.values())
    print("last %d dispatches: span %.1f us, busy %.1f us (%.1f %%)" % (len(rows), span, busy, 100 * busy / span))
    for k in dur:
        print("%-62s n %4d  median %8.2f us  gap before: median %6.2f us" % (
            k, len(dur[k]), np.median(dur[k]), np.median(gap[k]) if gap[k] else float("nan")))


if __name__ == "__main__":
    main()
