#!/usr/bin/env python3
"""Average duration per kernel family from rocprofv3 kernel_stats.csv files:
tools/kstats.py FILE ..."""
import csv
import sys

for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        short = n[:n.index("(cls::")] if "(cls::" in n else n
        short = short.replace("void ", "").replace("cls::(anonymous namespace)::", "")
        print("  %-60s calls %4s avg %9.1f us" % (short[:60], r["Calls"], float(r["AverageNs"]) / 1e3))
