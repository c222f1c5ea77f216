#!/usr/bin/env python3
"""One summary line per bench.py JSON file: tools/bsum.py FILE..."""
import json
import sys

for p in sys.argv[1:]:
    for line in open(p):
        if line.startswith("{"):
            d = json.loads(line)
            r = d["roofline"]
            print("%-40s %9.0f Mpps  step %.4f (med %.4s)  kern avg %.4f med %.4s  floor %s (shape %s)  frac %.4f  ar %s  settle %s"
                  % (p.split("/")[-1], d["value"], d["ms_per_step"], d.get("step_ms_median"), r["kernel_ms_avg"],
                     r.get("kernel_ms_median"), r.get("stream_floor_ms"), r.get("stream_floor_launch_shape_ms"), r["frac"],
                     r.get("allreduce_ms_median_max_rank"), d.get("settle_ms")))
