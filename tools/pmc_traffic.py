#!/usr/bin/env python3
"""Summarise rocprofv3 output for the classify kernel.

Usage:
  pmc_traffic.py stats  <kernel_stats.csv> <out.json>
  pmc_traffic.py pmc    <fetch counter_collection.csv> <write counter_collection.csv>
                        <config> <packets> <out.json>

HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of a
wide coalesced streaming read (128-B requests tallied at 64 B), so the read
side is doubled.  FETCH_SIZE and WRITE_SIZE are collected in separate passes.
"""
import csv
import json
import os
import sys

KERNEL = "classify4_cls"


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def _kname(r):
    return r.get("Kernel_Name") or r.get("Name") or r.get("KernelName") or ""


def stats(path, out):
    rows = [r for r in _rows(path) if KERNEL in _kname(r) or "classify" in _kname(r)]
    res = []
    for r in rows:
        res.append({"kernel": _kname(r), "calls": int(r["Calls"]),
                    "avg_ms": float(r["AverageNs"]) / 1e6, "total_ms": float(r["TotalDurationNs"]) / 1e6})
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


def _per_dispatch(path, counter, kernel=KERNEL):
    vals = {}
    for r in _rows(path):
        if kernel not in _kname(r):
            continue
        if r.get("Counter_Name") != counter:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def _source_hash():
    """The native sources measured (bench.py drops a summary of other sources)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from vpp_amd._abi import source_hash
    return source_hash()


def pmc(fetch_csv, write_csv, config, packets, out):
    # config 5 runs the 16-byte layout: classify16_cls, 35 B read per packet
    kernel, read_pp = ("classify16_cls", 35) if int(config) == 5 else (KERNEL, 11)
    f = _per_dispatch(fetch_csv, "FETCH_SIZE", kernel)
    w = _per_dispatch(write_csv, "WRITE_SIZE", kernel)
    fk = sum(f) / len(f)
    wk = sum(w) / len(w)
    read_bytes = 2.0 * fk * 1024        # gfx950 FETCH_SIZE half-count correction
    write_bytes = wk * 1024
    packets = int(packets)
    alg_read = packets * read_pp
    alg_write = packets * 1
    d = {"config": int(config), "packets": int(packets), "kernel": kernel,
         "dispatches": [len(f), len(w)], "fetch_kib_raw": fk, "write_kib_raw": wk,
         "hbm_read_bytes_per_launch": read_bytes, "hbm_write_bytes_per_launch": write_bytes,
         "hbm_bytes_per_launch": read_bytes + write_bytes,
         "algorithmic_read_bytes": alg_read, "algorithmic_write_bytes": alg_write,
         "read_ratio_vs_algorithmic": read_bytes / alg_read,
         "write_ratio_vs_algorithmic": write_bytes / alg_write,
         "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count, MI355X_MICROARCH.md HBM); "
                       "write = WRITE_SIZE KiB",
         "source_hash": _source_hash()}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    else:
        pmc(*sys.argv[2:7])
