#!/usr/bin/env python3
"""Does the placement of the five packet arrays in HBM change the stream rate?

Config 3 (256 Mi packets): src, dst (u32), dport (u16), proto (u8) and the
verdict (u8) either as five torch allocations (bench.py's layout) or carved
from one buffer back to back, with a stagger of S bytes added between arrays
(S = 0: every array starts at a multiple of its power-of-two size).  For each
layout: the stream floor (cls_stream_floor, best shape) and the classify
kernel (HIP events), one JSON line each.
usage: python tools/layout_bench.py [--staggers 0 4096 ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--staggers", type=int, nargs="+", default=[-1, 0, 4096, 65536 + 256, (1 << 20) + 12288])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--const", action="store_true", help="also: constant packet data (memset pattern)")
    a = ap.parse_args()
    import torch
    from vpp_amd import workload
    from vpp_amd.engine import Engine
    acl, spec, n = workload.config(3)
    eng = Engine(0)
    t = eng.put_table("g", acl.rules)
    sizes = [("src", 4, torch.int32), ("dst", 4, torch.int32), ("dport", 2, torch.int16),
             ("proto", 1, torch.uint8), ("verdict", 1, torch.uint8)]
    for st in a.staggers:
        if st < 0:
            arr = {k: torch.empty(n, dtype=dt, device="cuda") for k, _, dt in sizes}
            name = "separate allocations"
        else:
            total = sum(n * b for _, b, _ in sizes) + 5 * st + 4096
            buf = torch.empty(total, dtype=torch.uint8, device="cuda")
            arr, off = {}, 0
            for k, b, dt in sizes:
                arr[k] = buf[off:off + n * b].view(dt)
                off += n * b + st
            name = "one buffer, stagger %d B" % st
        eng.gen_traffic_v4(spec, 0, arr)
        torch.cuda.synchronize()
        floor = eng.stream_floor(arr["src"], arr["dst"], arr["dport"], arr["proto"], arr["verdict"])
        if a.const:
            cst = {k: torch.full_like(v, 1) for k, v in arr.items()}
            fc = eng.stream_floor(cst["src"], cst["dst"], cst["dport"], cst["proto"], cst["verdict"])
            half = {k: v.clone() for k, v in arr.items()}
            for k in half:
                half[k].view(torch.uint8)[1::2] = 0       # half the bytes zero
            fh = eng.stream_floor(half["src"], half["dst"], half["dport"], half["proto"], half["verdict"])
            print(json.dumps({"layout": name, "floor_random_ms": round(floor, 4), "floor_const_ms": round(fc, 4),
                              "floor_half_zero_ms": round(fh, 4)}), flush=True)
            del cst, half
        c = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
        for _ in range(3):
            eng.classify(t, arr["src"], arr["dst"], arr["dport"], arr["proto"], verdict=arr["verdict"], counters=c)
        torch.cuda.synchronize()
        eng.kernel_times(reset=True)
        for _ in range(a.iters):
            eng.classify(t, arr["src"], arr["dst"], arr["dport"], arr["proto"], verdict=arr["verdict"], counters=c,
                         timing=True)
        torch.cuda.synchronize()
        kms = float(np.mean(eng.kernel_times(reset=True)))
        print(json.dumps({"layout": name, "addr_mod_1GiB": [int(x.data_ptr() % (1 << 30)) for x in arr.values()],
                          "stream_floor_ms": round(floor, 4), "classify_ms": round(kms, 4),
                          "classify_GBps": round(12 * n / kms / 1e6, 1)}), flush=True)
        del arr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
