#!/usr/bin/env python3
"""A/B of classify kernel builds in ONE process, interleaved.

    python tools/ab_inproc.py [--config 3] [--rounds 6] lib_a.so lib_b.so ...

Every build (vpp_amd/csrc Makefile `variant`) is loaded side by side
(RTLD_LOCAL) with its own engine and table over the same device-resident
packets; rounds alternate the builds (10 timed launches each, HIP events), so
clock and box drift hit all of them alike.  Prints each build's median over
rounds of the per-round median kernel ms, and its verdicts/counters checked
against the first build's.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    import torch
    from vpp_amd import _abi, workload
    from vpp_amd.engine import Engine
    acl, spec, n = workload.config(a.config)
    gen = Engine(0)
    v16 = spec.get("layout", 4) == 16
    shape = (n, 16) if v16 else (n,)
    adt = torch.uint8 if v16 else torch.int32
    pk = {k: torch.empty(shape if k in ("src", "dst") else (n,), dtype=dt, device="cuda") for k, dt in
          (("src", adt), ("dst", adt), ("dport", torch.int16), ("proto", torch.uint8))}
    (gen.gen_traffic_v16 if v16 else gen.gen_traffic_v4)(spec, 0, pk)
    torch.cuda.synchronize()
    cr = _abi.CRules(acl.rules)
    p = lambda t: t.data_ptr()
    soa = (_abi.PktSoa(_abi.AF_V16, None, None, p(pk["src"]), p(pk["dst"]), None, p(pk["dport"]), p(pk["proto"]))
           if v16 else
           _abi.PktSoa(_abi.AF_V4, p(pk["src"]), p(pk["dst"]), None, None, None, p(pk["dport"]), p(pk["proto"])))
    builds = []
    for path in a.libs:
        L = _abi.bind(os.path.abspath(path), strict=False)
        h = C.c_void_p()
        assert L.cls_engine_create(C.byref(_abi.Config(0)), C.byref(h)) == 0
        tid = C.c_uint32()
        assert L.cls_table_put(h, b"t", cr.ptr(), cr.n, C.byref(tid)) == 0
        v = torch.empty(n, dtype=torch.uint8, device="cuda")
        c = torch.zeros(cr.n + 1, dtype=torch.int64, device="cuda")
        builds.append(dict(path=path, L=L, h=h, tid=tid.value, v=v, c=c, ms=[]))
    s = torch.cuda.current_stream().cuda_stream
    flags = _abi.F_DEVICE | _abi.F_TIMING
    for r in range(a.rounds + 1):                       # round 0 warms up
        for b in builds:
            L, h = b["L"], b["h"]
            L.cls_kernel_times_reset(h)
            for _ in range(10):
                assert L.cls_classify(h, b["tid"], C.byref(soa), n, p(b["v"]), p(b["c"]), flags, s) == 0
            cnt = C.c_uint32()
            buf = (C.c_float * 16)()
            L.cls_kernel_times(h, buf, 16, C.byref(cnt))
            if r:
                b["ms"].append(float(np.median(buf[:cnt.value])))
    torch.cuda.synchronize()
    base = builds[0]
    for b in builds:
        same = torch.equal(b["v"], base["v"]) and torch.equal(b["c"], base["c"])
        med = float(np.median(b["ms"]))
        print("%-40s median %.4f ms  (rounds %s)  %.1f Gpps  same results: %s" % (
            os.path.basename(b["path"]), med, " ".join("%.4f" % x for x in b["ms"]), n / med / 1e6, same),
            flush=True)


if __name__ == "__main__":
    main()
