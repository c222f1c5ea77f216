#!/usr/bin/env python3
"""Probe: do two connection batches overlap on the GPU when they run on two
streams?  A batch is classify4_pair (LDS-bound, one 1024-thread workgroup per
CU holding the large ACL's image) then connect_kernel (instruction-bound,
512-thread workgroups); if the hardware runs one batch's pair launch beside
another batch's connection launch, an engine that pipelines its batches over
two internal streams would take less than the sum of the two kernels per
batch.  Two engines (each its own scratch) on two streams stand in for that
engine here.  Prints per-batch times: one engine back to back, and the two
engines interleaved on two streams (and on one stream, as a control).
usage: python tools/conn_overlap_probe.py [--n 4194304] [--locals 12] [--iters 20]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from aclgen import random_traffic  # noqa: E402
from test_gpu_connect_scale import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--locals", type=int, default=12)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    from vpp_amd import _abi
    from vpp_amd.engine import Engine, _ptr
    engs = [Engine(0), Engine(0)]
    setups = [build(e, 0, cfg=3, n_local=a.locals) for e in engs]
    ifs, bind, by_name, pool, spec = setups[0]
    n = a.n
    tr = random_traffic(7, n, pool, other_proto=True)
    rng = np.random.default_rng(7)
    half = rng.random(n) < 0.5
    tr["src"][half] = rng.choice(spec["pod_ips"].astype(np.uint32), half.sum())
    dsts = spec["dst_addrs"].astype(np.uint32)
    tr["dst"][half] = rng.choice(dsts, half.sum()) | rng.integers(0, 256, half.sum()).astype(np.uint32)
    si = np.where(half, rng.integers(0, 2, n), rng.integers(0, len(ifs), n))
    di = rng.integers(0, len(ifs), n)
    calls = []
    for e, st in zip(engs, setups):
        ids = np.array([e.if_id(x) for x in st[0]], np.uint32)
        args = (ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"])
        d = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
             .to("cuda") for x in args]
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        pk = _abi.PktSoa(_abi.AF_V4, _ptr(d[2]), _ptr(d[3]), None, None, _ptr(d[5]), _ptr(d[6]), _ptr(d[4]))
        cs = _abi.ConnSoa(pk, _ptr(d[0]), _ptr(d[1]))
        calls.append((e, d, out, cs))
    fn = _abi.lib().cls_connect_batch
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def run(k, stream):
        e, d, out, cs = calls[k]
        assert fn(e.h, C.byref(cs), n, _ptr(out), _abi.F_DEVICE, C.c_void_p(stream.cuda_stream)) == 0

    for k in (0, 1):                        # warm-up (plans, uploads)
        for _ in range(3):
            run(k, streams[k])
    torch.cuda.synchronize()
    ref = calls[0][2].cpu().numpy()
    assert np.array_equal(ref, calls[1][2].cpu().numpy()), "the two engines differ"
    res = {}
    for name, plan in (("one_engine_one_stream", [(0, 0)] * 2),
                       ("two_engines_one_stream", [(0, 0), (1, 0)]),
                       ("two_engines_two_streams", [(0, 0), (1, 1)])):
        ts = []
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                for k, s in plan:
                    run(k, streams[s])
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / (2 * a.iters))
        res[name + "_ms_per_batch"] = round(float(np.median(ts)) * 1e3, 4)
    for k in (0, 1):
        assert np.array_equal(calls[k][2].cpu().numpy(), ref)
    print(json.dumps(dict(res, n=n, locals=a.locals)))


if __name__ == "__main__":
    main()
