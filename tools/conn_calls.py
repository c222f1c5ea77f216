#!/usr/bin/env python3
"""Wall time of each device connection batch (tools/conn_bench.py's setup):
python tools/conn_calls.py [--locals 64] [--n 4194304] [--calls 8]"""
import argparse
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
    ap.add_argument("--locals", type=int, default=64)
    ap.add_argument("--calls", type=int, default=8)
    a = ap.parse_args()
    import torch
    from vpp_amd.engine import Engine
    eng = Engine()
    ifs, bind, by_name, pool, spec = build(eng, 0, cfg=3, n_local=a.locals)
    n = a.n
    tr = random_traffic(7, n, pool, other_proto=True)
    rng = np.random.default_rng(7)
    ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
    si, di = rng.integers(0, len(ifs), n), rng.integers(0, len(ifs), n)
    args = (ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"])
    dargs = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
             .to("cuda") for x in args]
    torch.cuda.synchronize()
    for count in (False, True, False):
        ts = []
        for _ in range(a.calls):
            t0 = time.perf_counter()
            eng.connect_batch(*dargs, count=count)
            ts.append((time.perf_counter() - t0) * 1e3)
        print("count=%s ms per call:" % count, " ".join("%.3f" % t for t in ts), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
