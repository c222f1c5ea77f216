#!/usr/bin/env python3
"""Connection-path throughput (testConnection batches).

Layout: the config-3 global ACL (9963 rules) bound to if0/if1 (in) and
if0/if2 (out), 64 random local ACLs (1-300 rules) on 77 further interfaces,
half of the connections entering through a global-table interface.  Times
``Engine.connect_batch`` over N connections with host arrays in and out
(PCIe copies included; auto and linear modes) and with device-resident
tensors (CLS_F_DEVICE, ``hbm_resident``: the median wall time of --iters calls),
and the C oracle (one thread) on a sample.  Prints one JSON line.  --count 1 times CLS_F_COUNT batches (per-(ACL, rule) counters)
beside the plain ones; --locals sets the number of local ACLs (12: a rule
pool that fits LDS).
usage: python tools/conn_bench.py [--n 4194304] [--iters 5] [--locals 64]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from aclgen import random_traffic  # noqa: E402
from test_gpu_connect_scale import build, oracle_connections  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--iters", type=int, default=9)
    ap.add_argument("--cpu-sample", type=int, default=20000, help="connections checked on the literal oracle")
    ap.add_argument("--cpu-fast-sample", type=int, default=1 << 20,
                    help="connections timed on the OpenMP fast port (the CPU baseline)")
    ap.add_argument("--other-proto", type=int, default=1, help="6%% of packets with protocol > 2")
    ap.add_argument("--locals", type=int, default=64)
    ap.add_argument("--count", type=int, default=1)
    ap.add_argument("--no-check", action="store_true", help="diagnostic builds: skip the parity asserts")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="library tuning switch (cls_engine_set_option), repeatable")
    a = ap.parse_args()
    from vpp_amd.engine import Engine
    eng = Engine(options=dict(o.split("=", 1) for o in a.opt))
    ifs, bind, by_name, pool, spec = build(eng, 0, cfg=3, n_local=a.locals)
    n = a.n
    tr = random_traffic(7, n, pool, other_proto=bool(a.other_proto))
    rng = np.random.default_rng(7)
    half = rng.random(n) < 0.5
    tr["src"][half] = rng.choice(spec["pod_ips"].astype(np.uint32), half.sum())
    dsts = spec["dst_addrs"].astype(np.uint32)
    tr["dst"][half] = rng.choice(dsts, half.sum()) | rng.integers(0, 256, half.sum()).astype(np.uint32)
    ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
    si = np.where(half, rng.integers(0, 2, n), rng.integers(0, len(ifs), n))
    di = rng.integers(0, len(ifs), n)
    args = (ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"])
    res = {}
    for mode in ("linear", "auto"):
        out = eng.connect_batch(*args, mode=mode)        # warm-up (and table upload)
        t0 = time.perf_counter()
        for _ in range(a.iters):
            out = eng.connect_batch(*args, mode=mode)
        res[mode] = ((time.perf_counter() - t0) / a.iters, out)
    if not a.no_check:
        assert np.array_equal(res["linear"][1], res["auto"][1]), "linear and classifier modes differ"
    dt, out = res["auto"]
    # HBM-resident batch (CLS_F_DEVICE): no PCIe in the timed region
    import torch
    dargs = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
             .to("cuda") for x in (args[0], args[1], args[2], args[3], args[4], args[5], args[6])]
    torch.cuda.synchronize()
    dev_out = eng.connect_batch(*dargs)
    if not a.no_check:
        assert np.array_equal(dev_out.cpu().numpy(), out), "device batch differs"
    vout = torch.empty(n, dtype=torch.uint8, device="cuda")

    def per_call(count):
        """median wall time of a.iters device batches, each waited for (the
        call is stream-ordered: it returns once its launches are queued), the
        verdicts into one output tensor"""
        ts = []
        for _ in range(a.iters):
            t0 = time.perf_counter()
            eng.connect_batch(*dargs, count=count, out=vout)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))
    dev_dt = per_call(False)

    def per_call_abi(count):
        """the same batch through cls_connect_batch with the call's arguments
        built once (what a native host pays: no per-call Python marshalling)"""
        import ctypes as C
        from vpp_amd import _abi
        from vpp_amd.engine import _ptr
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        pk = _abi.PktSoa(_abi.AF_V4, _ptr(dargs[2]), _ptr(dargs[3]), None, None, _ptr(dargs[5]), _ptr(dargs[6]),
                         _ptr(dargs[4]))
        cs = _abi.ConnSoa(pk, _ptr(dargs[0]), _ptr(dargs[1]))
        fl = _abi.F_DEVICE | (_abi.F_COUNT if count else 0)
        fn, h, csr, op = _abi.lib().cls_connect_batch, eng.h, C.byref(cs), _ptr(out)
        sync = torch.cuda.synchronize
        ts = []
        for _ in range(a.iters + 1):
            t0 = time.perf_counter()
            rc = fn(h, csr, n, op, fl, None)
            sync()
            ts.append(time.perf_counter() - t0)
            assert rc == 0
        # pipelined: a.iters batches queued back to back, one wait at the end
        # (the stream-ordered device batch: the host work of a call overlaps
        # the GPU work of the one before)
        t0 = time.perf_counter()
        for _ in range(a.iters):
            assert fn(h, csr, n, op, fl, None) == 0
        sync()
        piped = (time.perf_counter() - t0) / a.iters
        if not a.no_check:
            assert np.array_equal(out.cpu().numpy(), dev_out.cpu().numpy())
        return float(np.median(ts[1:])), piped
    abi_dt, abi_piped = per_call_abi(False)
    counted = None
    if a.count:
        eng.connect_batch(*dargs, count=True)
        dt_c = per_call(True)
        abi_c, abi_c_piped = per_call_abi(True)
        counted = {"value": round(n / dt_c / 1e6, 3), "unit": "Mconn/s", "ms_per_batch": round(dt_c * 1e3, 3),
                   "abi_ms_per_batch": round(abi_c * 1e3, 4),
                   "abi_pipelined_ms_per_batch": round(abi_c_piped * 1e3, 4)}
        # how the counted calls spread over the (ACL, rule) counters: the
        # shares of the largest counters (contention of the counter atomics)
        cs = np.concatenate([eng.conn_counters(name).astype(np.float64) for name in by_name])
        tot = cs.sum()
        top = np.sort(cs)[::-1][:8] / max(tot, 1.0)
        counted["calls_per_connection"] = round(tot / (n * (3 * a.iters + 2)), 3)
        counted["top_counter_shares"] = [round(float(x), 4) for x in top]
        counted["nonzero_counters"] = int((cs > 0).sum())
    # roofline: the 22 algorithmic bytes of an IPv4 connection (src, dst,
    # src_if, dst_if 4 B each, sport, dport 2 B, proto 1 B read; the verdict
    # byte written) per HBM-resident batch, beside the stream floor of the
    # same arrays (cls_stream_floor_conn: the same reads and write, no
    # evaluation)
    # (the product path: device batches through the C ABI, back to back)
    floor = eng.stream_floor_conn(*dargs, reps=20)
    roof = {"bound": "hbm", "bytes_per_connection": 22, "peak": 8000.0, "unit": "GB/s",
            "achieved": round(22 * n / abi_piped / 1e9, 1), "frac": round(22 * n / abi_piped / 8e12, 4),
            "stream_floor_ms": round(floor, 4), "frac_of_stream_floor": round(floor / (abi_piped * 1e3), 4),
            "timed": "abi_pipelined_ms_per_batch"}
    k = a.cpu_sample
    t1 = time.perf_counter()
    want, _ = oracle_connections(bind, by_name, ifs, si[:k], di[:k], {f: v[:k] for f, v in tr.items()}, 4)
    cpu_dt = time.perf_counter() - t1
    if not a.no_check:
        assert np.array_equal(out[:k], want), "connection verdicts differ from the oracle"
    # the CPU baseline: the fast port (rules pre-parsed, orc_connect_fast)
    # over OpenMP on the cores this process may use, on a prefix of the batch
    import oracle
    from bench import cpu_share, host_cpu
    names = list(by_name)
    tabs = [oracle.FastTable(oracle.rules_to_c(by_name[x])) for x in names]
    if_ids = {x: i for i, x in enumerate(names)}
    if_in = [if_ids[bind[f][0]] if bind[f][0] else -1 for f in ifs]
    if_out = [if_ids[bind[f][1]] if bind[f][1] else -1 for f in ifs]
    kf = min(n, a.cpu_fast_sample)
    cores = cpu_share()
    trk = {f: v[:kf] for f, v in tr.items()}
    oracle.connect_fast(tabs, if_in, if_out, si[:1024], di[:1024], {f: v[:1024] for f, v in tr.items()},
                        nthreads=cores)
    t2 = time.perf_counter()
    fast = oracle.connect_fast(tabs, if_in, if_out, si[:kf], di[:kf], trk, nthreads=cores)
    fast_dt = time.perf_counter() - t2
    if not a.no_check:
        assert np.array_equal(fast, out[:kf]), "the fast CPU port differs from the GPU verdicts"
    print(json.dumps({
        "metric": "connections classified per second (testConnection, up to 4 ACL evaluations each)",
        "value": round(n / abi_piped / 1e6, 3), "unit": "Mconn/s", "n": n,
        "ms_per_batch": round(abi_piped * 1e3, 4),
        "timed": "device batches through cls_connect_batch, back to back (HBM-resident, stream-ordered)",
        "host_arrays": {"value": round(n / dt / 1e6, 3), "unit": "Mconn/s", "ms_per_batch": round(dt * 1e3, 3),
                        "pcie_included": True},
        "global_rules": len(by_name["global"]), "local_acls": a.locals,
        "other_proto": bool(a.other_proto), "hbm_resident_counted": counted,
        "hbm_resident": {"value": round(n / dev_dt / 1e6, 3), "unit": "Mconn/s",
                         "ms_per_batch": round(dev_dt * 1e3, 4), "abi_ms_per_batch": round(abi_dt * 1e3, 4),
                         "abi_pipelined_ms_per_batch": round(abi_piped * 1e3, 4)},
        "roofline": roof,
        "linear_scan": {"value": round(n / res["linear"][0] / 1e6, 3), "unit": "Mconn/s",
                        "ms_per_batch": round(res["linear"][0] * 1e3, 3)},
        "verdicts": np.bincount(out, minlength=4).tolist(),
        "cpu_baseline": {"value": round(kf / fast_dt / 1e6, 4), "unit": "Mconn/s", "cores": cores,
                         "kind": "port", "nproc": host_cpu()[0], "cpu_model": host_cpu()[1],
                         "sample": "%d connections of the batch, orc_connect_fast (ACLs pre-parsed, testConnection "
                                   "restated, OpenMP %d threads), %.1f s" % (kf, cores, fast_dt),
                         "faithful": {"value": round(k / cpu_dt / 1e6, 5), "unit": "Mconn/s", "cores": 1,
                                      "sample": "%d connections, orc_test_connection_hits (CIDR strings re-parsed "
                                                "per rule per call)" % k}},
        "parity": "first %d connections bit-exact vs oracle" % k}))
    eng.close()


if __name__ == "__main__":
    main()
