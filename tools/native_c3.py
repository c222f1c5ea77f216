#!/usr/bin/env python3
"""Config 3 through the C ABI alone, with no torch in the process.

The north-star host is Go over cgo: it may pass its memory only for the
duration of a call, so the HBM-resident path has to be reachable with
engine-owned batches (include/contivcls.h cls_batch_*).  This driver is that
host in Python/ctypes (CONTIVCLS_NO_TORCH=1: the library runs on /opt/rocm's
HIP runtime, and `torch` is never imported -- checked at the end):

  engine (one device, or --shards k: k shards on the devices of --devices)
  -> cls_table_put (the config-3 ~10k-rule global ACL, compiled once)
  -> cls_batch_create (256 Mi IPv4 packets in HBM, engine-owned)
  -> cls_batch_gen_traffic_v4 (the splitmix64 stream on the device)
  -> cls_classify_batch x (warmup + steps), CLS_F_TIMING
  -> cls_batch_download of --windows verdict windows, checked bit-exact
     against the oracle (test infrastructure) on the same stream packets.

It also times cls_classify on the batch's own device arrays (the raw-pointer
entry point, cls_batch_field) to show the batch path adds nothing to the
kernel, and prints one JSON line.  Used by tests/test_gpu_native.py and
bench.py --native.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ["CONTIVCLS_NO_TORCH"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402

from vpp_amd import _abi, workload  # noqa: E402
from vpp_amd.engine import Engine  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 5])
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--devices", type=str, default="0", help="comma-separated device list")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed calls first, for at least this much wall time (GPU clocks settle)")
    ap.add_argument("--windows", type=int, default=64)
    ap.add_argument("--window", type=int, default=4096)
    ap.add_argument("--rccl", action="store_true", help="cls_comm_init at one device (an RCCL group of one)")
    ap.add_argument("--no-raw", action="store_true", help="skip the raw-pointer cls_classify timing")
    return ap.parse_args()


def kernel_times(dev: Engine):
    return dev._timed(_abi.lib().cls_kernel_times)


def main():
    a = parse()
    acl, spec, n_default = workload.config(a.config)
    n = a.packets or n_default
    af = spec.get("layout", 4)
    devs = [int(x) for x in a.devices.split(",")]
    eng = Engine(devices=devs) if len(devs) > 1 else Engine(devs[0])
    if a.rccl:
        eng.comm_init()
    table = eng.put_table("contiv/vpp-policy-GLOBAL", acl.rules)
    R = table.n_rules
    b = eng.batch(n, af=af)
    t0 = time.perf_counter()
    b.gen_traffic(spec, 0)
    b.wait()
    gen_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < a.settle_ms:
        for _ in range(8):
            eng.classify_batch(table, b, counters=False)
        b.wait()
    for _ in range(a.warmup):
        eng.classify_batch(table, b, counters=False)
    b.wait()
    G = eng.n_devices()
    views = [eng.device_engine(g) for g in range(G)]
    for v in views:
        v.kernel_times(reset=True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.classify_batch(table, b, counters=False, timing=True)
    b.wait()
    wall = time.perf_counter() - t0
    kt = [kernel_times(v) for v in views]
    for v in views:
        v.kernel_times(reset=True)
    counters = b.counters(R)
    out = {"config": a.config, "packets": n, "rules": R, "devices": devs, "shards": [list(s) for s in b.shards()],
           "comm": list(eng.comm_info()), "steps": a.steps, "ms_per_step": wall / a.steps * 1e3,
           "gpps": n * a.steps / wall / 1e9, "gen_s": gen_s,
           "kernel_ms_avg": [float(np.mean(k)) if k else None for k in kt],
           "counter_sum": int(counters.sum()), "counters_sha": __import__("hashlib").sha256(
               counters.tobytes()).hexdigest()[:16]}
    # the raw-pointer entry point over the same device arrays (shard 0)
    if not a.no_raw:
        d0 = views[0]
        _, _, n0 = b.shards()[0]
        ptr = lambda f: b.field_ptr(0, f)  # noqa: E731
        if af == 16:
            pk = _abi.PktSoa(_abi.AF_V16, None, None, ptr(_abi.BF_SRC), ptr(_abi.BF_DST), None,
                             ptr(_abi.BF_DPORT), ptr(_abi.BF_PROTO))
        else:
            pk = _abi.PktSoa(_abi.AF_V4, ptr(_abi.BF_SRC), ptr(_abi.BF_DST), None, None, None,
                             ptr(_abi.BF_DPORT), ptr(_abi.BF_PROTO))
        L = _abi.lib()
        flags = _abi.F_DEVICE | _abi.F_TIMING
        vd = ptr(_abi.BF_VERDICT)            # the same verdict array: the same bytes moved
        # alternate the two entry points (a clock drift hits both alike):
        # device 0's timed kernels are then batch, raw, batch, raw, ...
        b.wait()
        d0.kernel_times(reset=True)
        for i in range(a.steps):
            eng.classify_batch(table, b, counters=False, timing=True)
            d0._check(L.cls_classify(d0.h, table.id, C.byref(pk), n0, vd, None, flags, None))
        b.wait()
        ab = kernel_times(d0)
        d0.kernel_times(reset=True)
        out["ab_batch_kernel_ms_avg"] = float(np.mean(ab[0::2]))
        out["raw_kernel_ms_avg"] = float(np.mean(ab[1::2]))
    # verdict windows vs the oracle (test infrastructure: only as the checker)
    if a.windows:
        import oracle
        cr = oracle.rules_to_c(acl.rules)
        ft = oracle.FastTable(cr)
        gen = oracle.gen_traffic_v16 if af == 16 else oracle.gen_traffic_v4
        w = min(a.window, n)
        starts = sorted(set(int(x) for x in np.linspace(0, n - w, a.windows)))
        bad = 0
        for s in starts:
            got = b.download(_abi.BF_VERDICT, s, w)
            tr = gen(spec, s, w)
            want = ft.classify(tr["src"], tr["dst"], tr["dport"], tr["proto"], af=af)[0]
            bad += int(np.count_nonzero(got != want))
        out["windows"] = len(starts)
        out["window"] = w
        out["window_mismatches"] = bad
    out["torch_imported"] = "torch" in sys.modules
    b.close()
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
