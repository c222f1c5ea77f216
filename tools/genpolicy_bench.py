#!/usr/bin/env python3
"""Classification rate on rule lists from the gen-policy.py workload
(tests/policy/perf/gen-policy.py restated as vpp_amd.configurator.gen_policy).

For each block count: the configurator generates the pod's egress list
(source = the policy's IP blocks minus excepts, x 20 ports), the list is
compiled onto the classifier (TestTraffic semantics, renderer/traffic.py),
and 64 Mi device-resident IPv4 packets around the blocks are classified,
timed with the engine's HIP events.  Prints one JSON line per block count.
usage: python tools/genpolicy_bench.py [--blocks 20 60 200] [--packets 67108864]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, nargs="+", default=[20, 60, 200])
    ap.add_argument("--packets", type=int, default=1 << 26)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import torch
    from vpp_amd import configurator as C
    from vpp_amd.engine import Engine
    from vpp_amd.renderer.api import PodID
    from vpp_amd.renderer.traffic import compile_rules
    eng = Engine()
    n = a.packets
    for nb in a.blocks:
        rng = random.Random(nb)
        pol = C.gen_policy(rng, num_cidrs=nb)
        pod = PodID("db", "default")
        txn = C.PolicyConfigurator({pod: "10.1.1.1"}).new_txn(False)
        t0 = time.perf_counter()
        rules = txn.generate_rules(C.MATCH_INGRESS, [pol])       # the vswitch egress list
        t_gen = time.perf_counter() - t0
        t0 = time.perf_counter()
        table = eng.put_table("gen%d" % nb, compile_rules(rules))
        t_put = time.perf_counter() - t0
        info = table.info()
        g = np.random.default_rng(nb)
        blk = g.integers(0, nb + nb // 10 + 1, n, dtype=np.uint64)
        src = (((blk + 0x100) << 16) | g.integers(0, 1 << 16, n, dtype=np.uint64)).astype(np.uint32)
        dst = g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        ports = np.array([p.number for p in pol.matches[0].ports], np.uint16)
        dport = np.where(g.random(n) < 0.5, g.choice(ports, n), g.integers(0, 65536, n)).astype(np.uint16)
        proto = g.integers(0, 2, n).astype(np.uint8)
        d = {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else
                                 (v.view(np.int16) if v.dtype == np.uint16 else v)).to("cuda")
             for k, v in dict(src=src, dst=dst, dport=dport, proto=proto).items()}
        verdict = torch.empty(n, dtype=torch.uint8, device="cuda")
        counters = torch.zeros(table.n_rules + 1, dtype=torch.int64, device="cuda")
        eng.classify(table, d["src"], d["dst"], d["dport"], d["proto"], verdict, counters)
        torch.cuda.synchronize()
        eng.kernel_times(reset=True)
        t0 = time.perf_counter()
        for _ in range(a.iters):
            eng.classify(table, d["src"], d["dst"], d["dport"], d["proto"], verdict, counters, timing=True)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.iters
        kms = eng.kernel_times(reset=True)
        k_avg = sum(kms) / max(1, len(kms))
        vh = np.bincount(verdict.cpu().numpy(), minlength=3).tolist()
        print(json.dumps({
            "workload": "gen-policy.py, %d blocks x 5 excepts x 20 ports: pod egress list" % nb,
            "rules": len(rules), "gen_s": round(t_gen, 2), "compile_s": round(t_put, 2),
            "kernel": info.get("kernel"), "lds_resident": info.get("lds_resident"),
            "packets": n, "Gpps_wall": round(n / wall / 1e9, 2), "kernel_ms": round(k_avg, 4),
            "Gpps_kernel": round(n / (k_avg * 1e-3) / 1e9, 2) if k_avg else None,
            "hbm_frac_kernel": round(12 * n / (k_avg * 1e-3) / 8e12, 3) if k_avg else None,
            "verdicts_deny_permit_unmatched": vh}), flush=True)
        del d, verdict, counters
        eng.del_table(table)
    eng.close()


if __name__ == "__main__":
    main()
