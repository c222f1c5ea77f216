#!/usr/bin/env python3
"""Classification rate on rule lists from the gen-policy.py workload
(tests/policy/perf/gen-policy.py restated as vpp_amd.configurator.gen_policy).

For each block count and direction: the configurator generates the pod's
list (ingress: the policy's IP blocks minus excepts as sources; egress: as
destinations; x 20 ports), the list is compiled onto the classifier
(TestTraffic semantics, renderer/traffic.py), and 64 Mi device-resident IPv4
packets around the blocks (TCP/UDP, 10 % ICMP, 1 % protocol 47) are
classified, timed with the engine's HIP events.  One JSON line per list.
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


def bench_list(eng, pol, txn, nb, match, n, iters, mix=(0.445, 0.445, 0.1, 0.01), layout=4, v6=0.0):
    """Classify n device-resident packets against one of the pod's lists
    (layout 16: the 16-byte SoA, IPv4-mapped addresses with a share v6 of
    IPv6 ones)."""
    import torch
    from vpp_amd import configurator as C
    from vpp_amd.renderer.traffic import compile_rules
    t0 = time.perf_counter()
    # MATCH_INGRESS: the list keyed on the blocks as sources; MATCH_EGRESS: as destinations
    rules = txn.generate_rules(C.MATCH_INGRESS if match == "ingress" else C.MATCH_EGRESS, [pol])
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    table = eng.put_table("gen%d" % nb, compile_rules(rules))
    t_put = time.perf_counter() - t0
    info = table.info()
    g = np.random.default_rng(nb)
    blk = g.integers(0, nb + nb // 10 + 1, n, dtype=np.uint64)
    inblk = (((blk + 0x100) << 16) | g.integers(0, 1 << 16, n, dtype=np.uint64)).astype(np.uint32)
    other = g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    src, dst = (inblk, other) if match == "ingress" else (other, inblk)
    if layout == 16:
        def wide(x):
            is6 = g.random(n) < v6
            hi = np.where(is6, np.uint64(0xFD000000 << 32), np.uint64(0))
            lo = np.where(is6, x.astype(np.uint64), np.uint64(0xFFFF << 32) | x.astype(np.uint64))
            out = np.empty((n, 16), np.uint8)
            out[:, :8] = hi.astype(">u8").view(np.uint8).reshape(n, 8)
            out[:, 8:] = lo.astype(">u8").view(np.uint8).reshape(n, 8)
            return out
        src, dst = wide(src), wide(dst)
    ports = np.array([p.number for p in pol.matches[0].ports], np.uint16)
    dport = np.where(g.random(n) < 0.5, g.choice(ports, n), g.integers(0, 65536, n)).astype(np.uint16)
    # default: TCP/UDP, 10 % ICMP, 1 % protocol 47
    proto = g.choice(np.array([0, 1, 2, 47], np.uint8), n, p=mix)
    d = {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else
                             (v.view(np.int16) if v.dtype == np.uint16 else v)).to("cuda")
         for k, v in dict(src=src, dst=dst, dport=dport, proto=proto).items()}
    verdict = torch.empty(n, dtype=torch.uint8, device="cuda")
    counters = torch.zeros(table.n_rules + 1, dtype=torch.int64, device="cuda")
    eng.classify(table, d["src"], d["dst"], d["dport"], d["proto"], verdict, counters)
    torch.cuda.synchronize()
    eng.kernel_times(reset=True)
    t0 = time.perf_counter()
    for _ in range(iters):
        eng.classify(table, d["src"], d["dst"], d["dport"], d["proto"], verdict, counters, timing=True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters
    kms = eng.kernel_times(reset=True)
    k_avg = sum(kms) / max(1, len(kms))
    vh = np.bincount(verdict.cpu().numpy(), minlength=3).tolist()
    eng.del_table(table)
    bpp = 12 if layout == 4 else 36                    # algorithmic bytes per packet
    return {
        "workload": "gen-policy.py, %d blocks x 5 excepts x 20 ports: the pod's %s list" % (nb, match),
        "proto_mix_tcp_udp_icmp_47": list(mix),
        "rules": len(rules), "gen_s": round(t_gen, 2), "compile_s": round(t_put, 2),
        "layout": "IPv4 SoA, 12 B/packet" if layout == 4 else "16-byte SoA, 36 B/packet (%.0f %% IPv6)" % (100 * v6),
        "kernel": info.get("kernel"),
        "lds_resident": info.get("lds_resident") if layout == 4 else info.get("lds_resident_v16"),
        "list_mode": info.get("list_mode"), "dst_keyed": info.get("swap"), "ctr16": info.get("ctr16"),
        "lds_slots": info.get("n_lctr"), "slots": info.get("n_slots"),
        "packets": n, "Gpps_wall": round(n / wall / 1e9, 2), "kernel_ms": round(k_avg, 4),
        "Gpps_kernel": round(n / (k_avg * 1e-3) / 1e9, 2) if k_avg else None,
        "hbm_frac_kernel": round(bpp * n / (k_avg * 1e-3) / 8e12, 3) if k_avg else None,
        "verdicts_deny_permit_unmatched": vh}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, nargs="+", default=[20, 60, 200])
    ap.add_argument("--packets", type=int, default=1 << 26)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--match", nargs="+", default=["ingress", "egress"])
    ap.add_argument("--mix", type=float, nargs=4, default=[0.445, 0.445, 0.1, 0.01],
                    help="shares of TCP, UDP, ICMP, protocol 47")
    ap.add_argument("--layout", type=int, default=4, choices=[4, 16])
    ap.add_argument("--v6", type=float, default=0.0, help="16-byte layout: share of IPv6 addresses")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="library tuning switch (cls_engine_set_option), repeatable")
    a = ap.parse_args()
    from vpp_amd import configurator as C
    from vpp_amd.engine import Engine
    from vpp_amd.renderer.api import PodID
    eng = Engine(options=dict(o.split("=", 1) for o in a.opt))
    for nb in a.blocks:
        pol = C.gen_policy(random.Random(nb), num_cidrs=nb)
        txn = C.PolicyConfigurator({PodID("db", "default"): "10.1.1.1"}).new_txn(False)
        for match in a.match:
            print(json.dumps(bench_list(eng, pol, txn, nb, match, a.packets, a.iters, tuple(a.mix), a.layout, a.v6)),
                  flush=True)
    eng.close()


if __name__ == "__main__":
    main()
