#!/usr/bin/env python3
"""Diagnostics: time classify4_cls builds A/B.

  tools/ablate.py CFG lib1.so lib2.so ...   one child process per library
  (build them with `make -C vpp_amd/csrc variant V=name F=...`; stage ablation
  is a build flag, F=-DCLS_ABLATE=bits: 1 counters, 2 candidate scan, 4 source
  lookup, 8 verdict store -- results of ablated builds are wrong by
  construction; only kernel times matter).  tools/build_ablate.sh builds the
  usual set."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from vpp_amd import workload
    from vpp_amd.engine import Engine
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    acl, spec, n = workload.config(cfg)
    n = int(os.environ.get("PKTS", n))
    eng = Engine(0)
    t = eng.put_table("t", acl.rules)
    print("info", t.info())
    pk = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
          (("src", torch.int32), ("dst", torch.int32), ("dport", torch.int16), ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, 0, pk)
    verdict = torch.empty(n, dtype=torch.uint8, device="cuda")
    counters = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
    for rep in range(2):       # the first round warms clocks up
        for _ in range(3):
            eng.classify(t, pk["src"], pk["dst"], pk["dport"], pk["proto"], verdict=verdict, counters=counters)
        eng.kernel_times(reset=True)
        for _ in range(10):
            eng.classify(t, pk["src"], pk["dst"], pk["dport"], pk["proto"], verdict=verdict,
                         counters=counters, timing=True)
        ks = eng.kernel_times(reset=True)
        ms = float(np.median(ks))
        print("kernel median %.3f ms (min %.3f)  %.1f Gpps  %.1f GB/s" % (ms, min(ks), n / ms / 1e6, n * 12 / ms / 1e6))


def ab_libs():
    """tools/ablate.py CFG lib1.so lib2.so ...: A/B the kernel build variants
    (vpp_amd/csrc/Makefile `variant`), one child process per library."""
    import subprocess
    for so in sys.argv[2:]:
        print("==", so, flush=True)
        env = dict(os.environ, CONTIVCLS_LIB=os.path.abspath(so))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), sys.argv[1]], env=env)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    if len(sys.argv) > 2:
        ab_libs()
    else:
        main()
