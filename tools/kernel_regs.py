#!/usr/bin/env python3
"""VGPR / SGPR / scratch of every kernel in a gfx950 assembly listing
(hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S), filtered
by a substring: the register budget behind a kernel's waves per SIMD.
usage: python tools/kernel_regs.py file.s [substring]"""
import re
import subprocess
import sys


def main():
    s = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = {}
    for m in re.finditer(r"^\s*\.set\s+(\S+)\.(num_vgpr|num_agpr|numbered_sgpr|private_seg_size),\s*(\d+)", s, re.M):
        vals.setdefault(m.group(1), {})[m.group(2)] = int(m.group(3))
    names = {}
    if vals:
        dem = subprocess.run(["c++filt"], input="\n".join(vals), capture_output=True, text=True).stdout.splitlines()
        names = dict(zip(vals, dem))
    for k, v in sorted(vals.items(), key=lambda kv: names.get(kv[0], kv[0])):
        n = names.get(k, k)
        if pat in n:
            print("%-80s vgpr %3d agpr %3d sgpr %3d scratch %d" % (n.rsplit("(", 1)[0].replace("(anonymous namespace)::", "")[-80:], v.get("num_vgpr", -1),
                                                                  v.get("num_agpr", -1), v.get("numbered_sgpr", -1),
                                                                  v.get("private_seg_size", -1)))


if __name__ == "__main__":
    main()
