#!/usr/bin/env python3
"""LDS bank-conflict model of classify4_cls (diagnostics, CPU only).

Replays the LDS address stream the hot kernel issues for a packet stream
(vpp_amd/csrc/kernels.hip, list mode 3 + hash LPM) and prices every wave
instruction with the gfx950 banking rules of MI355X_MICROARCH.md "LDS":
  ds_read_b32 / ds_read_u8 / ds_add_u32: 2 groups x 32 lanes, bank (a/4) mod 32
  ds_read_b64: 2 groups x 32 lanes, bank (a/4) mod 64, two dwords per lane
  one LDS cycle per group when conflict-free, +1 per extra distinct dword on a bank.
The lane -> packet map is the kernel's: lane l of a wave-step holds packets
4l..4l+3 of a 256-packet tile; instruction q touches packet q of every lane.
(On the round-1 list mode 2 kernel this model predicted 274 LDS cycles per
wave-step; rocprofv3 SQ_LDS_IDX_ACTIVE measured 274.)

usage: tools/lds_sim.py [config] [packets]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def group_cycles(addr, active, nbanks, width_dw, same_addr_serial=False):
    """addr, active: (I, 32) byte addresses / mask of one lane group.
    Returns cycles per group (I,)."""
    dw = (addr >> 2).astype(np.int64)
    I = addr.shape[0]
    counts = np.zeros((I, nbanks), np.int64)
    rows = np.repeat(np.arange(I), 32).reshape(I, 32)
    for k in range(width_dw):
        d = dw + k
        bank = d % nbanks
        if same_addr_serial:
            np.add.at(counts, (rows[active], bank[active]), 1)
        else:
            # distinct dwords per bank
            key = np.where(active, bank * (1 << 40) + d, -1)
            key.sort(axis=1)
            first = np.ones_like(key, bool)
            first[:, 1:] = key[:, 1:] != key[:, :-1]
            valid = first & (key >= 0)
            b = np.where(valid, key >> 40, 0)
            np.add.at(counts, (rows[valid], b[valid]), 1)
    cyc = counts.max(axis=1)
    return np.where(active.any(axis=1), np.maximum(cyc, 1), 0)


def inst_cycles(addr64, active64, kind):
    """addr64, active64: (I, 64).  kind: b32 | b64 | u8 | atomic."""
    tot = 0
    for g in (slice(0, 32), slice(32, 64)):
        a, m = addr64[:, g], active64[:, g]
        if kind == "b64":
            c = group_cycles(a, m, 64, 2)
        elif kind == "atomic":
            c = group_cycles(a, m, 32, 1, same_addr_serial=True)
        else:
            c = group_cycles(a & ~3, m, 32, 1)
        tot = tot + c
    return tot


def address_stream(cfg, npk):
    """(ops, header): ops = [(name, kind, byte address per packet)]."""
    import oracle
    from vpp_amd import _abi, workload
    import cls_image
    acl, spec, _ = workload.config(cfg)
    im = cls_image.Image(cls_image.compile_blob(_abi.CRules(acl.rules)))
    h = im.h
    assert h.mode == 1 and h.list_mode == 3, "model covers hash LPM + list mode 3"
    tr = oracle.gen_traffic_v4(spec, 0, npk)
    src, dst = tr["src"].astype(np.int64), tr["dst"].astype(np.int64)
    dport, proto = tr["dport"].astype(np.int64), tr["proto"].astype(np.int64)
    img = np.frombuffer(im._img, np.uint32).astype(np.int64)
    b8 = np.frombuffer(im._img, np.uint8).astype(np.int64)
    ops = []
    a_top = 4 * (dport >> 8)                       # port radix at LDS address 0
    a_win = img[a_top // 4] + (dport & 0xFF)
    pc4 = b8[a_win]
    ops += [("ptop", "b32", a_top), ("window", "u8", a_win)]
    row = np.full(npk, h.default_row, np.int64)
    for i, (mask, shift, cap, tab, mul) in enumerate(im.hash):
        L = 32 - shift
        key = src & mask
        p = (key * mul) & 0xFFFFFFFF
        a0 = h.off_hash[i] + 8 * (p >> shift)
        a1 = h.off_hash[i] + 8 * cap + 8 * ((p >> (32 - 2 * L)) & (cap - 1))
        ops += [("hash0", "b64", a0), ("hash1", "b64", a1)]
        row = np.where(img[a0 // 4] == key, img[a0 // 4 + 1],
                       np.where(img[a1 // 4] == key, img[a1 // 4 + 1], row))
    a_cell = row + 4 * np.minimum(proto, 2)
    cell = img[a_cell // 4]
    a_ptr = (cell & 0xFFFF) + pc4
    st = img[a_ptr // 4]
    ops += [("cell", "b32", a_cell), ("ptr", "b32", a_ptr)]
    for k in range(h.bv_steps_d - 1, -1, -1):
        a = (st >> 13) + (8 << k)
        ops.append(("step%d" % k, "b64", a))
        st = np.where(img[a // 4] < dst, img[a // 4 + 1], st)
    slot = (cell >> 16) + ((st >> 2) & 63)
    lane = (np.arange(npk) // 4) % 64
    a_ctr = np.where(slot < h.n_hot, h.off_hot + 4 * lane + 256 * slot, h.img_bytes + 4 * slot)
    ops.append(("atomic", "atomic", a_ctr))
    return ops, h


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    npk = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
    ops, h = address_stream(cfg, npk)
    ntile = npk // 256
    total = 0
    print("config %d: %d packets, D=%d, n_hot=%d, LDS %d B" % (cfg, npk, h.bv_steps_d, h.n_hot, h.lds_bytes))
    print("%-8s %-6s %8s" % ("op", "kind", "cyc/inst"))
    for name, kind, a in ops:
        A = a[: ntile * 256].reshape(ntile, 64, 4).transpose(0, 2, 1).reshape(-1, 64)
        c = inst_cycles(A, np.ones_like(A, bool), kind)
        total += c.mean() * 4
        print("%-8s %-6s %8.2f" % (name, kind, c.mean()))
    print("LDS cycles per wave-step (256 packets): %.1f  -> %.3f cycles/packet" % (total, total / 256))


if __name__ == "__main__":
    main()
