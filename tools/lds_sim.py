#!/usr/bin/env python3
"""LDS bank-conflict model of classify4_cls (diagnostics, CPU only).

Replays the LDS address stream the hot kernel issues for a packet stream
(vpp_amd/csrc/kernels.hip, list mode 2 + hash LPM) and prices every wave
instruction with the gfx950 banking rules of MI355X_MICROARCH.md "LDS":
  ds_read_b32 / ds_read_u8 / ds_add_u32: 2 groups x 32 lanes, bank (a/4) mod 32
  ds_read_b64: 2 groups x 32 lanes, bank (a/4) mod 64, two dwords per lane
  one LDS cycle per group when conflict-free, +1 per extra distinct dword on a bank.
The lane -> packet map is the kernel's: lane l of a wave-step holds packets
4l..4l+3 of a 256-packet tile; instruction q touches packet q of every lane.

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
    cyc = np.zeros(I, np.int64)
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
    any_active = active.any(axis=1)
    return np.where(any_active, np.maximum(cyc, 1), 0)


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


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    npk = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
    import oracle
    from vpp_amd import _abi, workload
    import cls_image
    acl, spec, _ = workload.config(cfg)
    im = cls_image.Image(cls_image.compile_blob(_abi.CRules(acl.rules)))
    h = im.h
    assert h.mode == 1 and h.list_mode == 2, "model covers hash LPM + list mode 2"
    tr = oracle.gen_traffic_v4(spec, 0, npk)
    src, dst = tr["src"].astype(np.int64), tr["dst"].astype(np.int64)
    dport, proto = tr["dport"].astype(np.int64), tr["proto"].astype(np.int64)
    img = np.frombuffer(im._img, np.uint32).astype(np.int64)
    b8 = np.frombuffer(im._img, np.uint8).astype(np.int64)
    V = set(os.environ.get("VARIANT", "").split(","))
    ops = []   # (name, kind, addr per packet[, active per packet])
    # port class
    a_top = h.off_ptop + 4 * (dport >> 8)
    tp = img[a_top // 4]
    a_sub = (tp & 0xFFFFF) + (dport & 0xFF)
    pc = (tp >> 20) + b8[a_sub]
    if "uniform" in V:      # uniform 256-port chunks read one fixed byte
        a_sub = np.where((tp & 0xFFFFF) == h.off_ptop + 1024, h.off_ptop + 1024, a_sub)
    ops += [("ptop", "b32", a_top), ("psub", "u8", a_sub)]
    # hash probes
    cls_true = im.source_class(tr["src"]).astype(np.int64)
    cls = np.full(npk, h.default_class, np.int64)
    for i in range(h.n_hash):
        mask, shift, cap = h.hash_mask[i], h.hash_shift[i], h.hash_cap[i]
        key = src & mask
        h0 = ((key * 0x9E3779B1) & 0xFFFFFFFF) >> shift
        h1 = (((key ^ 0x5BD1E995) * 0xC2B2AE35) & 0xFFFFFFFF) >> shift
        a0 = h.off_hash[i] + 8 * h0
        a1 = h.off_hash[i] + 8 * (cap + h1)
        hact = np.ones(npk, bool)
        if "filter" in V:   # 64-bit filter on src >> 26 (kernel argument)
            hact = np.isin(src >> 26, np.unique(key[cls_true != h.default_class] >> 26))
        ops += [("hash0", "b64", a0, hact), ("hash1", "b64", a1, hact)]
        e1k, e1v = img[a1 // 4], img[a1 // 4 + 1]
        e0k, e0v = img[a0 // 4], img[a0 // 4 + 1]
        cls = np.where(e1k == key, e1v, cls)
        cls = np.where(e0k == key, e0v, cls)
    a_cell = h.off_cells + 4 * (cls * 3 + np.minimum(proto, 2))
    cell = img[a_cell // 4]
    ops.append(("cell", "b32", a_cell, cls != h.default_class if "hotcell" in V else None))
    S = h.bv_steps_d
    ad = (cell & 0xFFFF) * 8
    ap = ad + (8 << S)
    if "nod0" not in V:
        ops.append(("d0", "b64", ad.copy()))
    a_mp = ap + 4 + pc * 4
    ops.append(("pmask", "b64" if "nod0" in V else "b32", a_mp & ~7 if "nod0" in V else a_mp))
    md = img[ad // 4 + 1]
    # per-list search depth: intervals in the block (bounds < sentinel)
    nint = np.ones(npk, np.int64)
    for i in range(1, 1 << S):
        nint += img[ad // 4 + 2 * i] != 0xFFFFFFFF
    sl = np.zeros(npk, np.int64)
    while True:
        more = (1 << sl) < nint
        if not more.any():
            break
        sl += more
    for i in range(S - 1, -1, -1):
        step = 8 << i
        a = ad + step
        ops.append(("dstep%d" % i, "b64", a, (i < sl) if "mask" in V else None))
        take = img[a // 4] <= dst
        md = np.where(take, img[a // 4 + 1], md)
        ad = np.where(take, a, ad)
    mp = img[a_mp // 4]
    m = md & mp
    j = np.zeros(npk, np.int64)
    nz = m != 0
    j[nz] = np.log2((m[nz] & -m[nz]).astype(np.float64)).astype(np.int64)
    slot = np.where(nz, (cell >> 16) + j, 0)
    lane = (np.arange(npk) // 4) % 64
    hot_base = h.lds_bytes - 0  # rows live after the counters: off_hot (not exported) = lds - n_hot*256
    n_hot = 0
    # n_hot is not in the exported header: recover it from lds_bytes
    ctr_end = h.img_bytes + ((h.n_ctr * 4 + 15) & ~15)
    n_hot = (h.lds_bytes - ctr_end) // 256
    a_ctr = np.where(slot < n_hot, ctr_end + 4 * (lane + slot * 64), h.img_bytes + 4 * slot)
    ops.append(("atomic", "atomic", a_ctr))

    # group into wave instructions: tile of 256 packets, instruction q -> packets 4l+q
    ntile = npk // 256
    total = 0
    print("config %d: %d packets, S=%d, n_hot=%d, hash caps %s" % (cfg, npk, S, n_hot, list(h.hash_cap)[:h.n_hash]))
    print("%-8s %-6s %8s %8s" % ("op", "kind", "cyc/inst", "ideal"))
    for op in ops:
        name, kind, a = op[:3]
        act = op[3] if len(op) > 3 and op[3] is not None else np.ones(npk, bool)
        A = a[: ntile * 256].reshape(ntile, 64, 4).transpose(0, 2, 1).reshape(-1, 64)
        act = act[: ntile * 256].reshape(ntile, 64, 4).transpose(0, 2, 1).reshape(-1, 64)
        c = inst_cycles(A, act, kind)
        ideal = 2
        total += c.mean() * 4
        print("%-8s %-6s %8.2f %8d" % (name, kind, c.mean(), ideal))
    print("LDS cycles per wave-step (256 packets): %.1f  -> %.3f cycles/packet" % (total, total / 256))


if __name__ == "__main__":
    main()
