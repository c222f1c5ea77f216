"""CPU interpreter of the compiled IPv4 device layouts (test infrastructure).

Reads the blob of ``cls_compile_v4`` (include/contivcls.h) and evaluates it
exactly as the gfx950 kernels do (vpp_amd/csrc/kernels.hip: classify4_cls's
branch-free interval search -> class -> cell -> candidate list; protocols >
2 on the OTHER image; linear_one for tables without a classifier), so the
rule compiler can be checked against the oracle without a GPU.  Never used
by the product.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from vpp_amd import _abi


def compile_blob(crules, fn="cls_compile_v4", options=None) -> bytes:
    """The compiler's image blob, under the test's library switches
    (libopts.CURRENT, the ``libopt`` fixture) and ``options``."""
    from libopts import option_string
    f = getattr(_abi.lib(), fn)
    need = C.c_uint64(0)
    opt = option_string(options)
    rc = f(crules.ptr(), crules.n, None, 0, C.byref(need), opt)
    if rc != 0:
        raise RuntimeError("%s rc=%d" % (fn, rc))
    buf = C.create_string_buffer(need.value)
    rc = f(crules.ptr(), crules.n, buf, need.value, C.byref(need), opt)
    if rc != 0:
        raise RuntimeError("%s rc=%d" % (fn, rc))
    return buf.raw


class Image:
    def __init__(self, blob: bytes):
        h = _abi.ImageHeader.from_buffer_copy(blob)
        assert h.magic in (0x434C5334, 0x434C3136, 0x434C534F)
        self.h = h
        self.n_rules = h.n_rules
        lin = np.frombuffer(blob, np.uint32, count=h.n_lin * 12, offset=h.off_lin).reshape(-1, 12)
        self.lin = lin
        self.has_cls = bool(h.has_cls)
        if self.has_cls:
            img = blob[h.off_image:h.off_image + h.img_bytes]
            self._img = img
            top = h.search_top
            if h.mode == 0:
                self.bounds = np.frombuffer(img, np.uint32, count=2 * top, offset=h.off_bounds)
                self.iclass = np.frombuffer(img, np.uint16, count=2 * top, offset=h.off_iclass)
            # cells per class: 3 (TCP, UDP, ICMP) or 1 (the OTHER image)
            self.ncell = h.row_bytes // (8 if h.list_mode in (0, 5, 6) else 4)
            if h.list_mode == 0:                   # uint2 cells
                self.cells = np.frombuffer(img, np.uint32, count=h.n_classes * 2 * self.ncell,
                                           offset=h.off_cells).reshape(-1, 2)
            if h.list_mode == 0:
                self.lists = np.frombuffer(img, np.uint16, count=h.n_list_entries, offset=h.off_lists)
                self.tmpl = np.frombuffer(img, np.uint32, count=h.n_tmpl * 4,
                                          offset=h.off_tmpl).reshape(-1, 4)
            self.ctr_rule = np.frombuffer(blob, np.uint32, count=h.n_ctr, offset=h.off_ctr_rule)
            self.hash = []
            for i in range(h.n_hash):
                cap = h.hash_cap[i]
                tab = np.frombuffer(img, np.uint32, count=4 * cap, offset=h.off_hash[i]).reshape(-1, 2)
                self.hash.append((h.hash_mask[i], h.hash_shift[i], cap, tab, h.hash_mul[i]))
        # list modes 5, 6: wide cells (uint2 {pointer table address, counter base}) in global memory
        self.gcells = (np.frombuffer(blob, np.uint32, count=h.n_gcells, offset=h.off_gcells).reshape(-1, 2)
                       if h.n_gcells else None)
        # protocols > 2: the OTHER image (its own blob inside this one)
        self.other = Image(blob[h.off_other:]) if h.off_other else None

    @staticmethod
    def _h0(k, mul, shift):
        return ((k.astype(np.uint64) * mul) & 0xFFFFFFFF) >> np.uint64(shift)

    @staticmethod
    def _h1(k, mul, shift):
        L = 32 - shift
        return (((k.astype(np.uint64) * mul) & 0xFFFFFFFF) >> np.uint64(32 - 2 * L)) & ((1 << L) - 1)

    def trie_class(self, src):
        """The source trie at h.off_trie (compile.cpp build_trie): class per
        host-order IPv4 address."""
        h = self.h
        img = np.frombuffer(self._img, np.uint32).astype(np.int64)
        s = np.asarray(src, np.uint32).astype(np.int64)
        a = img[(h.off_trie + ((s >> 22) & 0x3FC)) // 4]
        a = img[(a + ((s >> 14) & 0x3FC)) // 4]
        ln = (a & 0xFF) + 1
        a = a >> 8
        x = s & 0xFFFF
        for _ in range(h.trie_depth):
            half = ln >> 1
            c = a + 4 * half
            a = np.where((img[c // 4] & 0xFFFF) < x, c, a)
            ln = ln - half
        return img[a // 4] >> 16

    def source_class(self, src):
        h = self.h
        if h.mode == 4:
            # source trie (compile.cpp build_trie): level 1 -> node -> leaf
            # {address << 8 | m - 1}; branch-free lower bound for trie_depth steps
            img = np.frombuffer(self._img, np.uint32).astype(np.int64)
            s = src.astype(np.int64)
            a = img[(h.off_trie + ((s >> 22) & 0x3FC)) // 4]
            a = img[(a + ((s >> 14) & 0x3FC)) // 4]
            ln = (a & 0xFF) + 1
            a = a >> 8
            x = s & 0xFFFF
            for _ in range(h.trie_depth):
                half = ln >> 1
                c = a + 4 * half
                a = np.where((img[c // 4] & 0xFFFF) < x, c, a)
                ln = ln - half
            return img[a // 4] >> 16
        if h.mode == 1:
            # entries hold the byte address of the class's cell row
            row = np.full(len(src), h.default_row, np.int64)
            for mask, shift, cap, tab, mul in self.hash:
                key = src & np.uint32(mask)
                e0 = tab[self._h0(key, mul, shift).astype(np.int64)]
                e1 = tab[cap + self._h1(key, mul, shift).astype(np.int64)]
                row = np.where(e0[:, 0] == key, e0[:, 1].astype(np.int64),
                               np.where(e1[:, 0] == key, e1[:, 1].astype(np.int64), row))
            return (row - h.off_cells) // h.row_bytes
        k = np.zeros(len(src), np.int64)
        s = h.search_top
        while s:
            c = k + s
            k = np.where(self.bounds[c] <= src, c, k)
            s >>= 1
        return self.iclass[k].astype(np.int64)

    @staticmethod
    def _port_in(dport, pw):
        return ((dport.astype(np.uint32) - (pw & 0xFFFF)) & 0xFFFF) <= (pw >> 16)

    def _classify_bv(self, cls, src, dst, dport, proto, counters):
        """Bit-vector lists: per list, masks of the entries covering the dst
        interval and the port interval; first match = lowest common bit."""
        img = np.frombuffer(self._img, np.uint32)
        pr = np.minimum(proto, self.ncell - 1).astype(np.int64)
        cells1 = np.frombuffer(self._img, np.uint32, count=self.h.n_classes * self.ncell,
                               offset=self.h.off_cells)
        cell = cells1[cls * self.ncell + pr]
        cb = (cell >> 16).astype(np.int64)
        d_off = ((cell & 0xFFFF).astype(np.int64) * 8) // 4
        S = int(self.h.bv_steps_d)
        sd = np.full(len(cls), S, np.int64)
        sp = np.full(len(cls), S, np.int64)
        p_off = d_off + 2 * (np.int64(1) << sd)
        res_bits = img[d_off].astype(np.uint64) | (img[p_off].astype(np.uint64) << np.uint64(32))
        lm2 = self.h.list_mode == 2
        if lm2:
            pc = self._port_class(dport)

        def search(off, steps, x):
            k = np.zeros(len(x), np.int64)
            m = img[off + 1]
            for i in range(int(steps.max()) if len(x) else 0, -1, -1):
                st = np.where(i < steps, np.int64(1) << i, 0)
                c = k + st
                b = img[off + 2 * c]
                take = b <= x
                k = np.where(take, c, k)
                m = np.where(take, img[off + 2 * c + 1], m)
            return m

        md = search(d_off, sd, dst.astype(np.uint32))
        if lm2:
            mp = img[p_off + 1 + pc]
        else:
            mp = search(p_off, sp, dport.astype(np.uint32))
        m = (md & mp).astype(np.uint64)
        found = m != 0
        low = m & (~m + np.uint64(1))
        j = np.zeros(len(m), np.int64)
        nz = low != 0
        j[nz] = np.log2(low[nz].astype(np.float64)).astype(np.int64)
        res = np.where(found, (res_bits >> (2 * j).astype(np.uint64)) & np.uint64(3), 0).astype(np.uint32)
        slot = np.where(found, cb + j, 0)
        np.add.at(counters, self.ctr_rule[slot].astype(np.int64), 1)
        return res.astype(np.uint8), counters

    def _port_class(self, dport):
        """Global port class: top[p >> 8] = byte address of a 256-byte window
        of classes (x 4 in list mode 3)."""
        img = np.frombuffer(self._img, np.uint32)
        b8 = np.frombuffer(self._img, np.uint8)
        dp = dport.astype(np.int64)
        tp = img[self.h.off_ptop // 4 + (dp >> 8)].astype(np.int64)
        return b8[tp + (dp & 0xFF)].astype(np.int64)

    def _port_class4(self, dport):
        """List modes 3, 4: merged port class x 4 (mode 4: perfect hash at 0;
        5, 6 as 4, 3)."""
        if self.h.list_mode in (3, 6):
            return self._port_class(dport)
        img = np.frombuffer(self._img, np.uint32).astype(np.int64)
        dp = dport.astype(np.int64)
        e = img[(((dp * self.h.port_mul) >> 32) & self.h.port_mask4) // 4]
        return np.where((e & 0xFFFF) == dp, e >> 16, self.h.port_dflt)

    def _classify_bv3(self, cls, src, dst, dport, proto, counters):
        """List mode 3 (port-filtered sublists): cell u32 {pointer table word
        offset | counter base << 14}; table[port class] = initial state
        {outcome | entry slot << 16} (state >> 13 = entry byte address);
        entries {start - 1, state}, a probe of step i reads 8 << i bytes on and
        moves the state when start - 1 < dst; outcome = result | (j + 1) << 2."""
        img = np.frombuffer(self._img, np.uint32).astype(np.int64)
        pr = np.minimum(proto, self.ncell - 1).astype(np.int64)
        pc4 = self._port_class4(dport)                # class x 4
        if self.h.list_mode >= 5:
            # wide cells (list modes 5, 6) in global memory: {pointer table byte address, counter base}
            wc = self.gcells[cls * self.ncell + pr].astype(np.int64)
            st = img[(wc[:, 0] + pc4) // 4]
            base = wc[:, 1]
        else:
            cell = img[(self.h.off_cells + cls * self.h.row_bytes + pr * 4) // 4]
            st = img[((cell & 0x3FFF) * 4 + pc4) // 4]
            base = cell >> 14
        d = dst.astype(np.int64)
        for i in range(int(self.h.bv_steps_d) - 1, -1, -1):
            a = ((st >> 13) + (8 << i)) // 4
            st = np.where(img[a] < d, img[a + 1], st)
        res = (st & 3).astype(np.uint32)
        slot = base + ((st >> 2) & 63)               # the cell's no-match slot when j + 1 == 0
        np.add.at(counters, self.ctr_rule[slot].astype(np.int64), 1)
        return res.astype(np.uint8), counters

    def linear(self, src, dst, dport, proto):
        n = len(src)
        p = np.where(proto <= 2, proto, 3).astype(np.uint32)
        res = np.zeros(n, np.uint32)
        rule = np.full(n, self.n_rules, np.int64)
        done = np.zeros(n, bool)
        for r in self.lin:
            meta = (r[8] >> (8 * p)) & 0xFF
            pw = r[4 + p]
            m = (~done & ((meta & 0x80) != 0) & (((src ^ r[0]) & r[1]) == 0) &
                 (((dst ^ r[2]) & r[3]) == 0) & self._port_in(dport, pw))
            res[m] = meta[m] & 3
            rule[m] = r[9]
            done |= m
            if done.all():
                break
        return res, rule

    def classify(self, src, dst, dport, proto, cls=None, framed=False):
        """Returns (verdict u8[n], counters u64[R+1]).  cls: the packets'
        source classes when found by a front end (core mode 3).  A
        destination-keyed image (h.swap) sees src and dst exchanged, unless
        the caller already did that (framed)."""
        src = np.asarray(src, np.uint32)
        dst = np.asarray(dst, np.uint32)
        if self.h.swap and not framed:
            src, dst = dst, src
        dport = np.asarray(dport, np.uint16)
        proto = np.asarray(proto, np.uint8)
        oth = proto > 2
        if self.other is not None and oth.any():
            # the kernels classify protocols > 2 on the OTHER image (one cell per class)
            keep = ~oth
            v = np.zeros(len(src), np.uint8)
            v[keep], c = self.classify(src[keep], dst[keep], dport[keep], proto[keep],
                                       None if cls is None else cls[keep], framed=True)
            v[oth], c2 = self.other.classify(src[oth], dst[oth], dport[oth], np.zeros(int(oth.sum()), np.uint8),
                                             framed=True)
            return v, c + c2
        n = len(src)
        counters = np.zeros(self.n_rules + 1, np.uint64)
        if not self.has_cls:
            res, rule = self.linear(src, dst, dport, proto)
            np.add.at(counters, rule, 1)
            return res.astype(np.uint8), counters
        if cls is None:
            cls = self.source_class(src)
        if self.h.list_mode >= 3:
            return self._classify_bv3(cls, src, dst, dport, proto, counters)
        if self.h.list_mode >= 1:
            return self._classify_bv(cls, src, dst, dport, proto, counters)
        pr = np.minimum(proto, self.ncell - 1).astype(np.int64)
        cell = self.cells[cls * self.ncell + pr]
        start = (cell[:, 0] & 0xFFFF).astype(np.int64)
        ln = (cell[:, 0] >> 16).astype(np.int64)
        base = cell[:, 1].astype(np.int64)
        res = np.zeros(n, np.uint32)
        slot = np.zeros(n, np.int64)
        done = np.zeros(n, bool)
        for j in range(int(ln.max()) if n else 0):
            act = ~done & (j < ln)
            if not act.any():
                break
            tid = self.lists[np.where(act, start + j, 0)]
            tm = self.tmpl[tid]
            m = act & (((dst ^ tm[:, 0]) & tm[:, 1]) == 0) & self._port_in(dport, tm[:, 2])
            res[m] = tm[m, 3]
            slot[m] = base[m] + j
            done |= m
        np.add.at(counters, self.ctr_rule[slot].astype(np.int64), 1)
        return res.astype(np.uint8), counters


class Image16:
    """The 16-byte layout (cls_compile_v16): the front end maps each address to
    its 32-bit representative (kernels.hip fe_rep: binary search over 128-bit
    interval starts) or, src_mode 1, the source straight to its class row
    (src_hash16: host-route cuckoo hashes); the core image classifies."""

    def __init__(self, blob: bytes):
        h = _abi.Image16Header.from_buffer_copy(blob)
        assert h.core.magic == 0x434C3136
        self.h = h
        self.core = Image(blob)
        img = blob[h.core.off_image:h.core.off_image + h.core.img_bytes]
        self._img = img
        self.keys, self.vals = [None, None], [None, None]

        def table(src, koff, voff, top, k8, nval):
            if k8:                                     # 8-B keys over key8(address)
                k = np.frombuffer(src, np.uint32, count=2 * top, offset=koff).reshape(-1, 2)
                keys = [int(b) << 32 | int(a) for a, b in k]
            else:
                k = np.frombuffer(src, np.uint32, count=4 * top, offset=koff).reshape(-1, 4)
                hi = (k[:, 1].astype(object) << 32) | k[:, 0].astype(object)
                lo = (k[:, 3].astype(object) << 32) | k[:, 2].astype(object)
                keys = [int(a) << 64 | int(b) for a, b in zip(hi, lo)]
            if nval is None:                           # the real keys, then all-ones padding
                pad = (1 << 64) - 1 if k8 else (1 << 128) - 1
                nval = 1 + sum(1 for x in keys[1:] if x != pad)
            return keys, np.frombuffer(src, np.uint32, count=nval, offset=voff)

        for sd in range(2):
            src = img
            koff, voff = h.fe_key[sd], h.fe_val[sd]
            if sd == 0 and h.src_mode == 1:           # source interval table in the trailer
                src, koff = blob, h.off_src_search
                voff = koff + h.src_search_val
            self.keys[sd], self.vals[sd] = table(src, koff, voff, h.fe_top[sd], h.fe_k8[sd], h.fe_n[sd])
        # src_mode 2: side 0 above is the non-IPv4 search (values: rows); the
        # whole table with reps is in the trailer (protocols > 2)
        self.gtab = None
        if h.src_mode == 2:
            self.gtab = table(blob, h.off_src_search, h.off_src_search + h.src_search_val, h.src_search_top,
                              h.src_search_k8, None)

    def rep(self, sd: int, addrs, table=None) -> np.ndarray:
        keys, vals, top = self.keys[sd], self.vals[sd], self.h.fe_top[sd]
        k8 = self.h.fe_k8[sd]
        if table is not None:
            (keys, vals), top, k8 = table, self.h.src_search_top, self.h.src_search_k8
        if k8:
            # vectorised: the branch-free search lands on the number of keys
            # [1, top) below key8(address) (keys ascending, padding all ones)
            a = np.ascontiguousarray(addrs, np.uint8).reshape(-1, 16)
            hi = a[:, :8].copy().view(">u8").ravel().astype(np.uint64)
            lo = a[:, 8:].copy().view(">u8").ravel().astype(np.uint64)
            k48 = np.uint64(1 << 48)
            x = np.where(hi == 0, np.minimum(lo, k48), k48 + np.minimum(hi, np.uint64((1 << 64) - 1 - (1 << 48))))
            kk = np.array(keys[1:top], np.uint64)
            pos = np.searchsorted(kk, x, side="left")
            return np.asarray(vals, np.uint32)[pos]
        out = np.empty(len(addrs), np.uint32)
        for i, a in enumerate(addrs):
            x = int.from_bytes(bytes(a), "big")
            if k8:
                hi, lo = x >> 64, x & ((1 << 64) - 1)
                x = min(lo, 1 << 48) if hi == 0 else (1 << 48) + min(hi, (1 << 64) - 1 - (1 << 48))
            pos, s = 0, top >> 1
            while s:
                if keys[pos + s] < x:
                    pos += s
                s >>= 1
            out[i] = vals[pos]
        return out

    def src_rows(self, addrs) -> np.ndarray:
        """src_mode 1: kernels.hip src_hash16."""
        h = self.h
        w = np.frombuffer(np.ascontiguousarray(addrs).tobytes(), "<u4").reshape(-1, 4).astype(np.uint64)
        M = np.uint64(0xFFFFFFFF)
        L4, L6 = h.cap4.bit_length() - 1, h.cap6.bit_length() - 1
        t4 = np.frombuffer(self._img, np.uint32, count=4 * h.cap4, offset=h.h4).reshape(-1, 2)
        x = w[:, 3]
        g = (x * np.uint64(h.mul4)) & M
        e0 = t4[(g >> np.uint64(32 - L4)).astype(np.int64)]
        e1 = t4[h.cap4 + ((g >> np.uint64(32 - 2 * L4)) & np.uint64(h.cap4 - 1)).astype(np.int64)]
        r4 = np.where(e0[:, 0] == x, e0[:, 1], np.where(e1[:, 0] == x, e1[:, 1], h.dflt_row[0]))
        k6 = np.frombuffer(self._img, np.uint32, count=8 * h.cap6, offset=h.k6).reshape(-1, 4)
        r6t = np.frombuffer(self._img, np.uint32, count=2 * h.cap6, offset=h.r6)
        f = ((w[:, 0] * np.uint64(h.fold[0])) & M) ^ ((w[:, 1] * np.uint64(h.fold[1])) & M) ^ \
            ((w[:, 2] * np.uint64(h.fold[2])) & M) ^ w[:, 3]
        g = (f * np.uint64(h.mul6)) & M
        p0 = (g >> np.uint64(32 - L6)).astype(np.int64)
        p1 = h.cap6 + ((g >> np.uint64(32 - 2 * L6)) & np.uint64(h.cap6 - 1)).astype(np.int64)
        m0 = (k6[p0] == w).all(1)
        m1 = (k6[p1] == w).all(1)
        r6 = np.where(m0, r6t[p0], np.where(m1, r6t[p1], h.dflt_row[1]))
        is4 = (w[:, 0] == 0) & (w[:, 1] == 0) & (w[:, 2] == 0xFFFF0000)
        return np.where(is4, r4, r6).astype(np.int64)

    def classify(self, src16, dst16, dport, proto):
        src16 = np.asarray(src16, np.uint8).reshape(-1, 16)
        dst16 = np.asarray(dst16, np.uint8).reshape(-1, 16)
        if self.h.core.swap:                           # destination-keyed
            src16, dst16 = dst16, src16
        drep = self.rep(1, dst16)
        if self.h.src_mode == 2:
            # kernels_dev.hpp src_trie16: IPv4-mapped sources by the trie over
            # their IPv4 word, the others by the non-IPv4 search (rows);
            # protocol > 2 takes the rep from the whole table
            srep = self.rep(0, src16, table=self.gtab)
            w = np.frombuffer(np.ascontiguousarray(src16).tobytes(), "<u4").reshape(-1, 4)
            is4 = (w[:, 0] == 0) & (w[:, 1] == 0) & (w[:, 2] == 0xFFFF0000)
            ip = src16[:, 12:16].astype(np.uint32)
            ip = (ip[:, 0] << 24) | (ip[:, 1] << 16) | (ip[:, 2] << 8) | ip[:, 3]
            c4 = self.core.trie_class(ip)
            rows6 = self.rep(0, src16).astype(np.int64)
            c6 = (rows6 - self.core.h.off_cells) // self.core.h.row_bytes
            cls = np.where(is4, c4, c6)
            return self.core.classify(srep, drep, dport, proto, cls=cls, framed=True)
        srep = self.rep(0, src16)
        if self.h.src_mode == 1:
            rows = self.src_rows(src16)
            # the hashed row must be the class row of the rep (what the core's
            # own source lookup would give), protocol > 2 takes the rep
            cls = (rows - self.core.h.off_cells) // self.core.h.row_bytes
            return self.core.classify(srep, drep, dport, proto, cls=cls, framed=True)
        return self.core.classify(srep, drep, dport, proto, framed=True)
