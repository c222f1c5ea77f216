"""Random ACL and traffic generators for parity tests (test infrastructure).

``random_acl`` produces adversarial rule lists that exercise every branch of
evalACL (mock/aclengine/aclengine_mock.go:480-667): nested and disjoint
prefixes of every length, IPv6 and IPv4-mapped strings, malformed CIDRs,
missing/extra protocol sections and port ranges, non-full source ranges,
reversed and wide destination ranges (with uint16 truncation), ICMP
code/type ranges, Icmpv6, MAC-IP / Other sections, unknown actions.
"""
from __future__ import annotations

import random

import numpy as np

from vpp_amd import model as M


def _v4(a):
    return "%d.%d.%d.%d" % ((a >> 24) & 255, (a >> 16) & 255, (a >> 8) & 255, a & 255)


class PrefixPool:
    def __init__(self, rng: random.Random, n=24):
        self.rng = rng
        self.v4 = []
        base = [rng.getrandbits(32) for _ in range(max(2, n // 4))]
        for _ in range(n):
            b = rng.choice(base)
            ln = rng.choice([0, 1, 8, 12, 16, 20, 24, 24, 28, 30, 31, 32, 32, 32])
            b ^= rng.getrandbits(32) >> max(ln, 1) if rng.random() < 0.5 else 0
            mask = (0xFFFFFFFF << (32 - ln)) & 0xFFFFFFFF if ln else 0
            self.v4.append((b & mask, ln))

    def cidr(self, allow_weird=True) -> str:
        rng = self.rng
        r = rng.random()
        if not allow_weird or r < 0.80:
            a, ln = rng.choice(self.v4)
            if rng.random() < 0.1:                       # host bits set: ParseCIDR masks them
                a |= rng.getrandbits(32) & ((1 << (32 - ln)) - 1 if ln < 32 else 0)
            return "%s/%d" % (_v4(a), ln)
        if r < 0.86:                                      # IPv4-mapped IPv6 spelling
            a, ln = rng.choice(self.v4)
            return "::ffff:%s/%d" % (_v4(a), 96 + ln)
        if r < 0.90:
            return rng.choice(["fd00:10::/64", "::/0", "2001:db8::1/128", "::ffff:0:0/95"])
        return rng.choice(["10.0.0.0/33", "10.0.0/8", "garbage", "1.2.3.4", "300.1.1.1/8",
                           "10.0.0.0/", "/8", "::ffff:10.0.0.0/95", "010.001.0.0/16"])


def random_rule(rng: random.Random, pool: PrefixPool, weird: float = 0.15) -> M.Rule:
    w = lambda: rng.random() < weird
    action = rng.choice([M.DENY, M.PERMIT, M.PERMIT, M.REFLECT])
    if w():
        action = rng.choice([3, -1, 7])
    actions = None if w() and rng.random() < 0.3 else M.Actions(action)
    if w() and rng.random() < 0.15:
        return M.Rule(actions=actions, matches=M.Matches(macip_rule=M.MacIpRule()))
    if w() and rng.random() < 0.1:
        return M.Rule(actions=actions, matches=M.Matches())
    ip = M.Ip(source_network=pool.cidr(weird > 0) if rng.random() < 0.7 else "",
              destination_network=pool.cidr(weird > 0) if rng.random() < 0.6 else "")
    ipr = M.IpRule(ip=None if (w() and rng.random() < 0.1) else ip)
    kind = rng.choice(["tcp", "udp", "tcp", "udp", "icmp"] + (["none", "both", "other"] if w() else []))

    def prange(src=False):
        if src:
            if w():
                return rng.choice([None, M.PortRange(0, 1000), M.PortRange(1, 65535)])
            return M.PortRange(0, 65535)
        r = rng.random()
        if r < 0.35:
            return M.PortRange(0, 65535)
        if r < 0.75:
            p = rng.choice([22, 53, 80, 161, 443, 8080, rng.randint(1, 65535)])
            return M.PortRange(p, p)
        lo = rng.randint(0, 65535)
        hi = rng.randint(lo, 65535)
        if w():
            return rng.choice([None, M.PortRange(hi, lo), M.PortRange(70000, 80000),
                               M.PortRange(65536 + 80, 65536 + 90)])
        return M.PortRange(lo, hi)

    if kind in ("tcp", "both"):
        ipr.tcp = M.Tcp(destination_port_range=prange(), source_port_range=prange(True))
    if kind in ("udp", "both"):
        ipr.udp = M.Udp(destination_port_range=prange(), source_port_range=prange(True))
    if kind == "icmp":
        code = M.IcmpRange(0, 5) if not w() else rng.choice([None, M.IcmpRange(0, 4)])
        typ = M.IcmpRange(0, 16) if not w() else rng.choice([None, M.IcmpRange(1, 16)])
        ipr.icmp = M.Icmp(icmpv6=w() and rng.random() < 0.3, icmp_code_range=code,
                          icmp_type_range=typ)
    if kind == "other":
        ipr.other = M.Other(protocol=47)
    return M.Rule(actions=actions, matches=M.Matches(ip_rule=ipr))


def random_acl(seed: int, n_rules: int, weird: float = 0.15, n_prefixes: int = 24):
    rng = random.Random(seed)
    pool = PrefixPool(rng, n_prefixes)
    return [random_rule(rng, pool, weird) for _ in range(n_rules)], pool


def long_list_acl(seed: int, n_rules: int = 300, n_src: int = 3):
    """Rules with few source prefixes and no catch-all: every cell's candidate
    list is long (> 32), which selects the template-scan list mode."""
    rng = random.Random(seed)
    pool = PrefixPool(rng, 32)
    srcs = [pool.v4[i] for i in range(n_src)]
    rules = []
    for _ in range(n_rules):
        a, ln = rng.choice(srcs)
        da, dl = rng.choice(pool.v4[n_src:])
        dl = max(dl, 1)
        proto = rng.choice(["tcp", "udp"])
        p = rng.choice([22, 53, 80, 443, rng.randint(1, 65535)])
        hi = p if rng.random() < 0.7 else min(65535, p + rng.randint(1, 1000))
        rules.append(M.l4_rule(rng.choice([M.DENY, M.PERMIT, M.REFLECT]), "%s/%d" % (_v4(a), ln),
                               "%s/%d" % (_v4(da), dl), proto, 0, 65535, p, hi))
    return rules, pool


def many_ports_acl(seed: int, n_rules: int = 400, n_src: int = 40, host_src: bool = True):
    """Short candidate lists over many distinct port ranges: more than 256
    global port classes, which selects bit vectors with per-list port search
    (list_mode 1).  host_src: /32 sources (hash LPM), else the pool's mixed
    prefix lengths (interval search)."""
    rng = random.Random(seed)
    pool = PrefixPool(rng, 48)
    if host_src:
        srcs = [(a | rng.randint(0, 255) if ln <= 24 else a, 32) for a, ln in pool.v4[:n_src]]
    else:                                   # 5 lengths, random (rarely nested) prefixes
        lens = (16, 20, 24, 28, 32)
        srcs = [(rng.getrandbits(32) & ((0xFFFFFFFF << (32 - lens[i % 5])) & 0xFFFFFFFF), lens[i % 5])
                for i in range(n_src)]
        pool.v4 = srcs + pool.v4[n_src:]
    rules = []
    for _ in range(n_rules):
        a, ln = rng.choice(srcs)
        da, dl = rng.choice(pool.v4[n_src:])
        proto = rng.choice(["tcp", "udp"])
        lo = rng.randint(0, 64000)
        hi = lo + rng.randint(0, 1500)
        rules.append(M.l4_rule(rng.choice([M.DENY, M.PERMIT, M.REFLECT]), "%s/%d" % (_v4(a), ln),
                               "%s/%d" % (_v4(da), max(dl, 1)), proto, 0, 65535, lo, hi))
    return rules, pool


def random_traffic(seed: int, n: int, pool: PrefixPool, other_proto: bool = True):
    """IPv4 packets biased towards the prefixes' edges."""
    rng = np.random.default_rng(seed)
    pfx = np.array([a for a, _ in pool.v4], np.uint64)
    size = np.array([(1 << (32 - ln)) for _, ln in pool.v4], np.uint64)

    def addrs():
        choice = rng.integers(0, 5, n)
        i = rng.integers(0, len(pfx), n)
        inside = (pfx[i] + rng.integers(0, 1 << 62, n, dtype=np.uint64) % size[i]) & 0xFFFFFFFF
        first = pfx[i]
        last = (pfx[i] + size[i] - 1) & 0xFFFFFFFF
        past = (pfx[i] + size[i]) & 0xFFFFFFFF
        uni = rng.integers(0, 1 << 32, n, dtype=np.uint64)
        out = np.select([choice == 0, choice == 1, choice == 2, choice == 3],
                        [inside, first, last, past], uni)
        edge = rng.random(n) < 0.01
        out[edge] = rng.choice(np.array([0, 0xFFFFFFFF], np.uint64), edge.sum())
        return out.astype(np.uint32)

    src, dst = addrs(), addrs()
    ports = np.array([0, 1, 22, 53, 79, 80, 81, 161, 443, 8080, 65535], np.uint16)
    dport = np.where(rng.random(n) < 0.6, rng.choice(ports, n),
                     rng.integers(0, 65536, n)).astype(np.uint16)
    pvals = [0, 1, 2, 3, 17] if other_proto else [0, 1, 2]
    pw = [0.4, 0.4, 0.14, 0.03, 0.03] if other_proto else [0.43, 0.43, 0.14]
    proto = rng.choice(np.array(pvals, np.uint8), n, p=pw)
    sport = rng.integers(1024, 65536, n).astype(np.uint16)
    return dict(src=src, dst=dst, dport=dport, proto=proto, sport=sport)


def single_port_acl(seed: int, n_rules: int = 120, n_prefixes: int = 8):
    """Rules in renderACL's shape (acl_renderer.go:342-374): dst port a single
    port or any (ContivRule.DestPort, 0 = any), no source port.  Port classes
    then merge into few, and the compiler picks the hashed port lookup (list
    mode 4)."""
    rng = random.Random(seed)
    pool = PrefixPool(rng, n_prefixes)
    ports = [22, 53, 80, 161, 443, 8080, rng.randint(1, 65535), rng.randint(1, 65535)]
    rules = []
    for _ in range(n_rules):
        a, ln = rng.choice(pool.v4)
        src = "%s/%d" % (_v4(a), ln) if rng.random() < 0.8 else ""
        da, dl = rng.choice(pool.v4)
        dst = "%s/%d" % (_v4(da), dl) if rng.random() < 0.7 else ""
        p = rng.choice(ports) if rng.random() < 0.7 else 0
        rules.append(M.l4_rule(rng.choice([M.DENY, M.PERMIT, M.REFLECT]), src, dst,
                               rng.choice(["tcp", "udp"]), 0, 65535, p, p if p else 65535))
    return rules, pool


# ---------------------------------------------------------------------------
# mixed-family tables and 16-byte traffic (the CLS_AF_V16 path)

V4_MAPPED = 0xFFFF << 32


def _v6(x: int) -> str:
    import ipaddress
    return str(ipaddress.IPv6Address(x))


class PrefixPool16(PrefixPool):
    """IPv4 prefixes (PrefixPool) plus IPv6 ones: nested /32../128 under a few
    bases, IPv4-mapped and IPv4-compatible spellings, and the ranges around the
    v4-mapped block (::ffff:0:0/96 is an IPv4 network for Go, /95 and /80 are
    IPv6 networks that numerically contain it)."""

    def __init__(self, rng: random.Random, n=24):
        super().__init__(rng, n)
        bases = [0xFD000010 << 96, 0xFD000020 << 96, 0x20010DB8 << 96, 0, V4_MAPPED]
        self.v6 = []
        for _ in range(n):
            b = rng.choice(bases[:3])
            ln = rng.choice([32, 48, 56, 64, 64, 96, 112, 120, 127, 128, 128, 128])
            a = b | (rng.getrandbits(128 - 32) if ln > 32 else 0)
            host = (1 << (128 - ln)) - 1
            self.v6.append((a & ~host & ((1 << 128) - 1), ln))
        self.v6 += [(0, 0), (0, 80), (V4_MAPPED & ~((1 << 33) - 1), 95), (0, 96), (1, 128)]

    def cidr(self, allow_weird=True) -> str:
        rng = self.rng
        r = rng.random()
        if r < 0.45:
            a, ln = rng.choice(self.v6)
            return "%s/%d" % (_v6(a), ln)
        if r < 0.52:
            return rng.choice(["::ffff:0:0/96", "::ffff:0.0.0.0/96", "::ffff:0:0/95", "::/0",
                               "::ffff:10.1.0.0/112", "::10.1.2.3/128", "0.0.0.0/0"])
        return super().cidr(allow_weird)

    def addr16(self, np_rng, n):
        """n addresses (as python ints) biased towards the prefixes' edges."""
        out = []
        for _ in range(n):
            c = np_rng.integers(0, 10)
            if c < 4:
                a, ln = self.v4[np_rng.integers(0, len(self.v4))]
                size = 1 << (32 - ln)
                k = np_rng.integers(0, 4)
                x = [a + int(np_rng.integers(0, size)), a, a + size - 1, a + size][k] & 0xFFFFFFFF
                out.append(V4_MAPPED | x)
            elif c < 8:
                a, ln = self.v6[np_rng.integers(0, len(self.v6))]
                size = 1 << (128 - ln)
                k = np_rng.integers(0, 4)
                off = int.from_bytes(np_rng.bytes(16), "big") % size
                out.append([a + off, a, a + size - 1, a + size][k] & ((1 << 128) - 1))
            elif c < 9:
                out.append(int(np_rng.choice([0, 1, V4_MAPPED - 1, V4_MAPPED, V4_MAPPED | 0xFFFFFFFF,
                                              (V4_MAPPED | 0xFFFFFFFF) + 1, (1 << 128) - 1,
                                              0x0A010203])))
            else:
                out.append(int.from_bytes(np_rng.bytes(16), "big"))
        return out


def random_acl16(seed: int, n_rules: int, weird: float = 0.15, n_prefixes: int = 24):
    rng = random.Random(seed)
    pool = PrefixPool16(rng, n_prefixes)
    return [random_rule(rng, pool, weird) for _ in range(n_rules)], pool


def to16(addrs) -> np.ndarray:
    return np.frombuffer(b"".join(int(a).to_bytes(16, "big") for a in addrs), np.uint8).reshape(-1, 16).copy()


def random_traffic16(seed: int, n: int, pool: PrefixPool16, other_proto: bool = True):
    rng = np.random.default_rng(seed)
    src, dst = to16(pool.addr16(rng, n)), to16(pool.addr16(rng, n))
    ports = np.array([0, 1, 22, 53, 79, 80, 81, 161, 443, 8080, 65535], np.uint16)
    dport = np.where(rng.random(n) < 0.6, rng.choice(ports, n),
                     rng.integers(0, 65536, n)).astype(np.uint16)
    pvals = [0, 1, 2, 3, 17] if other_proto else [0, 1, 2]
    pw = [0.4, 0.4, 0.14, 0.03, 0.03] if other_proto else [0.43, 0.43, 0.14]
    proto = rng.choice(np.array(pvals, np.uint8), n, p=pw)
    sport = rng.integers(1024, 65536, n).astype(np.uint16)
    return dict(src=src, dst=dst, dport=dport, proto=proto, sport=sport)


V6_TWIN = 0xFD000030 << 96          # fd00:30::/96 + IPv4 address: an IPv6 twin of the IPv4 space


def _twin_cidr(c: str, rng: random.Random) -> str:
    """a.b.c.d/n -> fd00:30::a.b.c.d/(96+n) (an IPv6 network of the same shape), other strings as is."""
    import ipaddress
    try:
        net = ipaddress.IPv4Network(c, strict=False)
        if "/" not in c or c.count(".") != 3 or rng.random() < 0.5:
            return c
        return "%s/%d" % (_v6(V6_TWIN | int(net.network_address)), 96 + net.prefixlen)
    except ValueError:
        return c


def mix_families(rules, traffic, seed: int, frac: float = 0.5):
    """A mixed-family version of an IPv4 table and batch: about `frac` of the
    networks become their fd00:30::/96 twins, every packet address becomes
    16 bytes -- its twin with probability frac, else IPv4-mapped -- so list
    shapes (and the compiler's list modes) stay those of the IPv4 table."""
    import copy
    rng = random.Random(seed)
    out = []
    for r in rules:
        r = copy.deepcopy(r)
        ip = r.matches.ip_rule.ip if r.matches is not None and r.matches.ip_rule is not None else None
        if ip is not None:
            ip.source_network = _twin_cidr(ip.source_network, rng) if ip.source_network else ip.source_network
            ip.destination_network = (_twin_cidr(ip.destination_network, rng) if ip.destination_network
                                      else ip.destination_network)
        out.append(r)
    nrng = np.random.default_rng(seed)
    n = len(traffic["src"])

    def widen(a):
        twin = nrng.random(n) < frac
        hi = np.where(twin, np.uint64(V6_TWIN >> 64), np.uint64(0))
        lo = np.where(twin, np.uint64(0), np.uint64(0xFFFF << 32)) | a.astype(np.uint64)
        b = np.empty((n, 16), np.uint8)
        b[:, :8] = hi.astype(">u8").view(np.uint8).reshape(n, 8)
        b[:, 8:] = lo.astype(">u8").view(np.uint8).reshape(n, 8)
        return b

    tr = dict(traffic)
    tr["src"], tr["dst"] = widen(traffic["src"]), widen(traffic["dst"])
    return out, tr
