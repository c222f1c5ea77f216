"""Go 1.9 ``net`` semantics needed by the renderer layer.

The Contiv renderer builds ``*net.IPNet`` values, orders them
(plugins/policy/utils/utils.go:187-239) and prints them with
``IPNet.String()`` into the ACL's CIDR strings
(renderer/acl/acl_renderer.go:336-341).  This module restates exactly those
stdlib behaviours (Go 1.9.x, .travis.yml:7-8): ParseIP, ParseCIDR, CIDRMask,
IP.To4/To16/Mask/Equal/String, IPMask.Size, IPNet.Contains/String.

IPs are ``bytes`` of length 0 (nil), 4 or 16; masks likewise.
"""
from __future__ import annotations

from typing import Optional, Tuple

IPV4LEN = 4
IPV6LEN = 16
_BIG = 0xFFFFFF
V4_IN_V6_PREFIX = bytes([0] * 10 + [0xFF, 0xFF])


def _dtoi(s: str) -> Tuple[int, int, bool]:
    n = 0
    i = 0
    while i < len(s) and "0" <= s[i] <= "9":
        n = n * 10 + (ord(s[i]) - 48)
        if n >= _BIG:
            return _BIG, i, False
        i += 1
    if i == 0:
        return 0, 0, False
    return n, i, True


def _xtoi(s: str) -> Tuple[int, int, bool]:
    n = 0
    i = 0
    while i < len(s):
        c = s[i]
        if "0" <= c <= "9":
            n = n * 16 + (ord(c) - 48)
        elif "a" <= c <= "f":
            n = n * 16 + (ord(c) - 97) + 10
        elif "A" <= c <= "F":
            n = n * 16 + (ord(c) - 65) + 10
        else:
            break
        if n >= _BIG:
            return 0, i, False
        i += 1
    if i == 0:
        return 0, i, False
    return n, i, True


def ipv4(a: int, b: int, c: int, d: int) -> bytes:
    return V4_IN_V6_PREFIX + bytes([a, b, c, d])


def parse_ipv4(s: str) -> Optional[bytes]:
    p = []
    for i in range(IPV4LEN):
        if len(s) == 0:
            return None
        if i > 0:
            if s[0] != ".":
                return None
            s = s[1:]
        n, c, ok = _dtoi(s)
        if not ok or n > 0xFF:
            return None
        s = s[c:]
        p.append(n)
    if len(s) != 0:
        return None
    return ipv4(*p)


def parse_ipv6(s: str) -> Optional[bytes]:
    ip = bytearray(IPV6LEN)
    ellipsis = -1
    if len(s) >= 2 and s[0] == ":" and s[1] == ":":
        ellipsis = 0
        s = s[2:]
        if len(s) == 0:
            return bytes(ip)
    i = 0
    while i < IPV6LEN:
        n, c, ok = _xtoi(s)
        if not ok or n > 0xFFFF:
            return None
        if c < len(s) and s[c] == ".":
            if ellipsis < 0 and i != IPV6LEN - IPV4LEN:
                return None
            if i + IPV4LEN > IPV6LEN:
                return None
            ip4 = parse_ipv4(s)
            if ip4 is None:
                return None
            ip[i:i + 4] = ip4[12:16]
            s = ""
            i += IPV4LEN
            break
        ip[i] = (n >> 8) & 0xFF
        ip[i + 1] = n & 0xFF
        i += 2
        s = s[c:]
        if len(s) == 0:
            break
        if s[0] != ":" or len(s) == 1:
            return None
        s = s[1:]
        if s[0] == ":":
            if ellipsis >= 0:
                return None
            ellipsis = i
            s = s[1:]
            if len(s) == 0:
                break
    if len(s) != 0:
        return None
    if i < IPV6LEN:
        if ellipsis < 0:
            return None
        n = IPV6LEN - i
        for j in range(i - 1, ellipsis - 1, -1):
            ip[j + n] = ip[j]
        for j in range(ellipsis + n - 1, ellipsis - 1, -1):
            ip[j] = 0
    elif ellipsis >= 0:
        return None
    return bytes(ip)


def parse_ip(s: str) -> Optional[bytes]:
    """net.ParseIP"""
    for ch in s:
        if ch == ".":
            return parse_ipv4(s)
        if ch == ":":
            return parse_ipv6(s)
    return None


def cidr_mask(ones: int, bits: int) -> bytes:
    if bits != 8 * IPV4LEN and bits != 8 * IPV6LEN:
        return b""
    if ones < 0 or ones > bits:
        return b""
    m = bytearray(bits // 8)
    n = ones
    for i in range(len(m)):
        if n >= 8:
            m[i] = 0xFF
            n -= 8
            continue
        m[i] = (~(0xFF >> n)) & 0xFF
        n = 0
    return bytes(m)


def to4(ip: bytes) -> Optional[bytes]:
    if len(ip) == IPV4LEN:
        return ip
    if len(ip) == IPV6LEN and ip[:12] == V4_IN_V6_PREFIX:
        return ip[12:16]
    return None


def to16(ip: bytes) -> Optional[bytes]:
    if len(ip) == IPV4LEN:
        return V4_IN_V6_PREFIX + ip
    if len(ip) == IPV6LEN:
        return ip
    return None


def ip_mask(ip: bytes, mask: bytes) -> Optional[bytes]:
    if len(mask) == IPV6LEN and len(ip) == IPV4LEN and all(b == 0xFF for b in mask[:12]):
        mask = mask[12:]
    if len(mask) == IPV4LEN and len(ip) == IPV6LEN and ip[:12] == V4_IN_V6_PREFIX:
        ip = ip[12:]
    if len(ip) != len(mask):
        return None
    return bytes(a & b for a, b in zip(ip, mask))


def ip_equal(a: bytes, b: bytes) -> bool:
    if len(a) == len(b):
        return a == b
    if len(a) == IPV4LEN and len(b) == IPV6LEN:
        return b[:12] == V4_IN_V6_PREFIX and a == b[12:]
    if len(a) == IPV6LEN and len(b) == IPV4LEN:
        return a[:12] == V4_IN_V6_PREFIX and a[12:] == b
    return False


def simple_mask_length(mask: bytes) -> int:
    n = 0
    for i, v in enumerate(mask):
        if v == 0xFF:
            n += 8
            continue
        while v & 0x80:
            n += 1
            v = (v << 1) & 0xFF
        if v != 0:
            return -1
        for w in mask[i + 1:]:
            if w != 0:
                return -1
        break
    return n


def mask_size(mask: bytes) -> Tuple[int, int]:
    ones, bits = simple_mask_length(mask), len(mask) * 8
    if ones == -1:
        return 0, 0
    return ones, bits


def ip_string(ip: bytes) -> str:
    """net.IP.String (Go 1.9)."""
    if len(ip) == 0:
        return "<nil>"
    p4 = to4(ip)
    if p4 is not None and len(p4) == IPV4LEN:
        return "%d.%d.%d.%d" % tuple(p4)
    if len(ip) != IPV6LEN:
        return "?" + ip.hex()
    e0, e1 = -1, -1
    i = 0
    while i < IPV6LEN:
        j = i
        while j < IPV6LEN and ip[j] == 0 and ip[j + 1] == 0:
            j += 2
        if j > i and j - i > e1 - e0:
            e0, e1 = i, j
            i = j
        i += 2
    if e1 - e0 <= 2:
        e0, e1 = -1, -1
    out = []
    i = 0
    while i < IPV6LEN:
        if i == e0:
            out.append("::")
            i = e1
            if i >= IPV6LEN:
                break
        elif i > 0:
            out.append(":")
        out.append("%x" % ((ip[i] << 8) | ip[i + 1]))
        i += 2
    return "".join(out)


class IPNet:
    """``net.IPNet``; ``IPNet()`` is the empty network (``&net.IPNet{}``)."""

    __slots__ = ("ip", "mask")

    def __init__(self, ip: bytes = b"", mask: bytes = b""):
        self.ip = bytes(ip)
        self.mask = bytes(mask)

    def __repr__(self) -> str:
        return "IPNet(%s)" % (self.string() if self.ip else "ANY")

    def _network_number_and_mask(self):
        ip = to4(self.ip)
        if ip is None:
            ip = self.ip
            if len(ip) != IPV6LEN:
                return None, None
        m = self.mask
        if len(m) == IPV4LEN:
            if len(ip) != IPV4LEN:
                return None, None
        elif len(m) == IPV6LEN:
            if len(ip) == IPV4LEN:
                m = m[12:]
        else:
            return None, None
        return ip, m

    def contains(self, ip: bytes) -> bool:
        nn, m = self._network_number_and_mask()
        if nn is None:
            return False
        x = to4(ip)
        if x is not None:
            ip = x
        if len(ip) != len(nn):
            return False
        return all((a & k) == (b & k) for a, b, k in zip(nn, ip, m))

    def string(self) -> str:
        nn, m = self._network_number_and_mask()
        if nn is None or m is None:
            return "<nil>"
        length = simple_mask_length(m)
        if length == -1:
            return ip_string(nn) + "/" + m.hex()
        return ip_string(nn) + "/" + str(length)

    __str__ = string

    def copy(self) -> "IPNet":
        return IPNet(self.ip, self.mask)


def parse_cidr(s: str) -> Tuple[Optional[bytes], Optional[IPNet]]:
    """net.ParseCIDR; returns (ip, network) or (None, None) on error."""
    i = s.find("/")
    if i < 0:
        return None, None
    addr, mask = s[:i], s[i + 1:]
    iplen = IPV4LEN
    ip = parse_ipv4(addr)
    if ip is None:
        iplen = IPV6LEN
        ip = parse_ipv6(addr)
    n, j, ok = _dtoi(mask)
    if ip is None or not ok or j != len(mask) or n < 0 or n > 8 * iplen:
        return None, None
    m = cidr_mask(n, 8 * iplen)
    return ip, IPNet(ip_mask(ip, m), m)


def ip_network(s: str) -> IPNet:
    """testdata.IpNetwork (renderer/testdata/testdata.go:257-263)."""
    if s == "":
        return IPNet()
    _, net = parse_cidr(s)
    return net


def one_host_subnet(host: str) -> Optional[IPNet]:
    """utils.GetOneHostSubnet (plugins/policy/utils/utils.go:271-283)."""
    ip = parse_ip(host)
    if ip is None:
        return None
    if to4(ip) is not None:
        return IPNet(ip, cidr_mask(32, 32))
    return IPNet(ip, cidr_mask(128, 128))
