"""Renderer API: ContivRule, its total order, and the PolicyRendererAPI shape.

Restates plugins/policy/renderer/api.go (ContivRule :65-77, Compare
:114-136, ActionType :139-147, ProtocolType :161-169) and the comparators of
plugins/policy/utils/utils.go:175-257 that define the first-match order of a
ContivRuleTable.
"""
from __future__ import annotations

from typing import NamedTuple

from .. import gonet
from ..gonet import IPNet

# ActionType (api.go:139-147)
ACTION_DENY = 0
ACTION_PERMIT = 1

# ProtocolType (api.go:161-169)
TCP = 0
UDP = 1

ANY_PORT = 0


class PodID(NamedTuple):
    """podmodel.ID"""
    name: str
    namespace: str

    def __str__(self) -> str:
        return "%s/%s" % (self.namespace, self.name)


class ContivRule:
    """n-tuple with the most basic policy rule definition (api.go:65-77)."""

    __slots__ = ("action", "src_network", "dest_network", "protocol", "src_port", "dest_port")

    def __init__(self, action: int = ACTION_DENY, src_network: IPNet = None,
                 dest_network: IPNet = None, protocol: int = TCP, src_port: int = 0,
                 dest_port: int = 0):
        self.action = action
        self.src_network = src_network if src_network is not None else IPNet()
        self.dest_network = dest_network if dest_network is not None else IPNet()
        self.protocol = protocol
        self.src_port = src_port & 0xFFFF
        self.dest_port = dest_port & 0xFFFF

    def copy(self) -> "ContivRule":
        """Copy (api.go:104-108): shallow; networks are shared pointers in Go."""
        r = ContivRule.__new__(ContivRule)
        r.action = self.action
        r.src_network = self.src_network
        r.dest_network = self.dest_network
        r.protocol = self.protocol
        r.src_port = self.src_port
        r.dest_port = self.dest_port
        return r

    def compare(self, other: "ContivRule") -> int:
        """Compare (api.go:114-136)."""
        o = compare_ints(self.protocol, other.protocol)
        if o:
            return o
        o = compare_ipnets(self.src_network, other.src_network)
        if o:
            return o
        o = compare_ipnets(self.dest_network, other.dest_network)
        if o:
            return o
        o = compare_ports(self.src_port, other.src_port)
        if o:
            return o
        o = compare_ports(self.dest_port, other.dest_port)
        if o:
            return o
        return compare_ints(self.action, other.action)

    def __repr__(self) -> str:
        net = lambda n: n.string() if len(n.ip) else "ANY"
        port = lambda p: str(p) if p else "ANY"
        proto = {TCP: "TCP", UDP: "UDP"}.get(self.protocol, "INVALID")
        act = {ACTION_DENY: "DENY", ACTION_PERMIT: "PERMIT"}.get(self.action, "INVALID")
        return "Rule <%s %s[%s:%s] -> %s[%s:%s]>" % (
            act, net(self.src_network), proto, port(self.src_port),
            net(self.dest_network), proto, port(self.dest_port))


def compare_ints(a: int, b: int) -> int:
    """utils.CompareInts (utils.go:175-183)."""
    return -1 if a < b else (1 if a > b else 0)


def _bytes_compare(a: bytes, b: bytes) -> int:
    return -1 if a < b else (1 if a > b else 0)


def compare_ipnets(a: IPNet, b: IPNet) -> int:
    """utils.CompareIPNets (utils.go:187-239)."""
    if len(a.ip) == 0:
        return 0 if len(b.ip) == 0 else 1
    if len(b.ip) == 0:
        return -1
    a4 = gonet.to4(a.ip)
    b4 = gonet.to4(b.ip)
    if a4 is not None:
        if b4 is None:
            return -1
        a_ip, a_mask = a4, a.mask
    else:
        a_ip, a_mask = gonet.to16(a.ip), a.mask
    if b4 is not None:
        if a4 is None:
            return 1
        b_ip, b_mask = b4, b.mask
    else:
        b_ip, b_mask = gonet.to16(b.ip), b.mask
    a_ones, bits = gonet.mask_size(a_mask)
    b_ones, _ = gonet.mask_size(b_mask)
    common = min(a_ones, b_ones)
    cm = gonet.cidr_mask(common, bits)
    am = gonet.ip_mask(a_ip, cm)
    bm = gonet.ip_mask(b_ip, cm)
    if gonet.ip_equal(am or b"", bm or b""):
        return compare_ints(b_ones, a_ones)
    o = _bytes_compare(b_mask, a_mask)
    if o:
        return o
    return _bytes_compare(a_ip, b_ip)


def compare_ports(a: int, b: int) -> int:
    """utils.ComparePorts (utils.go:243-257): 0 = any port sorts last."""
    if a == b:
        return 0
    if a == 0:
        return 1
    if b == 0:
        return -1
    return -1 if a < b else 1


def net_key(n: IPNet):
    """A sort key of ``n`` consistent with compare_ipnets (equal keys <=>
    compare_ipnets == 0), or None where the key form does not apply (a
    non-canonical mask, a mask whose width differs from the address's):
    IPv4 before IPv6, longer prefix first, then the masked address; the
    empty network last.  For disjoint prefixes of one length the masked and
    the unmasked address order agree (they differ inside the prefix)."""
    if n is None:
        return None
    ck = (n.ip, n.mask)
    k = _NET_KEYS.get(ck, _MISSING)
    if k is _MISSING:
        if len(_NET_KEYS) > 1 << 20:
            _NET_KEYS.clear()
        k = _NET_KEYS[ck] = _net_key(n)
    return k


_NET_KEYS = {}
_MISSING = object()


def _net_key(n: IPNet):
    if len(n.ip) == 0:
        return (2, 0, 0)
    a4 = gonet.to4(n.ip)
    if a4 is not None:
        if len(n.mask) != 4:
            return None
        ip = a4
        fam = 0
    else:
        if len(n.ip) != 16 or len(n.mask) != 16:
            return None
        ip = n.ip
        fam = 1
    ones, bits = gonet.mask_size(n.mask)
    if bits == 0:
        return None
    x = int.from_bytes(ip, "big") & int.from_bytes(n.mask, "big")
    return (fam, -ones, x)


def rule_key(r: ContivRule):
    """Sort key of a rule consistent with ContivRule.compare, or None."""
    s, d = net_key(r.src_network), net_key(r.dest_network)
    if s is None or d is None:
        return None
    return (r.protocol, s, d, r.src_port or 0x10000, r.dest_port or 0x10000, r.action)


def compare_rule_lists(a, b) -> int:
    """compareRuleLists (renderer/cache/local_tables.go:242-263)."""
    if a is None and b is None:
        return 0
    if a is None:
        return -1
    if b is None:
        return 1
    o = compare_ints(len(a), len(b))
    if o:
        return o
    for x, y in zip(a, b):
        o = x.compare(y)
        if o:
            return o
    return 0


# Test-set helpers (renderer/testdata/testdata.go:265-311)
def allow_all_tcp() -> ContivRule:
    return ContivRule(ACTION_PERMIT, IPNet(), IPNet(), TCP, 0, 0)


def allow_all_udp() -> ContivRule:
    return ContivRule(ACTION_PERMIT, IPNet(), IPNet(), UDP, 0, 0)


def deny_all_tcp() -> ContivRule:
    return ContivRule(ACTION_DENY, IPNet(), IPNet(), TCP, 0, 0)


def deny_all_udp() -> ContivRule:
    return ContivRule(ACTION_DENY, IPNet(), IPNet(), UDP, 0, 0)
