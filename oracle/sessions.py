"""CPU restatement of session-rule packet evaluation -- TEST INFRASTRUCTURE.

Only tests/ may import this module; the product path (vpp_amd/renderer/
sessions.py) compiles installed session rules onto the GPU classifier and
never calls into oracle/.

The reference holds no evaluator for VPP session rules (the session-rule
mock stores rules and answers HasRule, mock/sessionrules/sessionrules_mock.go;
VPP's lookup is external), so this oracle restates the build's definition
(vpp_amd/renderer/sessions.py module doc) literally, per packet, over the
installed SessionRule fields: parity unpinned.

  * order: the ContivRule Compare order (renderer/api.go:114-136) of the rule
    each session rule describes -- protocol, source network, destination
    network (utils.go:187-239 CompareIPNets: IPv4 first, covering prefixes
    after the prefixes they cover, disjoint ones by mask then address),
    source port, destination port (utils.go:243-257: 0 = any last), action
    (deny first); equal ones keep the first installed;
  * match: transport protocol equal (TCP 0, UDP 1; other packet protocols
    never match), the rule's family (IsIP4) equal to the packet's (IPv4 or
    IPv4-mapped = IPv4, Go's To4), prefixes containing the addresses --
    global scope: lcl = destination, rmt = source; local scope: lcl =
    source, rmt = destination -- and ports 0 or equal (local port of a
    global rule = destination port, remote port of a local rule =
    destination port, the other one any);
  * the first matching rule's action (ALLOW 1, DENY 0); none: ALLOW.
"""
from __future__ import annotations

import functools

SCOPE_GLOBAL = 1
ACTION_ALLOW_IDX = 0xFFFFFFFF - 2
ALLOW, DENY = 1, 0


def _addr16(a) -> bytes:
    """A packet address as 16 bytes (IPv4 host-order int -> v4-mapped)."""
    if isinstance(a, (int,)) or hasattr(a, "dtype") and getattr(a, "ndim", 0) == 0:
        return bytes(10) + b"\xff\xff" + int(a).to_bytes(4, "big")
    return bytes(bytearray(a))


def _is4(a16: bytes) -> bool:
    return a16[:12] == bytes(10) + b"\xff\xff"


def _contains(ip: bytes, plen: int, a16: bytes, is_ip4: int) -> bool:
    a = a16[12:] if is_ip4 else a16
    bits = 8 * len(a)
    plen = min(plen, bits)
    x = int.from_bytes(a, "big") >> (bits - plen) if plen else 0
    y = int.from_bytes(ip[:len(a)], "big") >> (bits - plen) if plen else 0
    return x == y


def _sides(r):
    """(src ip, src plen, dst ip, dst plen, src port, dst port) of the rule
    in the packet's frame."""
    if r.scope == SCOPE_GLOBAL:
        return r.rmt_ip, r.rmt_plen, r.lcl_ip, r.lcl_plen, r.rmt_port, r.lcl_port
    return r.lcl_ip, r.lcl_plen, r.rmt_ip, r.rmt_plen, r.lcl_port, r.rmt_port


def _cmp(a, b):
    return (a > b) - (a < b)


def _cmp_net(fa, ia, pa, fb, ib, pb):
    """CompareIPNets (utils.go:187-239) on family-bound prefixes."""
    if fa != fb:
        return -1 if fa else 1                    # IPv4 first
    n = 4 if fa else 16
    bits = 8 * n
    pa, pb = min(pa, bits), min(pb, bits)
    xa, xb = int.from_bytes(ia[:n], "big"), int.from_bytes(ib[:n], "big")
    common = min(pa, pb)
    cm = ((1 << common) - 1) << (bits - common) if common else 0
    if xa & cm == xb & cm:
        return _cmp(pb, pa)                       # more specific first
    ma = ((1 << pa) - 1) << (bits - pa) if pa else 0
    mb = ((1 << pb) - 1) << (bits - pb) if pb else 0
    o = _cmp(mb, ma)                              # masks, bytes compared: longer mask first
    return o if o else _cmp(xa, xb)


def _cmp_port(a, b):
    if a == b:
        return 0
    if a == 0:
        return 1
    if b == 0:
        return -1
    return -1 if a < b else 1


def _cmp_rule(a, b):
    o = _cmp(a.transport_proto, b.transport_proto)
    if o:
        return o
    sa, sb = _sides(a), _sides(b)
    o = _cmp_net(a.is_ip4, sa[0], sa[1], b.is_ip4, sb[0], sb[1])
    if o:
        return o
    o = _cmp_net(a.is_ip4, sa[2], sa[3], b.is_ip4, sb[2], sb[3])
    if o:
        return o
    o = _cmp_port(sa[4], sb[4])
    if o:
        return o
    o = _cmp_port(sa[5], sb[5])
    if o:
        return o
    act = lambda r: 1 if r.action_index == ACTION_ALLOW_IDX else 0
    return _cmp(act(a), act(b))


def order(rules):
    """Indices of the rules in first-match order; equal rules: the first installed."""
    idx = sorted(range(len(rules)), key=functools.cmp_to_key(lambda i, j: _cmp_rule(rules[i], rules[j]) or (i - j)))
    out = []
    for i in idx:
        if out and _cmp_rule(rules[out[-1]], rules[i]) == 0:
            continue
        out.append(i)
    return out


def evaluate(rules, src, dst, proto, dport):
    """Per packet: (verdicts ALLOW/DENY, hits per rule, unmatched count).
    src/dst: IPv4 host-order ints or 16-byte addresses; proto ProtocolType."""
    seq = order(rules)
    hits = [0] * len(rules)
    verdict = []
    unmatched = 0
    for s, d, p, dp in zip(src, dst, proto, dport):
        s16, d16 = _addr16(s), _addr16(d)
        v = None
        if int(p) in (0, 1) and _is4(s16) == _is4(d16):
            for i in seq:
                r = rules[i]
                si, sl, di, dl, sport_r, dport_r = _sides(r)
                if r.transport_proto != int(p) or bool(r.is_ip4) != _is4(s16):
                    continue
                if not (_contains(si, sl, s16, r.is_ip4) and _contains(di, dl, d16, r.is_ip4)):
                    continue
                if sport_r != 0 or (dport_r != 0 and dport_r != int(dp)):
                    continue                          # source port: the batch carries none -- any only
                v = ALLOW if r.action_index == ACTION_ALLOW_IDX else DENY
                hits[i] += 1
                break
        if v is None:
            v = ALLOW
            unmatched += 1
        verdict.append(v)
    return verdict, hits, unmatched
