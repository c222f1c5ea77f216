"""Random ContivRule lists and packets for the TestTraffic tests.

Networks mix IPv4, IPv6 and IPv4-mapped forms (4- and 16-byte masks), a few
with host bits set, and "dead" networks whose Contains never holds; packets
are drawn near the rules' networks so that most rules get hits.
"""
from __future__ import annotations

import random

from vpp_amd import gonet
from vpp_amd.gonet import IPNet
from vpp_amd.renderer.api import ACTION_DENY, ACTION_PERMIT, TCP, UDP, ContivRule

PORTS = [22, 53, 80, 443, 8080, 65535]


def _rand_net(rng: random.Random) -> IPNet:
    k = rng.random()
    if k < 0.25:
        return IPNet()
    if k < 0.6:                                     # IPv4, 4-byte mask
        ones = rng.choice([0, 8, 16, 20, 24, 28, 32])
        ip = bytes([10, rng.randrange(4), rng.randrange(4), rng.randrange(256)])
        return IPNet(ip, gonet.cidr_mask(ones, 32))
    if k < 0.75:                                    # IPv4-mapped, 16-byte mask
        ones = rng.choice([96, 104, 112, 120, 128, 64])
        ip = gonet.V4_IN_V6_PREFIX + bytes([10, rng.randrange(4), rng.randrange(4), rng.randrange(256)])
        return IPNet(ip, gonet.cidr_mask(ones, 128))
    if k < 0.97:                                    # IPv6
        ones = rng.choice([0, 16, 48, 64, 96, 120, 128])
        ip = bytes([0xFD, 0, 0, 0x10] + [0] * 4 + [0, 0, 0, 0, 0, 0, rng.randrange(4), rng.randrange(256)])
        return IPNet(ip, gonet.cidr_mask(ones, 128))
    # dead: IPv6 address with a 4-byte mask (networkNumberAndMask -> nil)
    return IPNet(bytes([0xFD] + [0] * 15), gonet.cidr_mask(8, 32))


def rand_rules(rng: random.Random, n: int):
    out = []
    for _ in range(n):
        out.append(ContivRule(ACTION_PERMIT if rng.random() < 0.6 else ACTION_DENY,
                              _rand_net(rng), _rand_net(rng), rng.choice([TCP, UDP]), 0,
                              rng.choice(PORTS + [0, 0])))
    return out


def _near(rng: random.Random, net: IPNet) -> bytes:
    nn, m = net._network_number_and_mask() if len(net.ip) else (None, None)
    if nn is None:
        fam4 = rng.random() < 0.5
        nn = bytes([10, rng.randrange(4), rng.randrange(4), rng.randrange(256)]) if fam4 else \
            bytes([0xFD, 0, 0, 0x10] + [0] * 10 + [rng.randrange(4), rng.randrange(256)])
        m = bytes(len(nn))
    host = bytes((a & k) | (rng.randrange(256) & ~k & 0xFF) for a, k in zip(nn, m))
    if rng.random() < 0.1:
        host = bytes(x ^ 1 for x in host)
    return host


def rand_packets(rng: random.Random, rules, n: int):
    """Returns lists of (src, dst) net.IP byte strings (4 or 16 bytes, IPv4 sometimes
    in mapped form), protocol (0..4), sport, dport."""
    src, dst, proto, sport, dport = [], [], [], [], []
    for _ in range(n):
        r = rng.choice(rules) if rules and rng.random() < 0.85 else None
        s = _near(rng, r.src_network if r else IPNet())
        d = _near(rng, r.dest_network if r else IPNet())
        if len(s) == 4 and rng.random() < 0.3:
            s = gonet.V4_IN_V6_PREFIX + s
        if len(d) == 4 and rng.random() < 0.3:
            d = gonet.V4_IN_V6_PREFIX + d
        src.append(s)
        dst.append(d)
        p = rng.random()
        proto.append((r.protocol if r else TCP) if p < 0.8 else rng.choice([0, 1, 2, 3, 4]))
        sport.append(rng.randrange(1024, 65536))
        dport.append(r.dest_port if (r and r.dest_port and rng.random() < 0.7) else rng.choice(PORTS + [1234]))
    return src, dst, proto, sport, dport
