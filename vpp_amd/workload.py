"""Synthetic policy renders for the benchmark configurations (BASELINE.json configs 2-4).

A node with ``n_pods`` pods (IPs 10.{1..4}.x.y) grouped into ``n_apps``
applications (K8s NetworkPolicies select pods by label, so every replica of
an app carries the same ContivRules).  Each app gets ``rules_per_pod`` ingress
ContivRules: TCP/UDP permits towards destination networks drawn from a pool
of service CIDRs (/16-/24) and ports from common service ports, closed by
DenyAllTCP + DenyAllUDP (renderer/testdata/testdata.go:289-311 shape).
The global table is built exactly as the renderer cache builds it
(installGlobalRules with src = pod /32, allow-all TCP/UDP appended,
cache_impl.go:638-673) and rendered by renderACL (acl_renderer.go:312-402),
so R = #distinct (pod, rule) + 2 allow-all + 1 ICMP.

Config 2: 100 pods x 10 rules (~1k).  Config 3: 1000 pods x 10 rules (~10k).
Config 5: the config 3 shape with mixed address families --
every other app (so half the pods) IPv6, pods at fd00:10::/64 hosts,
IPv6 apps' destination networks from fd00:20::/32 (/48-/64) -- destination
port ranges in the ACL form (some named ports widened to [p, p+w], the same
for every rule naming p), 10% ICMP, packets in the 16-byte layout.
Traffic pools (pod IPs, rule destination prefixes, rule ports) feed the
splitmix64 generator (DESIGN.md "Traffic").
"""
from __future__ import annotations

import copy
import random

import numpy as np

from . import gonet
from .renderer import api
from .renderer.acl import render_acl
from .renderer.cache import build_global_table

TCP_PORTS = [22, 80, 443, 3306, 5432, 6379, 8080, 8443, 9090, 9200]
UDP_PORTS = [53, 67, 123, 161, 514, 1812, 4789, 5353]
SEEDS = {2: 0xC0175EED02, 3: 0xC0175EED03, 4: 0xC0175EED04, 5: 0xC0175EED05}
CONFIGS = {
    2: dict(n_pods=100, rules_per_pod=10, n_apps=10, packets=16 << 20),
    3: dict(n_pods=1000, rules_per_pod=10, n_apps=100, packets=256 << 20),
    # config 4: the config 3 table, one 2 Gi-packet batch sharded over the GPUs
    4: dict(n_pods=1000, rules_per_pod=10, n_apps=100, packets=2 << 30, table=3),
    5: dict(n_pods=1000, rules_per_pod=10, n_apps=100, packets=256 << 20, mixed=True),
}
V6_PODS = 0xFD000010 << 96          # fd00:10::/64
V6_SVC = 0xFD000020 << 96           # fd00:20::/32


def pod_ip(k: int) -> int:
    b = 1 + (k % 4)
    j = k // 4
    return (10 << 24) | (b << 16) | ((j // 254) << 8) | (j % 254 + 1)


def _v4(a: int) -> str:
    return "%d.%d.%d.%d" % ((a >> 24) & 255, (a >> 16) & 255, (a >> 8) & 255, a & 255)


def service_cidrs(rng: random.Random, n: int = 256):
    out = []
    for _ in range(n):
        ln = rng.choice([16, 20, 22, 24, 24, 24])
        base = rng.choice([0xAC100000, 0xC0A80000, 0x64400000, 0x0A000000 | (rng.randrange(16, 256) << 16)])
        a = (base | rng.getrandbits(16)) & ((0xFFFFFFFF << (32 - ln)) & 0xFFFFFFFF)
        out.append("%s/%d" % (_v4(a), ln))
    return out


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def pod_ip6(k: int) -> int:
    """Pod k's IPv6 address: a host of fd00:10::/64."""
    return V6_PODS | _mix64(k)


def _v6(a: int) -> str:
    import ipaddress
    return str(ipaddress.IPv6Address(a))


def service_cidrs6(rng: random.Random, n: int = 256):
    out = []
    for _ in range(n):
        ln = rng.choice([48, 56, 60, 64, 64, 64])
        a = (V6_SVC | (rng.getrandbits(32) << 64)) & ~((1 << (128 - ln)) - 1)
        out.append("%s/%d" % (_v6(a), ln))
    return out


def port_range_of(p: int) -> tuple:
    """Config 5: the dst port range a named port stands for in the ACL form."""
    h = _mix64(p * 0x10001)
    w = (0, 0, 0, 1, 7, 63, 1023)[h % 7]
    return p, min(65535, p + w)


def app_rules(rng: random.Random, cidrs, rules_per_pod: int):
    rules = []
    for _ in range(max(0, rules_per_pod - 2)):
        tcp = rng.random() < 0.6
        port = rng.choice(TCP_PORTS if tcp else UDP_PORTS) if rng.random() < 0.9 else 0
        dst = gonet.ip_network(rng.choice(cidrs)) if rng.random() < 0.85 else gonet.IPNet()
        rules.append(api.ContivRule(api.ACTION_PERMIT, gonet.IPNet(), dst,
                                    api.TCP if tcp else api.UDP, 0, port))
    rules.append(api.deny_all_tcp())
    rules.append(api.deny_all_udp())
    return rules


def render_global(n_pods: int, rules_per_pod: int, n_apps: int, seed: int, mixed: bool = False):
    """Returns (acl: vpp_amd.model.Acl, traffic pools dict).  mixed: config 5
    (odd apps IPv6, port ranges; pools as 16-byte addresses)."""
    rng = random.Random(seed)
    cidrs = service_cidrs(rng)
    cidrs6 = service_cidrs6(rng) if mixed else None
    apps = [app_rules(rng, cidrs6 if mixed and a % 2 else cidrs, rules_per_pod) for a in range(n_apps)]
    pods = []
    for k in range(n_pods):
        v6 = mixed and (k % n_apps) % 2 == 1
        ip = gonet.one_host_subnet(_v6(pod_ip6(k)) if v6 else _v4(pod_ip(k)))
        pods.append((ip, apps[k % n_apps]))
    table = build_global_table(pods)
    acl = render_acl(table, None)
    if mixed:
        return acl, _widen_and_pools(acl, table, pods)
    dst = sorted({(int.from_bytes(r.dest_network.ip[-4:], "big"), gonet.mask_size(r.dest_network.mask)[0])
                  for r in table.rules if len(r.dest_network.ip)})
    ports = sorted({r.dest_port for r in table.rules if r.dest_port})
    pools = dict(pod_ips=np.array([pod_ip(k) for k in range(n_pods)], np.uint32),
                 dst_addrs=np.array([a for a, _ in dst], np.uint32),
                 dst_lens=np.array([ln for _, ln in dst], np.uint8),
                 ports=np.array(ports, np.uint16))
    return acl, pools


def _widen_and_pools(acl, table, pods):
    """Config 5: dst port ranges in the ACL form, and the 16-byte pools."""
    # rendered rules are shared read-only messages: widen editable copies
    for i, r in enumerate(acl.rules):
        ipr = r.matches.ip_rule if r.matches is not None else None
        for sec in (ipr.tcp, ipr.udp) if ipr is not None else ():
            if sec is not None and sec.destination_port_range is not None:
                pr = sec.destination_port_range
                if pr.lower_port == pr.upper_port and pr.lower_port != 0:
                    r = acl.rules[i] = copy.deepcopy(r)
                    ipr = r.matches.ip_rule
                    pr = (ipr.tcp or ipr.udp).destination_port_range
                    pr.lower_port, pr.upper_port = port_range_of(pr.lower_port)
                    break

    def b16(net) -> bytes:
        ip = bytes(net.ip)
        return ip if len(ip) == 16 else bytes(10) + b"\xff\xff" + ip

    dst = sorted({(b16(r.dest_network), gonet.mask_size(r.dest_network.mask)[0] +
                   (96 if len(r.dest_network.ip) == 4 else 0))
                  for r in table.rules if len(r.dest_network.ip)})
    ports = sorted({r.dest_port for r in table.rules if r.dest_port})
    return dict(pod_ips=np.frombuffer(b"".join(b16(ip) for ip, _ in pods), np.uint8).reshape(-1, 16).copy(),
                dst_addrs=np.frombuffer(b"".join(a for a, _ in dst), np.uint8).reshape(-1, 16).copy(),
                dst_lens=np.array([ln for _, ln in dst], np.uint8),
                ports=np.array(ports, np.uint16))


def config(cfg: int):
    """(acl, traffic spec dict, default packet count) of BASELINE config 2, 3,
    4 or 5 (config 4: the config 3 table, its own stream seed and the whole
    2 Gi-packet batch -- bench.py shards it; config 5: 16-byte pools,
    spec["layout"] == 16)."""
    c = CONFIGS[cfg]
    mixed = c.get("mixed", False)
    acl, pools = render_global(c["n_pods"], c["rules_per_pod"], c["n_apps"], seed=c.get("table", cfg),
                               mixed=mixed)
    spec = dict(seed=SEEDS[cfg], pct_pod_src=60, pct_rule_dst=50, pct_table_port=50,
                pct_icmp=10 if mixed else 0, layout=16 if mixed else 4, **pools)
    return acl, spec, c["packets"]
