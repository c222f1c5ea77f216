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
Traffic pools (pod IPs, rule destination prefixes, rule ports) feed the
splitmix64 generator (DESIGN.md "Traffic").
"""
from __future__ import annotations

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
}


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


def render_global(n_pods: int, rules_per_pod: int, n_apps: int, seed: int):
    """Returns (acl: vpp_amd.model.Acl, traffic pools dict)."""
    rng = random.Random(seed)
    cidrs = service_cidrs(rng)
    apps = [app_rules(rng, cidrs, rules_per_pod) for _ in range(n_apps)]
    pods = []
    for k in range(n_pods):
        ip = gonet.one_host_subnet(_v4(pod_ip(k)))
        pods.append((ip, apps[k % n_apps]))
    table = build_global_table(pods)
    acl = render_acl(table, None)
    dst = sorted({(int.from_bytes(r.dest_network.ip[-4:], "big"), gonet.mask_size(r.dest_network.mask)[0])
                  for r in table.rules if len(r.dest_network.ip)})
    ports = sorted({r.dest_port for r in table.rules if r.dest_port})
    pools = dict(pod_ips=np.array([pod_ip(k) for k in range(n_pods)], np.uint32),
                 dst_addrs=np.array([a for a, _ in dst], np.uint32),
                 dst_lens=np.array([ln for _, ln in dst], np.uint8),
                 ports=np.array(ports, np.uint16))
    return acl, pools


def config(cfg: int):
    """(acl, traffic spec dict, default packet count) of BASELINE config 2 or 3."""
    c = CONFIGS[cfg]
    acl, pools = render_global(c["n_pods"], c["rules_per_pod"], c["n_apps"], seed=cfg)
    spec = dict(seed=SEEDS[cfg], pct_pod_src=60, pct_rule_dst=50, pct_table_port=50, pct_icmp=0,
                **pools)
    return acl, spec, c["packets"]
