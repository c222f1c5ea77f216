"""First match over raw ContivRule lists on the GPU.

Restates the evaluator of mock/renderer/renderer_mock.go (MockRenderer
:39-183, TestTraffic :105-145, TrafficAction :25-37) as a drop-in renderer
whose TestTraffic runs on the gfx950 classifier.  The configurator tests use
this evaluator; the build also uses it for the IngressOrientation tables that
the VPPTCP renderer exports as session rules.

TestTraffic's semantics for a packet (src, dst, proto, sport, dport), rule by
rule in list order:
  * a non-empty SrcNetwork / DestNetwork must Contain the address (Go 1.9
    IPNet.Contains);
  * Protocol must equal the packet's protocol exactly;
  * SrcPort / DestPort 0 match any port, otherwise exact equality;
  * the first matching rule gives ALLOWED (Permit) or DENIED (any other
    action); no match gives UNMATCHED.

The GPU path does not add a kernel for this: a rule list compiles into an
ACL whose evalACL semantics (aclengine_mock.go:473-668) reproduce TestTraffic
bit for bit, and the ACL goes through the same classifier image as rendered
ACLs.  The translation (``compile_rules``):

  index 0    sentinel: networks any, Tcp + Udp + Icmp sections, REFLECT.
             TCP/UDP/ICMP packets skip it (evalACL's "other section present"
             branches); a packet protocol > 2 has no case in evalACL's switch
             and matches it -> REFLECT = UNMATCHED (no ContivRule protocol
             equals it).
  1 + i      ContivRule i: the network strings are the ones ParseCIDR turns
             back into the same Contains test; TCP -> Tcp section, UDP -> Udp
             section; src range [0, 65535]; dst range [p, p] or [0, 65535];
             Permit -> PERMIT, else DENY.  A network whose Contains can never
             hold (Go's networkNumberAndMask gives nil) becomes a rule that
             no packet reaches: Tcp + Udp + Icmp sections.
  n+1..n+3   catch-all TCP, UDP and ICMP rules with action REFLECT: whatever
             reaches them is UNMATCHED.

Verdicts then read directly as TrafficAction: DENY 0 = DeniedTraffic,
PERMIT 1 = AllowedTraffic, REFLECT 2 = UnmatchedTraffic.  The hit counters of
rule i are the ACL's counters at 1 + i; the unmatched count is the sum of the
sentinel, the three catch-alls and the default slot.

Not expressible through the ACL form, rejected with ValueError at compile time
(never silently approximated):
  * SrcPort != 0 -- evalACL fails any rule whose source range is not full,
    and the packet batch carries no source port.  No reference producer sets
    it (configurator_impl.go:312-472 and testdata.go always use SrcPort 0);
  * Protocol outside renderer.ProtocolType {TCP, UDP} (api.go:161-169);
  * a non-contiguous network mask (IPNet.String gives a hex mask that
    ParseCIDR rejects, while Contains would still apply it).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from .. import gonet, model
from ..gonet import IPNet
from .api import ACTION_PERMIT, TCP, UDP, ContivRule, PodID

# TrafficDirection (renderer_mock.go:14-22): from the vswitch point of view
INGRESS_TRAFFIC = 0
EGRESS_TRAFFIC = 1

# TrafficAction (renderer_mock.go:25-37) == the ACL verdict of the translation
DENIED_TRAFFIC = 0
ALLOWED_TRAFFIC = 1
UNMATCHED_TRAFFIC = 2

FIRST_RULE = 1          # ACL index of ContivRule 0
N_TAIL = 3              # catch-all TCP, UDP, ICMP


def _full(lo: int = 0, hi: int = model.MAX_PORT) -> model.PortRange:
    return model.PortRange(lo, hi)


def _dead_rule(action: int) -> model.Rule:
    """A rule no TCP/UDP/ICMP packet reaches: every protocol section present
    (evalACL :528-642 skips it); protocols > 2 stop at the sentinel first."""
    icmp = model.Icmp(icmpv6=False, icmp_code_range=model.IcmpRange(0, model.MAX_ICMP_CODE),
                      icmp_type_range=model.IcmpRange(0, model.MAX_ICMP_TYPE))
    ipr = model.IpRule(ip=model.Ip(),
                       tcp=model.Tcp(destination_port_range=_full(), source_port_range=_full()),
                       udp=model.Udp(destination_port_range=_full(), source_port_range=_full()),
                       icmp=icmp)
    return model.Rule(actions=model.Actions(action), matches=model.Matches(ip_rule=ipr))


def network_string(net: IPNet) -> Optional[str]:
    """The CIDR string whose ParseCIDR + Contains equals ``net.Contains``,
    "" for the empty network (match all), None when Contains never holds.
    Go 1.9 IPNet.String prints networkNumberAndMask's (nn, m), which is what
    Contains compares against; only a non-contiguous mask cannot round-trip."""
    if len(net.ip) == 0:
        return ""
    nn, m = net._network_number_and_mask()
    if nn is None:
        return None
    if gonet.simple_mask_length(m) == -1:
        raise ValueError("non-contiguous network mask %s: not expressible as a CIDR" % m.hex())
    return net.string()


def compile_rules(rules: List[ContivRule]) -> List[model.Rule]:
    """ContivRule list -> ACL rules with TestTraffic semantics (module doc)."""
    out = [_dead_rule(model.REFLECT)]
    out[0].matches.ip_rule.ip = model.Ip()                   # sentinel: networks any
    for i, r in enumerate(rules):
        if r.src_port != 0:
            raise ValueError("rule %d: SrcPort %d is not supported by the compiled path" % (i, r.src_port))
        if r.protocol not in (TCP, UDP):
            raise ValueError("rule %d: protocol %r outside renderer.ProtocolType" % (i, r.protocol))
        action = model.PERMIT if r.action == ACTION_PERMIT else model.DENY
        src, dst = network_string(r.src_network), network_string(r.dest_network)
        if src is None or dst is None:
            out.append(_dead_rule(action))
            continue
        drange = _full(r.dest_port, r.dest_port) if r.dest_port else _full()
        sec = dict(destination_port_range=drange, source_port_range=_full())
        ipr = model.IpRule(ip=model.Ip(destination_network=dst, source_network=src))
        if r.protocol == TCP:
            ipr.tcp = model.Tcp(**sec)
        else:
            ipr.udp = model.Udp(**sec)
        out.append(model.Rule(actions=model.Actions(action), matches=model.Matches(ip_rule=ipr)))
    out.append(model.l4_rule(model.REFLECT, "", "", "tcp", 0, model.MAX_PORT, 0, model.MAX_PORT))
    out.append(model.l4_rule(model.REFLECT, "", "", "udp", 0, model.MAX_PORT, 0, model.MAX_PORT))
    out.append(model.icmp_rule(model.REFLECT))
    return out


def rule_counters(acl_counters, n_rules: int):
    """ACL hit counters (len n_rules + 5) -> (per-ContivRule counters, unmatched)."""
    c = acl_counters
    per_rule = c[FIRST_RULE:FIRST_RULE + n_rules]
    unmatched = int(c[0]) + int(sum(int(x) for x in c[FIRST_RULE + n_rules:]))
    return per_rule, unmatched


class RuleTable:
    """One ContivRule list compiled onto the engine."""

    def __init__(self, engine, name: str, rules: List[ContivRule]):
        self.rules = list(rules)
        self.engine = engine
        self.table = engine.put_table(name, compile_rules(self.rules))

    def test_traffic_batch(self, src, dst, proto, dport, verdict=None, counters=None, stream=None):
        """TestTraffic over a packet batch (the classify SoA: IPv4 uint32 host
        order or uint8[n,16]; proto = renderer.ProtocolType values).  numpy in:
        returns (TrafficAction uint8[n], per-rule counters, unmatched).  Device
        tensors: verdict / counters (int64[len(rules) + 5]) are written on the
        stream and returned as given."""
        v, c = self.engine.classify(self.table, src, dst, dport, proto, verdict=verdict,
                                    counters=counters, stream=stream)
        if isinstance(v, np.ndarray):
            per_rule, unmatched = rule_counters(c, len(self.rules))
            return v, per_rule, unmatched
        return v, c

    def close(self):
        if self.table is not None:
            self.engine.del_table(self.table)
            self.table = None


class _PodConfig:
    __slots__ = ("ip", "ingress", "egress")

    def __init__(self, ip, ingress, egress):
        self.ip, self.ingress, self.egress = ip, list(ingress), list(egress)


class TrafficRenderer:
    """MockRenderer (renderer_mock.go:39-183) with TestTraffic on the GPU.
    Render stores a pod's rule lists; Commit compiles them onto the engine;
    TestTraffic evaluates one packet, TestTrafficBatch a batch."""

    def __init__(self, name: str, engine):
        self.name = name
        self.engine = engine
        self.config: Dict[PodID, _PodConfig] = {}
        self.tables: Dict[tuple, RuleTable] = {}

    def new_txn(self, resync: bool) -> "TrafficRendererTxn":
        return TrafficRendererTxn(self, resync)

    def get_pod_ip(self, pod: PodID):
        """GetPodIP (:84-100)."""
        cfg = self.config.get(pod)
        if cfg is None or cfg.ip is None:
            return "", 0
        ones, _ = gonet.mask_size(cfg.ip.mask)
        return gonet.ip_string(cfg.ip.ip), ones

    def _table(self, pod: PodID, direction: int) -> Optional[RuleTable]:
        return self.tables.get((pod, direction))

    def test_traffic(self, pod: PodID, direction: int, src_ip: bytes, dst_ip: bytes, protocol: int,
                     src_port: int, dst_port: int) -> int:
        """TestTraffic (:105-145) for one packet.  ``src_port`` is accepted for
        the reference's signature; compiled tables carry no SrcPort (module doc)."""
        t = self._table(pod, direction)
        if t is None:
            return UNMATCHED_TRAFFIC
        if not t.rules:
            return UNMATCHED_TRAFFIC
        s, d = _addr16(src_ip), _addr16(dst_ip)
        v, _, _ = t.test_traffic_batch(s[None, :], d[None, :], np.array([protocol], np.uint8),
                                       np.array([dst_port], np.uint16))
        return int(v[0])

    def test_traffic_batch(self, pod: PodID, direction: int, src, dst, proto, dport, **kw):
        t = self._table(pod, direction)
        if t is None:
            raise KeyError("pod %s has no %s rules committed" % (pod, "ingress" if direction == 0 else "egress"))
        return t.test_traffic_batch(src, dst, proto, dport, **kw)

    def close(self):
        for t in self.tables.values():
            t.close()
        self.tables.clear()


class TrafficRendererTxn:
    """MockRendererTxn (renderer_mock.go:49-55, Render :148-163, Commit :166-183)."""

    def __init__(self, renderer: TrafficRenderer, resync: bool):
        self.renderer = renderer
        self.resync = resync
        self.config: Dict[PodID, _PodConfig] = {}

    def render(self, pod: PodID, pod_ip: IPNet, ingress, egress, removed: bool) -> "TrafficRendererTxn":
        """Render (:148-165): a removed pod only leaves *this txn's* config;
        the renderer forgets it on a resync commit alone, as in the reference."""
        if removed:
            self.config.pop(pod, None)
        else:
            self.config[pod] = _PodConfig(pod_ip, ingress, egress)
        return self

    def commit(self) -> None:
        r = self.renderer
        if self.resync:
            for key in list(r.tables):
                r.tables.pop(key).close()
            r.config = {}
        for pod, cfg in self.config.items():
            for d in (INGRESS_TRAFFIC, EGRESS_TRAFFIC):
                old = r.tables.pop((pod, d), None)
                if old is not None:
                    old.close()
            r.config[pod] = cfg
            for d, rules in ((INGRESS_TRAFFIC, cfg.ingress), (EGRESS_TRAFFIC, cfg.egress)):
                r.tables[(pod, d)] = RuleTable(r.engine, "%s/%s/%d" % (r.name, pod, d), rules)


def _addr16(ip) -> np.ndarray:
    """Go net.IP (4 or 16 bytes) -> the 16-byte SoA row (IPv4 as IPv4-mapped,
    which the classifier treats as IPv4 exactly as Go's To4 does)."""
    b = bytes(ip)
    if len(b) == 4:
        b = gonet.V4_IN_V6_PREFIX + b
    if len(b) != 16:
        raise ValueError("IP of %d bytes" % len(b))
    return np.frombuffer(b, np.uint8).copy()
