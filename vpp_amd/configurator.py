"""Policy configurator: ContivPolicy sets -> ordered ContivRule lists.

Restates plugins/policy/configurator/ (configurator_api.go types :41-275,
configurator_impl.go Commit :129-239, generateRules :248-479, appendRule(s)
:482-498, ContivPolicies order/equality :507-541, subtractSubnet :563-595).
This is the producer of the rule lists that the renderers compile onto the
classifier; it is host-side list construction (at most a few rules per peer
and port), so it stays in Python next to the renderer restatements.

Renderers are anything with ``new_txn(resync)`` returning a txn with
``render(pod, pod_ip, ingress, egress, removed)`` and ``commit()`` --
``vpp_amd.renderer.traffic.TrafficRenderer`` (GPU TestTraffic), the ACL and
VPPTCP renderers.  Rules are generated from the *vswitch* point of view:
the policy's ingress becomes the pod's egress rule list and vice versa
(configurator_impl.go:183-186).
"""
from __future__ import annotations

from typing import Dict, List, NamedTuple, Optional, Sequence

from . import gonet
from .gonet import IPNet
from .renderer.api import ACTION_DENY, ACTION_PERMIT, TCP as R_TCP, UDP as R_UDP, ContivRule, PodID

# PolicyType (configurator_api.go:166-175)
POLICY_INGRESS = 0
POLICY_EGRESS = 1
POLICY_ALL = 2

# MatchType (configurator_api.go:195-201)
MATCH_INGRESS = 0
MATCH_EGRESS = 1

# ProtocolType of a policy port (configurator_api.go:217-223)
TCP = 0
UDP = 1


class PolicyID(NamedTuple):
    """policymodel.ID"""
    name: str
    namespace: str


class Port(NamedTuple):
    """Port (configurator_api.go:240-244); Number 0 = any port."""
    protocol: int
    number: int


class IPBlock:
    """IPBlock (configurator_api.go:258-264): Network minus the Except subnets."""

    __slots__ = ("network", "excepts")

    def __init__(self, network: IPNet, excepts: Sequence[IPNet] = ()):
        self.network = network
        self.excepts = list(excepts)


class Match:
    """Match (configurator_api.go:104-116).  ``pods`` / ``ip_blocks`` None is Go's
    nil (= match anything on L3 when both are nil); an empty list is not nil."""

    __slots__ = ("type", "pods", "ip_blocks", "ports")

    def __init__(self, type: int, pods: Optional[List[PodID]] = None,
                 ip_blocks: Optional[List[IPBlock]] = None, ports: Optional[List[Port]] = None):
        self.type = type
        self.pods = pods
        self.ip_blocks = ip_blocks
        self.ports = ports


class ContivPolicy:
    """ContivPolicy (configurator_api.go:78-88)."""

    __slots__ = ("id", "type", "matches")

    def __init__(self, id: PolicyID, type: int, matches: Sequence[Match] = ()):
        self.id = id
        self.type = type
        self.matches = list(matches)


def _policy_key(p: ContivPolicy):
    """ContivPolicies.Less (configurator_impl.go:531-541): namespace, then name."""
    return (p.id.namespace, p.id.name)


def _policies_equal(a: List[ContivPolicy], b: List[ContivPolicy]) -> bool:
    """ContivPolicies.Equals (configurator_impl.go:508-518): same IDs in order."""
    return len(a) == len(b) and all(x.id == y.id for x, y in zip(a, b))


def subtract_subnet(net1: IPNet, net2: IPNet) -> List[IPNet]:
    """subtractSubnet (configurator_impl.go:563-595): the subnets covering
    every address of net1 that is not in net2."""
    ones1, _ = gonet.mask_size(net1.mask)
    ones2, _ = gonet.mask_size(net2.mask)
    if ones1 > ones2:                                   # net2 above net1 in the tree
        return [] if net2.contains(net1.ip) else [net1]
    if ones1 == ones2:                                  # same level
        return [] if gonet.ip_equal(net1.ip, net2.ip) else [net1]
    if not net1.contains(net2.ip):                      # net2 below net1, elsewhere
        return [net1]
    out = []
    bits = len(net2.mask) * 8
    for bit in range(ones1, ones2):                     # net2 under net1: :583-590
        mask = gonet.cidr_mask(bit + 1, bits)
        ip = bytearray(gonet.ip_mask(net2.ip, mask))
        ip[bit // 8] ^= 1 << (7 - bit % 8)              # flip the last bit of the prefix
        out.append(IPNet(bytes(ip), mask))
    return out


def _net_key(net: IPNet):
    """A key with key(a) == key(b) iff CompareIPNets(a, b) == 0, for the
    networks where that is easy to state (empty, or a contiguous mask of the
    address family's width); None otherwise."""
    if len(net.ip) == 0:
        return ()
    ip4 = gonet.to4(net.ip)
    if ip4 is not None and len(net.mask) == 4:
        ip, bits = ip4, 32
    elif ip4 is None and len(net.ip) == 16 and len(net.mask) == 16:
        ip, bits = net.ip, 128
    else:
        return None
    ones = gonet.simple_mask_length(net.mask)
    if ones < 0:
        return None
    return (bits, ones, gonet.ip_mask(ip, gonet.cidr_mask(ones, bits)))


def _rule_key(r: ContivRule):
    s, d = _net_key(r.src_network), _net_key(r.dest_network)
    if s is None or d is None:
        return None
    return (r.protocol, s, d, r.src_port, r.dest_port, r.action)


class _RuleList(list):
    """A rule list with appendRule's duplicate test (Compare == 0) answered
    from a key set -- O(1) per append instead of a scan of the list -- while
    every rule has a key; any keyless rule switches back to the scan."""

    def __init__(self):
        super().__init__()
        self.keys = set()
        self.keyless = False

    def append_unique(self, n: ContivRule) -> None:
        k = None if self.keyless else _rule_key(n)
        if k is None:
            self.keyless = True
            if any(r.compare(n) == 0 for r in self):
                return
        elif k in self.keys:
            return
        else:
            self.keys.add(k)
        self.append(n)


def _append_rules(rules: List[ContivRule], *new: ContivRule) -> List[ContivRule]:
    """appendRule(s) (configurator_impl.go:482-498): skip exact duplicates."""
    keyed = getattr(rules, "append_unique", None)
    for n in new:
        if keyed is not None:
            keyed(n)
        elif not any(r.compare(n) == 0 for r in rules):
            rules.append(n)
    return rules


def _rule(action: int, protocol: int, dest_port: int = 0, src: IPNet = None, dst: IPNet = None) -> ContivRule:
    return ContivRule(action=action, src_network=src if src is not None else IPNet(),
                      dest_network=dst if dst is not None else IPNet(),
                      protocol=protocol, src_port=0, dest_port=dest_port)


def _port_proto(port: Port) -> int:
    return R_TCP if port.protocol == TCP else R_UDP


class PolicyConfigurator:
    """PolicyConfigurator (configurator_impl.go:39-115).

    ``cache`` is the policy cache's LookupPod as a mapping PodID -> IP string
    (the mock/policycache AddPodConfig data); a missing pod or "" is a pod
    without an address."""

    def __init__(self, cache: Dict[PodID, str], parallel_rendering: bool = False):
        self.cache = cache
        self.renderers = []
        self.parallel_rendering = parallel_rendering   # Go goroutines; commits run in order here
        self.pod_ip_addresses: Dict[PodID, IPNet] = {}

    def register_renderer(self, renderer) -> None:
        self.renderers.append(renderer)

    def new_txn(self, resync: bool) -> "PolicyConfiguratorTxn":
        return PolicyConfiguratorTxn(self, resync)

    def lookup_pod(self, pod: PodID):
        ip = self.cache.get(pod)
        return (ip is not None), (ip or "")


class PolicyConfiguratorTxn:
    """PolicyConfiguratorTxn (configurator_impl.go:54-60, 102-239)."""

    def __init__(self, configurator: PolicyConfigurator, resync: bool):
        self.configurator = configurator
        self.resync = resync
        self.config: Dict[PodID, List[ContivPolicy]] = {}
        self.pod_ip_addresses = dict(configurator.pod_ip_addresses)
        self.generated: Dict[PodID, tuple] = {}   # pod -> (ingress, egress) rendered (inspection)

    def configure(self, pod: PodID, policies: Sequence[ContivPolicy]) -> "PolicyConfiguratorTxn":
        """Configure (:119-126): replaces the pod's policy set."""
        self.config[pod] = list(policies)
        return self

    def commit(self) -> None:
        """Commit (:129-239).  Renderer errors propagate (the last one in Go)."""
        processed = []                                    # [(policies, ingress, egress)]
        txns = []
        for pod, unordered in self.config.items():
            ingress: List[ContivRule] = []
            egress: List[ContivRule] = []
            removed = False
            pod_ipnet = self.pod_ip_addresses.get(pod)
            found, ip = self.configurator.lookup_pod(pod)
            if not found or ip == "":                     # :146-156
                if pod_ipnet is None:
                    continue                              # already un-configured
                removed = True
                del self.pod_ip_addresses[pod]
            if not removed:
                pod_ipnet = gonet.one_host_subnet(ip)     # :159-165
                if pod_ipnet is None:
                    continue                              # invalid IP: warn and skip
                self.pod_ip_addresses[pod] = pod_ipnet
                policies = sorted(unordered, key=_policy_key)   # stable, like sort.Sort on distinct IDs
                hit = None
                for entry in processed:                   # :172-179
                    if _policies_equal(entry[0], policies):
                        hit = entry
                if hit is not None:
                    ingress, egress = hit[1], hit[2]
                else:                                     # :182-194
                    egress = self.generate_rules(MATCH_INGRESS, policies)
                    ingress = self.generate_rules(MATCH_EGRESS, policies)
                    processed.append((policies, ingress, egress))
            if not txns:                                  # :198-202
                txns = [r.new_txn(self.resync) for r in self.configurator.renderers]
            for t in txns:                                # :205-207 (deep copies)
                t.render(pod, pod_ipnet, [r.copy() for r in ingress], [r.copy() for r in egress], removed)
            self.generated[pod] = (ingress, egress)
        err = None
        for t in txns:                                    # :211-233
            try:
                t.commit()
            except Exception as e:                        # noqa: BLE001 -- Go keeps the last error
                err = e
        self.configurator.pod_ip_addresses = dict(self.pod_ip_addresses)   # :236
        if err is not None:
            raise err

    def generate_rules(self, direction: int, policies: List[ContivPolicy]) -> List[ContivRule]:
        """generateRules (configurator_impl.go:248-479)."""
        rules: List[ContivRule] = _RuleList()
        has_policy = False
        all_allowed = False
        for policy in policies:
            if ((policy.type == POLICY_INGRESS and direction == MATCH_EGRESS)
                    or (policy.type == POLICY_EGRESS and direction == MATCH_INGRESS)):
                continue                                  # :254-258
            has_policy = True
            for match in policy.matches:
                if match.type != direction:
                    continue
                peers = []                                # :266-286
                for peer in match.pods or ():
                    found, ip = self.configurator.lookup_pod(peer)
                    if not found or ip == "":
                        continue
                    peer_net = gonet.one_host_subnet(ip)
                    if peer_net is None:
                        continue
                    peers.append(peer_net)
                subnets_all = []                          # :288-300
                for block in match.ip_blocks or ():
                    subnets = [block.network]
                    for exc in block.excepts:
                        subnets = [s for net in subnets for s in subtract_subnet(net, exc)]
                    subnets_all.extend(subnets)
                ports = match.ports or []
                if match.pods is None and match.ip_blocks is None:   # :302-343
                    if not ports:
                        _append_rules(rules, _rule(ACTION_PERMIT, R_TCP), _rule(ACTION_PERMIT, R_UDP))
                        all_allowed = True
                    else:
                        for port in ports:
                            _append_rules(rules, _rule(ACTION_PERMIT, _port_proto(port), port.number))
                # peers (:345-398), then IP blocks (:400-453): same shape
                for net in peers + subnets_all:
                    src = net if direction == MATCH_INGRESS else None
                    dst = None if direction == MATCH_INGRESS else net
                    if not ports:
                        _append_rules(rules, _rule(ACTION_PERMIT, R_TCP, 0, src, dst),
                                      _rule(ACTION_PERMIT, R_UDP, 0, src, dst))
                    else:
                        for port in ports:
                            _append_rules(rules, _rule(ACTION_PERMIT, _port_proto(port), port.number, src, dst))
        if has_policy and not all_allowed:                # :457-476 deny the rest
            _append_rules(rules, _rule(ACTION_DENY, R_TCP), _rule(ACTION_DENY, R_UDP))
        return list(rules)


def gen_policy(rng, num_cidrs: int = 1000, num_excepts: int = 5, num_ports: int = 20,
               name: str = "test-network-policy", namespace: str = "default") -> ContivPolicy:
    """The NetworkPolicy of tests/policy/perf/gen-policy.py (:8-65) as the
    ContivPolicy the policy processor would hand the configurator: ingress
    from and egress to ``num_cidrs`` IP blocks (block i inside (i + 256) << 16,
    /16-/24) with ``num_excepts`` excepts each (/24-/32 inside the block), and
    ``num_ports`` random TCP/UDP ports per direction.  ``rng``: random.Random."""

    def mask(a, ln):
        return a & (0xFFFFFFFF ^ ((1 << (32 - ln)) - 1))

    def net(a, ln):
        return IPNet(a.to_bytes(4, "big"), gonet.cidr_mask(ln, 32))

    def blocks():
        out = []
        for i in range(num_cidrs):
            prefix = (i + 0x100) << 16
            ln = rng.randint(16, 24)
            cidr = mask(rng.randint(prefix, prefix | 0xFFFF), ln)
            excepts = []
            for _ in range(num_excepts):
                e = rng.randint(cidr, cidr | ((1 << (32 - ln)) - 1))
                eln = rng.randint(24, 32)
                excepts.append(net(mask(e, eln), eln))
            out.append(IPBlock(net(cidr, ln), excepts))
        return out

    def ports():
        return [Port(TCP if rng.randint(0, 1) == 0 else UDP, rng.randint(0, 65535)) for _ in range(num_ports)]

    ingress = Match(MATCH_INGRESS, ip_blocks=blocks(), ports=ports())
    egress = Match(MATCH_EGRESS, ip_blocks=blocks(), ports=ports())
    return ContivPolicy(PolicyID(name, namespace), POLICY_ALL, [ingress, egress])
