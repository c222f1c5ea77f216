"""Policy configurator (configurator_impl.go) on CPU.

1. The reference's own configurator tests (configurator_test.go, 10 tests,
   115 TestTraffic verdicts + GetPodIP checks) replayed from
   tests/golden/configurator_scenarios.json into
   a. the literal TestTraffic oracle (oracle/traffic.py) over the raw
      ContivRule lists -- this also pins that oracle to reference
      expectations for the first time;
   b. the GPU renderer's own code (vpp_amd/renderer/traffic.py: compile_rules,
      bookkeeping, verdict mapping) with the C evalACL oracle standing in for
      the device classify.
2. subtractSubnet (configurator_impl.go:563-595) against a brute-force set
   difference over every address of small IPv4 and IPv6 prefixes.
3. generateRules details: duplicate suppression, "allow all" suppressing the
   trailing deny, policy direction filtering, processed-set reuse and pod
   removal in Commit.
"""
import random

import numpy as np
import pytest

import oracle
from oracle import traffic as otraffic
from configurator_replay import load, mismatches, replay
from vpp_amd import configurator as C
from vpp_amd import gonet
from vpp_amd.gonet import IPNet
from vpp_amd.renderer import traffic as T
from vpp_amd.renderer.api import ACTION_DENY, ACTION_PERMIT, TCP, UDP, PodID

SCENARIOS = load()["scenarios"]


class _BookkeepingEngine:
    """Tables are never evaluated: the literal renderer reads r.config."""

    def __init__(self):
        self.n = 0

    def put_table(self, name, rules):
        self.n += 1
        return self.n

    def del_table(self, t):
        pass


class LiteralRenderer(T.TrafficRenderer):
    """MockRenderer with TestTraffic = the literal oracle over the raw lists."""

    def __init__(self, name):
        super().__init__(name, _BookkeepingEngine())

    def test_traffic(self, pod, direction, src_ip, dst_ip, protocol, src_port, dst_port):
        cfg = self.config.get(pod)
        if cfg is None:
            return otraffic.UNMATCHED
        rules = cfg.ingress if direction == T.INGRESS_TRAFFIC else cfg.egress
        a, _ = otraffic.test_traffic(rules, src_ip, dst_ip, protocol, src_port, dst_port)
        return a


class _EvalAclTable:
    def __init__(self, rules):
        self.cr = oracle.rules_to_c(rules)

    def info(self):
        return {}


class EvalAclEngine:
    """The renderer's engine calls, answered by the C evalACL oracle."""

    def put_table(self, name, rules):
        return _EvalAclTable(rules)

    def del_table(self, t):
        pass

    def classify(self, t, src, dst, dport, proto, verdict=None, counters=None, stream=None):
        return oracle.classify_faithful(t.cr, np.ascontiguousarray(src), np.ascontiguousarray(dst),
                                        np.asarray(dport, np.uint16), np.asarray(proto, np.uint8), af=16)


def test_fixture_covers_reference_tests():
    data = load()
    assert len(SCENARIOS) == 10 and data["n_traffic"] == 115


@pytest.mark.parametrize("scn", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_reference_scenarios_literal_oracle(scn):
    _, checks = replay(scn, LiteralRenderer)
    assert checks and not mismatches(checks)


@pytest.mark.parametrize("scn", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_reference_scenarios_gpu_translation_on_eval_acl(scn):
    eng = EvalAclEngine()
    _, checks = replay(scn, lambda name: T.TrafficRenderer(name, eng))
    assert checks and not mismatches(checks)


def _addr_int(ip):
    return int.from_bytes(ip, "big")


@pytest.mark.parametrize("bits", [32, 128])
def test_subtract_subnet_bruteforce(bits):
    rng = random.Random(bits)
    nbytes = bits // 8
    base = bytes(rng.randrange(256) for _ in range(nbytes))
    for _ in range(300):
        l1 = bits - rng.randrange(0, 9)
        l2 = bits - rng.randrange(0, 9)
        a = bytearray(base)
        b = bytearray(base)
        a[-1] = rng.randrange(256)
        b[-1] = rng.randrange(256)
        if rng.random() < 0.2:
            b[-2] ^= 1                                          # disjoint upper bits
        m1, m2 = gonet.cidr_mask(l1, bits), gonet.cidr_mask(l2, bits)
        n1 = IPNet(gonet.ip_mask(bytes(a), m1), m1)
        n2 = IPNet(gonet.ip_mask(bytes(b), m2), m2)
        out = C.subtract_subnet(n1, n2)
        lo = _addr_int(n1.ip)
        want = {x for x in range(lo, lo + (1 << (bits - l1)))
                if not n2.contains(x.to_bytes(nbytes, "big"))}
        got = []
        for s in out:
            ones, _ = gonet.mask_size(s.mask)
            s_lo = _addr_int(s.ip)
            got.extend(range(s_lo, s_lo + (1 << (bits - ones))))
        assert len(got) == len(set(got)), "subnets overlap"
        assert set(got) == want, (n1, n2, out)


def _cfg(cache):
    return C.PolicyConfigurator(cache)


def test_generate_rules_allow_all_and_duplicates():
    pod1, pod2 = PodID("p1", "ns"), PodID("p2", "ns")
    cache = {pod1: "10.0.0.1", pod2: "10.0.0.2"}
    txn = _cfg(cache).new_txn(False)
    any_l3 = C.Match(C.MATCH_INGRESS)                           # nil pods + nil blocks, no ports
    dup = C.Match(C.MATCH_INGRESS, pods=[pod2, pod2], ports=[C.Port(C.TCP, 80), C.Port(C.TCP, 80)])
    p = C.ContivPolicy(C.PolicyID("a", "ns"), C.POLICY_INGRESS, [dup, any_l3])
    rules = txn.generate_rules(C.MATCH_INGRESS, [p])
    assert [(r.action, r.protocol, r.dest_port, str(r.src_network) if r.src_network.ip else "") for r in rules] == [
        (ACTION_PERMIT, TCP, 80, "10.0.0.2/32"), (ACTION_PERMIT, TCP, 0, ""), (ACTION_PERMIT, UDP, 0, "")]
    # ingress-only policy: nothing for the other direction, and no deny either
    assert txn.generate_rules(C.MATCH_EGRESS, [p]) == []
    # an empty-but-non-nil pod list is not "match anything": only the deny tail
    q = C.ContivPolicy(C.PolicyID("b", "ns"), C.POLICY_ALL, [C.Match(C.MATCH_EGRESS, pods=[])])
    rules = txn.generate_rules(C.MATCH_EGRESS, [q])
    assert [(r.action, r.protocol) for r in rules] == [(ACTION_DENY, TCP), (ACTION_DENY, UDP)]


class _RecordingRenderer:
    def __init__(self):
        self.calls = []
        self.commits = 0

    def new_txn(self, resync):
        outer = self

        class Txn:
            def render(self, pod, ip, ingress, egress, removed):
                outer.calls.append((pod, ip, ingress, egress, removed))
                return self

            def commit(self):
                outer.commits += 1
        return Txn()


def test_commit_reuse_and_removal():
    pods = [PodID("p%d" % i, "ns") for i in range(3)]
    cache = {p: "10.0.0.%d" % (i + 1) for i, p in enumerate(pods)}
    conf = _cfg(cache)
    rec = _RecordingRenderer()
    conf.register_renderer(rec)
    pa = C.ContivPolicy(C.PolicyID("a", "ns"), C.POLICY_INGRESS,
                        [C.Match(C.MATCH_INGRESS, pods=[pods[2]], ports=[C.Port(C.UDP, 53)])])
    pb = C.ContivPolicy(C.PolicyID("b", "ns"), C.POLICY_EGRESS, [C.Match(C.MATCH_EGRESS, ports=[C.Port(C.TCP, 1)])])
    txn = conf.new_txn(False)
    txn.configure(pods[0], [pb, pa]).configure(pods[1], [pa, pb])   # same set, other order
    txn.commit()
    assert rec.commits == 1 and len(rec.calls) == 2
    g0, g1 = txn.generated[pods[0]], txn.generated[pods[1]]
    assert g0[0] is g1[0] and g0[1] is g1[1]                       # processed-set reuse
    # the policy's ingress is the vswitch's egress list
    assert [(r.protocol, r.dest_port) for r in g0[1]][:1] == [(UDP, 53)]
    assert str(conf.pod_ip_addresses[pods[0]]) == "10.0.0.1/32"
    # pod disappears from the cache: rendered as removed with its old address
    del cache[pods[0]]
    rec.calls.clear()
    conf.new_txn(False).configure(pods[0], []).configure(PodID("ghost", "ns"), [pa]).commit()
    assert len(rec.calls) == 1
    pod, ip, ingress, egress, removed = rec.calls[0]
    assert pod == pods[0] and removed and str(ip) == "10.0.0.1/32" and ingress == [] and egress == []
    assert pods[0] not in conf.pod_ip_addresses


@pytest.mark.parametrize("seed", range(3))
def test_random_policy_sets_translation_matches_literal(seed):
    from configurator_replay import random_packets, random_policy_set
    from vpp_amd.renderer import traffic as TT
    rng = random.Random(seed)
    cache, assign = random_policy_set(rng)
    lit, gpuish = LiteralRenderer("L"), T.TrafficRenderer("E", EvalAclEngine())
    conf = C.PolicyConfigurator(cache)
    conf.register_renderer(lit)
    conf.register_renderer(gpuish)
    txn = conf.new_txn(True)
    for pod, pols in assign.items():
        txn.configure(pod, pols)
    txn.commit()
    src, dst, proto, sport, dport = random_packets(rng, cache, 300)
    rows = lambda ips: np.frombuffer(b"".join(gonet.V4_IN_V6_PREFIX + x if len(x) == 4 else x for x in ips),
                                     np.uint8).reshape(-1, 16)
    checked = 0
    for pod in list(gpuish.config)[:12]:
        for d in (TT.INGRESS_TRAFFIC, TT.EGRESS_TRAFFIC):
            rules = gpuish.config[pod].ingress if d == TT.INGRESS_TRAFFIC else gpuish.config[pod].egress
            if not rules:
                continue
            want, want_c, want_u = otraffic.test_traffic_batch(rules, src, dst, proto, sport, dport)
            v, c, u = gpuish.test_traffic_batch(pod, d, rows(src), rows(dst), np.array(proto, np.uint8),
                                                np.array(dport, np.uint16))
            assert list(v) == want and [int(x) for x in c] == want_c and u == want_u
            checked += 1
    assert checked >= 5


def test_rule_key_agrees_with_compare():
    from vpp_amd.renderer.api import ContivRule
    rng = random.Random(11)

    def net():
        k = rng.randrange(6)
        if k == 0:
            return IPNet()
        if k in (1, 2):                                     # IPv4, 4- or 16-byte address
            ones = rng.choice([0, 8, 16, 24, 30, 32])
            ip = bytes([10, rng.randrange(2), rng.randrange(2), rng.randrange(4)])
            return IPNet(ip if k == 1 else gonet.V4_IN_V6_PREFIX + ip, gonet.cidr_mask(ones, 32))
        if k == 3:                                          # IPv6
            ones = rng.choice([0, 64, 120, 128])
            ip = bytes([0xfd] + [0] * 14 + [rng.randrange(4)])
            return IPNet(ip, gonet.cidr_mask(ones, 128))
        if k == 4:                                          # non-contiguous mask
            return IPNet(bytes([10, 0, 0, rng.randrange(4)]), bytes([255, 0, 255, 0]))
        return IPNet(bytes([10, 0, rng.randrange(2), 0]), gonet.cidr_mask(rng.choice([16, 24]), 128))

    rules = [ContivRule(rng.randrange(2), net(), net(), rng.randrange(2), 0, rng.choice([0, 80])) for _ in range(400)]
    for a in rules:
        for b in rules[:120]:
            ka, kb = C._rule_key(a), C._rule_key(b)
            if ka is not None and kb is not None:
                assert (ka == kb) == (a.compare(b) == 0), (a, b)


@pytest.mark.parametrize("seed", range(4))
def test_generate_rules_keyed_equals_scan(seed):
    from configurator_replay import random_policy_set
    rng = random.Random(seed)
    cache, assign = random_policy_set(rng, n_pods=200, n_policies=60)
    txn = C.PolicyConfigurator(cache).new_txn(False)
    pols = sorted({id(p): p for ps in assign.values() for p in ps}.values(), key=C._policy_key)
    fast = txn.generate_rules(C.MATCH_INGRESS, pols) + txn.generate_rules(C.MATCH_EGRESS, pols)
    orig = C._RuleList
    try:
        C._RuleList = list                                  # the reference's linear scan
        slow = txn.generate_rules(C.MATCH_INGRESS, pols) + txn.generate_rules(C.MATCH_EGRESS, pols)
    finally:
        C._RuleList = orig
    assert len(fast) == len(slow) and all(a.compare(b) == 0 for a, b in zip(fast, slow))


def test_gen_policy_small_translation_matches_literal():
    """gen-policy.py shape at 3 blocks: the GPU renderer's translation (on the
    C evalACL oracle) equals the literal TestTraffic oracle packet by packet."""
    from configurator_replay import gen_policy_packets
    rng = random.Random(3)
    pol = C.gen_policy(rng, num_cidrs=3, num_ports=4)
    pod = PodID("db", "default")
    conf = C.PolicyConfigurator({pod: "10.1.1.1"})
    r = T.TrafficRenderer("gen", EvalAclEngine())
    conf.register_renderer(r)
    conf.new_txn(False).configure(pod, [pol]).commit()
    src, dst, proto, dport, s16, d16 = gen_policy_packets(rng, 400, 3)
    ports = [p.number for m in pol.matches for p in m.ports]
    dport = [rng.choice(ports) if rng.random() < 0.5 else p for p in dport]
    sport = [1000] * len(src)
    for d in (T.INGRESS_TRAFFIC, T.EGRESS_TRAFFIC):
        rules = r.config[pod].ingress if d == T.INGRESS_TRAFFIC else r.config[pod].egress
        want, want_c, want_u = otraffic.test_traffic_batch(rules, src, dst, proto, sport, dport)
        v, c, u = r.test_traffic_batch(pod, d, s16, d16, np.array(proto, np.uint8), np.array(dport, np.uint16))
        assert list(v) == want and [int(x) for x in c] == want_c and u == want_u
