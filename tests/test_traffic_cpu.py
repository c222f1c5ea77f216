"""TestTraffic (mock/renderer/renderer_mock.go:105-145) on CPU.

1. The oracle restatement (oracle/traffic.py) is pinned against the evalACL
   oracle on rule lists both can express: renderACL + evalACL gives the same
   Permit/Deny, and evalACL's default DENY where TestTraffic is UNMATCHED.
2. The ACL translation the GPU path runs (vpp_amd/renderer/traffic.py
   compile_rules), evaluated by the C evalACL oracle, equals TestTraffic
   packet by packet, hit index included -- IPv6, IPv4-mapped, dead networks
   and protocols > 2 included.
3. Inputs the translation cannot express are rejected, never approximated.
4. MockRendererTxn bookkeeping (Render/Commit, resync, removed pods).
"""
import random

import numpy as np
import pytest

import oracle
from oracle import traffic as otraffic
from traffic_gen import rand_packets, rand_rules
from vpp_amd import gonet
from vpp_amd.gonet import IPNet
from vpp_amd.renderer import traffic as T
from vpp_amd.renderer.acl import render_acl
from vpp_amd.renderer.api import ACTION_PERMIT, TCP, UDP, ContivRule, PodID
from vpp_amd.renderer.cache import ContivRuleTable
from vpp_amd import model


@pytest.mark.parametrize("seed", range(6))
def test_oracle_agrees_with_render_acl_eval_acl(seed):
    rng = random.Random(seed)
    rules = [r for r in rand_rules(rng, 24)
             if T.network_string(r.src_network) is not None and T.network_string(r.dest_network) is not None]
    table = ContivRuleTable("LOCAL-x")
    table.rules = rules
    acl = render_acl(table, model.Interfaces())
    cr = oracle.rules_to_c(acl.rules)
    src, dst, proto, sport, dport = rand_packets(rng, rules, 1500)
    checked = 0
    for s, d, p, sp, dp in zip(src, dst, proto, sport, dport):
        if p not in (TCP, UDP):
            continue               # renderACL's trailing ICMP rule and evalACL's fall-through differ
        a, i = otraffic.test_traffic(rules, s, d, p, sp, dp)
        b, j = oracle.eval_acl(cr, False, s, d, p, dp)
        if a == otraffic.UNMATCHED:
            assert (b, j) == (0, len(acl.rules)), (s, d, p, dp)
        else:
            assert (a, i) == (b, j), (s, d, p, dp)
        checked += 1
    assert checked > 1000


@pytest.mark.parametrize("seed", range(8))
def test_translation_matches_test_traffic(seed):
    rng = random.Random(100 + seed)
    rules = rand_rules(rng, rng.choice([1, 5, 30, 80]))
    acl_rules = T.compile_rules(rules)
    assert len(acl_rules) == len(rules) + 1 + T.N_TAIL
    cr = oracle.rules_to_c(acl_rules)
    src, dst, proto, sport, dport = rand_packets(rng, rules, 2000)
    seen = set()
    for s, d, p, sp, dp in zip(src, dst, proto, sport, dport):
        a, i = otraffic.test_traffic(rules, s, d, p, sp, dp)
        b, j = oracle.eval_acl(cr, False, s, d, p, dp)
        assert a == b, (seed, s, d, p, dp)
        if i >= 0:
            assert j == T.FIRST_RULE + i
        else:
            assert j == 0 or j >= T.FIRST_RULE + len(rules)
        seen.add(a)
    assert T.UNMATCHED_TRAFFIC in seen and len(seen) >= 2


def test_translation_counters_fold():
    rng = random.Random(7)
    rules = rand_rules(rng, 40)
    cr = oracle.rules_to_c(T.compile_rules(rules))
    src, dst, proto, sport, dport = rand_packets(rng, rules, 3000)
    want_v, want_c, want_u = otraffic.test_traffic_batch(rules, src, dst, proto, sport, dport)
    rows = [(gonet.V4_IN_V6_PREFIX + x if len(x) == 4 else x) for x in src]
    rowd = [(gonet.V4_IN_V6_PREFIX + x if len(x) == 4 else x) for x in dst]
    s16 = np.frombuffer(b"".join(rows), np.uint8).reshape(-1, 16)
    d16 = np.frombuffer(b"".join(rowd), np.uint8).reshape(-1, 16)
    v, c = oracle.classify_faithful(cr, s16, d16, np.array(dport, np.uint16), np.array(proto, np.uint8), af=16)
    per_rule, unmatched = T.rule_counters(c, len(rules))
    assert list(v) == want_v
    assert [int(x) for x in per_rule] == want_c
    assert unmatched == want_u


def test_rejects_what_the_acl_form_cannot_express():
    net = gonet.ip_network("10.0.0.0/8")
    with pytest.raises(ValueError):
        T.compile_rules([ContivRule(ACTION_PERMIT, net, IPNet(), TCP, 1234, 0)])
    with pytest.raises(ValueError):
        T.compile_rules([ContivRule(ACTION_PERMIT, net, IPNet(), 2, 0, 0)])
    with pytest.raises(ValueError):
        T.compile_rules([ContivRule(ACTION_PERMIT, IPNet(bytes([10, 0, 0, 0]), bytes([255, 0, 255, 0])),
                                    IPNet(), TCP, 0, 0)])


def test_network_string_round_trips_contains():
    rng = random.Random(3)
    from traffic_gen import _near, _rand_net
    for _ in range(400):
        net = _rand_net(rng)
        s = T.network_string(net)
        if s is None or s == "":
            continue
        _, parsed = gonet.parse_cidr(s)
        assert parsed is not None, s
        for _ in range(5):
            ip = _near(rng, net)
            assert parsed.contains(ip) == net.contains(ip), (s, ip)


class _StubEngine:
    def __init__(self):
        self.live = set()
        self.n = 0

    def put_table(self, name, rules):
        self.n += 1
        self.live.add(self.n)
        return self.n

    def del_table(self, t):
        self.live.remove(t)


def test_renderer_txn_bookkeeping():
    eng = _StubEngine()
    r = T.TrafficRenderer("mock", eng)
    p1, p2 = PodID("pod1", "default"), PodID("pod2", "default")
    ip1 = gonet.one_host_subnet("10.10.1.1")
    rule = ContivRule(ACTION_PERMIT, IPNet(), IPNet(), TCP, 0, 80)
    r.new_txn(False).render(p1, ip1, [rule], [], False).render(p2, ip1, [], [rule], False).commit()
    assert set(r.config) == {p1, p2} and len(eng.live) == 4
    assert r.get_pod_ip(p1) == ("10.10.1.1", 32)
    # removed in a non-resync txn: the renderer keeps the pod (renderer_mock.go:157-181)
    r.new_txn(False).render(p1, None, [], [], True).commit()
    assert set(r.config) == {p1, p2} and len(eng.live) == 4
    r.new_txn(True).render(p2, ip1, [rule], [], False).commit()
    assert set(r.config) == {p2} and len(eng.live) == 2
    assert r.test_traffic(p1, T.INGRESS_TRAFFIC, b"\x0a\0\0\1", b"\x0a\0\0\2", TCP, 1, 80) == T.UNMATCHED_TRAFFIC
    r.close()
    assert not eng.live
