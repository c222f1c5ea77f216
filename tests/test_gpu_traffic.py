"""GPU parity of TestTraffic (mock/renderer/renderer_mock.go:105-145, SURVEY
8(a10)): ContivRule lists compiled onto the classifier
(vpp_amd/renderer/traffic.py) against the literal oracle (oracle/traffic.py).
Bar: TrafficAction per packet, per-rule hit counts and the unmatched count
bit-exact, in the 16-byte and the IPv4 layouts, device and host buffers.
"""
import random

import numpy as np
import pytest

from oracle import traffic as otraffic
from traffic_gen import rand_packets, rand_rules
from vpp_amd import gonet
from vpp_amd.renderer import traffic as T
from vpp_amd.renderer.api import ACTION_DENY, ACTION_PERMIT, TCP, UDP, ContivRule, PodID

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from vpp_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


def _rows(ips):
    return np.frombuffer(b"".join(gonet.V4_IN_V6_PREFIX + x if len(x) == 4 else x for x in ips),
                         np.uint8).reshape(-1, 16)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("n_rules", [1, 12, 90, 400])
def test_rule_lists_v16(eng, seed, n_rules):
    rng = random.Random(seed * 1000 + n_rules)
    rules = rand_rules(rng, n_rules)
    src, dst, proto, sport, dport = rand_packets(rng, rules, 5003)
    want_v, want_c, want_u = otraffic.test_traffic_batch(rules, src, dst, proto, sport, dport)
    t = T.RuleTable(eng, "tt", rules)
    try:
        v, c, u = t.test_traffic_batch(_rows(src), _rows(dst), np.array(proto, np.uint8),
                                       np.array(dport, np.uint16))
    finally:
        t.close()
    assert list(v) == want_v
    assert [int(x) for x in c] == want_c
    assert u == want_u


def test_rule_lists_v4_device(eng):
    """IPv4-only rules and packets through device tensors (the bench layout)."""
    import torch
    rng = random.Random(5)
    rules = [r for r in rand_rules(rng, 300)
             if all(len(n.ip) == 0 or (gonet.to4(n.ip) is not None and len(n.mask) == 4)
                    for n in (r.src_network, r.dest_network))]
    src, dst, proto, sport, dport = rand_packets(rng, rules, 40000)
    keep = [i for i in range(len(src)) if gonet.to4(src[i]) is not None and gonet.to4(dst[i]) is not None]
    src = [gonet.to4(src[i]) for i in keep]
    dst = [gonet.to4(dst[i]) for i in keep]
    proto, sport, dport = ([x[i] for i in keep] for x in (proto, sport, dport))
    want_v, want_c, want_u = otraffic.test_traffic_batch(rules, src, dst, proto, sport, dport)
    dev = torch.device("cuda", 0)
    s = torch.tensor(np.array([int.from_bytes(x, "big") for x in src], np.uint32).view(np.int32), device=dev)
    d = torch.tensor(np.array([int.from_bytes(x, "big") for x in dst], np.uint32).view(np.int32), device=dev)
    pr = torch.tensor(np.array(proto, np.uint8), device=dev)
    dp = torch.tensor(np.array(dport, np.uint16).view(np.int16), device=dev)
    v = torch.empty(len(src), dtype=torch.uint8, device=dev)
    c = torch.zeros(len(rules) + 1 + T.N_TAIL + 1, dtype=torch.int64, device=dev)
    t = T.RuleTable(eng, "tt4", rules)
    try:
        t.test_traffic_batch(s, d, pr, dp, verdict=v, counters=c)
        torch.cuda.synchronize()
    finally:
        t.close()
    per_rule, unmatched = T.rule_counters(c.cpu().numpy(), len(rules))
    assert v.cpu().numpy().tolist() == want_v
    assert [int(x) for x in per_rule] == want_c
    assert unmatched == want_u


def test_mock_renderer_single_packets(eng):
    """The TrafficRenderer drop-in: Render/Commit then TestTraffic per packet,
    with the rules of renderer testdata Ts3-style lists."""
    p1 = PodID("pod1", "default")
    ip1 = gonet.one_host_subnet("10.10.1.1")
    ingress = [ContivRule(ACTION_PERMIT, gonet.ip_network("10.10.0.0/16"), gonet.ip_network(""), TCP, 0, 80),
               ContivRule(ACTION_DENY, gonet.ip_network(""), gonet.ip_network(""), TCP, 0, 0)]
    egress = [ContivRule(ACTION_PERMIT, gonet.ip_network(""), gonet.ip_network("192.168.0.0/16"), UDP, 0, 53)]
    r = T.TrafficRenderer("gpu", eng)
    r.new_txn(False).render(p1, ip1, ingress, egress, False).commit()
    a, b = gonet.parse_ip("10.10.5.5"), gonet.parse_ip("10.10.1.1")
    cases = [(T.INGRESS_TRAFFIC, a, b, TCP, 80), (T.INGRESS_TRAFFIC, a, b, TCP, 81),
             (T.INGRESS_TRAFFIC, a, b, UDP, 80), (T.EGRESS_TRAFFIC, b, gonet.parse_ip("192.168.3.4"), UDP, 53),
             (T.EGRESS_TRAFFIC, b, gonet.parse_ip("192.169.3.4"), UDP, 53)]
    try:
        for d, s_ip, d_ip, p, dp in cases:
            rules = ingress if d == T.INGRESS_TRAFFIC else egress
            want, _ = otraffic.test_traffic(rules, s_ip, d_ip, p, 5000, dp)
            assert r.test_traffic(p1, d, s_ip, d_ip, p, 5000, dp) == want
    finally:
        r.close()


def test_vpptcp_committed_tables_on_gpu(eng):
    """Session-rule renderer: the IngressOrientation tables it
    commits are compiled onto the engine; packets against a pod's local table
    and the global table match TestTraffic over the same rule lists."""
    from test_vpptcp_cpu import EG1, EG2, IN1, IN2, IN3, POD1, POD1_IP, POD1_NS, POD2, POD2_IP, POD2_NS, contiv, host
    from vpp_amd.renderer import vpptcp as V
    sink = V.SessionRuleTables()
    rend = V.Renderer(contiv((POD1, POD1_NS), (POD2, POD2_NS)), sink, engine=eng).init()
    txn = rend.new_txn(False)
    txn.render(POD1, host(POD1_IP), [IN1(), IN2()], [EG1(), EG2()], False)
    txn.render(POD2, host(POD2_IP), [IN1(), IN3()], [], False)
    txn.commit()
    rng = random.Random(11)
    try:
        tables = [rend.local_rule_table(POD1), rend.local_rule_table(POD2), rend.global_rule_table()]
        assert all(t is not None for t in tables)
        for t in tables:
            src, dst, proto, sport, dport = rand_packets(rng, t.rules, 3001)
            want_v, want_c, want_u = otraffic.test_traffic_batch(t.rules, src, dst, proto, sport, dport)
            v, c, u = t.test_traffic_batch(_rows(src), _rows(dst), np.array(proto, np.uint8),
                                           np.array(dport, np.uint16))
            assert list(v) == want_v
            assert [int(x) for x in c] == want_c and u == want_u
    finally:
        rend.close()
