"""VPPTCP renderer + session-rule sink replayed against the
reference's own expectations.

Each test restates one test of
plugins/policy/renderer/vpptcp/vpptcp_renderer_test.go statement by statement
(same rules, pods, namespace indices, channel buffer sizes and transaction
sequence), and checks every GetErrCount / GetReqCount / NumOfRules / HasRule
expectation it makes: 6 tests, 49 HasRule checks plus the counts.  The
session-rule sink is the restated mock/sessionrules store.
"""
import pytest

from vpp_amd import gonet
from vpp_amd.renderer.acl import ContivIfs
from vpp_amd.renderer.api import ACTION_DENY, ACTION_PERMIT, TCP, UDP, ContivRule, PodID
from vpp_amd.renderer import vpptcp as V

NS = "default"
POD1, POD1_IP, POD1_NS = PodID("pod1", NS), "192.168.1.1", 10
POD2, POD2_IP, POD2_NS = PodID("pod2", NS), "192.168.1.2", 15

HAS_RULE_CHECKS = [0]


def net(s):
    return gonet.ip_network(s)


def rule(action, src, dst, proto, dport):
    return ContivRule(action, net(src), net(dst), proto, 0, dport)


def host(ip):
    return gonet.one_host_subnet(ip)


def check(sink, err, req, local=None, glob=None):
    assert sink.err_count == err
    assert sink.req_count == req
    for ns, (n, rules) in (local or {}).items():
        assert sink.num_of_rules(ns) == n, ns
        for r in rules:
            HAS_RULE_CHECKS[0] += 1
            assert sink.has_rule(ns, *r), (ns, r)
    if glob is not None:
        n, rules = glob
        assert sink.num_of_rules() == n
        for r in rules:
            HAS_RULE_CHECKS[0] += 1
            assert sink.has_rule(None, *r), r


@pytest.fixture
def sink():
    return V.SessionRuleTables(V.SESSION_RULE_TAG_PREFIX)


def contiv(*pods):
    c = ContivIfs()
    for pod, ns in pods:
        c.set_pod_app_ns_index(pod, ns)
    return c


def test_single_egress_rule_single_pod(sink):                       # :54-107
    r = rule(ACTION_DENY, "192.168.2.0/24", "", TCP, 80)
    rend = V.Renderer(contiv((POD1, POD1_NS)), sink, chan_buf_size=20).init()
    rend.new_txn(False).render(POD1, host(POD1_IP), [], [r], False).commit()
    check(sink, 0, 1, {POD1_NS: (0, [])},
          (1, [(POD1_IP, 80, "192.168.2.0/24", 0, "TCP", "DENY")]))


def test_single_ingress_rule_single_pod(sink):                      # :109-162
    r = rule(ACTION_DENY, "", "10.0.0.0/8", TCP, 22)
    rend = V.Renderer(contiv((POD1, POD1_NS)), sink, chan_buf_size=2).init()
    rend.new_txn(False).render(POD1, host(POD1_IP), [r], [], False).commit()
    check(sink, 0, 1, {POD1_NS: (1, [("", 0, "10.0.0.0/8", 22, "TCP", "DENY")])}, (0, []))


IN1 = lambda: rule(ACTION_DENY, "", "10.0.0.0/8", TCP, 22)
IN2 = lambda: rule(ACTION_DENY, "", "10.1.0.0/16", TCP, 80)
IN3 = lambda: rule(ACTION_DENY, "", "", TCP, 0)
EG1 = lambda: rule(ACTION_PERMIT, "192.168.2.0/24", "", TCP, 23)
EG2 = lambda: rule(ACTION_DENY, "", "", UDP, 0)

SPLIT_UDP = lambda ip: [(ip, 0, "0.0.0.0/1", 0, "UDP", "DENY"), (ip, 0, "128.0.0.0/1", 0, "UDP", "DENY")]
SPLIT_TCP_LOCAL = [("", 0, "0.0.0.0/1", 0, "TCP", "DENY"), ("", 0, "128.0.0.0/1", 0, "TCP", "DENY")]


def test_multiple_rules_single_pod_with_data_change(sink):          # :164-274
    in1, in2, eg1, eg2, in3 = IN1(), IN2(), EG1(), EG2(), IN3()
    rend = V.Renderer(contiv((POD1, POD1_NS)), sink, chan_buf_size=5).init()
    rend.new_txn(False).render(POD1, host(POD1_IP), [in1, in2], [eg1, eg2], False).commit()
    check(sink, 0, 5,
          {POD1_NS: (2, [("", 0, "10.0.0.0/8", 22, "TCP", "DENY"), ("", 0, "10.1.0.0/16", 80, "TCP", "DENY")])},
          (3, [(POD1_IP, 23, "192.168.2.0/24", 0, "TCP", "ALLOW")] + SPLIT_UDP(POD1_IP)))
    rend.new_txn(False).render(POD1, host(POD1_IP), [in1, in3], [eg2], False).commit()
    check(sink, 0, 9, {POD1_NS: (3, [("", 0, "10.0.0.0/8", 22, "TCP", "DENY")] + SPLIT_TCP_LOCAL)},
          (2, SPLIT_UDP(POD1_IP)))


def _two_pods_first_txn(rend, sink):
    in1, in2, eg1, eg2 = IN1(), IN2(), EG1(), EG2()
    txn = rend.new_txn(False)
    txn.render(POD1, host(POD1_IP), [in1, in2], [eg1, eg2], False)
    txn.render(POD2, host(POD2_IP), [in1], [eg2], False)
    txn.commit()
    check(sink, 0, 8,
          {POD1_NS: (2, [("", 0, "10.0.0.0/8", 22, "TCP", "DENY"), ("", 0, "10.1.0.0/16", 80, "TCP", "DENY")]),
           POD2_NS: (1, [("", 0, "10.0.0.0/8", 22, "TCP", "DENY")])},
          (5, [(POD1_IP, 23, "192.168.2.0/24", 0, "TCP", "ALLOW")] + SPLIT_UDP(POD1_IP) + SPLIT_UDP(POD2_IP)))


def _two_pods_second_txn(rend, resync):
    in1, eg2, in3 = IN1(), EG2(), IN3()
    txn = rend.new_txn(resync)
    txn.render(POD1, host(POD1_IP), [in1], [eg2], False)
    txn.render(POD2, host(POD2_IP), [in1, in3], [], False)
    txn.commit()


SECOND_LOCAL = {POD1_NS: (1, [("", 0, "10.0.0.0/8", 22, "TCP", "DENY")]),
                POD2_NS: (3, [("", 0, "10.0.0.0/8", 22, "TCP", "DENY")] + SPLIT_TCP_LOCAL)}


def test_multiple_rules_multiple_pods_with_data_change(sink):       # :276-407
    c = contiv((POD1, POD1_NS), (POD2, POD2_NS))
    rend = V.Renderer(c, sink).init()
    _two_pods_first_txn(rend, sink)
    _two_pods_second_txn(rend, False)
    check(sink, 0, 14, SECOND_LOCAL, (2, SPLIT_UDP(POD1_IP)))


def test_multiple_rules_multiple_pods_with_resync(sink):            # :409-551
    c = contiv((POD1, POD1_NS), (POD2, POD2_NS))
    rend = V.Renderer(c, sink, chan_buf_size=12).init()
    _two_pods_first_txn(rend, sink)
    rend = V.Renderer(c, sink).init()                                # simulate restart (I)
    _two_pods_second_txn(rend, True)
    check(sink, 0, 16, SECOND_LOCAL, (2, SPLIT_UDP(POD1_IP)))


def test_single_pod_with_resync(sink):                              # :553-681
    in1 = rule(ACTION_PERMIT, "", "10.0.0.0/8", TCP, 22)
    in2 = rule(ACTION_PERMIT, "", "10.0.0.0/8", TCP, 23)
    eg1 = rule(ACTION_DENY, "192.168.2.0/24", "", TCP, 80)
    c = contiv((POD1, POD1_NS))
    first = ({POD1_NS: (2, [("", 0, "10.0.0.0/8", 22, "TCP", "ALLOW"), ("", 0, "10.0.0.0/8", 23, "TCP", "ALLOW")])},
             (1, [(POD1_IP, 80, "192.168.2.0/24", 0, "TCP", "DENY")]))
    rend = V.Renderer(c, sink).init()
    rend.new_txn(False).render(POD1, host(POD1_IP), [in1, in2], [eg1], False).commit()
    check(sink, 0, 3, *first)
    rend = V.Renderer(c, sink).init()                                # restart (I)
    rend.new_txn(True).render(POD1, host(POD1_IP), [in1, in2], [eg1], False).commit()
    check(sink, 0, 5, *first)                                        # + dump + ping
    rend = V.Renderer(c, sink).init()                                # restart (II)
    eg2 = rule(ACTION_PERMIT, "192.168.3.0/24", "", UDP, 0)
    rend.new_txn(True).render(POD1, host(POD1_IP), [in2], [eg1, eg2], False).commit()
    check(sink, 0, 9, {POD1_NS: (1, [("", 0, "10.0.0.0/8", 23, "TCP", "ALLOW")])},
          (2, [(POD1_IP, 80, "192.168.2.0/24", 0, "TCP", "DENY"),
               (POD1_IP, 0, "192.168.3.0/24", 0, "UDP", "ALLOW")]))


def test_export_import_round_trip():
    """ImportSessionRules(ExportSessionRules(t)) rebuilds the table in table
    order, the split deny-all merged back into one rule; export drops the
    allow-all and self-destination rules."""
    from vpp_amd.renderer.cache import ContivRuleTable
    c = contiv((POD1, POD1_NS))
    rules = [IN1(), IN2(), IN3(), rule(ACTION_DENY, "", "fd00:10::/64", UDP, 53)]
    dropped = [rule(ACTION_PERMIT, "", "", UDP, 0), rule(ACTION_DENY, "", POD1_IP + "/32", TCP, 8)]
    exported = V.export_session_rules(rules + dropped, POD1, gonet.parse_ip(POD1_IP), c)
    assert len(exported) == 5
    tables = V.import_session_rules(exported, c)
    local = [t for t in tables if t.id != V.GLOBAL_TABLE_ID]
    assert len(local) == 1 and local[0].pods.has(POD1)
    ref = ContivRuleTable("x")
    for r in rules:
        ref.insert_rule(r)
    got = local[0].rules[:local[0].num_of_rules]
    assert [repr(x) for x in got] == [repr(x) for x in ref.rules[:ref.num_of_rules]]


def test_committed_tables_follow_the_cache(sink):
    """With an engine the renderer keeps one compiled table per committed
    IngressOrientation table (pod-group locals + global), replaced on change,
    and one per installed session-rule table (global + per app namespace)."""
    from test_traffic_cpu import _StubEngine
    eng = _StubEngine()
    c = contiv((POD1, POD1_NS), (POD2, POD2_NS))
    rend = V.Renderer(c, sink, engine=eng).init()
    _two_pods_first_txn(rend, sink)
    assert rend.local_rule_table(POD1) is not None and rend.local_rule_table(POD2) is not None
    g = rend.global_rule_table()
    assert [repr(r) for r in g.rules] == [repr(r) for r in rend.cache.get_global_table().rules]
    n_sess = len(rend.sessions.tables)
    assert n_sess == 1 + sum(1 for t in sink.local_table.values() if t)
    assert len(eng.live) == 3 + n_sess
    _two_pods_second_txn(rend, False)
    assert rend.global_rule_table() is not g
    assert len(eng.live) == 3 + len(rend.sessions.tables)
    rend.close()
    assert not eng.live
