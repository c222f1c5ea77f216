"""Installed VPP session rules evaluated on packets, on CPU.

vpp_amd/renderer/sessions.py turns a session-rule table into the rule list
the GPU classifier runs (TestTraffic's ACL form, vpp_amd/renderer/traffic.py);
here that list is evaluated by the C evalACL oracle and compared with the
literal per-packet restatement oracle/sessions.py (parity unpinned: the
reference has no session-rule evaluator).  The export's own
effects (session_rule.go:201-331) are checked where they change verdicts: the
deny-all split into 0.0.0.0/1 + 128.0.0.0/1 covers IPv4 only, allow-all and
self rules are not installed.
"""
import random

import numpy as np
import pytest

import oracle
from oracle import sessions as osess
from vpp_amd import gonet
from vpp_amd.gonet import IPNet
from vpp_amd.renderer import sessions as S
from vpp_amd.renderer import traffic as T
from vpp_amd.renderer.api import ACTION_DENY, ACTION_PERMIT, TCP, UDP, ContivRule, PodID
from vpp_amd.renderer.vpptcp import SessionRuleTables, export_session_rules


class _Contiv:
    def __init__(self, ns):
        self.ns = ns

    def get_ns_index(self, namespace, name):
        pod = PodID(name, namespace)
        return self.ns.get(pod, 0), pod in self.ns


def _net(rng, fam4):
    if rng.random() < 0.25:
        return IPNet()
    if fam4:
        ones = rng.choice([8, 16, 24, 28, 32])
        ip = bytes([10, rng.randrange(4), rng.randrange(4), rng.randrange(256)])
        return IPNet(ip, gonet.cidr_mask(ones, 32))
    ones = rng.choice([16, 48, 64, 120, 128])
    ip = bytes([0xFD, 0, 0, 0x10] + [0] * 10 + [rng.randrange(4), rng.randrange(256)])
    return IPNet(ip, gonet.cidr_mask(ones, 128))


def random_contiv_rules(rng, n):
    out = []
    for _ in range(n):
        fam4 = rng.random() < 0.6
        out.append(ContivRule(ACTION_PERMIT if rng.random() < 0.5 else ACTION_DENY, _net(rng, fam4),
                              _net(rng, fam4), rng.choice([TCP, UDP]), 0,
                              rng.choice([0, 0, 22, 53, 80, 443])))
    return out


def installed(rng, n_rules, pod_ip=None, scope="global"):
    """A sink holding the export of a random ContivRule table."""
    sink = SessionRuleTables()
    pod = PodID("p", "default")
    contiv = _Contiv({pod: 7})
    rules = random_contiv_rules(rng, n_rules)
    for sr in export_session_rules(rules, None if scope == "global" else pod, pod_ip, contiv):
        sink.add_del(sr, True)
    return sink, rules


def packets(rng, rules, n):
    """16-byte packets near the rules' networks, both families, protocols 0-3."""
    src, dst, proto, dport = [], [], [], []
    for _ in range(n):
        r = rng.choice(rules)
        out = []
        for net in (r.src_network, r.dest_network):
            if len(net.ip) == 0 or rng.random() < 0.2:
                fam4 = rng.random() < 0.5
                a = (bytes(10) + b"\xff\xff" + bytes([10, rng.randrange(4), rng.randrange(4), rng.randrange(256)])
                     if fam4 else bytes([0xFD, 0, 0, 0x10] + [0] * 10 + [rng.randrange(4), rng.randrange(256)]))
            else:
                ip = gonet.to16(net.ip)
                m = net.mask if len(net.mask) == 16 else b"\xff" * 12 + net.mask
                a = bytes((x & k) | (rng.randrange(256) & ~k & 0xFF) for x, k in zip(ip, m))
            out.append(a)
        src.append(out[0])
        dst.append(out[1])
        proto.append(r.protocol if rng.random() < 0.85 else rng.choice([0, 1, 2, 3]))
        dport.append(r.dest_port if r.dest_port and rng.random() < 0.7 else rng.choice([22, 53, 80, 443, 999]))
    a16 = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(-1, 16)
    return a16(src), a16(dst), np.array(proto, np.uint8), np.array(dport, np.uint16)


def gpu_form_on_cpu(table_rules, s16, d16, p8, dp16):
    """The GPU path's list, evaluated by the C evalACL oracle instead of the
    classifier: (session verdicts, hits per session rule, unmatched)."""
    rl, origin = S.ordered(table_rules)
    v, c = oracle.classify_faithful(oracle.rules_to_c(T.compile_rules(rl)), s16, d16, dp16, p8, af=16)
    per_rule, unmatched = T.rule_counters(c, len(rl))
    hits = np.zeros(len(table_rules), np.uint64)
    for i, k in enumerate(origin):
        hits[k] += np.uint64(per_rule[i])
    return np.where(v == T.DENIED_TRAFFIC, S.SESSION_DENY, S.SESSION_ALLOW), hits, unmatched


@pytest.mark.parametrize("seed", range(10))
@pytest.mark.parametrize("scope", ["global", "local"])
def test_compiled_session_tables_match_oracle(seed, scope):
    rng = random.Random(seed)
    pod_ip = bytes([10, 1, 1, rng.randrange(1, 255)])
    sink, rules = installed(rng, 60, pod_ip, scope)
    table = sink.global_table if scope == "global" else sink.local_table.get(7, [])
    if not table:
        pytest.skip("nothing installed")
    s16, d16, p8, dp16 = packets(rng, rules, 3000)
    v, hits, unmatched = gpu_form_on_cpu(table, s16, d16, p8, dp16)
    ov, oh, ou = osess.evaluate(table, list(s16), list(d16), p8, dp16)
    assert np.array_equal(v, np.array(ov, np.uint8))
    assert hits.tolist() == oh and unmatched == ou
    assert len(set(ov)) == 2


def _sink_of(rules, pod=None, pod_ip=None):
    sink = SessionRuleTables()
    contiv = _Contiv({PodID("p", "default"): 3})
    for sr in export_session_rules(rules, pod, pod_ip, contiv):
        sink.add_del(sr, True)
    return sink


def test_deny_all_split_covers_ipv4_only():
    """An empty remote network exports as 0.0.0.0/1 + 128.0.0.0/1 (IsIP4):
    an IPv6 source is not denied by the global deny-all, an IPv4 one is."""
    dst = gonet.ip_network("fd00:10::5/128")
    dst4 = gonet.ip_network("10.1.1.5/32")
    rules = [ContivRule(ACTION_DENY, IPNet(), dst4, TCP, 0, 0), ContivRule(ACTION_DENY, IPNet(), dst, TCP, 0, 0)]
    sink = _sink_of(rules)
    assert len(sink.global_table) == 4                       # two split pairs
    v6 = bytes.fromhex("fd000010000000000000000000000005")
    s6 = bytes.fromhex("fd000010000000000000000000000099")
    v4 = bytes(10) + b"\xff\xff" + bytes([10, 1, 1, 5])
    s4 = bytes(10) + b"\xff\xff" + bytes([10, 9, 9, 9])
    a16 = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(-1, 16)
    src, dst_ = a16([s4, s6, s6]), a16([v4, v6, v4])
    p8, dp = np.zeros(3, np.uint8), np.array([80, 80, 80], np.uint16)
    v, _, _ = gpu_form_on_cpu(sink.global_table, src, dst_, p8, dp)
    ov, _, _ = osess.evaluate(sink.global_table, list(src), list(dst_), p8, dp)
    assert list(v) == ov == [S.SESSION_DENY, S.SESSION_ALLOW, S.SESSION_ALLOW]
    # the ContivRule list itself (TestTraffic) denies the IPv6 packet
    tv, _ = oracle.classify_faithful(oracle.rules_to_c(T.compile_rules(rules)), src, dst_, dp, p8, af=16)
    assert tv[1] == T.DENIED_TRAFFIC


def test_self_and_allow_all_rules_not_installed():
    pod, ip = PodID("p", "default"), bytes([10, 1, 1, 7])
    rules = [ContivRule(ACTION_DENY, IPNet(), gonet.ip_network("10.1.1.7/32"), TCP, 0, 80),   # self
             ContivRule(ACTION_PERMIT, IPNet(), IPNet(), UDP, 0, 0),                          # allow-all
             ContivRule(ACTION_DENY, IPNet(), gonet.ip_network("10.2.0.0/16"), TCP, 0, 0)]
    sink = _sink_of(rules, pod, ip)
    table = sink.local_table[3]
    assert len(table) == 1
    a16 = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(-1, 16)
    me = bytes(10) + b"\xff\xff" + ip
    src = a16([me, me, me])
    dst = a16([me, bytes(10) + b"\xff\xff" + bytes([10, 2, 3, 4]), bytes(10) + b"\xff\xff" + bytes([8, 8, 8, 8])])
    p8, dp = np.array([0, 0, 1], np.uint8), np.array([80, 80, 53], np.uint16)
    v, _, _ = gpu_form_on_cpu(table, src, dst, p8, dp)
    ov, _, _ = osess.evaluate(table, list(src), list(dst), p8, dp)
    assert list(v) == ov == [S.SESSION_ALLOW, S.SESSION_DENY, S.SESSION_ALLOW]


def test_icmp_and_other_protocols_are_allowed():
    rules = [ContivRule(ACTION_DENY, IPNet(), IPNet(), TCP, 0, 0), ContivRule(ACTION_DENY, IPNet(), IPNet(), UDP, 0, 0)]
    sink = _sink_of(rules)
    a16 = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(-1, 16)
    a = bytes(10) + b"\xff\xff" + bytes([10, 0, 0, 1])
    src = dst = a16([a] * 4)
    p8, dp = np.array([0, 1, 2, 47], np.uint8), np.full(4, 80, np.uint16)
    v, _, _ = gpu_form_on_cpu(sink.global_table, src, dst, p8, dp)
    ov, _, _ = osess.evaluate(sink.global_table, list(src), list(dst), p8, dp)
    assert list(v) == ov == [S.SESSION_DENY, S.SESSION_DENY, S.SESSION_ALLOW, S.SESSION_ALLOW]
