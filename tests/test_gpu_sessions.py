"""GPU: installed VPP session rules evaluated on packets.

vpp_amd.renderer.sessions runs each session-rule table of the sink on the
classifier; verdicts and per-session-rule hits must equal the literal
restatement oracle/sessions.py (parity unpinned) on random
exported tables, and the same compiled list under the C evalACL oracle on the
config-5 global table exported as session rules (mixed IPv4 / IPv6 pods).
The VPPTCP renderer keeps an evaluator of its sink after every commit.
"""
import random

import numpy as np
import pytest

import oracle
from oracle import sessions as osess
from test_sessions_cpu import _Contiv, gpu_form_on_cpu, installed, packets

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from vpp_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("scope", ["global", "local"])
def test_session_tables_on_gpu_match_oracle(eng, seed, scope):
    from vpp_amd.renderer.sessions import SessionEvaluator
    rng = random.Random(100 + seed)
    sink, rules = installed(rng, 80, bytes([10, 1, 1, rng.randrange(1, 255)]), scope)
    ns = None if scope == "global" else 7
    table = sink.global_table if ns is None else sink.local_table.get(ns, [])
    if not table:
        pytest.skip("nothing installed")
    ev = SessionEvaluator(eng, sink)
    try:
        ev.sync()
        s16, d16, p8, dp16 = packets(rng, rules, 4000)
        v, hits, unmatched = ev.evaluate(ns, s16, d16, p8, dp16)
        ov, oh, ou = osess.evaluate(table, list(s16), list(d16), p8, dp16)
        assert np.array_equal(v, np.array(ov, np.uint8))
        assert hits.tolist() == oh and unmatched == ou
    finally:
        ev.close()


def test_config5_global_table_as_session_rules(eng):
    """The config-5 global ContivRule table (1000 pods, half IPv6) exported to
    session rules and evaluated on 16-byte packets of the config-5 stream."""
    from vpp_amd import gonet, workload
    from vpp_amd.renderer.cache import build_global_table
    from vpp_amd.renderer.sessions import SessionEvaluator
    from vpp_amd.renderer.vpptcp import SessionRuleTables, export_session_rules
    c = workload.CONFIGS[5]
    rng = random.Random(5)
    cidrs, cidrs6 = workload.service_cidrs(rng), workload.service_cidrs6(rng)
    apps = [workload.app_rules(rng, cidrs6 if a % 2 else cidrs, c["rules_per_pod"]) for a in range(c["n_apps"])]
    pods = []
    for k in range(c["n_pods"]):
        v6 = (k % c["n_apps"]) % 2 == 1
        ip = gonet.one_host_subnet(workload._v6(workload.pod_ip6(k)) if v6 else workload._v4(workload.pod_ip(k)))
        pods.append((ip, apps[k % c["n_apps"]]))
    table = build_global_table(pods)
    sink = SessionRuleTables()
    for sr in export_session_rules(table.rules, None, None, _Contiv({})):
        sink.add_del(sr, True)
    assert len(sink.global_table) > 5000
    _, spec, _ = workload.config(5)
    tr = oracle.gen_traffic_v16(spec, 0, 1 << 14)
    s16, d16 = tr["src"].reshape(-1, 16), tr["dst"].reshape(-1, 16)
    # destinations on the pods: the global table is about traffic into them
    d16 = s16[::-1].copy()
    ev = SessionEvaluator(eng, sink)
    try:
        ev.sync()
        v, hits, unmatched = ev.evaluate(None, s16, d16, tr["proto"], tr["dport"])
        wv, wh, wu = gpu_form_on_cpu(sink.global_table, s16, d16, tr["proto"], tr["dport"])
        assert np.array_equal(v, wv)
        assert np.array_equal(hits, wh) and unmatched == wu
        assert len(set(v.tolist())) == 2
    finally:
        ev.close()


def test_vpptcp_renderer_keeps_session_evaluator(eng):
    """A VPPTCP renderer with an engine evaluates what its sink holds."""
    from vpp_amd import gonet
    from vpp_amd.renderer.acl import ContivIfs
    from vpp_amd.renderer.api import ACTION_DENY, TCP, ContivRule, PodID
    from vpp_amd.renderer.vpptcp import Renderer, SessionRuleTables
    contiv = ContivIfs()
    pod = PodID("web", "default")
    contiv.set_pod_app_ns_index(pod, 4)
    sink = SessionRuleTables()
    r = Renderer(contiv, sink, engine=eng).init()
    try:
        deny = ContivRule(ACTION_DENY, gonet.IPNet(), gonet.IPNet(), TCP, 0, 0)
        r.new_txn(False).render(pod, gonet.one_host_subnet("10.1.1.3"), [deny], [deny], False).commit()
        assert r.sessions is not None and None in r.sessions.tables
        a16 = lambda xs: np.frombuffer(b"".join(xs), np.uint8).reshape(-1, 16)
        v4 = bytes(10) + b"\xff\xff" + bytes([10, 1, 1, 3])
        v6 = bytes.fromhex("fd000010000000000000000000000003")
        for ns in r.sessions.tables:
            v, _, _ = r.sessions.evaluate(ns, a16([v4, v6]), a16([v4, v6]), np.zeros(2, np.uint8),
                                          np.full(2, 80, np.uint16))
            want, _, _ = osess.evaluate(sink.global_table if ns is None else sink.local_table[ns],
                                        [v4, v6], [v4, v6], [0, 0], [80, 80])
            assert list(v) == want
    finally:
        r.close()
