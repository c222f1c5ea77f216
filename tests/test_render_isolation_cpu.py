"""Rendered ACLs do not depend on process history.

Go's renderACL allocates fresh rule messages per call
(plugins/policy/renderer/acl/acl_renderer.go:319-335), so nothing a caller
does with one rendered or dumped ACL can change another render.  These tests
pin that for the restatement: the benchmark tables rendered in one process in
the order 5, 2, 3 equal their fresh-interpreter digests
(tests/golden/rule_list_hashes.json, tests/golden/make_rule_hashes.py), and
editing rendered / dumped ACLs in place leaves later renders unchanged.
"""
import copy
import json
import os

import pytest

from rule_hash import rule_list_digest
from vpp_amd import gonet, model, workload
from vpp_amd.renderer import api
from vpp_amd.renderer.acl import ContivIfs, Renderer, TxnTracker, render_acl
from vpp_amd.renderer.cache import ContivRuleTable

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rule_list_hashes.json")


def _golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_configs_rendered_in_one_process_match_fresh_digests():
    want = _golden()
    for cfg in (5, 2, 3, 5):      # config 5 widens its own ports; it must not leak into 2 or 3
        acl, _, _ = workload.config(cfg)
        assert len(acl.rules) == want[str(cfg)]["n_rules"]
        assert rule_list_digest(acl.rules) == want[str(cfg)]["sha256"], "config %d" % cfg


def _table(rules, tid="T1"):
    t = ContivRuleTable(tid)
    for r in rules:
        t.insert_rule(r)
    return t


def _rules():
    net = gonet.ip_network
    return [api.ContivRule(api.ACTION_PERMIT, net("10.1.1.1/32"), net("192.168.0.0/16"), api.TCP, 0, 80),
            api.ContivRule(api.ACTION_DENY, net("10.1.1.1/32"), gonet.IPNet(), api.UDP, 0, 53),
            api.deny_all_tcp(), api.deny_all_udp()]


def _edits(r):
    """Every in-place edit of one rule message's fields."""
    ipr = r.matches.ip_rule
    sec = ipr.tcp or ipr.udp
    dpr, spr = sec.destination_port_range, sec.source_port_range
    return [lambda: setattr(r.actions, "acl_action", 2),
            lambda: setattr(ipr.ip, "source_network", "1.2.3.4/32"),
            lambda: setattr(ipr.ip, "destination_network", "5.6.7.8/32"),
            lambda: setattr(dpr, "lower_port", 7),
            lambda: setattr(dpr, "upper_port", 9),
            lambda: setattr(spr, "lower_port", 1),
            lambda: setattr(sec, "destination_port_range", None),
            lambda: setattr(ipr, "tcp", None),
            lambda: setattr(r, "actions", None)]


def _scribble(acl):
    """Try every in-place edit of every rule: a shared rendered rule refuses
    each one (FrozenMessageError); the renderer's own trailing ICMP rule and
    deep copies are editable and may be edited."""
    for r in acl.rules:
        if r.matches.ip_rule.icmp is not None:
            r.actions.acl_action = 2
            continue
        for e in _edits(r):
            with pytest.raises(model.FrozenMessageError):
                e()
        c = copy.deepcopy(r)
        assert c == r
        for e in _edits(c):
            e()
        assert c != r


def test_editing_a_rendered_acl_does_not_change_a_later_render():
    first = render_acl(_table(_rules()), None)
    pristine = copy.deepcopy(first)
    _scribble(first)
    again = render_acl(_table(_rules(), "T2"), None)
    assert rule_list_digest(again.rules) == rule_list_digest(pristine.rules)


def test_workload_widening_does_not_touch_shared_rules():
    a5, _, _ = workload.config(5)
    assert any(type(r) is model.Rule for r in a5.rules)          # the widened copies
    # every point dst range of a shared (read-only) rule is still a point
    for r in a5.rules:
        if type(r) is not model.Rule:
            pr = (r.matches.ip_rule.tcp or r.matches.ip_rule.udp).destination_port_range
            assert pr.lower_port == 0 or pr.lower_port != pr.upper_port or \
                workload.port_range_of(pr.lower_port)[1] == pr.lower_port


class _PointerEngine:
    """Stores the ACL messages it is given, as MockACLEngine.PutACL stores the
    *AccessLists_Acl pointer (mock/aclengine/aclengine_mock.go:713)."""

    def __init__(self):
        self.by_name = {}

    def apply_txn(self, ops):
        for key, value in ops:
            name = key.split("/")[-1] if value is None else value.acl_name
            if value is None:
                self.by_name.pop(name, None)
            else:
                self.by_name[name] = value
        return None

    def dump_acls(self):
        return list(self.by_name.values())

    def get_acl_by_name(self, name):
        return self.by_name.get(name)


def _commit(renderer, pods):
    txn = renderer.new_txn(True)
    for pod, ip, ingress in pods:
        txn.render(pod, gonet.one_host_subnet(ip), ingress, [], False)
    txn.commit()


def test_editing_dumped_acls_does_not_change_a_later_render():
    contiv = ContivIfs(main_if="GbE", vxlan_bvi="VXLAN-BVI", host_interconnect="VPP-Host")
    pods = []
    for k in range(4):
        pod = api.PodID("pod%d" % k, "default")
        contiv.set_pod_if_name(pod, "tap%d" % k)
        pods.append((pod, "10.1.1.%d" % (k + 1), _rules()[:1] + [api.deny_all_tcp(), api.deny_all_udp()]))

    def run(scribble_between):
        eng = _PointerEngine()
        r = Renderer(contiv, TxnTracker(eng.apply_txn).new_linux_data_change_txn).init()
        _commit(r, pods)
        before = sorted(rule_list_digest(a.rules) for a in eng.dump_acls())
        if scribble_between:
            for a in eng.dump_acls():
                _scribble(a)
            _scribble(eng.get_acl_by_name(sorted(eng.by_name)[0]))
        # a second renderer over the same pods renders every table again
        eng2 = _PointerEngine()
        r2 = Renderer(contiv, TxnTracker(eng2.apply_txn).new_linux_data_change_txn).init()
        _commit(r2, pods)
        # table ids come from a process-wide counter, so compare the rule lists
        return before, sorted(rule_list_digest(a.rules) for a in eng2.dump_acls())

    clean_before, clean_after = run(False)
    before, after = run(True)
    assert clean_before == clean_after == before == after
    assert len(after) >= 3
