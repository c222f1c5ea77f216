"""Replay of the reference's ACL renderer scenarios (tests/golden/acl_scenarios.json).

Mirrors the structure of plugins/policy/renderer/acl/acl_renderer_test.go:
mock Contiv interfaces, a verdict engine, a TxnTracker whose commits go to the
engine's ApplyTxn, the ACL Renderer, renderer transactions and restarts, and
the expectations.  The verdict engine is pluggable: the CPU oracle
(oracle.OracleACLEngine) or the GPU engine (vpp_amd.engine.ACLEngine).
"""
from __future__ import annotations

import json
import os

from vpp_amd import gonet
from vpp_amd.renderer import api
from vpp_amd.renderer.acl import (ACL_NAME_PREFIX, REFLECTIVE_ACL_NAME, ContivIfs, Renderer,
                                  TxnTracker)
from vpp_amd.renderer.cache import GLOBAL_TABLE_ID

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "acl_scenarios.json")
PROTO = {"TCP": 0, "UDP": 1, "ICMP": 2}
CONN = {"DenySyn": 0, "DenySynAck": 1, "Allow": 2, "Failure": 3}


def load_scenarios():
    with open(GOLDEN) as f:
        return json.load(f)["tests"]


def contiv_rule(spec) -> api.ContivRule:
    return api.ContivRule(api.ACTION_PERMIT if spec["action"] == "PERMIT" else api.ACTION_DENY,
                          gonet.ip_network(spec["src"]), gonet.ip_network(spec["dst"]),
                          api.TCP if spec["proto"] == "TCP" else api.UDP,
                          spec["sport"], spec["dport"])


def pod_id(p) -> api.PodID:
    return api.PodID(p["name"], p["namespace"])


def _conn_args(step):
    fn, a = step["fn"], step["args"]
    if fn == "ConnectionPodToPod":
        return fn, (pod_id(a[0]), pod_id(a[1]), PROTO[a[2]], a[3], a[4])
    if fn == "ConnectionPodToInternet":
        return fn, (pod_id(a[0]), a[1], PROTO[a[2]], a[3], a[4])
    return fn, (a[0], pod_id(a[1]), PROTO[a[2]], a[3], a[4])


def replay(test, make_engine, check_conn=None):
    """Run one scenario.  Returns (n_checked, failures).  ``check_conn`` may
    evaluate every expectation of a phase in one batch: it receives the engine
    and a list of (fn, args) and returns a list of ConnectionActions."""
    contiv = ContivIfs()
    engine = None
    tracker = None
    renderer = None
    vpp_acls = []
    failures = []
    checked = 0
    pending_conn = []

    def flush_conns():
        nonlocal checked
        if not pending_conn:
            return
        calls = [_conn_args(s) for s in pending_conn]
        if check_conn is not None:
            got = check_conn(engine, calls)
        else:
            got = [getattr(engine, {"ConnectionPodToPod": "connection_pod_to_pod",
                                    "ConnectionPodToInternet": "connection_pod_to_internet",
                                    "ConnectionInternetToPod": "connection_internet_to_pod"}[fn])(*args)
                   for fn, args in calls]
        for s, g in zip(pending_conn, got):
            checked += 1
            if g != CONN[s["want"]]:
                failures.append("%s:%d %s%s want %s got %s" % (test["name"], s["line"], s["fn"],
                                                              tuple(s["args"]), s["want"], g))
        pending_conn.clear()

    for st in test["steps"]:
        op = st["op"]
        if op != "expect_conn":
            flush_conns()
        if op == "set_main_if":
            contiv.main_if = st["name"]
        elif op == "set_vxlan_if":
            contiv.vxlan_bvi = st["name"]
        elif op == "set_host_if":
            contiv.host_interconnect = st["name"]
        elif op == "set_pod_if":
            contiv.set_pod_if_name(pod_id(st["pod"]), st["if"])
        elif op == "new_engine":
            engine = make_engine(contiv)
        elif op == "register_pod":
            engine.register_pod(pod_id(st["pod"]), st["ip"], st["another_node"])
        elif op == "dump_to_vpp":
            vpp_acls.extend(a.clone() for a in engine.dump_acls())
        elif op == "init_renderer":
            tracker = TxnTracker(engine.apply_txn)
            renderer = Renderer(contiv, tracker.new_linux_data_change_txn,
                                vpp_dump=lambda: list(vpp_acls)).init()
        elif op == "txn":
            txn = renderer.new_txn(st["resync"])
            for r in st["renders"]:
                txn.render(pod_id(r["pod"]), gonet.one_host_subnet(r["ip"]),
                           [contiv_rule(x) for x in r["ingress"]],
                           [contiv_rule(x) for x in r["egress"]], r["removed"])
            txn.commit()
        elif op == "expect_conn":
            pending_conn.append(st)
            continue
        elif op == "expect_num_acls":
            checked += 1
            if engine.get_num_of_acls() != st["n"]:
                failures.append("%s:%d GetNumOfACLs want %d got %d" % (
                    test["name"], st["line"], st["n"], engine.get_num_of_acls()))
        elif op == "expect_num_changes":
            checked += 1
            if engine.get_num_of_acl_changes() != st["n"]:
                failures.append("%s:%d GetNumOfACLChanges want %d got %d" % (
                    test["name"], st["line"], st["n"], engine.get_num_of_acl_changes()))
        elif op == "expect_committed":
            checked += 1
            if len(tracker.committed) != st["n"]:
                failures.append("%s:%d CommittedTxns want %d got %d" % (
                    test["name"], st["line"], st["n"], len(tracker.committed)))
        elif op == "expect_pending":
            checked += 1
            if tracker.pending != st["n"]:
                failures.append("%s:%d PendingTxns want %d got %d" % (
                    test["name"], st["line"], st["n"], tracker.pending))
        elif op == "expect_reflective":
            checked += 1
            err = _verify_reflective(engine, contiv, st["if"], st["on_output_ifs"], st["present"])
            if err:
                failures.append("%s:%d verifyReflectiveACL: %s" % (test["name"], st["line"], err))
        elif op == "expect_global":
            checked += 1
            err = _verify_global(engine, contiv, st["present"])
            if err:
                failures.append("%s:%d verifyGlobalTable: %s" % (test["name"], st["line"], err))
        else:
            raise ValueError(op)
    flush_conns()
    return checked, failures


def _verify_reflective(engine, contiv, if_name, on_output_ifs, present):
    """verifyReflectiveACL (acl_renderer_test.go:51-143), structure subset."""
    ifs = []
    if on_output_ifs:
        ifs = contiv.get_other_physical_if_names() + [contiv.get_vxlan_bvi_if_name(),
                                                      contiv.get_main_physical_if_name(),
                                                      contiv.get_host_interconnect_if_name()]
    ifs.append(if_name)
    acl = engine.get_inbound_acl(if_name)
    if not present:
        return None if acl is None else "expected no inbound ACL"
    if acl is None:
        return "missing inbound ACL"
    if acl.acl_name != ACL_NAME_PREFIX + REFLECTIVE_ACL_NAME:
        return "wrong name %s" % acl.acl_name
    if len(acl.rules) != 3:
        return "expected 3 rules"
    for x in ifs:
        if x not in acl.interfaces.ingress:
            return "missing ingress if %s" % x
    if acl.interfaces.egress:
        return "unexpected egress ifs"
    r1, r2, r3 = acl.rules
    ok = (r1.actions.acl_action == 2 and r1.matches.ip_rule.tcp is not None and
          r1.matches.ip_rule.udp is None and r1.matches.ip_rule.icmp is None and
          r1.matches.ip_rule.tcp.source_port_range.upper_port == 0xFFFF and
          r2.actions.acl_action == 2 and r2.matches.ip_rule.udp is not None and
          r3.actions.acl_action == 2 and r3.matches.ip_rule.icmp is not None and
          r3.matches.ip_rule.icmp.icmp_code_range.last == 5 and
          r3.matches.ip_rule.icmp.icmp_type_range.last == 16)
    return None if ok else "rule content"


def _verify_global(engine, contiv, present):
    """verifyGlobalTable (acl_renderer_test.go:145-164)."""
    ifs = contiv.get_other_physical_if_names() + [contiv.get_vxlan_bvi_if_name(),
                                                  contiv.get_main_physical_if_name(),
                                                  contiv.get_host_interconnect_if_name()]
    acl = engine.get_acl_by_name(ACL_NAME_PREFIX + GLOBAL_TABLE_ID)
    if not present:
        return None if acl is None else "expected no global ACL"
    if acl is None or len(acl.rules) == 0:
        return "missing global ACL"
    if acl.interfaces.ingress:
        return "unexpected ingress"
    if sorted(acl.interfaces.egress) != sorted(ifs):
        return "egress %s != %s" % (acl.interfaces.egress, ifs)
    return None
