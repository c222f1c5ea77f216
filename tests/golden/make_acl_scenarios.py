#!/usr/bin/env python3
"""Generate tests/golden/acl_scenarios.json from the reference's ACL renderer tests.

Run in the build container only (needs /root/reference, which does not
exist on the GPU box):

    python tests/golden/make_acl_scenarios.py /root/reference

It reads plugins/policy/renderer/acl/acl_renderer_test.go as TEXT and
translates its seven test functions (TestEgressRulesOnePod :166 ...
TestCombinedRulesWithRemovedPods :839) statement by statement into a small
step language: mock set-up, renderer transactions, simulated restarts and
every expectation (Connection* verdicts, ACL counts, change counts,
reflective/global ACL presence).  The rule sets Ts3/Ts4/Ts5 and the pod data
of plugins/policy/renderer/testdata/testdata.go:24-253 are transcribed below
as data.  Output: inputs and expected outputs only -- no reference source.
"""
import json
import os
import re
import sys

# --- testdata.go:24-80 -------------------------------------------------------
PODS = {"Pod%d" % (i + 1): {"name": "pod%d" % (i + 1),
                             "namespace": "default" if i < 5 else "namespace2"}
        for i in range(6)}
POD_IPS = {"Pod1IP": "10.10.1.1", "Pod2IP": "10.10.1.2", "Pod3IP": "10.10.2.1",
           "Pod4IP": "10.10.2.2", "Pod5IP": "10.10.2.3", "Pod6IP": "10.10.10.1"}
POD_IFS = {"Pod1IfName": "node1-tap1", "Pod2IfName": "node1-tap2", "Pod3IfName": "node1-tap3",
           "Pod4IfName": "node1-tap4", "Pod5IfName": "node1-tap5", "Pod6IfName": "node2-tap1"}
CONSTS = {"mainIfName": "GbE", "vxlanIfName": "VXLAN-BVI", "hostInterIfName": "VPP-Host",
          "googleDNS": "8.8.8.8", "somePort": 500, "somePort2": 600}


def R(action, src, dst, proto, sport, dport):
    return {"action": action, "src": src, "dst": dst, "proto": proto, "sport": sport,
            "dport": dport}


DENY_ALL_TCP = R("DENY", "", "", "TCP", 0, 0)     # testdata.go:289-299
DENY_ALL_UDP = R("DENY", "", "", "UDP", 0, 0)     # testdata.go:301-311
RULES = {                                         # testdata.go:87-156
    "Ts1.Rule": R("PERMIT", "192.168.0.0/16", "", "TCP", 0, 80),
    "Ts2.Rule": R("PERMIT", "", "192.168.0.0/16", "TCP", 0, 80),
    "Ts3.Rule1": R("PERMIT", "10.10.0.0/16", "", "TCP", 0, 0),
    "Ts3.Rule2": R("PERMIT", "10.10.0.0/16", "", "UDP", 0, 0),
    "Ts3.Rule3": DENY_ALL_TCP, "Ts3.Rule4": DENY_ALL_UDP,
    "Ts4.Rule1": R("PERMIT", "", "10.10.0.0/16", "TCP", 0, 0),
    "Ts4.Rule2": R("PERMIT", "", "10.10.0.0/16", "UDP", 0, 0),
    "Ts4.Rule3": DENY_ALL_TCP, "Ts4.Rule4": DENY_ALL_UDP,
}
RULE_LISTS = {                                    # testdata.go:164-253
    "Ts5.Pod1Ingress": [R("PERMIT", "", "10.10.0.0/16", "TCP", 0, 80),
                        R("PERMIT", "", "", "UDP", 0, 161), DENY_ALL_TCP, DENY_ALL_UDP],
    "Ts5.Pod1Egress": [R("PERMIT", "10.0.0.0/8", "", "UDP", 0, 53),
                       R("PERMIT", "192.168.0.0/16", "", "UDP", 0, 514), DENY_ALL_TCP, DENY_ALL_UDP],
    "Ts5.Pod3Ingress": [R("PERMIT", "", "10.10.1.1/32", "UDP", 0, 0),
                        R("PERMIT", "", "", "TCP", 0, 22), DENY_ALL_TCP, DENY_ALL_UDP],
    "Ts5.Pod3Egress": [R("PERMIT", "10.0.0.0/8", "", "TCP", 0, 80),
                       R("PERMIT", "10.0.0.0/8", "", "TCP", 0, 443),
                       R("PERMIT", "", "", "UDP", 0, 67), DENY_ALL_TCP, DENY_ALL_UDP],
}
CONN = {"ConnActionDenySyn": "DenySyn", "ConnActionDenySynAck": "DenySynAck",
        "ConnActionAllow": "Allow", "ConnActionFailure": "Failure"}


def rule_list(expr, env):
    expr = re.sub(r"/\*.*?\*/", "", expr).strip()
    if expr in env:
        return env[expr]
    m = re.fullmatch(r"\[\]\*renderer\.ContivRule\{(.*)\}", expr)
    if m:
        items = [x.strip() for x in m.group(1).split(",") if x.strip()]
        return [RULES[x] for x in items]
    m = re.fullmatch(r"(Ts5\.\w+)(\[(\d*):(\d*)\])?", expr)
    if m:
        lst = RULE_LISTS[m.group(1)]
        if m.group(2):
            lo = int(m.group(3)) if m.group(3) else 0
            hi = int(m.group(4)) if m.group(4) else len(lst)
            lst = lst[lo:hi]
        return list(lst)
    m = re.fullmatch(r"(\w+)\.(Ingress|Egress)", expr)
    if m:
        return env[m.group(1)][m.group(2).lower()]
    raise ValueError("rule list: %r" % expr)


def pod_ip(expr, env):
    m = re.fullmatch(r"GetOneHostSubnet\((\w+)\)", expr.strip())
    if m:
        return POD_IPS[m.group(1)]
    m = re.fullmatch(r"(\w+)\.PodIP", expr.strip())
    if m:
        return env[m.group(1)]["ip"]
    raise ValueError(expr)


def val(tok):
    tok = tok.strip()
    if tok in PODS:
        return PODS[tok]
    if tok in POD_IPS:
        return POD_IPS[tok]
    if tok in POD_IFS:
        return POD_IFS[tok]
    if tok in CONSTS:
        return CONSTS[tok]
    if tok in ("TCP", "UDP", "ICMP"):
        return tok
    if tok.startswith('"'):
        return tok.strip('"')
    return int(tok)


def split_args(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out]


def translate(src_text):
    lines = src_text.split("\n")
    tests = []
    cur = None
    env = {}
    pending_txn = None
    i = 0
    while i < len(lines):
        raw = lines[i]
        lineno = i + 1
        line = raw.strip()
        i += 1
        m = re.match(r"func (Test\w+)\(t \*testing\.T\)", line)
        if m:
            cur = {"name": m.group(1), "line": lineno, "steps": []}
            tests.append(cur)
            env = {}
            continue
        if cur is None or line.startswith("//") or not line:
            continue
        steps = cur["steps"]
        # multi-line PodConfig literal
        m = re.match(r"(\w+) := &cache\.PodConfig\{", line)
        if m:
            body = ""
            while not lines[i].strip().startswith("}"):
                body += lines[i].strip()
                i += 1
            i += 1
            fields = dict(re.findall(r"(\w+):\s*([^,]+),", body))
            env[m.group(1)] = {"ip": pod_ip(fields["PodIP"], env),
                               "ingress": rule_list(fields["Ingress"], env),
                               "egress": rule_list(fields["Egress"], env)}
            continue
        m = re.match(r"(ingress|egress) := (.*)$", line)
        if m:
            env[m.group(1)] = rule_list(m.group(2), env)
            continue
        m = re.match(r"contiv\.Set(MainPhysicalIfName|VxlanBVIIfName|HostInterconnectIfName)\((\w+)\)", line)
        if m:
            steps.append({"op": "set_" + {"MainPhysicalIfName": "main_if", "VxlanBVIIfName": "vxlan_if",
                                          "HostInterconnectIfName": "host_if"}[m.group(1)],
                          "name": val(m.group(2))})
            continue
        m = re.match(r"contiv\.SetPodIfName\((\w+), (\w+)\)", line)
        if m:
            steps.append({"op": "set_pod_if", "pod": val(m.group(1)), "if": val(m.group(2))})
            continue
        m = re.match(r"aclEngine\.RegisterPod\((\w+), (\w+), (true|false)\)", line)
        if m:
            steps.append({"op": "register_pod", "pod": val(m.group(1)), "ip": val(m.group(2)),
                          "another_node": m.group(3) == "true"})
            continue
        if re.match(r"aclEngine := NewMockACLEngine", line):
            steps.append({"op": "new_engine"})
            continue
        if line.startswith("acls := aclEngine.DumpACLs()"):
            steps.append({"op": "dump_to_vpp"})
            continue
        if line.startswith("aclRenderer.Init()"):
            steps.append({"op": "init_renderer"})
            continue
        # one-shot txn: [err :=|err =] aclRenderer.NewTxn(b).Render(args).Commit()
        m = re.match(r"err :?= aclRenderer\.NewTxn\((true|false)\)\.Render\((.*)\)\.Commit\(\)$", line)
        if m:
            a = split_args(m.group(2))
            steps.append({"op": "txn", "resync": m.group(1) == "true", "line": lineno,
                          "renders": [{"pod": val(a[0]), "ip": pod_ip(a[1], env),
                                       "ingress": rule_list(a[2], env), "egress": rule_list(a[3], env),
                                       "removed": a[4] == "true"}]})
            continue
        m = re.match(r"txn :?= aclRenderer\.NewTxn\((true|false)\)$", line)
        if m:
            pending_txn = {"op": "txn", "resync": m.group(1) == "true", "renders": []}
            continue
        m = re.match(r"txn\.Render\((.*)\)$", line)
        if m:
            a = split_args(m.group(1))
            pending_txn["renders"].append({"pod": val(a[0]), "ip": pod_ip(a[1], env),
                                           "ingress": rule_list(a[2], env),
                                           "egress": rule_list(a[3], env),
                                           "removed": a[4] == "true"})
            continue
        if re.match(r"err :?= txn\.Commit\(\)$", line):
            pending_txn["line"] = lineno
            steps.append(pending_txn)
            pending_txn = None
            continue
        m = re.match(r"gomega\.Expect\(aclEngine\.(Connection\w+)\((.*)\)\)\.To\(gomega\.Equal\((\w+)\)\)", line)
        if m:
            a = [val(x) for x in split_args(m.group(2))]
            steps.append({"op": "expect_conn", "fn": m.group(1), "args": a,
                          "want": CONN[m.group(3)], "line": lineno})
            continue
        m = re.match(r"gomega\.Expect\(aclEngine\.(GetNumOfACLs|GetNumOfACLChanges)\(\)\)\.To\(gomega\.Equal\((\d+)\)\)", line)
        if m:
            steps.append({"op": "expect_" + {"GetNumOfACLs": "num_acls",
                                             "GetNumOfACLChanges": "num_changes"}[m.group(1)],
                          "n": int(m.group(2)), "line": lineno})
            continue
        m = re.match(r"gomega\.Expect\(txnTracker\.CommittedTxns\)\.To\(gomega\.HaveLen\((\d+)\)\)", line)
        if m:
            steps.append({"op": "expect_committed", "n": int(m.group(1)), "line": lineno})
            continue
        m = re.match(r"gomega\.Expect\(txnTracker\.PendingTxns\)\.To\(gomega\.HaveLen\((\d+)\)\)", line)
        if m:
            steps.append({"op": "expect_pending", "n": int(m.group(1)), "line": lineno})
            continue
        m = re.match(r"verifyReflectiveACL\(aclEngine, contiv, (\w+|\"\"), (true|false), (true|false)\)", line)
        if m:
            steps.append({"op": "expect_reflective", "if": val(m.group(1)),
                          "on_output_ifs": m.group(2) == "true", "present": m.group(3) == "true",
                          "line": lineno})
            continue
        m = re.match(r"verifyGlobalTable\(aclEngine, contiv, (true|false)\)", line)
        if m:
            steps.append({"op": "expect_global", "present": m.group(1) == "true", "line": lineno})
            continue
    return tests


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    path = os.path.join(ref, "plugins/policy/renderer/acl/acl_renderer_test.go")
    with open(path) as f:
        tests = translate(f.read())
    n_conn = sum(1 for t in tests for s in t["steps"] if s["op"] == "expect_conn")
    out = {"source": "plugins/policy/renderer/acl/acl_renderer_test.go",
           "generator": "tests/golden/make_acl_scenarios.py",
           "n_tests": len(tests), "n_connection_expectations": n_conn, "tests": tests}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "acl_scenarios.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote %s: %d tests, %d Connection* expectations" % (dst, len(tests), n_conn))


if __name__ == "__main__":
    main()
