#!/usr/bin/env python3
"""Generate tests/golden/configurator_scenarios.json from the reference's configurator tests.

Run in the build container only (needs /root/reference, which does not
exist on the GPU box):

    python tests/golden/make_configurator_scenarios.py /root/reference

It reads plugins/policy/configurator/configurator_test.go as TEXT and turns
each of its test functions (TestSinglePolicySinglePod :47 ...
TestMultiplePodsSpecialCases :1225) into data: the pods and addresses put
into the mock policy cache, the ContivPolicy literals (parsed by a small
Go composite-literal reader below), the configurator/renderer steps in
source order, and every expectation -- GetPodIP address + mask length and
each TestTraffic verdict with its source line.  Output: inputs and expected
outputs only -- no reference source.
"""
import json
import os
import re
import sys

TEST_FILE = "plugins/policy/configurator/configurator_test.go"


def strip_comments(text):
    text = re.sub(r"/\*.*?\*/", lambda m: " " * len(m.group(0)) if "\n" not in m.group(0)
                  else "\n" * m.group(0).count("\n"), text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


# --- Go composite literal reader ------------------------------------------------
_TOK = re.compile(r'\s*(\[\]\*?|[{}(),:&*]|"[^"]*"|[A-Za-z_][\w.]*|\d+)')


def tokenize(s):
    out, pos = [], 0
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m:
            if s[pos:].strip() == "":
                break
            raise ValueError("cannot tokenize at %r" % s[pos:pos + 30])
        out.append(m.group(1))
        pos = m.end()
    return out


class Lit:
    def __init__(self, type_, keyed, items):
        self.type, self.keyed, self.items = type_, keyed, items


def parse_value(toks, i):
    """-> (value, next index).  Values: Lit, ('id', name), ('str', s), ('num', n),
    ('call', fn, arg)."""
    if toks[i] == "&":
        i += 1
    type_ = None
    if toks[i].startswith("[]"):
        type_ = toks[i] + toks[i + 1]
        i += 2
    elif toks[i] != "{" and i + 1 < len(toks) and toks[i + 1] == "{" and re.match(r"[A-Za-z_]", toks[i]):
        type_ = toks[i]
        i += 1
    if toks[i] == "{":
        i += 1
        items, keyed = [], None
        while toks[i] != "}":
            if i + 1 < len(toks) and toks[i + 1] == ":" and re.match(r"[A-Za-z_]\w*$", toks[i]):
                key = toks[i]
                v, i = parse_value(toks, i + 2)
                items.append((key, v))
                keyed = True
            else:
                v, i = parse_value(toks, i)
                items.append(v)
                keyed = False if keyed is None else keyed
            if toks[i] == ",":
                i += 1
        return Lit(type_, bool(keyed), items), i + 1
    t = toks[i]
    if t.startswith('"'):
        return ("str", t[1:-1]), i + 1
    if t.isdigit():
        return ("num", int(t)), i + 1
    if i + 1 < len(toks) and toks[i + 1] == "(":
        arg, j = parse_value(toks, i + 2)
        assert toks[j] == ")", toks[j:j + 3]
        return ("call", t, arg), j + 1
    return ("id", t), i + 1


def literal_at(body, start):
    """The balanced {...} literal that begins at the first '{' at/after start."""
    i = body.index("{", start)
    depth = 0
    for j in range(i, len(body)):
        depth += {"{": 1, "}": -1}.get(body[j], 0)
        if depth == 0:
            return body[start:j + 1]
    raise ValueError("unbalanced literal")


# --- translation ------------------------------------------------------------------
ENUMS = {"PolicyIngress": "INGRESS", "PolicyEgress": "EGRESS", "PolicyAll": "ALL",
         "MatchIngress": "INGRESS", "MatchEgress": "EGRESS", "TCP": "TCP", "UDP": "UDP"}


def scalar(v, env):
    kind = v[0]
    if kind == "str" or kind == "num":
        return v[1]
    if kind == "id":
        if v[1] in env:
            return env[v[1]]
        if v[1] in ENUMS:
            return ENUMS[v[1]]
        raise KeyError(v[1])
    if kind == "call" and v[1] == "parseIPNet":
        return scalar(v[2], env)
    raise ValueError(v)


def fields(lit):
    assert lit.keyed, lit.items
    return dict(lit.items)


def policy_json(lit, env):
    f = fields(lit)
    pid = fields(f["ID"])
    out = {"name": scalar(pid["Name"], env), "namespace": scalar(pid["Namespace"], env),
           "type": scalar(f["Type"], env), "matches": []}
    for m in f["Matches"].items:
        mf = fields(m)
        match = {"type": scalar(mf["Type"], env), "pods": None, "ip_blocks": None, "ports": None}
        if "Pods" in mf:
            match["pods"] = [scalar(p, env) for p in mf["Pods"].items]
        if "IPBlocks" in mf:
            match["ip_blocks"] = []
            for b in mf["IPBlocks"].items:
                bf = fields(b)
                match["ip_blocks"].append({
                    "network": scalar(bf["Network"], env),
                    "except": [scalar(e, env) for e in bf["Except"].items] if "Except" in bf else []})
        if "Ports" in mf:
            match["ports"] = [[scalar(fields(p)["Protocol"], env), scalar(fields(p)["Number"], env)]
                              for p in mf["Ports"].items]
        out["matches"].append(match)
    return out


STEP_RES = [
    ("renderer", r'(\w+) := NewMockRenderer\("(\w+)", logger\)'),
    ("init", r"configurator\.Init\((true|false)\)"),
    ("register", r"configurator\.RegisterRenderer\((\w+)\)"),
    ("new_txn", r"\w+ :?= configurator\.NewTxn\((true|false)\)"),
    ("configure", r"txn\.Configure\((\w+), (\w+)\)"),
    ("commit", r"txn\.Commit\(\)"),
    ("cache", r"cache\.AddPodConfig\((\w+), (\w+)\)"),
    ("pod_ip", r"ip, masklen :?= (\w+)\.GetPodIP\((\w+)\)\s*"
               r"gomega\.Expect\(masklen\)\.To\(gomega\.BeEquivalentTo\(net\.IPv(4|6)len \* 8\)\)\s*"
               r"gomega\.Expect\(ip\)\.To\(gomega\.BeEquivalentTo\((\w+)\)\)"),
    ("traffic", r"action :?= (\w+)\.TestTraffic\((\w+), (\w+),\s*parseIP\(([^)]*)\), parseIP\(([^)]*)\), "
                r"rendererAPI\.(\w+), (\d+), (\d+)\)\s*"
                r"gomega\.Expect\(action\)\.To\(gomega\.BeEquivalentTo\((\w+)\)\)"),
]


def translate(name, body, line0):
    env = {}
    for m in re.finditer(r"const \((.*?)\n\s*\)", body, re.S):
        for c in re.finditer(r'(\w+)\s*=\s*"([^"]*)"', m.group(1)):
            env[c.group(1)] = c.group(2)
    pods = {}
    for m in re.finditer(r"(\w+) := podmodel\.ID\{Name: (\w+), Namespace: (\w+)\}", body):
        env[m.group(1)] = [env[m.group(2)], env[m.group(3)]]
        pods[m.group(1)] = env[m.group(1)]
    policies = {}
    for m in re.finditer(r"(\w+) := &ContivPolicy\{", body):
        text = literal_at(body, m.start(0) + len(m.group(1)) + 4)
        lit, _ = parse_value(tokenize(text), 0)
        policies[m.group(1)] = policy_json(lit, env)
    lists = {}
    for m in re.finditer(r"(\w+) := \[\]\*ContivPolicy\{([^}]*)\}", body):
        lists[m.group(1)] = [policies[p.strip()]["name"] for p in m.group(2).split(",") if p.strip()]

    def ip_arg(a):
        a = a.strip()
        return a[1:-1] if a.startswith('"') else env[a]

    found = []
    for kind, rx in STEP_RES:
        for m in re.finditer(rx, body):
            g = m.groups()
            line = line0 + body.count("\n", 0, m.start())
            if kind == "renderer":
                step = {"op": kind, "var": g[0], "name": g[1]}
            elif kind in ("init", "new_txn"):
                step = {"op": kind, "flag": g[0] == "true"}
            elif kind == "register":
                step = {"op": kind, "renderer": g[0]}
            elif kind == "configure":
                step = {"op": kind, "pod": env[g[0]], "policies": lists[g[1]]}
            elif kind == "commit":
                step = {"op": kind}
            elif kind == "cache":
                step = {"op": kind, "pod": env[g[0]], "ip": env[g[1]]}
            elif kind == "pod_ip":
                step = {"op": kind, "renderer": g[0], "pod": env[g[1]],
                        "masklen": 32 if g[2] == "4" else 128, "ip": env[g[3]]}
            else:
                step = {"op": kind, "renderer": g[0], "pod": env[g[1]],
                        "dir": {"EgressTraffic": "EGRESS", "IngressTraffic": "INGRESS"}[g[2]],
                        "src": ip_arg(g[3]), "dst": ip_arg(g[4]), "proto": g[5],
                        "sport": int(g[6]), "dport": int(g[7]),
                        "expect": {"AllowedTraffic": "ALLOWED", "DeniedTraffic": "DENIED",
                                   "UnmatchedTraffic": "UNMATCHED"}[g[8]]}
            step["line"] = line
            found.append((m.start(), step))
    found.sort(key=lambda x: x[0])
    steps = [s for _, s in found]
    n_traffic = sum(1 for s in steps if s["op"] == "traffic")
    n_pod_ip = sum(1 for s in steps if s["op"] == "pod_ip")
    assert n_traffic == body.count(".TestTraffic("), (name, n_traffic)
    assert n_pod_ip == body.count(".GetPodIP("), (name, n_pod_ip)
    assert sum(1 for s in steps if s["op"] == "configure") == body.count("txn.Configure(")
    by_name = {p["name"]: p for p in policies.values()}
    return {"name": name, "line": line0, "pods": pods, "policies": by_name, "steps": steps}


def main(ref_root):
    path = os.path.join(ref_root, TEST_FILE)
    text = strip_comments(open(path).read())
    starts = [(m.start(), m.group(1)) for m in re.finditer(r"^func (Test\w+)\(t \*testing\.T\) \{", text, re.M)]
    scenarios = []
    for k, (pos, name) in enumerate(starts):
        end = starts[k + 1][0] if k + 1 < len(starts) else len(text)
        scenarios.append(translate(name, text[pos:end], text.count("\n", 0, pos) + 1))
    out = {"source": TEST_FILE, "generator": "tests/golden/make_configurator_scenarios.py",
           "n_traffic": sum(1 for s in scenarios for st in s["steps"] if st["op"] == "traffic"),
           "scenarios": scenarios}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configurator_scenarios.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("%d scenarios, %d TestTraffic expectations -> %s" % (len(scenarios), out["n_traffic"], dst))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
