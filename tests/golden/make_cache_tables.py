#!/usr/bin/env python3
"""Generate tests/golden/cache_tables.json from the reference's renderer-cache tests.

Run in the build container only (needs /root/reference, which does not
exist on the GPU box):

    python tests/golden/make_cache_tables.py /root/reference

It reads plugins/policy/renderer/cache/cache_test.go as TEXT, rewrites each
of its 14 test functions from the Go subset they use (short variable
declarations, composite literals, append, range loops, if/else, gomega
expectations) into Python, and runs that once against a recorder:

  * every cache operation (Init, NewTxn, Update, Commit, GetChanges, Flush,
    Resync, the getters) becomes a step, performed on this build's own
    renderer cache (vpp_amd/renderer/cache.py) so that the tests'
    data-dependent control flow (which change holds Pod1's table) resolves;
  * every expectation (verifyRules and the other verify* helpers, :60-181;
    gomega.Expect) becomes a check step holding the EXPECTED value the test
    computes -- ordered rule lists, pod sets, pod configs, change counts --
    and is also asserted on the spot, so a fixture is only written when the
    build's cache agrees with every reference expectation.

Tables and changes are referred to by labels bound when a step obtains them
(a change by its table type, pods and previous pods, never by its position,
which in Go follows map iteration).  The fixture holds inputs, steps and
expected outputs only -- no reference source; the rule data of testdata.go
comes from make_acl_scenarios.py's transcription.
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, HERE]

from make_acl_scenarios import RULE_LISTS, RULES, POD_IPS   # noqa: E402  (testdata.go transcription)

from vpp_amd import gonet                                      # noqa: E402
from vpp_amd.renderer import api                               # noqa: E402
from vpp_amd.renderer import cache as CA                       # noqa: E402

ORDER = ["Pod1", "Pod2", "Pod3", "Pod4", "Pod5", "Pod6"]


# --- rule / pod data ---------------------------------------------------------
def mk_rule(d):
    return api.ContivRule(api.ACTION_PERMIT if d["action"] == "PERMIT" else api.ACTION_DENY,
                          gonet.ip_network(d["src"]) if d["src"] else gonet.IPNet(),
                          gonet.ip_network(d["dst"]) if d["dst"] else gonet.IPNet(),
                          api.TCP if d["proto"] == "TCP" else api.UDP, d["sport"], d["dport"])


def rule_json(r):
    def net(n):
        return "" if not len(n.ip) else "%s/%d" % (gonet.ip_string(n.ip), gonet.mask_size(n.mask)[0])
    return {"action": "PERMIT" if r.action == api.ACTION_PERMIT else "DENY", "src": net(r.src_network),
            "dst": net(r.dest_network), "proto": "TCP" if r.protocol == api.TCP else "UDP",
            "sport": r.src_port, "dport": r.dest_port}


class NS:
    def __init__(self, **kw):
        self.__dict__.update(kw)


POD = {p: api.PodID("pod%d" % (i + 1), "default" if i < 5 else "namespace2") for i, p in enumerate(ORDER)}
POD_NAME = {v: k for k, v in POD.items()}
IPS = [POD_IPS["Pod%dIP" % (i + 1)] for i in range(6)]


def pod_json(p):
    return POD_NAME[p]


def pods_json(ps):
    return sorted(pod_json(p) for p in ps)


def cfg_json(c):
    if c is None:
        return None
    return {"pod_ip": "" if c.pod_ip is None or not len(c.pod_ip.ip) else
            "%s/%d" % (gonet.ip_string(c.pod_ip.ip), gonet.mask_size(c.pod_ip.mask)[0]),
            "ingress": [rule_json(r) for r in c.ingress], "egress": [rule_json(r) for r in c.egress],
            "removed": c.removed}


def env():
    """The Go test package's names (testdata.go, cache_test.go:34-112)."""
    ts = {}
    for k, d in RULES.items():
        obj, attr = k.split(".")
        ts.setdefault(obj, {})[attr] = mk_rule(d)
    for k, lst in RULE_LISTS.items():
        obj, attr = k.split(".")
        ts.setdefault(obj, {})[attr] = [mk_rule(d) for d in lst]
    e = {name: NS(**attrs) for name, attrs in ts.items()}
    e.update(POD)
    e["PodIDs"] = [POD[p] for p in ORDER]
    e["PodIPs"] = list(IPS)
    for i, ip in enumerate(IPS):
        e["Pod%dIP" % (i + 1)] = ip

    def one_host(ip):
        return gonet.one_host_subnet(ip)

    def with_net(rule, src=None, dst=None):
        c = rule.copy()
        if src is not None:
            c.src_network = one_host(src)
        if dst is not None:
            c.dest_network = one_host(dst)
        return c

    def mk(action, src, dst, port, proto):
        return api.ContivRule(action, one_host(src) if src else gonet.IPNet(),
                              one_host(dst) if dst else gonet.IPNet(), proto, 0, port)
    e.update(
        GetOneHostSubnet=one_host, NewPodSet=lambda *ps: CA.PodSet(ps), EmptyPodSet=CA.PodSet(),
        EmptyRules=[], AllowAllTCP=api.allow_all_tcp, AllowAllUDP=api.allow_all_udp,
        modifySrc=lambda ip, *rules: [with_net(r, src=ip) for r in rules],
        modifyDst=lambda rule, *ips: [with_net(rule, dst=ip) for ip in ips],
        allowPodEgress=lambda ip, port, proto: mk(api.ACTION_PERMIT, ip, None, port, proto),
        blockPodEgress=lambda ip, proto: mk(api.ACTION_DENY, ip, None, 0, proto),
        allowPodIngress=lambda ip, port, proto: mk(api.ACTION_PERMIT, None, ip, port, proto),
        blockPodIngress=lambda ip, proto: mk(api.ACTION_DENY, None, ip, 0, proto),
        TCP=api.TCP, UDP=api.UDP, GlobalTableID=CA.GLOBAL_TABLE_ID,
        EgressOrientation=CA.EGRESS_ORIENTATION, IngressOrientation=CA.INGRESS_ORIENTATION,
        append=lambda lst, *items: list(lst) + list(items), len=len, range=range, logger=None)
    return e


# --- recorder ------------------------------------------------------------------
class Rec:
    def __init__(self):
        self.steps = []
        self.n = 0
        self.labels = {}         # id(obj) -> label (the last binding)

    def label(self, kind):
        self.n += 1
        return "%s%d" % (kind, self.n)

    def step(self, **kw):
        self.steps.append(kw)

    def check(self, ok, **kw):
        if not ok:
            raise AssertionError("reference expectation fails on this build: %r" % (kw,))
        self.steps.append(kw)


R = Rec()


class TableRef:
    """A table a step obtained (label) -- or a table the test itself built."""

    def __init__(self, t, label):
        self.t, self.label = t, label

    @property
    def Pods(self):
        return PodSetView(self.t.pods, self)

    def InsertRule(self, rule):
        self.t.insert_rule(rule)
        R.step(op="table_insert", table=self.label, rule=rule_json(rule))


class PodSetView:
    def __init__(self, ps, owner=None):
        self.ps, self.owner = ps, owner

    def Has(self, p):
        return p in self.ps

    def Add(self, p):
        self.ps.add(p)
        R.step(op="table_add_pod", table=self.owner.label, pod=pod_json(p))

    def __len__(self):
        return len(self.ps)


def new_table(tid):
    lab = R.label("T")
    R.step(op="new_table", id=tid, bind=lab)
    return TableRef(CA.ContivRuleTable(tid), lab)


class ChangeRef:
    def __init__(self, c, label):
        self.c, self.label = c, label
        self._table = None

    @property
    def Table(self):
        if self._table is None:
            lab = R.label("T")
            R.step(op="change_table", change=self.label, bind=lab)
            self._table = TableRef(self.c.table, lab)
        return self._table

    @property
    def PreviousPods(self):
        return PodSetView(self.c.previous_pods)


class Changes:
    def __init__(self, lst, label):
        self.lst, self.label = lst, label
        self.refs = {}

    def __len__(self):
        return len(self.lst)

    def __getitem__(self, i):
        if i not in self.refs:
            c = self.lst[i]
            lab = R.label("X")
            R.step(op="change", changes=self.label, bind=lab,
                   locate={"global": c.table.type == CA.GLOBAL, "pods": pods_json(c.table.pods),
                           "prev": pods_json(c.previous_pods)})
            self.refs[i] = ChangeRef(c, lab)
        return self.refs[i]


class View:
    """RendererCache or its Txn, as the test sees it (cache_api.go:51-190)."""

    def __init__(self, obj, who):
        self.o, self.who = obj, who

    def GetGlobalTable(self):
        lab = R.label("T")
        R.step(op="global_table", on=self.who, bind=lab)
        return TableRef(self.o.get_global_table(), lab)

    def GetLocalTableByPod(self, p):
        lab = R.label("T")
        R.step(op="local_table", on=self.who, pod=pod_json(p), bind=lab)
        t = self.o.get_local_table_by_pod(p)
        return None if t is None else TableRef(t, lab)

    def GetPodConfig(self, p):
        return self.o.get_pod_config(p)

    def GetAllPods(self):
        return self.o.get_all_pods()

    def GetIsolatedPods(self):
        return self.o.get_isolated_pods()


class Txn(View):
    def __init__(self, o):
        super().__init__(o, "txn")

    def Update(self, p, cfg):
        R.step(op="update", pod=pod_json(p), cfg=cfg_json(cfg))
        self.o.update(p, cfg)

    def GetUpdatedPods(self):
        return self.o.get_updated_pods()

    def GetRemovedPods(self):
        return self.o.get_removed_pods()

    def GetChanges(self):
        lab = R.label("C")
        R.step(op="changes", bind=lab)
        return Changes(self.o.get_changes(), lab)

    def Commit(self):
        R.step(op="commit")
        self.o.commit()
        return None


class Cache(View):
    def __init__(self, **deps):           # &RendererCache{Deps: ...}: the logger is not needed
        super().__init__(CA.RendererCache(), "cache")

    def Init(self, orientation):
        R.step(op="init", orientation="egress" if orientation == CA.EGRESS_ORIENTATION else "ingress")
        self.o.init(orientation)

    def Flush(self):
        R.step(op="flush")
        self.o.flush()

    def NewTxn(self):
        R.step(op="new_txn")
        return Txn(self.o.new_txn())

    def Resync(self, tables):
        R.step(op="resync", tables=[t.label for t in tables])
        try:
            self.o.resync([t.t for t in tables])
        except ValueError as e:
            return e
        return None


def rules_equal(table, rules):
    a = table.t.rules[:table.t.num_of_rules]
    return len(a) == len(rules) and all(x.compare(y) == 0 for x, y in zip(a, rules))


def deep_equal(a, b):
    """gomega.Equal on two *ContivRuleTable: reflect.DeepEqual of the tables."""
    x, y = a.t, b.t
    return (x.id == y.id and x.type == y.type and set(x.pods) == set(y.pods) and
            len(x.rules) == len(y.rules) and all(p.compare(q) == 0 for p, q in zip(x.rules, y.rules)))


# the verify helpers of cache_test.go:60-181, as recorded checks
def verifyRules(table, rules):
    R.check(rules_equal(table, rules), check="rules", table=table.label, rules=[rule_json(r) for r in rules])


def verifyCachedPods(view, all_, isolated):
    R.check(set(view.GetAllPods()) == set(all_), check="all_pods", on=view.who, pods=pods_json(all_))
    R.check(set(view.GetIsolatedPods()) == set(isolated), check="isolated_pods", on=view.who,
            pods=pods_json(isolated))


def verifyUpdatedPods(txn, updated, removed):
    R.check(set(txn.GetUpdatedPods()) == set(updated), check="updated_pods", pods=pods_json(updated))
    R.check(set(txn.GetRemovedPods()) == set(removed), check="removed_pods", pods=pods_json(removed))


def _table_basics(table, local):
    R.check(table is not None, check="not_nil", table=None if table is None else table.label)
    t = table.t
    if local:
        R.check(t.id != "" and t.id != CA.GLOBAL_TABLE_ID and t.type == CA.LOCAL, check="local", table=table.label)
    else:
        R.check(t.id == CA.GLOBAL_TABLE_ID and t.type == CA.GLOBAL, check="global", table=table.label)


def verifyLocalTableChange(change, exp, rules, prev, new):
    R.check(change is not None, check="change_not_nil")
    verifyLocalTable(change.Table, exp, rules, new)
    R.check(set(change.c.previous_pods) == set(prev), check="previous_pods", change=change.label,
            pods=pods_json(prev))


def verifyPodLocalTable(view, pod, exp, rules, pods):
    table = view.GetLocalTableByPod(pod)
    if table is None:
        R.check(False, check="local_table_missing", pod=pod_json(pod))
    if exp is not None:
        R.check(deep_equal(table, exp), check="table_equal", a=table.label, b=exp.label)
    _table_basics(table, True)
    verifyRules(table, rules)
    R.check(set(table.t.pods) == set(pods), check="pods", table=table.label, pods=pods_json(pods))


def verifyPodNilLocalTable(view, pod):
    t = view.o.get_local_table_by_pod(pod)
    R.check(t is None, check="no_local_table", on=view.who, pod=pod_json(pod))


def verifyLocalTable(table, exp, rules, pods):
    _table_basics(table, True)
    if exp is not None:
        R.check(table.t.id == exp.t.id, check="same_id", a=table.label, b=exp.label)
    verifyRules(table, rules)
    R.check(set(table.t.pods) == set(pods), check="pods", table=table.label, pods=pods_json(pods))


def verifyGlobalTableChange(change, exp, not_exp, rules):
    R.check(change is not None, check="change_not_nil")
    verifyGlobalTable(change.Table, exp, not_exp, rules)
    R.check(len(change.c.previous_pods) == 0, check="previous_pods", change=change.label, pods=[])


def verifyGlobalTable(table, exp, not_exp, rules):
    R.check(table is not None, check="not_nil", table=table.label)
    if exp is not None:
        R.check(deep_equal(table, exp), check="table_equal", a=table.label, b=exp.label)
    if not_exp is not None:
        R.check(not deep_equal(table, not_exp), check="table_not_equal", a=table.label, b=not_exp.label)
    _table_basics(table, False)
    verifyRules(table, rules)
    R.check(len(table.t.pods) == 0, check="pods", table=table.label, pods=[])


def verifyPodConfig(view, pod, cfg):
    got = view.GetPodConfig(pod)
    same = (got is None and cfg is None) or (got is not None and cfg is not None and cfg_json(got) == cfg_json(cfg))
    R.check(same, check="pod_config", on=view.who, pod=pod_json(pod), cfg=cfg_json(cfg))


class Expect:
    def __init__(self, v):
        self.v = v

    def To(self, m):
        m(self.v, True)

    def ToNot(self, m):
        m(self.v, False)


def HaveLen(n):
    def m(v, pos):
        assert pos
        R.check(len(v) == n, check="changes_len", changes=v.label, n=n)
    return m


def BeNil():
    def m(v, pos):
        if isinstance(v, (ChangeRef, TableRef)) or v is None and not pos:
            R.check((v is None) == pos, check="nil" if pos else "not_nil_ref",
                    ref=None if v is None else v.label)
        else:
            R.check((v is None) == pos, check="no_error" if pos else "error")
    return m


def BeTrue():
    def m(v, pos):
        R.check(bool(v) == pos, check="test_flag", value=pos)
    return m


def BeFalse():
    def m(v, pos):
        R.check((not v) == pos, check="test_flag", value=not pos)
    return m


# --- Go subset -> Python ---------------------------------------------------------
LIT_TYPES = (r"\[\]\*renderer\.ContivRule", r"\[\]\*PodConfig", r"\[\]\*ContivRuleTable", r"&PodConfig",
             r"&RendererCache", r"Deps")


def go_to_python(body: str) -> str:
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    body = re.sub(r"//[^\n]*", "", body)
    # composite literals: Type{...} -> Ctor(...)
    out, stack, i = [], [], 0
    ctor = {r"\[\]\*renderer\.ContivRule": "L(", r"\[\]\*PodConfig": "L(", r"\[\]\*ContivRuleTable": "L(",
            r"&PodConfig": "PodConfig(", r"&RendererCache": "Cache(", r"Deps": "dict("}
    while i < len(body):
        hit = None
        for pat in LIT_TYPES:
            m = re.match(pat + r"\{", body[i:])
            if m and not re.match(r"\w", body[i - 1:i] or " "):
                hit = (pat, m.end())
                break
        if hit:
            out.append(ctor[hit[0]])
            stack.append("lit")
            i += hit[1]
            continue
        ch = body[i]
        if ch == "{":
            stack.append("blk")
            out.append("{")
        elif ch == "}":
            kind = stack.pop()
            out.append(")" if kind == "lit" else "}")
        else:
            out.append(ch)
        i += 1
    src = "".join(out)
    # statements, one per line, with block structure from { }
    lines, depth = [], 0
    for raw in src.split("\n"):
        s = raw.strip()
        if not s:
            continue
        if s == "}":
            depth -= 1
            continue
        if s.startswith("} else {"):
            lines.append("    " * (depth - 1) + "else:")
            continue
        opens = s.endswith("{")
        if opens:
            s = s[:-1].rstrip()
        s = translate_stmt(s)
        if s is not None:
            lines.append("    " * depth + s + (":" if opens else ""))
        elif opens:
            lines.append("    " * depth + "if True:")
        if opens:
            depth += 1
    return "\n".join(lines)


def translate_stmt(s: str):
    if re.match(r"(gomega\.RegisterTestingT|logger)", s) or s.startswith("logger :="):
        return None
    m = re.fullmatch(r"for (\w+) := 0; \1 < (.+); \1\+\+", s)
    if m:
        return "for %s in range(%s)" % (m.group(1), expr(m.group(2)))
    m = re.fullmatch(r"for (\w+) := range (.+)", s)
    if m:
        return "for %s in range(len(%s))" % (m.group(1), expr(m.group(2)))
    m = re.fullmatch(r"for _, (\w+) := range (.+)", s)
    if m:
        return "for %s in %s" % (m.group(1), expr(m.group(2)))
    m = re.fullmatch(r"if (.+)", s)
    if m:
        return "if %s" % expr(m.group(1))
    m = re.fullmatch(r"var ([\w, ]+) (\S+)", s)
    if m:
        init = {"bool": "False", "int": "0"}.get(m.group(2), "[]" if m.group(2).startswith("[]") else "None")
        return " = ".join(v.strip() for v in m.group(1).split(",")) + " = " + init
    m = re.fullmatch(r"([\w, ]+) :?= (.+)", s, flags=re.S)
    if m:
        return "%s = %s" % (m.group(1), expr(m.group(2)))
    return expr(s)


def expr(e: str) -> str:
    e = re.sub(r"\s+", " ", e).strip()
    e = e.replace("gomega.", "").replace("renderer.", "")
    e = re.sub(r"(\w+)\.\.\.", r"*\1", e)                 # f(x...) spreads
    e = re.sub(r"\*(\w+\[[^\]]*\])\.\.\.", r"*\1", e)
    e = re.sub(r"([\w\]\)]+\[[^\]]*\])\.\.\.", r"*\1", e)
    e = re.sub(r"(\w+\([^()]*\))\.\.\.", r"*\1", e)
    e = re.sub(r"\b(\w+): ", r"\1=", e)                    # PodConfig{Key: v} keyword arguments
    e = re.sub(r"\bnil\b", "None", e).replace("true", "True").replace("false", "False")
    e = re.sub(r"NewContivRuleTable\(", "new_table(", e)
    e = e.replace("PodIP=", "pod_ip=").replace("Ingress=", "ingress=").replace("Egress=", "egress=")
    e = e.replace("Removed=", "removed=")
    return e


def L(*items):
    return list(items)


class GoPodConfig(CA.PodConfig):
    """cache.PodConfig with the Go field names the tests read."""
    Ingress = property(lambda self: self.ingress)
    Egress = property(lambda self: self.egress)
    PodIP = property(lambda self: self.pod_ip)
    Removed = property(lambda self: self.removed)


def PodConfig(pod_ip=None, ingress=None, egress=None, removed=False):
    return GoPodConfig(pod_ip, ingress, egress, removed)


def run_test(name, pysrc):
    global R
    R = Rec()
    g = env()
    g.update({k: v for k, v in globals().items() if k[:1].islower() or k[:1].isupper()})
    g.update(env())
    g["new_table"] = new_table
    exec(compile("def _t():\n" + "\n".join("    " + ln for ln in pysrc.split("\n")) + "\n", name, "exec"), g)
    g["_t"]()
    return R.steps


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    text = open(os.path.join(ref, "plugins/policy/renderer/cache/cache_test.go")).read()
    tests = []
    for m in re.finditer(r"^func (Test\w+)\(t \*testing\.T\) \{\n(.*?)^\}", text, re.S | re.M):
        name = m.group(1)
        line = text[:m.start()].count("\n") + 1
        py = go_to_python(m.group(2))
        steps = run_test(name, py)
        tests.append({"name": name, "line": line, "steps": steps})
        n_rules = sum(1 for s in steps if s.get("check") == "rules")
        print("%-52s :%-5d %4d steps, %3d rule-order checks" % (name, line, len(steps), n_rules))
    out = os.path.join(HERE, "cache_tables.json")
    with open(out, "w") as f:                      # one step per line
        f.write('{"source": "plugins/policy/renderer/cache/cache_test.go (generated by make_cache_tables.py)",\n')
        f.write(' "tests": [\n')
        for i, t in enumerate(tests):
            f.write('  {"name": %s, "line": %d, "steps": [\n' % (json.dumps(t["name"]), t["line"]))
            f.write(",\n".join("   " + json.dumps(st, separators=(",", ":")) for st in t["steps"]))
            f.write("]}%s\n" % ("," if i + 1 < len(tests) else ""))
        f.write(" ]}\n")
    print("wrote", out, sum(1 for t in tests for s in t["steps"] if s.get("check") == "rules"), "rule-order checks")


if __name__ == "__main__":
    main()
