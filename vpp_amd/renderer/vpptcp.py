"""VPPTCP renderer: ContivRuleTables -> VPP session rules.

Restates plugins/policy/renderer/vpptcp:
  * rule/session_rule.go -- SessionRule (:70-83), Compare (:156-197),
    ExportSessionRules (:201-331), ImportSessionRules (:335-436), constants
    (:32-67);
  * vpptcp_renderer.go   -- Renderer.Init with IngressOrientation (:62-73),
    NewTxn/Render (:80-102), Commit (:106-192), dumpRules (:195-238),
    updateRules (:270-327, requests sent in batches of GoVPPChanBufSize);
and the session-rule sink the rules are sent to, restated from
mock/sessionrules/sessionrules_mock.go (add/del :270-362, HasRule :123-228,
dump :241-251, request / error counters).

Session rules are the control-plane encoding only: the reference never
evaluates a packet against them (the mock stores rules and answers HasRule;
VPP's session-table lookup is external).  With an engine the renderer
evaluates packets two ways on the GPU (parity unpinned by reference
fixtures):
  * TestTraffic semantics (renderer_mock.go:105-145) over the
    IngressOrientation tables it commits -- each pod's local table and the
    global table (vpp_amd.renderer.traffic.RuleTable, ``rule_tables``);
  * the session rules the sink holds, as exported (deny-all split covering
    IPv4 only, allow-all and self rules not installed):
    vpp_amd.renderer.sessions.SessionEvaluator, ``sessions``.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from .. import gonet
from ..gonet import IPNet
from .api import ACTION_DENY, ACTION_PERMIT, TCP, UDP, ContivRule, PodID, compare_ints
from .cache import GLOBAL_TABLE_ID, INGRESS_ORIENTATION, ContivRuleTable, PodConfig, RendererCache

SESSION_RULE_TAG_PREFIX = "contiv/vpp-policy-"
SPLIT_SESSION_RULE_TAG = "SPLIT"
SCOPE_GLOBAL = 1
SCOPE_LOCAL = 2
SCOPE_BOTH = 3
ACTION_DO_NOTHING = 0xFFFFFFFF
ACTION_DENY_IDX = 0xFFFFFFFF - 1
ACTION_ALLOW_IDX = 0xFFFFFFFF - 2
PROTO_TCP = 0
PROTO_UDP = 1
TAG_LEN = 64


def _tag(s: str) -> bytes:
    b = s.encode()[:TAG_LEN]
    return b + bytes(TAG_LEN - len(b))


def _ip16(ip: Optional[bytes]) -> bytes:
    """copy(rule.XxxIP[:], ip): 4 or 16 bytes at the start of a [16]byte."""
    ip = ip or b""
    return ip[:16] + bytes(16 - min(16, len(ip)))


class SessionRule:
    """SessionRule (session_rule.go:70-83)."""

    __slots__ = ("transport_proto", "is_ip4", "lcl_ip", "lcl_plen", "rmt_ip", "rmt_plen",
                 "lcl_port", "rmt_port", "action_index", "appns_index", "scope", "tag")

    def __init__(self, **kw):
        self.transport_proto = 0
        self.is_ip4 = 0
        self.lcl_ip = bytes(16)
        self.lcl_plen = 0
        self.rmt_ip = bytes(16)
        self.rmt_plen = 0
        self.lcl_port = 0
        self.rmt_port = 0
        self.action_index = 0
        self.appns_index = 0
        self.scope = 0
        self.tag = bytes(TAG_LEN)
        for k, v in kw.items():
            setattr(self, k, v)

    def copy(self) -> "SessionRule":
        return SessionRule(**{k: getattr(self, k) for k in self.__slots__})

    def tag_string(self) -> str:
        i = self.tag.find(b"\0")
        return (self.tag if i < 0 else self.tag[:i]).decode(errors="replace")

    def compare(self, other: "SessionRule", compare_tag: bool) -> int:
        """Compare (session_rule.go:156-197)."""
        for a, b in ((self.appns_index, other.appns_index), (self.scope, other.scope),
                     (self.action_index, other.action_index), (self.is_ip4, other.is_ip4)):
            o = compare_ints(a, b)
            if o:
                return o
        for (ap, ai), (bp, bi) in (((self.lcl_plen, self.lcl_ip), (other.lcl_plen, other.lcl_ip)),
                                   ((self.rmt_plen, self.rmt_ip), (other.rmt_plen, other.rmt_ip))):
            o = compare_ints(ap, bp)                            # CompareIPNetsBytes (utils.go:261-267)
            if o:
                return o
            o = -1 if ai < bi else (1 if ai > bi else 0)
            if o:
                return o
        for a, b in ((self.transport_proto, other.transport_proto), (self.lcl_port, other.lcl_port),
                     (self.rmt_port, other.rmt_port)):
            o = compare_ints(a, b)
            if o:
                return o
        if compare_tag:
            return -1 if self.tag < other.tag else (1 if self.tag > other.tag else 0)
        return 0

    def __repr__(self) -> str:
        bits = 32 if self.is_ip4 else 128
        n = bits // 8
        lcl = IPNet(self.lcl_ip[:n], gonet.cidr_mask(self.lcl_plen, bits)).string()
        rmt = IPNet(self.rmt_ip[:n], gonet.cidr_mask(self.rmt_plen, bits)).string()
        scope = {0: "global", SCOPE_GLOBAL: "global", SCOPE_LOCAL: "local", SCOPE_BOTH: "both"}.get(self.scope, "invalid")
        action = {ACTION_DO_NOTHING: "do-nothing", ACTION_ALLOW_IDX: "allow",
                  ACTION_DENY_IDX: "deny"}.get(self.action_index, "fwd->%d" % self.action_index)
        proto = {PROTO_TCP: "TCP", PROTO_UDP: "UDP"}.get(self.transport_proto, "invalid")
        return "Rule <ns:%d scope:%s action:%s lcl:%s[%s:%d] rmt:%s:[%s:%d] tag:%s>" % (
            self.appns_index, scope, action, lcl, proto, self.lcl_port, rmt, proto, self.rmt_port,
            self.tag_string())


def export_session_rules(rules: List[ContivRule], pod: Optional[PodID], pod_ip: Optional[bytes],
                         contiv) -> List[SessionRule]:
    """ExportSessionRules (session_rule.go:201-331).  ``pod`` None = global table."""
    is_global = pod is None
    out: List[SessionRule] = []
    ns_index = 0
    if not is_global:
        ns_index, found = contiv.get_ns_index(pod.namespace, pod.name)
        if not found:
            return out
    for rule in rules:
        sr = SessionRule()
        if rule.dest_port == 0 and rule.action == ACTION_PERMIT and (
                (is_global and len(rule.src_network.ip) == 0) or
                (not is_global and len(rule.dest_network.ip) == 0)):
            continue                                             # allow-all: the stack default (:220-224)
        if not is_global and len(rule.dest_network.ip) > 0:
            ones, bits = gonet.mask_size(rule.dest_network.mask)
            if ones == bits and gonet.ip_equal(rule.dest_network.ip, pod_ip or b""):
                continue                                         # same source as destination (:226-232)
        sr.transport_proto = PROTO_UDP if rule.protocol == UDP else PROTO_TCP
        net = rule.src_network if is_global else rule.dest_network
        if len(net.ip) == 0 or gonet.to4(net.ip) is not None:
            sr.is_ip4 = 1
        if is_global:
            d = rule.dest_network
            sr.lcl_ip = _ip16(gonet.to4(d.ip) if sr.is_ip4 else gonet.to16(d.ip))
            sr.lcl_plen = gonet.mask_size(d.mask)[0] & 0xFF
            sr.lcl_port = rule.dest_port
        else:
            sr.lcl_port = rule.src_port                          # it is any
        rmt = rule.src_network if is_global else rule.dest_network
        if len(rmt.ip) > 0:
            sr.rmt_ip = _ip16(gonet.to4(rmt.ip) if sr.is_ip4 else gonet.to16(rmt.ip))
            sr.rmt_plen = gonet.mask_size(rmt.mask)[0] & 0xFF
        sr.rmt_port = rule.src_port if is_global else rule.dest_port
        sr.action_index = ACTION_ALLOW_IDX if rule.action == ACTION_PERMIT else ACTION_DENY_IDX
        sr.appns_index = ns_index
        sr.scope = SCOPE_GLOBAL if is_global else SCOPE_LOCAL
        if len(rmt.ip) == 0:
            # deny-all split into the two halves of the address space (:311-322)
            sr.rmt_plen = 1
            sr2 = sr.copy()
            sr.tag = _tag(SESSION_RULE_TAG_PREFIX + SPLIT_SESSION_RULE_TAG)
            out.append(sr)
            sr2.rmt_ip = bytes([0x80]) + sr2.rmt_ip[1:]
            sr2.tag = _tag(SESSION_RULE_TAG_PREFIX + SPLIT_SESSION_RULE_TAG)
            out.append(sr2)
        else:
            sr.tag = _tag(SESSION_RULE_TAG_PREFIX)
            out.append(sr)
    return out


def import_session_rules(rules: List[SessionRule], contiv) -> List[ContivRuleTable]:
    """ImportSessionRules (session_rule.go:335-436)."""
    global_table = ContivRuleTable(GLOBAL_TABLE_ID)
    local: Dict[PodID, ContivRuleTable] = {}
    for rule in rules:
        if rule.tag_string().endswith(SPLIT_SESSION_RULE_TAG):
            if rule.rmt_ip[0] != 0:
                continue                                         # skip this half
            rule.rmt_plen = 0                                    # merge
        cr = ContivRule()
        cr.protocol = UDP if rule.transport_proto == PROTO_UDP else TCP
        if rule.scope == SCOPE_GLOBAL:
            src_ip, src_plen, dst_ip, dst_plen = rule.rmt_ip, rule.rmt_plen, rule.lcl_ip, rule.lcl_plen
        else:
            src_ip, src_plen, dst_ip, dst_plen = rule.lcl_ip, rule.lcl_plen, rule.rmt_ip, rule.rmt_plen
        ip_len = 4 if rule.is_ip4 > 0 else 16
        cr.src_network = IPNet(src_ip[:ip_len], gonet.cidr_mask(src_plen, ip_len * 8)) if src_plen > 0 else IPNet()
        cr.dest_network = IPNet(dst_ip[:ip_len], gonet.cidr_mask(dst_plen, ip_len * 8)) if dst_plen > 0 else IPNet()
        if rule.scope == SCOPE_GLOBAL:
            cr.src_port, cr.dest_port = rule.rmt_port, rule.lcl_port
        else:
            cr.src_port, cr.dest_port = rule.lcl_port, rule.rmt_port
        cr.action = ACTION_PERMIT if rule.action_index == ACTION_ALLOW_IDX else ACTION_DENY
        if rule.scope == SCOPE_GLOBAL:
            global_table.insert_rule(cr)
        else:
            ns, name, ok = contiv.get_pod_by_app_ns_index(rule.appns_index)
            if not ok:
                continue
            pod = PodID(name, ns)
            if pod not in local:
                local[pod] = ContivRuleTable(str(pod))
                local[pod].pods.add(pod)
            local[pod].insert_rule(cr)
    return [global_table] + list(local.values())


class SessionRuleTables:
    """The session-rule sink (mock/sessionrules/sessionrules_mock.go:23-362):
    per-appns local tables and one global table, add/del by Compare, HasRule
    queries, and the request / error counters the reference tests check."""

    def __init__(self, tag_prefix: str = SESSION_RULE_TAG_PREFIX):
        self.tag_prefix = tag_prefix
        self.clear()

    def clear(self):
        self.local_table: Dict[int, List[SessionRule]] = {}
        self.global_table: List[SessionRule] = []
        self.err_count = 0
        self.req_count = 0

    # -- binary API ------------------------------------------------------------
    def dump(self) -> List[SessionRule]:
        """session_rules_dump + control_ping (:241-268): two requests."""
        self.req_count += 2
        out = [r.copy() for t in self.local_table.values() for r in t]
        return out + [r.copy() for r in self.global_table]

    def add_del(self, rule: SessionRule, is_add: bool) -> int:
        """session_rule_add_del (:270-333); returns the reply's retval."""
        self.req_count += 1
        rule = rule.copy()
        if not rule.tag_string().startswith(self.tag_prefix):
            self.err_count += 1
            return 1
        if rule.scope == SCOPE_LOCAL:
            table = self.local_table.setdefault(rule.appns_index, [])
        else:
            table = self.global_table
        if not _add_del_rule(table, rule, is_add):
            self.err_count += 1
            return 1
        return 0

    # -- checks ----------------------------------------------------------------
    def num_of_rules(self, ns_index: Optional[int] = None) -> int:
        if ns_index is None:
            return len(self.global_table)
        return len(self.local_table.get(ns_index, []))

    def has_rule(self, ns_index: Optional[int], lcl_ip: str, lcl_port: int, rmt_ip: str, rmt_port: int,
                 proto: str, action: str) -> bool:
        """LocalTable(ns).HasRule / GlobalTable().HasRule (:123-228); ns_index None = global."""
        if ns_index is None:
            table, scope, ns = self.global_table, SCOPE_GLOBAL, 0
        else:
            if ns_index not in self.local_table:
                return False
            table, scope, ns = self.local_table[ns_index], SCOPE_LOCAL, ns_index
        rule = SessionRule(lcl_port=lcl_port, rmt_port=rmt_port, appns_index=ns, scope=scope)
        rule.transport_proto = {"TCP": PROTO_TCP, "UDP": PROTO_UDP}.get(proto, 0)
        rule.action_index = {"ALLOW": ACTION_ALLOW_IDX, "DENY": ACTION_DENY_IDX}.get(action, 0)
        is_ip4 = 0
        for s, attr in ((lcl_ip, "lcl"), (rmt_ip, "rmt")):
            if s == "":
                continue
            if "/" not in s:
                net = gonet.one_host_subnet(s)
            else:
                _, net = gonet.parse_cidr(s)
                if net is None:
                    return False
            if gonet.to4(net.ip) is not None:
                is_ip4 = 1
                setattr(rule, attr + "_ip", _ip16(gonet.to4(net.ip)))
            else:
                setattr(rule, attr + "_ip", _ip16(gonet.to16(net.ip)))
            setattr(rule, attr + "_plen", gonet.mask_size(net.mask)[0])
        if lcl_ip == "" and rmt_ip == "":
            is_ip4 = 1
        rule.is_ip4 = is_ip4
        return any(rule.compare(r2, False) == 0 for r2 in table)


def _add_del_rule(table: List[SessionRule], rule: SessionRule, is_add: bool) -> bool:
    """addDelRule (sessionrules_mock.go:342-362): in place."""
    for idx, r2 in enumerate(table):
        if rule.compare(r2, not is_add) == 0:
            if is_add:
                return False                                     # already added
            del table[idx]
            return True
    if is_add:
        table.append(rule)
        return True
    return False


class Renderer:
    """vpptcp.Renderer (vpptcp_renderer.go:34-73).  ``sink`` plays GoVPPChan's
    peer (a SessionRuleTables); ``engine`` (optional) compiles the committed
    IngressOrientation tables for TestTraffic-semantics evaluation on the GPU."""

    def __init__(self, contiv, sink: SessionRuleTables, chan_buf_size: int = 0, engine=None):
        self.contiv = contiv
        self.sink = sink
        self.chan_buf_size = chan_buf_size
        self.engine = engine
        self.cache: Optional[RendererCache] = None
        self.rule_tables: Dict[str, object] = {}     # table id -> traffic.RuleTable
        self.sessions = None                         # sessions.SessionEvaluator of the sink's rules

    def init(self) -> "Renderer":
        self.cache = RendererCache()
        self.cache.init(INGRESS_ORIENTATION)
        return self

    def new_txn(self, resync: bool) -> "RendererTxn":
        return RendererTxn(self, resync)

    def update_rules(self, add: List[SessionRule], remove: List[SessionRule]) -> None:
        """updateRules (:270-327): deletions first, then additions, sent in
        batches of the channel buffer size; the first failed reply aborts."""
        requests = [(r, False) for r in remove] + [(r, True) for r in add]
        buf = self.chan_buf_size or 100
        i = 0
        while i < len(requests):
            batch = requests[i:i + buf]
            i += len(batch)
            retvals = [self.sink.add_del(r, is_add) for r, is_add in batch]
            if any(rv != 0 for rv in retvals):
                raise RuntimeError("failed to update VPPTCP session rule")

    # -- GPU evaluation of the committed tables ----------------------------------
    def _sync_rule_tables(self):
        if self.engine is None:
            return
        from .sessions import SessionEvaluator
        from .traffic import RuleTable
        if self.sessions is None:
            self.sessions = SessionEvaluator(self.engine, self.sink)
        self.sessions.sync()
        want = {}
        g = self.cache.get_global_table()
        want[GLOBAL_TABLE_ID] = g
        for t in self.cache.local_tables.tables:
            if len(t.pods):
                want[t.id] = t
        for tid in list(self.rule_tables):
            if tid not in want or self.rule_tables[tid].rules != want[tid].rules[:want[tid].num_of_rules]:
                self.rule_tables.pop(tid).close()
        for tid, t in want.items():
            if tid not in self.rule_tables:
                self.rule_tables[tid] = RuleTable(self.engine, "vpptcp/" + tid, t.rules[:t.num_of_rules])

    def local_rule_table(self, pod: PodID):
        t = self.cache.local_tables.lookup_by_pod(pod)
        return None if t is None else self.rule_tables.get(t.id)

    def global_rule_table(self):
        return self.rule_tables.get(GLOBAL_TABLE_ID)

    def close(self):
        for t in self.rule_tables.values():
            t.close()
        self.rule_tables.clear()
        if self.sessions is not None:
            self.sessions.close()


class RendererTxn:
    """vpptcp.RendererTxn (vpptcp_renderer.go:53-192)."""

    def __init__(self, renderer: Renderer, resync: bool):
        self.renderer = renderer
        self.cache_txn = renderer.cache.new_txn()
        self.resync = resync

    def render(self, pod: PodID, pod_ip: IPNet, ingress, egress, removed: bool) -> "RendererTxn":
        self.cache_txn.update(pod, PodConfig(pod_ip, list(ingress), list(egress), removed))
        return self

    def commit(self) -> None:
        r = self.renderer
        added: List[SessionRule] = []
        removed: List[SessionRule] = []
        if self.resync:
            tables = import_session_rules(self.dump_rules(), r.contiv)
            r.cache.resync(tables)
            txn_pods = self.cache_txn.get_updated_pods()
            for pod in list(r.cache.get_all_pods()):
                if not txn_pods.has(pod):
                    self.cache_txn.update(pod, PodConfig(removed=True))

        for pod in sorted(self.cache_txn.get_updated_pods(), key=tuple):
            new_rules: List[ContivRule] = []
            removed_rules: List[ContivRule] = []
            cfg = self.cache_txn.get_pod_config(pod)
            if cfg.removed:
                cfg = r.cache.get_pod_config(pod)
                if cfg is None:
                    continue
            orig = r.cache.get_local_table_by_pod(pod)
            new = self.cache_txn.get_local_table_by_pod(pod)
            if orig is None and new is not None:
                new_rules = new.rules[:new.num_of_rules]
            if orig is not None and new is None:
                removed_rules = orig.rules[:orig.num_of_rules]
            if orig is not None and new is not None and orig.id != new.id:
                removed_rules, new_rules = orig.diff_rules(new)
            pod_ip = cfg.pod_ip.ip if cfg.pod_ip is not None else None
            added.extend(export_session_rules(new_rules, pod, pod_ip, r.contiv))
            removed.extend(export_session_rules(removed_rules, pod, pod_ip, r.contiv))

        orig_g = r.cache.get_global_table()
        new_g = self.cache_txn.get_global_table()
        removed_rules, new_rules = orig_g.diff_rules(new_g)
        added.extend(export_session_rules(new_rules, None, None, r.contiv))
        removed.extend(export_session_rules(removed_rules, None, None, r.contiv))

        if added or removed:
            r.update_rules(added, removed)
        self.cache_txn.commit()
        r._sync_rule_tables()

    def dump_rules(self) -> List[SessionRule]:
        """dumpRules (:195-238): only rules tagged by this renderer."""
        return [x for x in self.renderer.sink.dump() if x.tag_string().startswith(SESSION_RULE_TAG_PREFIX)]
