"""Renderer cache: builds the ContivRuleTables whose first-match the engine evaluates.

Restates plugins/policy/renderer/cache/ (cache_api.go:199-329 ContivRuleTable,
cache_impl.go:31-713 RendererCache / RendererCacheTxn, local_tables.go:43-263
LocalTables, ports.go:25-161 Ports).  Host-side control plane: it produces
the tables that the ACL renderer turns into ACLs (acl.py) which are then
compiled and classified on the GPU.

Deviations (documented, no effect on rendered rules or verdicts):
  * Table IDs come from a deterministic counter instead of crypto/rand
    (cache_impl.go:676-689); they only name ACLs.
  * ``rules`` holds exactly NumOfRules entries (the Go slice may carry trailing
    nils after RemoveByIdx, which only perturbs LocalTables' internal order).
"""
from __future__ import annotations

import bisect
import itertools
from typing import Dict, Iterable, List, Optional

from ..gonet import IPNet
from .api import (ACTION_DENY, ACTION_PERMIT, ANY_PORT, TCP, UDP, ContivRule, PodID,
                  allow_all_tcp, allow_all_udp, compare_rule_lists, rule_key)
from .. import gonet

# Orientation (cache_api.go)
INGRESS_ORIENTATION = 0
EGRESS_ORIENTATION = 1

# TableType
LOCAL = 0
GLOBAL = 1
GLOBAL_TABLE_ID = "GLOBAL"


class PodSet(set):
    """cache.PodSet"""

    def has(self, pod) -> bool:
        return pod in self

    def copy(self) -> "PodSet":
        return PodSet(self)

    def join(self, other: Iterable) -> "PodSet":
        return PodSet(set(self) | set(other))

    def equals(self, other) -> bool:
        return set(self) == set(other)


class PodConfig:
    """cache.PodConfig: pod IP and its ingress/egress ContivRules."""

    def __init__(self, pod_ip: Optional[IPNet] = None, ingress=None, egress=None,
                 removed: bool = False):
        self.pod_ip = pod_ip
        self.ingress = list(ingress or [])
        self.egress = list(egress or [])
        self.removed = removed


class ContivRuleTable:
    """ContivRuleTable (cache_api.go:199-265,267-329)."""

    def __init__(self, table_id: str):
        self.id = table_id
        self.type = GLOBAL if table_id == GLOBAL_TABLE_ID else LOCAL
        self.pods = PodSet()
        self.rules: List[ContivRule] = []
        self.private = None

    @property
    def num_of_rules(self) -> int:
        return len(self.rules)

    def _rule_index(self, rule: ContivRule):
        lo, hi = 0, len(self.rules)
        while lo < hi:                      # sort.Search(compare <= 0)
            mid = (lo + hi) // 2
            if rule.compare(self.rules[mid]) <= 0:
                hi = mid
            else:
                lo = mid + 1
        found = lo < len(self.rules) and rule.compare(self.rules[lo]) == 0
        return lo, found

    def insert_rule(self, rule: ContivRule) -> bool:
        idx, found = self._rule_index(rule)
        if found:
            return False
        self.rules.insert(idx, rule)
        return True

    def remove_by_predicate(self, pred) -> int:
        before = len(self.rules)
        self.rules = [r for r in self.rules if not pred(r)]
        return before - len(self.rules)

    def has_rule(self, rule: ContivRule) -> bool:
        return self._rule_index(rule)[1]

    def diff_rules(self, other: "ContivRuleTable"):
        not_in_2 = [r for r in self.rules if not other.has_rule(r)]
        not_in_this = [r for r in other.rules if not self.has_rule(r)]
        return not_in_2, not_in_this

    def shallow_copy(self) -> "ContivRuleTable":
        t = ContivRuleTable(self.id)
        t.type = self.type
        t.rules = self.rules
        t.pods = self.pods.copy()
        t.private = self.private
        return t

    def __repr__(self) -> str:
        return "Rule Table %s <rules: %r, pods: %s>" % (self.id, self.rules, sorted(map(str, self.pods)))


class Ports(set):
    """cache.Ports (ports.go:25-103); 0 = AnyPort."""

    def has(self, port: int) -> bool:
        return ANY_PORT in self or port in self

    def is_subset_of(self, p2: "Ports") -> bool:
        if p2.has(ANY_PORT):
            return True
        if self.has(ANY_PORT):
            return False
        return all(p2.has(p) for p in self)

    def intersection(self, p2: "Ports") -> "Ports":
        if self.has(ANY_PORT):
            return p2
        if p2.has(ANY_PORT):
            return self
        return Ports(p for p in self if p2.has(p))


def get_allowed_egress_ports(src_ip: IPNet, egress) -> tuple:
    """getAllowedEgressPorts (ports.go:107-132)."""
    tcp, udp = Ports(), Ports()
    has_deny = False
    for rule in egress:
        if rule.action == ACTION_DENY:
            has_deny = True
            continue
        if len(rule.src_network.ip) > 0 and not rule.src_network.contains(src_ip.ip):
            continue
        (tcp if rule.protocol == TCP else udp).add(rule.dest_port)
    if not has_deny:
        return Ports([ANY_PORT]), Ports([ANY_PORT])
    return tcp, udp


def get_allowed_ingress_ports(dst_ip: IPNet, ingress) -> tuple:
    """getAllowedIngressPorts (ports.go:136-161)."""
    tcp, udp = Ports(), Ports()
    has_deny = False
    for rule in ingress:
        if rule.action == ACTION_DENY:
            has_deny = True
            continue
        if len(rule.dest_network.ip) > 0 and not rule.dest_network.contains(dst_ip.ip):
            continue
        (tcp if rule.protocol == TCP else udp).add(rule.dest_port)
    if not has_deny:
        return Ports([ANY_PORT]), Ports([ANY_PORT])
    return tcp, udp


class _KeyedRules(list):
    """A rule list built in keyed form, carrying its keys (valid while its
    length is unchanged)."""
    __slots__ = ("keys",)


def _list_keys(rules):
    """The rules' keys as one tuple (None if some rule has no key)."""
    if isinstance(rules, _KeyedRules) and len(rules.keys) == len(rules):
        return rules.keys
    keys = []
    for r in rules:
        k = rule_key(r)
        if k is None:
            return None
        keys.append(k)
    return tuple(keys)


def _table_keys(t: "ContivRuleTable"):
    c = getattr(t, "_rkeys", None)
    if c is not None and c[0] is t.rules and c[1] == len(t.rules):
        return c[2]
    k = _list_keys(t.rules)
    t._rkeys = (t.rules, len(t.rules), k)
    return k


class LocalTables:
    """LocalTables (local_tables.go:43-263): tables ordered by rule lists."""

    def __init__(self):
        self.tables: List[ContivRuleTable] = []
        self.by_id: Dict[str, ContivRuleTable] = {}
        self.by_pod: Dict[PodID, ContivRuleTable] = {}

    def _lookup_idx_by_rules(self, rules) -> int:
        # compareRuleLists by length, then rule by rule: with every rule keyed
        # (api.rule_key) the same order is one tuple comparison
        qk = _list_keys(rules) if KEYED else None
        lo, hi = 0, len(self.tables)
        while lo < hi:
            mid = (lo + hi) // 2
            tk = _table_keys(self.tables[mid]) if qk is not None else None
            if tk is not None:
                c = (len(rules) > len(tk)) - (len(rules) < len(tk)) or (qk > tk) - (qk < tk)
            else:
                c = compare_rule_lists(rules, self.tables[mid].rules)
            if c <= 0:
                hi = mid
            else:
                lo = mid + 1
        return lo

    def insert(self, table: ContivRuleTable) -> bool:
        if table.id in self.by_id:
            return False
        self.tables.insert(self._lookup_idx_by_rules(table.rules), table)
        self.by_id[table.id] = table
        for pod in list(table.pods):
            self.unassign_pod(None, pod)
            self.by_pod[pod] = table
        return True

    def remove(self, table: ContivRuleTable) -> bool:
        for i, t in enumerate(self.tables):
            if t is table:
                return self.remove_by_idx(i)
        return False

    def remove_by_idx(self, idx: int) -> bool:
        if idx >= len(self.tables):
            return False
        table = self.tables.pop(idx)
        self.by_id.pop(table.id, None)
        for pod in table.pods:
            self.by_pod.pop(pod, None)
        return True

    def assign_pod(self, table: ContivRuleTable, pod: PodID):
        self.unassign_pod(None, pod)
        table.pods.add(pod)
        self.by_pod[pod] = table

    def unassign_pod(self, table: Optional[ContivRuleTable], pod: PodID):
        if table is not None:
            table.pods.discard(pod)
        t2 = self.by_pod.get(pod)
        if t2 is not None and (table is None or table is t2):
            t2.pods.discard(pod)
            del self.by_pod[pod]

    def lookup_by_id(self, table_id: str) -> Optional[ContivRuleTable]:
        return self.by_id.get(table_id)

    def lookup_by_rules(self, rules) -> Optional[ContivRuleTable]:
        idx = self._lookup_idx_by_rules(rules)
        if idx < len(self.tables):
            t = self.tables[idx]
            qk = _list_keys(rules) if KEYED else None
            tk = _table_keys(t) if qk is not None else None
            if (qk == tk) if tk is not None else compare_rule_lists(rules, t.rules) == 0:
                return t
        return None

    def lookup_by_pod(self, pod: PodID) -> Optional[ContivRuleTable]:
        return self.by_pod.get(pod)

    def get_isolated_pods(self) -> PodSet:
        return PodSet(p for p, t in self.by_pod.items() if t.num_of_rules > 0)


class TxnChange:
    def __init__(self, table: ContivRuleTable, previous_pods: Optional[PodSet] = None):
        self.table = table
        self.previous_pods = previous_pods if previous_pods is not None else PodSet()


_ids = itertools.count(1)

# Keyed table construction (_LocalCtx, _rebuild_global_table); False: the
# literal InsertRule path only (tests compare the two).
KEYED = True


class RendererCache:
    """RendererCache (cache_impl.go:31-191)."""

    def __init__(self):
        self.orientation = EGRESS_ORIENTATION
        self.flush()

    def init(self, orientation: int):
        self.orientation = orientation
        self.flush()

    def flush(self):
        self.local_tables = LocalTables()
        self.global_table = ContivRuleTable(GLOBAL_TABLE_ID)
        self.allocated_ids = set()
        self.config: Dict[PodID, PodConfig] = {}

    def new_txn(self) -> "RendererCacheTxn":
        return RendererCacheTxn(self)

    def resync(self, tables) -> None:
        """Resync (cache_impl.go:102-147); raises ValueError like the Go error."""
        config, allocated = {}, set()
        local_tables = LocalTables()
        global_table = ContivRuleTable(GLOBAL_TABLE_ID)
        for table in tables:
            if table is None:
                continue
            if table.type == GLOBAL:
                global_table = table
                continue
            if len(table.pods) == 0:
                continue
            if table.id in allocated:
                raise ValueError("duplicate ContivRuleTable ID: %s" % table.id)
            allocated.add(table.id)
            local_tables.insert(table)
            for pod in table.pods:
                if pod in config:
                    raise ValueError("pod assigned to multiple local tables: %s" % (pod,))
                config[pod] = PodConfig()
        self.allocated_ids = allocated
        self.local_tables = local_tables
        self.global_table = global_table
        self.config = config

    def get_pod_config(self, pod: PodID) -> Optional[PodConfig]:
        return self.config.get(pod)

    def get_all_pods(self) -> PodSet:
        return PodSet(self.config.keys())

    def get_isolated_pods(self) -> PodSet:
        return self.local_tables.get_isolated_pods()

    def get_local_table_by_pod(self, pod: PodID) -> Optional[ContivRuleTable]:
        t = self.local_tables.lookup_by_pod(pod)
        if t is not None and t.num_of_rules == 0:
            return None
        return t

    def get_global_table(self) -> ContivRuleTable:
        return self.global_table


class RendererCacheTxn:
    """RendererCacheTxn (cache_impl.go:51-713)."""

    def __init__(self, cache: RendererCache):
        self.cache = cache
        self.local_tables = LocalTables()
        self.global_table: Optional[ContivRuleTable] = None
        self.up_to_date = False
        self.config: Dict[PodID, PodConfig] = {}

    def update(self, pod: PodID, cfg: PodConfig):
        self.config[pod] = cfg
        self.up_to_date = False

    def get_updated_pods(self) -> PodSet:
        return PodSet(self.config.keys())

    def get_removed_pods(self) -> PodSet:
        return PodSet(p for p, c in self.config.items() if c.removed)

    def get_changes(self) -> List[TxnChange]:
        if not self.up_to_date:
            self._refresh_tables()
        changes = []
        for txn_table in self.local_tables.tables:
            orig = self.cache.local_tables.lookup_by_id(txn_table.id)
            if txn_table.num_of_rules == 0:
                continue
            if len(txn_table.pods) == 0 and orig is None:
                continue
            if orig is not None and txn_table.pods.equals(orig.pods):
                continue
            changes.append(TxnChange(txn_table, orig.pods.copy() if orig is not None else PodSet()))
        if self.global_table is not None and compare_rule_lists(
                self.global_table.rules, self.cache.global_table.rules) != 0:
            changes.append(TxnChange(self.global_table))
        return changes

    def commit(self) -> None:
        if not self.up_to_date:
            self._refresh_tables()
        for txn_table in list(self.local_tables.tables):
            orig = self.cache.local_tables.lookup_by_id(txn_table.id)
            if orig is not None:
                if len(txn_table.pods) == 0:
                    self.cache.local_tables.remove(txn_table)
                elif not txn_table.pods.equals(orig.pods):
                    for pod in list(orig.pods):
                        if not txn_table.pods.has(pod):
                            self.cache.local_tables.unassign_pod(orig, pod)
                    for pod in list(txn_table.pods):
                        if not orig.pods.has(pod):
                            self.cache.local_tables.assign_pod(orig, pod)
                    orig.private = txn_table.private
            else:
                if len(txn_table.pods) != 0:
                    self.cache.local_tables.insert(txn_table)
        if self.global_table is not None and compare_rule_lists(
                self.global_table.rules, self.cache.global_table.rules) != 0:
            self.cache.global_table = self.global_table
        for pod, cfg in self.config.items():
            if cfg.removed:
                self.cache.config.pop(pod, None)
                self.cache.local_tables.unassign_pod(None, pod)
            else:
                self.cache.config[pod] = cfg

    def get_pod_config(self, pod: PodID) -> Optional[PodConfig]:
        if pod in self.config:
            return self.config[pod]
        return self.cache.get_pod_config(pod)

    def get_all_pods(self) -> PodSet:
        pods = self.cache.get_all_pods()
        for pod, cfg in self.config.items():
            if not cfg.removed:
                pods.add(pod)
            else:
                pods.discard(pod)
        return pods

    def get_isolated_pods(self) -> PodSet:
        if not self.up_to_date:
            self._refresh_tables()
        isolated = self.local_tables.get_isolated_pods()
        for pod in self.cache.get_isolated_pods():
            if self.local_tables.lookup_by_pod(pod) is None:
                isolated.add(pod)
        return isolated

    def get_local_table_by_pod(self, pod: PodID) -> Optional[ContivRuleTable]:
        if not self.up_to_date:
            self._refresh_tables()
        t = self.local_tables.lookup_by_pod(pod)
        if t is not None and t.num_of_rules == 0:
            return None
        if t is not None:
            return t
        return self.cache.get_local_table_by_pod(pod)

    def get_global_table(self) -> ContivRuleTable:
        if not self.up_to_date:
            self._refresh_tables()
        if self.global_table is not None:
            return self.global_table
        return self.cache.global_table

    # -- table construction (cache_impl.go:418-673) ---------------------------
    def _refresh_tables(self):
        self._ctx = _LocalCtx(self)
        for pod in sorted(self.get_all_pods().join(self.get_removed_pods()), key=tuple):
            cfg = self.get_pod_config(pod)
            new_table = self._build_local_table(pod, cfg)
            orig = self.cache.local_tables.lookup_by_pod(pod)
            if orig is not None and self.local_tables.lookup_by_id(orig.id) is None:
                self.local_tables.insert(orig.shallow_copy())
            txn_table = self.local_tables.lookup_by_rules(new_table.rules)
            if txn_table is not None:
                self.local_tables.assign_pod(txn_table, pod)
                self.cache.allocated_ids.discard(new_table.id)
                continue
            cache_table = self.cache.local_tables.lookup_by_rules(new_table.rules)
            if cache_table is not None:
                updated = cache_table.shallow_copy()
                updated.pods.add(pod)
                self.local_tables.insert(updated)
                self.cache.allocated_ids.discard(new_table.id)
                continue
            self.local_tables.insert(new_table)
        self._rebuild_global_table()
        self._ctx = None
        self.up_to_date = True

    def _build_local_table(self, dst_pod: PodID, dst_cfg: PodConfig) -> ContivRuleTable:
        table = ContivRuleTable(self._generate_table_id())
        table.pods.add(dst_pod)
        if dst_cfg.removed:
            return table
        ctx = getattr(self, "_ctx", None)
        if KEYED and ctx is not None and ctx.ok:
            try:
                table.rules = ctx.local_rules(dst_cfg)
                return table
            except ValueError:
                pass                        # outside the keyed form: the literal path
        rules = dst_cfg.egress if self.cache.orientation == EGRESS_ORIENTATION else dst_cfg.ingress
        for rule in rules:
            table.insert_rule(rule.copy())
        for src_pod in sorted(self.get_all_pods(), key=tuple):
            self._install_local_rules(table, dst_cfg, self.get_pod_config(src_pod))
        if table.num_of_rules > 0:
            all_tcp = all_udp = False
            for r in table.rules:
                if r.dest_port == 0 and len(r.src_network.ip) == 0 and len(r.dest_network.ip) == 0:
                    if r.protocol == TCP:
                        all_tcp = True
                    else:
                        all_udp = True
            if not all_tcp:
                table.insert_rule(allow_all_tcp())
            if not all_udp:
                table.insert_rule(allow_all_udp())
        return table

    def _install_local_rules(self, dst_table, dst_cfg: PodConfig, src_cfg: PodConfig):
        if self.cache.orientation == EGRESS_ORIENTATION:
            src_tcp, src_udp = get_allowed_ingress_ports(dst_cfg.pod_ip, src_cfg.ingress)
            dst_tcp, dst_udp = get_allowed_egress_ports(src_cfg.pod_ip, dst_cfg.egress)
        else:
            src_tcp, src_udp = get_allowed_egress_ports(dst_cfg.pod_ip, src_cfg.egress)
            dst_tcp, dst_udp = get_allowed_ingress_ports(src_cfg.pod_ip, dst_cfg.ingress)
        if not dst_tcp.is_subset_of(src_tcp):
            self._install_allowed_ports(dst_table, src_cfg.pod_ip, dst_tcp.intersection(src_tcp), TCP)
        if not dst_udp.is_subset_of(src_udp):
            self._install_allowed_ports(dst_table, src_cfg.pod_ip, dst_udp.intersection(src_udp), UDP)

    def _install_allowed_ports(self, dst_table, src_pod_ip: IPNet, allowed: Ports, protocol: int):
        egress = self.cache.orientation == EGRESS_ORIENTATION

        def pred(rule: ContivRule) -> bool:
            if rule.protocol != protocol:
                return False
            addr = rule.src_network if egress else rule.dest_network
            if len(addr.ip) == 0:
                return False
            ones, bits = gonet.mask_size(addr.mask)
            if ones != bits or not gonet.ip_equal(addr.ip, src_pod_ip.ip):
                return False
            return True

        dst_table.remove_by_predicate(pred)
        for port in sorted(allowed):
            r = ContivRule(ACTION_PERMIT, IPNet(), IPNet(), protocol, ANY_PORT, port)
            if egress:
                r.src_network = src_pod_ip
            else:
                r.dest_network = src_pod_ip
            dst_table.insert_rule(r)
        r = ContivRule(ACTION_DENY, IPNet(), IPNet(), protocol, ANY_PORT, ANY_PORT)
        if egress:
            r.src_network = src_pod_ip
        else:
            r.dest_network = src_pod_ip
        dst_table.insert_rule(r)

    def _rebuild_global_table(self):
        self.global_table = ContivRuleTable(GLOBAL_TABLE_ID)
        pods = sorted(self.get_all_pods(), key=tuple)
        # keyed form (one sort, first of equal rules kept -- InsertRule's
        # outcome) when every rule has a key; else sorted insertions
        egress = self.cache.orientation == EGRESS_ORIENTATION
        rules = []
        for pod in pods:
            cfg = self.get_pod_config(pod)
            for rule in (cfg.ingress if egress else cfg.egress):
                c = rule.copy()
                if egress:
                    c.src_network = cfg.pod_ip
                else:
                    c.dest_network = cfg.pod_ip
                rules.append(c)
        keys = [rule_key(r) for r in rules]
        if KEYED and all(k is not None for k in keys):
            if rules:
                rules += [allow_all_tcp(), allow_all_udp()]
                keys += [rule_key(rules[-2]), rule_key(rules[-1])]
            out, last = [], None
            for k, i in sorted((k, i) for i, k in enumerate(keys)):
                if k != last:
                    out.append(rules[i])
                    last = k
            self.global_table.rules = out
            return
        for pod in pods:
            self._install_global_rules(self.get_pod_config(pod))
        if self.global_table.num_of_rules > 0:
            self.global_table.insert_rule(allow_all_tcp())
            self.global_table.insert_rule(allow_all_udp())

    def _install_global_rules(self, cfg: PodConfig):
        egress = self.cache.orientation == EGRESS_ORIENTATION
        rules = cfg.ingress if egress else cfg.egress
        for rule in rules:
            c = rule.copy()
            if egress:
                c.src_network = cfg.pod_ip
            else:
                c.dest_network = cfg.pod_ip
            self.global_table.insert_rule(c)

    def _generate_table_id(self) -> str:
        while True:
            tid = "%010X" % next(_ids)
            if tid not in self.cache.allocated_ids:
                self.cache.allocated_ids.add(tid)
                return tid


class _LocalCtx:
    """One refresh's shared state for building local tables in sorted-key form.

    buildLocalTable (cache_impl.go:488-535) inserts the pod's own rules, then
    for every pod on the node (installLocalRules :543-571) removes the rules
    whose source (egress orientation; destination for ingress) is that pod's
    host route, and inserts its allowed-port permits and a deny
    (installAllowedPorts :576-634) -- every InsertRule a sorted insertion,
    O(R) each.  Here the same rule multiset is collected and sorted once by a
    key consistent with Compare (api.rule_key), keeping the first of equal
    rules as InsertRule does.  The allowed-port sets depend only on a rule
    list and one address, so they are computed once per (list content,
    address).  Exactness needs: every pod address a host route and distinct
    (the removals of one pod then touch only that pod's rules) and every rule
    keyable; otherwise ``ok`` is False and the literal path runs.
    Equivalence: tests/test_cache_fast_cpu.py."""

    def __init__(self, txn: "RendererCacheTxn"):
        self.egress = txn.cache.orientation == EGRESS_ORIENTATION
        pods = sorted(txn.get_all_pods(), key=tuple)
        self.src = []                  # (ip16, pod_ip, id of its opposite-side rule list)
        self.ok = True
        # Content caches, kept by the renderer cache across refreshes (a txn
        # rebuilds every local table, cache_impl.go:420-474, but the rule
        # lists, addresses and allowed-port sets mostly repeat): list content
        # -> id, (fn, list id, address) -> port sets, one object per
        # port-set content, table signature -> table.
        memo = getattr(txn.cache, "_local_memo", None)
        if memo is None or len(memo["pcache"]) > 4_000_000 or memo["egress"] != self.egress:
            memo = txn.cache._local_memo = {"egress": self.egress, "lists": {}, "pcache": {}, "pint": {},
                                            "built": {}}
        self._lists = memo["lists"]
        self._pcache = memo["pcache"]
        self._pint = memo["pint"]
        self._built = memo["built"]
        seen = set()
        for pod in pods:
            cfg = txn.get_pod_config(pod)
            ip16 = self._host16(cfg.pod_ip)
            if ip16 is None or ip16 in seen:
                self.ok = False
                return
            seen.add(ip16)
            lid = self._intern(cfg.ingress if self.egress else cfg.egress)
            if lid is None:
                self.ok = False
                return
            self.src.append((ip16, cfg.pod_ip, lid, cfg.ingress if self.egress else cfg.egress))
        # sources grouped by rule list: a destination's allowed-port sets are
        # computed once per distinct list, not once per source pod
        firsts = {}
        for k, (_, _, lid, rules) in enumerate(self.src):
            firsts.setdefault(lid, (len(firsts), rules))
        self.lids = [(lid, rules) for lid, (_, rules) in sorted(firsts.items(), key=lambda kv: kv[1][0])]
        self.src_slot = [firsts[lid][0] for _, _, lid, _ in self.src]
        sets = memo.setdefault("srcsets", {})
        self.srcset = sets.setdefault(tuple((ip16, lid) for ip16, _, lid, _ in self.src), len(sets))

    @staticmethod
    def _host16(net):
        if net is None or len(net.ip) == 0:
            return None
        ones, bits = gonet.mask_size(net.mask)
        if bits == 0 or ones != bits:
            return None
        return gonet.to16(net.ip)

    def _intern(self, rules):
        keys = []
        for r in rules:
            k = rule_key(r)
            if k is None:
                return None
            keys.append(k)
        return self._lists.setdefault(tuple(keys), len(self._lists))

    def _ports(self, fn, lid, rules, net, ip16):
        k = (fn is get_allowed_ingress_ports, lid, ip16)
        v = self._pcache.get(k)
        if v is None:
            v = fn(net, rules)
            v = self._pcache[k] = self._pint.setdefault((frozenset(v[0]), frozenset(v[1])), v)   # one object per content
        return v

    def local_rules(self, dst_cfg: PodConfig):
        """The sorted rules of the destination pod's local table, or raises
        if a rule is not keyable (the caller checked ok)."""
        egress = self.egress
        own = dst_cfg.egress if egress else dst_cfg.ingress
        dst16 = self._host16(dst_cfg.pod_ip)
        own_lid = self._intern(own)
        if dst16 is None or own_lid is None:
            raise ValueError("local table outside the keyed form")
        # The table depends on the destination pod only through its own rule
        # list and the source pods' allowed ports towards it: equal
        # signatures, equal tables (built once per refresh).
        sfn = get_allowed_ingress_ports if egress else get_allowed_egress_ports
        sp_lid = [self._ports(sfn, lid, rules, dst_cfg.pod_ip, dst16) for lid, rules in self.lids]
        # The table depends on the destination only through its own list and
        # the allowed-port sets; the source pods (addresses and lists) are
        # named by the refresh's interned source set.
        sig = (own_lid, self.srcset, tuple(map(id, sp_lid)))
        hit = self._built.get(sig)
        if hit is not None:
            return self._keyed(*hit)
        sp_all = [sp_lid[k] for k in self.src_slot]
        base = [r.copy() for r in own]
        # base rules a pod's installAllowedPorts would remove: (protocol, host ip16)
        removable = {}
        for i, r in enumerate(base):
            h = self._host16(r.src_network if egress else r.dest_network)
            if h is not None:
                removable.setdefault((r.protocol, h), []).append(i)
        dropped = set()
        installed = []
        dfn = get_allowed_egress_ports if egress else get_allowed_ingress_ports
        for (ip16, pod_ip, lid, rules), (src_tcp, src_udp) in zip(self.src, sp_all):
            dst_tcp, dst_udp = self._ports(dfn, own_lid, own, pod_ip, ip16)
            for proto, d, sp in ((TCP, dst_tcp, src_tcp), (UDP, dst_udp, src_udp)):
                if d.is_subset_of(sp):
                    continue
                dropped.update(removable.get((proto, ip16), ()))
                for port in sorted(d.intersection(sp)):
                    r = ContivRule(ACTION_PERMIT, IPNet(), IPNet(), proto, ANY_PORT, port)
                    if egress:
                        r.src_network = pod_ip
                    else:
                        r.dest_network = pod_ip
                    installed.append(r)
                r = ContivRule(ACTION_DENY, IPNet(), IPNet(), proto, ANY_PORT, ANY_PORT)
                if egress:
                    r.src_network = pod_ip
                else:
                    r.dest_network = pod_ip
                installed.append(r)
        rules = [r for i, r in enumerate(base) if i not in dropped] + installed
        if rules:
            all_tcp = all_udp = False
            for r in rules:
                if r.dest_port == 0 and len(r.src_network.ip) == 0 and len(r.dest_network.ip) == 0:
                    if r.protocol == TCP:
                        all_tcp = True
                    else:
                        all_udp = True
            if not all_tcp:
                rules.append(allow_all_tcp())
            if not all_udp:
                rules.append(allow_all_udp())
        keyed = sorted(((rule_key(r), i) for i, r in enumerate(rules)))   # stable: equal keys by position
        out, keys, last = [], [], None
        for k, i in keyed:
            if k != last:
                out.append(rules[i])
                keys.append(k)
                last = k
        self._built[sig] = (out, tuple(keys))
        return self._keyed(out, self._built[sig][1])

    @staticmethod
    def _keyed(rules, keys):
        r = _KeyedRules(rules)
        r.keys = keys
        return r


def build_global_table(pods) -> ContivRuleTable:
    """Fast path of rebuildGlobalTable for large synthetic renders (config 2/3).

    ``pods`` is an iterable of (pod_ip: IPNet, ingress rules).  Equivalent to
    RendererCacheTxn._rebuild_global_table in EgressOrientation
    (cache_impl.go:638-673), but sorts once (O(R log R)) instead of R sorted
    insertions; the resulting order is identical because Compare is a total
    order and duplicates (Compare == 0) keep the first inserted element.
    """
    import functools
    rules = []
    for pod_ip, ingress in pods:
        for r in ingress:
            c = r.copy()
            c.src_network = pod_ip
            rules.append(c)
    table = ContivRuleTable(GLOBAL_TABLE_ID)
    if not rules:
        return table
    rules.append(allow_all_tcp())
    rules.append(allow_all_udp())
    keyf = functools.cmp_to_key(lambda a, b: a.compare(b))
    order = sorted(range(len(rules)), key=lambda i: keyf(rules[i]))  # stable
    out = []
    for i in order:
        if out and rules[i].compare(out[-1]) == 0:
            continue
        out.append(rules[i])
    table.rules = out
    return table
