"""Packet evaluation of installed VPP session rules on the GPU.

The VPPTCP renderer exports ContivRules as VPP session rules
(plugins/policy/renderer/vpptcp/rule/session_rule.go:201-331) and the
session-rule sink stores them (mock/sessionrules/sessionrules_mock.go).  The
reference never evaluates a packet against session rules; VPP's session-table
lookup is external.  This module evaluates the rules *as exported*, so the
export's own effects reach the packets:

  * allow-all-destination rules are not installed (:220-224) -- the stack
    default (allow) answers for them;
  * local rules whose remote is the pod itself are not installed (:226-232);
  * an empty remote network is installed as the two halves 0.0.0.0/1 and
    128.0.0.0/1 with IsIP4 = 1 (:245-252, :311-322), so a deny-all covers
    IPv4 only;
  * every rule belongs to one address family (IsIP4): a 0-length local
    prefix still only matches addresses of that family.

Semantics (defined by this build -- parity unpinned):
  * a table is the global table or one app namespace's local table of the
    sink; its rules are taken in the reference's first-match order, the
    ContivRule Compare order (renderer/api.go:114-136) of the rule each
    session rule describes, and the first match decides: ALLOW or DENY;
  * global scope: the packet's destination is the local end (lcl prefix and
    port), its source the remote end (rmt prefix, port any);
  * local scope (connections made by the namespace's pod): the packet's
    destination is the remote end (rmt prefix and port), its source the
    local end (lcl = the family's 0/0);
  * a rule matches TCP or UDP packets of its transport protocol only; no
    rule matching (and every other protocol) gives ALLOW, the session
    layer's default.

GPU path: each session rule becomes the ContivRule-shaped rule it describes,
with the family kept (a 0-length prefix becomes 0.0.0.0/0 or ::/0, which
Go's IPNet.Contains restricts to that family), the table is sorted by
inserting them into a ContivRuleTable, and the list runs on the classifier
through vpp_amd.renderer.traffic (TestTraffic's ACL form; UNMATCHED reads as
ALLOW).  The CPU restatement the tests compare with is oracle/sessions.py.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from .. import gonet
from ..gonet import IPNet
from .api import ACTION_DENY, ACTION_PERMIT, TCP, UDP, ContivRule
from .cache import ContivRuleTable
from .traffic import DENIED_TRAFFIC, RuleTable
from .vpptcp import ACTION_ALLOW_IDX, PROTO_UDP, SCOPE_GLOBAL, SessionRule, SessionRuleTables

SESSION_DENY = 0
SESSION_ALLOW = 1


def _net(ip16: bytes, plen: int, is_ip4: int) -> IPNet:
    """A session rule prefix as a family-bound network (plen 0 included)."""
    n = 4 if is_ip4 else 16
    return IPNet(bytes(ip16[:n]), gonet.cidr_mask(min(plen, 8 * n), 8 * n))


def eval_rule(sr: SessionRule) -> ContivRule:
    """The ContivRule-shaped rule one installed session rule applies, in the
    frame of a packet (src, dst, dport): global scope src = rmt, dst = lcl,
    dport = lcl port; local scope src = lcl, dst = rmt, dport = rmt port."""
    lcl = _net(sr.lcl_ip, sr.lcl_plen, sr.is_ip4)
    rmt = _net(sr.rmt_ip, sr.rmt_plen, sr.is_ip4)
    glob = sr.scope == SCOPE_GLOBAL
    cr = ContivRule()
    cr.action = ACTION_PERMIT if sr.action_index == ACTION_ALLOW_IDX else ACTION_DENY
    cr.protocol = UDP if sr.transport_proto == PROTO_UDP else TCP
    cr.src_network, cr.dest_network = (rmt, lcl) if glob else (lcl, rmt)
    cr.src_port = sr.rmt_port if glob else sr.lcl_port
    cr.dest_port = sr.lcl_port if glob else sr.rmt_port
    return cr


def ordered(rules: List[SessionRule]) -> Tuple[List[ContivRule], List[int]]:
    """The table's rules in first-match order: (eval rules, index of the
    session rule each came from).  Equal eval rules (Compare == 0) keep the
    first; the shadowed duplicates never match."""
    t = ContivRuleTable("session")
    origin = {}
    for k, sr in enumerate(rules):
        cr = eval_rule(sr)
        if t.insert_rule(cr):
            origin[id(cr)] = k
    rl = t.rules[:t.num_of_rules]
    return rl, [origin[id(r)] for r in rl]


class SessionTable:
    """One installed session-rule table compiled onto the engine."""

    def __init__(self, engine, name: str, rules: List[SessionRule]):
        self.session_rules = [r.copy() for r in rules]
        self.rules, self.origin = ordered(self.session_rules)
        self.table = RuleTable(engine, name, self.rules)

    def evaluate(self, src, dst, proto, dport):
        """A packet batch (IPv4 uint32 host order or uint8[n, 16]; proto =
        ProtocolType) -> (SESSION_DENY / SESSION_ALLOW uint8[n], hits per
        session rule as given (u64), packets no rule matched)."""
        v, per_rule, unmatched = self.table.test_traffic_batch(src, dst, proto, dport)
        verdict = np.where(v == DENIED_TRAFFIC, SESSION_DENY, SESSION_ALLOW).astype(np.uint8)
        hits = np.zeros(len(self.session_rules), np.uint64)
        for i, k in enumerate(self.origin):
            hits[k] += np.uint64(per_rule[i])
        return verdict, hits, unmatched

    def close(self):
        self.table.close()


class SessionEvaluator:
    """The sink's installed tables on the GPU: the global table and one local
    table per app namespace, recompiled when their rules change."""

    def __init__(self, engine, sink: SessionRuleTables):
        self.engine = engine
        self.sink = sink
        self.tables: Dict[Optional[int], SessionTable] = {}
        self._sig: Dict[Optional[int], list] = {}

    def sync(self) -> None:
        want: Dict[Optional[int], List[SessionRule]] = {None: self.sink.global_table}
        for ns, rules in self.sink.local_table.items():
            if rules:
                want[ns] = rules
        for ns in list(self.tables):
            if ns not in want:
                self.tables.pop(ns).close()
                self._sig.pop(ns)
        for ns, rules in want.items():
            sig = [repr(r) for r in rules]
            if self._sig.get(ns) != sig:
                if ns in self.tables:
                    self.tables.pop(ns).close()
                self.tables[ns] = SessionTable(self.engine, "session/%s" % ("global" if ns is None else ns), rules)
                self._sig[ns] = sig

    def evaluate(self, ns_index: Optional[int], src, dst, proto, dport):
        """``ns_index`` None: the global table (packets arriving at a local
        destination); else that namespace's local table (connections its pod
        makes).  A namespace without rules allows everything."""
        t = self.tables.get(ns_index)
        if t is None:
            n = len(dport)
            return np.full(n, SESSION_ALLOW, np.uint8), np.zeros(0, np.uint64), n
        return t.evaluate(src, dst, proto, dport)

    def close(self):
        for t in self.tables.values():
            t.close()
        self.tables.clear()
        self._sig.clear()
