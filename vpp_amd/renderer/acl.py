"""ACL renderer: ContivRuleTables -> vpp_acl ACLs, committed through a txn sink.

Restates plugins/policy/renderer/acl/acl_renderer.go (Renderer :49-88,
RendererTxn.Render :109-119, Commit :124-264, reflectiveACL :267-295,
getNodeOutputInterfaces :299-309, renderACL :312-402, renderInterfaces
:406-426, dumpVppACLConfig :430-598).  The PolicyRendererAPI shape
(NewTxn(resync) -> Render(...) -> Commit()) is kept (renderer/api.go:33-61).

``acl_txn_factory`` plays the role of ``Deps.ACLTxnFactory``: it returns a
DataChangeDSL whose ``send()`` delivers the put/delete operations to the verdict
backend -- in the reference the MockACLEngine via localclient.TxnTracker
(mock/localclient/txn.go:48-131), here the GPU engine (vpp_amd.engine) or,
in tests, the CPU oracle.
"""
from __future__ import annotations

from typing import Callable, List, Optional

from .. import model
from ..gonet import IPNet
from .api import ACTION_DENY, ACTION_PERMIT, TCP, UDP, ContivRule, PodID
from .cache import (EGRESS_ORIENTATION, GLOBAL, LOCAL, ContivRuleTable, PodConfig, PodSet,
                    RendererCache)
from .. import gonet

ACL_NAME_PREFIX = "contiv/vpp-policy-"
REFLECTIVE_ACL_NAME = "REFLECTION"
MAX_PORT = 0xFFFF
MAX_ICMP_CODE = 5
MAX_ICMP_TYPE = 16


class ContivIfs:
    """The subset of contiv.API the ACL renderer and the engine use
    (mock/contiv/contiv_mock.go:14-220)."""

    def __init__(self, main_if: str = "", vxlan_bvi: str = "", host_interconnect: str = "",
                 other_physical=None):
        self.main_if = main_if
        self.vxlan_bvi = vxlan_bvi
        self.host_interconnect = host_interconnect
        self.other_physical = list(other_physical or [])
        self.pod_if = {}
        self.pod_app_ns = {}

    def set_pod_if_name(self, pod: PodID, if_name: str):
        self.pod_if[pod] = if_name

    def set_pod_app_ns_index(self, pod: PodID, ns_index: int):
        """SetPodAppNsIndex (contiv_mock.go:50-52)."""
        self.pod_app_ns[pod] = ns_index

    def get_ns_index(self, namespace: str, name: str):
        """GetNsIndex (contiv_mock.go:134-137)."""
        idx = self.pod_app_ns.get(PodID(name, namespace))
        return (0, False) if idx is None else (idx, True)

    def get_pod_by_app_ns_index(self, ns_index: int):
        """GetPodByAppNsIndex (contiv_mock.go:150-157)."""
        for pod, idx in self.pod_app_ns.items():
            if idx == ns_index:
                return pod.namespace, pod.name, True
        return "", "", False

    def get_if_name(self, namespace: str, name: str):
        name_if = self.pod_if.get(PodID(name, namespace))
        return name_if, name_if is not None

    def get_pod_by_if(self, if_name: str):
        for pod, name in self.pod_if.items():
            if name == if_name:
                return pod.namespace, pod.name, True
        return "", "", False

    def get_main_physical_if_name(self) -> str:
        return self.main_if

    def get_other_physical_if_names(self):
        return list(self.other_physical)

    def get_host_interconnect_if_name(self) -> str:
        return self.host_interconnect

    def get_vxlan_bvi_if_name(self) -> str:
        return self.vxlan_bvi


class DataChangeDSL:
    """linux.DataChangeDSL subset: Put().ACL / Delete().ACL / Send()."""

    def __init__(self, on_send: Callable[[list], None]):
        self.ops: List[tuple] = []   # (key, Acl or None)
        self._on_send = on_send

    def put_acl(self, acl: model.Acl):
        self.ops.append((model.acl_key(acl.acl_name), acl))

    def delete_acl(self, name: str):
        self.ops.append((model.acl_key(name), None))

    def send(self):
        self._on_send(self.ops)


class TxnTracker:
    """localclient.TxnTracker (mock/localclient/txn.go:16-131): records committed
    transactions and forwards each to ``on_commit`` (the engine's ApplyTxn)."""

    def __init__(self, on_commit):
        self.on_commit = on_commit
        self.committed = []
        self.pending = 0

    def new_linux_data_change_txn(self) -> DataChangeDSL:
        self.pending += 1

        def _send(ops):
            err = None
            if self.on_commit is not None:
                err = self.on_commit(ops)
            self.pending -= 1
            self.committed.append(ops)
            if err:
                raise RuntimeError(err)
        return DataChangeDSL(_send)


class Renderer:
    """acl.Renderer (acl_renderer.go:49-104)."""

    def __init__(self, contiv: ContivIfs, acl_txn_factory: Callable[[], DataChangeDSL],
                 vpp_dump: Optional[Callable[[], list]] = None):
        self.contiv = contiv
        self.acl_txn_factory = acl_txn_factory
        self.vpp_dump = vpp_dump or (lambda: [])
        self.cache: Optional[RendererCache] = None
        self.pod_interfaces = {}

    def init(self):
        self.cache = RendererCache()
        self.cache.init(EGRESS_ORIENTATION)
        self.pod_interfaces = {}
        return self

    def new_txn(self, resync: bool) -> "RendererTxn":
        return RendererTxn(self, resync)


class RendererTxn:
    """acl.RendererTxn (acl_renderer.go:66-426)."""

    def __init__(self, renderer: Renderer, resync: bool):
        self.renderer = renderer
        self.cache_txn = renderer.cache.new_txn()
        self.resync = resync

    def render(self, pod: PodID, pod_ip: IPNet, ingress, egress, removed: bool) -> "RendererTxn":
        self.cache_txn.update(pod, PodConfig(pod_ip, list(ingress), list(egress), removed))
        return self

    def commit(self) -> None:
        r = self.renderer
        global_table = None
        if self.resync:
            acl_dump, has_reflective = self._dump_vpp_acl_config()
            r.cache.resync(acl_dump)
            txn_pods = self.cache_txn.get_updated_pods()
            for pod in list(r.cache.get_all_pods()):
                if not txn_pods.has(pod):
                    self.cache_txn.update(pod, PodConfig(removed=True))
        else:
            has_reflective = (r.cache.get_global_table().num_of_rules != 0
                              or len(r.cache.get_isolated_pods()) > 0)

        changes = self.cache_txn.get_changes()
        if not self.resync and len(changes) == 0:
            self.cache_txn.commit()
            return

        dsl = r.acl_txn_factory()
        for change in changes:
            if change.table.type == GLOBAL:
                global_table = change.table
                continue
            if len(change.previous_pods) == 0:
                dsl.put_acl(self.render_acl(change.table))
            elif len(change.table.pods) != 0:
                acl = change.table.private.clone()
                acl.interfaces = self.render_interfaces(change.table.pods, False)
                dsl.put_acl(acl)
            else:
                dsl.delete_acl(change.table.private.acl_name)

        if self.resync and global_table is None and r.cache.get_global_table().num_of_rules != 0:
            global_table = r.cache.get_global_table()

        gt_added_or_deleted = False
        if global_table is not None:
            global_acl = self.render_acl(global_table)
            if global_table.num_of_rules == 0:
                dsl.delete_acl(global_acl.acl_name)
                gt_added_or_deleted = True
            else:
                global_acl.interfaces.egress = self.get_node_output_interfaces()
                dsl.put_acl(global_acl)
                if r.cache.get_global_table().num_of_rules == 0:
                    gt_added_or_deleted = True

        if (self.resync or gt_added_or_deleted or
                not self.cache_txn.get_isolated_pods().equals(r.cache.get_isolated_pods())):
            refl = self.reflective_acl()
            if len(refl.interfaces.ingress) == 0:
                if has_reflective:
                    dsl.delete_acl(refl.acl_name)
            else:
                dsl.put_acl(refl)

        dsl.send()
        self.cache_txn.commit()

    def reflective_acl(self) -> model.Acl:
        table = ContivRuleTable(REFLECTIVE_ACL_NAME)
        table.rules = [ContivRule(ACTION_PERMIT, IPNet(), IPNet(), TCP, 0, 0),
                       ContivRule(ACTION_PERMIT, IPNet(), IPNet(), UDP, 0, 0)]
        table.pods = self.cache_txn.get_isolated_pods()
        acl = self.render_acl(table)
        if self.cache_txn.get_global_table().num_of_rules > 0:
            acl.interfaces.ingress.extend(self.get_node_output_interfaces())
        return acl

    def get_node_output_interfaces(self) -> List[str]:
        c = self.renderer.contiv
        ifs = [c.get_host_interconnect_if_name(), c.get_main_physical_if_name()]
        ifs.extend(c.get_other_physical_if_names())
        if c.get_vxlan_bvi_if_name() != "":
            ifs.append(c.get_vxlan_bvi_if_name())
        return ifs

    def render_acl(self, table: ContivRuleTable) -> model.Acl:
        return render_acl(table, self.render_interfaces(table.pods, table.id == REFLECTIVE_ACL_NAME))

    def render_interfaces(self, pods: PodSet, ingress: bool) -> model.Interfaces:
        ifs = model.Interfaces()
        for pod in sorted(pods, key=tuple):
            if_name = self.renderer.pod_interfaces.get(pod)
            if if_name is None:
                if_name, found = self.renderer.contiv.get_if_name(pod.namespace, pod.name)
                if not found:
                    continue
            self.renderer.pod_interfaces[pod] = if_name
            (ifs.ingress if ingress else ifs.egress).append(if_name)
        return ifs

    def _dump_vpp_acl_config(self):
        tables = []
        has_reflective = False
        for acl in self.renderer.vpp_dump():
            if not acl.acl_name.startswith(ACL_NAME_PREFIX):
                continue
            name = acl.acl_name[len(ACL_NAME_PREFIX):]
            if name == REFLECTIVE_ACL_NAME:
                has_reflective = True
                continue
            table = ContivRuleTable(name)
            if table.type == LOCAL:
                if acl.interfaces is None or len(acl.interfaces.ingress) > 0:
                    continue
                if len(acl.interfaces.egress) == 0:
                    continue
                for if_name in acl.interfaces.egress:
                    ns, pname, ok = self.renderer.contiv.get_pod_by_if(if_name)
                    if ok:
                        table.pods.add(PodID(pname, ns))
            for ar in acl.rules:
                rule = _dump_rule(ar)
                if rule is not None:
                    table.insert_rule(rule)
            table.private = acl
            tables.append(table)
        return tables, has_reflective


def _dump_rule(ar: model.Rule) -> Optional[ContivRule]:
    """One iteration of dumpVppACLConfig's rule loop (acl_renderer.go:482-588)."""
    rule = ContivRule()
    if ar.actions is None:
        return None
    if ar.actions.acl_action == model.PERMIT:
        rule.action = ACTION_PERMIT
    elif ar.actions.acl_action == model.DENY:
        rule.action = ACTION_DENY
    else:
        return None
    if ar.matches is None or ar.matches.ip_rule is None:
        return None
    ipr = ar.matches.ip_rule
    rule.src_network, rule.dest_network = IPNet(), IPNet()
    if ipr.ip is not None:
        if ipr.ip.source_network != "":
            _, n = gonet.parse_cidr(ipr.ip.source_network)
            if n is None:
                return None
            rule.src_network = n
        if ipr.ip.destination_network != "":
            _, n = gonet.parse_cidr(ipr.ip.destination_network)
            if n is None:
                return None
            rule.dest_network = n
    if ipr.other is not None:
        return None
    if ipr.icmp is not None:
        return None
    for sec, proto in ((ipr.tcp, TCP), (ipr.udp, UDP)):
        if sec is None:
            continue
        rule.protocol = proto
        for rng, attr in ((sec.source_port_range, "src_port"), (sec.destination_port_range, "dest_port")):
            if rng is None:
                continue
            if rng.lower_port != rng.upper_port and (rng.lower_port != 0 or rng.upper_port != MAX_PORT):
                return None
            setattr(rule, attr, rng.lower_port & 0xFFFF)
        break
    return rule


# Rendered rules by their exact rendering inputs: a txn re-renders whole
# tables (the global one has ~10k rules at 1000 pods) of which few rules
# changed, so equal rules share one message.  Shared messages are read-only
# (model.frozen): a caller that edits a rendered or dumped ACL's rule gets
# FrozenMessageError instead of silently rewriting every ACL that shares it,
# and copy.deepcopy gives an editable copy.  (Go's renderACL allocates fresh
# messages per call, acl_renderer.go:324; building 10k fresh messages per
# render costs ~20x the memoised render here.)
_rendered = {}


def render_acl(table: ContivRuleTable, interfaces: model.Interfaces) -> model.Acl:
    """renderACL (acl_renderer.go:312-402)."""
    acl = model.Acl(acl_name=ACL_NAME_PREFIX + table.id, interfaces=interfaces)
    reflective = table.id == REFLECTIVE_ACL_NAME
    if len(_rendered) > 1_000_000:
        _rendered.clear()
    out = acl.rules
    for rule in table.rules:
        k = (rule.action, reflective, bytes(rule.src_network.ip), bytes(rule.src_network.mask),
             bytes(rule.dest_network.ip), bytes(rule.dest_network.mask), rule.protocol, rule.src_port,
             rule.dest_port)
        r = _rendered.get(k)
        if r is None:
            r = _rendered[k] = _build_rule(_recipe(rule, reflective))
        out.append(r)
    if table.num_of_rules > 0:
        out.append(model.icmp_rule(model.REFLECT if reflective else model.PERMIT))
    table.private = acl
    return acl


def _recipe(rule, reflective: bool) -> tuple:
    """What one ContivRule renders to (acl_renderer.go:324-375), as a tuple:
    (action, src network string, dst network string, is TCP, src lo, src hi,
    dst lo, dst hi)."""
    if rule.action == ACTION_DENY:
        action = model.DENY
    elif reflective:
        action = model.REFLECT
    else:
        action = model.PERMIT
    src = rule.src_network.string() if len(rule.src_network.ip) > 0 else ""
    dst = rule.dest_network.string() if len(rule.dest_network.ip) > 0 else ""
    return (action, src, dst, rule.protocol == TCP,
            rule.src_port, MAX_PORT if rule.src_port == 0 else rule.src_port,
            rule.dest_port, MAX_PORT if rule.dest_port == 0 else rule.dest_port)


def _build_rule(rec: tuple) -> model.Rule:
    """A read-only rule message from a recipe: TCP rules get a Tcp section,
    every other protocol a Udp section (acl_renderer.go:342-374)."""
    action, src, dst, tcp, slo, shi, dlo, dhi = rec
    F = model.frozen
    sec = F(model.Tcp if tcp else model.Udp,
            destination_port_range=F(model.PortRange, lower_port=dlo, upper_port=dhi),
            source_port_range=F(model.PortRange, lower_port=slo, upper_port=shi))
    ip = F(model.Ip, destination_network=dst, source_network=src)
    iprule = F(model.IpRule, ip=ip, tcp=sec) if tcp else F(model.IpRule, ip=ip, udp=sec)
    return F(model.Rule, actions=F(model.Actions, acl_action=action), matches=F(model.Matches, ip_rule=iprule))
