"""ACL data model: the vpp_acl protobuf messages the Contiv ACL renderer emits.

Mirrors ``AccessLists_Acl`` and its nested messages from the vendored
vpp-agent model (vendor/github.com/ligato/vpp-agent/plugins/defaultplugins/
common/model/acl/acl.proto:12-161, acl.pb.go).  ``None`` stands for a nil
sub-message: evalACL's semantics depend on nil-ness
(mock/aclengine/aclengine_mock.go:481-664), so the model keeps it.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field, fields
from typing import List, Optional

# vpp_acl.AclAction (acl.proto:4-8)
DENY = 0
PERMIT = 1
REFLECT = 2

# vpp_acl.KeyPrefix() (keys_agent_acl.go:3-14)
ACL_KEY_PREFIX = "vpp/config/v1/acl/"


def acl_key(name: str) -> str:
    return ACL_KEY_PREFIX + name


@dataclass
class PortRange:
    lower_port: int = 0
    upper_port: int = 0


@dataclass
class Tcp:
    destination_port_range: Optional[PortRange] = None
    source_port_range: Optional[PortRange] = None
    tcp_flags_mask: int = 0
    tcp_flags_value: int = 0


@dataclass
class Udp:
    destination_port_range: Optional[PortRange] = None
    source_port_range: Optional[PortRange] = None


@dataclass
class IcmpRange:
    first: int = 0
    last: int = 0


@dataclass
class Icmp:
    icmpv6: bool = False
    icmp_code_range: Optional[IcmpRange] = None
    icmp_type_range: Optional[IcmpRange] = None


@dataclass
class Other:
    protocol: int = 0


@dataclass
class Ip:
    destination_network: str = ""
    source_network: str = ""


@dataclass
class IpRule:
    ip: Optional[Ip] = None
    icmp: Optional[Icmp] = None
    tcp: Optional[Tcp] = None
    udp: Optional[Udp] = None
    other: Optional[Other] = None


@dataclass
class MacIpRule:
    source_address: str = ""
    source_address_prefix: int = 0
    source_mac_address: str = ""
    source_mac_address_mask: str = ""


@dataclass
class Matches:
    ip_rule: Optional[IpRule] = None
    macip_rule: Optional[MacIpRule] = None


@dataclass
class Actions:
    acl_action: int = DENY


@dataclass
class Rule:
    actions: Optional[Actions] = None
    matches: Optional[Matches] = None
    rule_name: str = ""


@dataclass
class Interfaces:
    egress: List[str] = field(default_factory=list)
    ingress: List[str] = field(default_factory=list)


@dataclass
class Acl:
    rules: List[Rule] = field(default_factory=list)
    acl_name: str = ""
    interfaces: Optional[Interfaces] = None

    def clone(self) -> "Acl":
        """proto.Clone equivalent (acl_renderer.go:189).  Rule messages are
        never modified once rendered, so the clone shares them; the rule list
        and the interfaces (which the renderer rewrites) are copies."""
        return Acl(rules=list(self.rules), acl_name=self.acl_name,
                   interfaces=copy.deepcopy(self.interfaces))


class FrozenMessageError(AttributeError):
    """An attempt to edit a read-only (shared) rule message."""


def _sealed_class(base):
    """A read-only variant of a message class: same fields, isinstance of
    ``base``, equal to a ``base`` message with equal fields; setting a field
    raises FrozenMessageError; ``copy.deepcopy`` returns a mutable ``base``
    copy (like proto.Clone)."""
    names = [f.name for f in fields(base)]

    def __setattr__(self, k, v):
        raise FrozenMessageError("%s is a shared rendered message; deepcopy it to edit" % base.__name__)

    def __delattr__(self, k):
        raise FrozenMessageError("%s is a shared rendered message" % base.__name__)

    def __eq__(self, other):
        if not isinstance(other, base):
            return NotImplemented
        return all(getattr(self, n) == getattr(other, n) for n in names)

    def __deepcopy__(self, memo):
        return base(**{n: copy.deepcopy(getattr(self, n), memo) for n in names})

    return type("Frozen" + base.__name__, (base,),
                dict(__setattr__=__setattr__, __delattr__=__delattr__, __eq__=__eq__, __hash__=None,
                     __deepcopy__=__deepcopy__))


_FROZEN = {c: _sealed_class(c) for c in (PortRange, Tcp, Udp, IcmpRange, Icmp, Ip, IpRule, Matches, Actions,
                                         Rule)}


def frozen(cls, **values):
    """A read-only ``cls`` message (cls one of the rule message classes).
    Rendered rules are shared between ACLs (renderer/acl.py memo), so they
    are built read-only: nobody can edit one ACL's rule and thereby another's."""
    o = object.__new__(_FROZEN[cls])
    d = o.__dict__
    for f in fields(cls):
        d[f.name] = values.get(f.name, f.default)
    return o


MAX_PORT = 0xFFFF
MAX_ICMP_CODE = 5
MAX_ICMP_TYPE = 16


def l4_rule(action: int, src: str, dst: str, proto: str, sport_lo: int, sport_hi: int,
            dport_lo: int, dport_hi: int) -> Rule:
    """Convenience constructor of a TCP/UDP ACL rule in renderACL's shape
    (acl_renderer.go:324-375)."""
    ip = Ip(destination_network=dst, source_network=src)
    sec_args = dict(destination_port_range=PortRange(dport_lo, dport_hi),
                    source_port_range=PortRange(sport_lo, sport_hi))
    if proto == "tcp":
        iprule = IpRule(ip=ip, tcp=Tcp(**sec_args))
    else:
        iprule = IpRule(ip=ip, udp=Udp(**sec_args))
    return Rule(actions=Actions(action), matches=Matches(ip_rule=iprule))


def icmp_rule(action: int, src: str = "", dst: str = "") -> Rule:
    """The trailing allow-ICMP rule of renderACL (acl_renderer.go:378-398)."""
    iprule = IpRule(ip=Ip(destination_network=dst, source_network=src),
                    icmp=Icmp(icmpv6=False,
                              icmp_code_range=IcmpRange(0, MAX_ICMP_CODE),
                              icmp_type_range=IcmpRange(0, MAX_ICMP_TYPE)))
    return Rule(actions=Actions(action), matches=Matches(ip_rule=iprule))
