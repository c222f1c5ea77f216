"""ORACLE -- MockACLEngine restated (test infrastructure only).

Follows mock/aclengine/aclengine_mock.go:94-728: ACLConfig (byName/byIf,
PutACL :699-728, DelACL :680-696, GetACLs :671-677), ApplyTxn :151-198,
RegisterPod :144-148, Connection{PodToPod,PodToInternet,InternetToPod}
:243-390 and testConnection :394-471.  Every ACL evaluation goes through
the C restatement of evalACL (aclengine_ref.c, orc_test_connection).
"""
from __future__ import annotations

import copy
import ctypes as C

CONN_DENY_SYN, CONN_DENY_SYN_ACK, CONN_ALLOW, CONN_FAILURE = 0, 1, 2, 3
ACL_KEY_PREFIX = "vpp/config/v1/acl/"


def _parse_ip(s: str):
    from . import lib
    buf = C.create_string_buffer(16)
    ln = C.c_int(0)
    if not lib().orc_parse_ip(s.encode(), buf, C.byref(ln)):
        return None
    return buf.raw[:ln.value]


class OracleACLEngine:
    def __init__(self, contiv):
        self.contiv = contiv
        self.pods = {}            # PodID -> (ip bytes | None, another_node)
        self.by_name = {}         # name -> Acl
        self.by_if = {}           # if -> [inbound Acl|None, outbound Acl|None]
        self.changes = 0
        self._crules = {}         # id(Acl) -> CRules

    # -- RegisterPod (:144-148) -------------------------------------------
    def register_pod(self, pod, pod_ip: str, another_node: bool):
        self.pods[pod] = (_parse_ip(pod_ip), another_node)

    # -- ApplyTxn (:151-198) ------------------------------------------------
    def apply_txn(self, ops):
        for key, value in ops:
            if not key.startswith(ACL_KEY_PREFIX):
                return "non-ACL changed in txn"
            name = key[len(ACL_KEY_PREFIX):]
            if value is not None:
                err = self.put_acl(copy.deepcopy(value))
            else:
                err = self.del_acl(name)
            if err:
                return err
        return None

    def put_acl(self, acl):
        if acl is None:
            return "ACL is nil"
        if acl.interfaces is None or (len(acl.interfaces.ingress) == 0 and len(acl.interfaces.egress) == 0):
            return "ACL with empty interfaces"
        if acl.acl_name in self.by_name:
            self.del_acl(acl.acl_name)
            self.changes -= 1
        self.by_name[acl.acl_name] = acl
        for ifn in acl.interfaces.ingress:
            self.by_if.setdefault(ifn, [None, None])[0] = acl
        for ifn in acl.interfaces.egress:
            self.by_if.setdefault(ifn, [None, None])[1] = acl
        self.changes += 1
        return None

    def del_acl(self, name):
        if name not in self.by_name:
            return "cannot find ACL: %s" % name
        del self.by_name[name]
        for cfg in self.by_if.values():
            if cfg[0] is not None and cfg[0].acl_name == name:
                cfg[0] = None
            if cfg[1] is not None and cfg[1].acl_name == name:
                cfg[1] = None
        self.changes += 1
        return None

    # -- getters (:201-239) ------------------------------------------------
    def dump_acls(self):
        return list(self.by_name.values())

    def get_num_of_acls(self):
        return len(self.by_name)

    def get_num_of_acl_changes(self):
        return self.changes

    def get_inbound_acl(self, if_name):
        return self.by_if.get(if_name, [None, None])[0]

    def get_outbound_acl(self, if_name):
        return self.by_if.get(if_name, [None, None])[1]

    def get_acl_by_name(self, name):
        return self.by_name.get(name)

    # -- Connection* (:243-390) -------------------------------------------
    def _node_output_if(self):
        ifn = self.contiv.get_vxlan_bvi_if_name()
        if ifn == "":
            ifn = self.contiv.get_main_physical_if_name()
        return ifn

    def _pod_if(self, pod, cfg):
        if cfg[1]:
            ifn = self._node_output_if()
            return ifn if ifn != "" else None
        ifn, ok = self.contiv.get_if_name(pod.namespace, pod.name)
        return ifn if ok else None

    def connection_pod_to_pod(self, src_pod, dst_pod, proto, sport, dport):
        s, d = self.pods.get(src_pod), self.pods.get(dst_pod)
        if s is None or d is None:
            return CONN_FAILURE
        sif, dif = self._pod_if(src_pod, s), self._pod_if(dst_pod, d)
        if sif is None or dif is None:
            return CONN_FAILURE
        return self.test_connection(sif, s[0], dif, d[0], proto, sport, dport)

    def connection_pod_to_internet(self, src_pod, dst_ip: str, proto, sport, dport):
        s = self.pods.get(src_pod)
        if s is None or s[1]:
            return CONN_FAILURE
        sif, ok = self.contiv.get_if_name(src_pod.namespace, src_pod.name)
        if not ok:
            return CONN_FAILURE
        dif = self._node_output_if()
        if dif == "":
            return CONN_FAILURE
        dip = _parse_ip(dst_ip)
        if dip is None:
            return CONN_FAILURE
        return self.test_connection(sif, s[0], dif, dip, proto, sport, dport)

    def connection_internet_to_pod(self, src_ip: str, dst_pod, proto, sport, dport):
        d = self.pods.get(dst_pod)
        if d is None or d[1]:
            return CONN_FAILURE
        sif = self._node_output_if()
        if sif == "":
            return CONN_FAILURE
        sip = _parse_ip(src_ip)
        if sip is None:
            return CONN_FAILURE
        dif, ok = self.contiv.get_if_name(dst_pod.namespace, dst_pod.name)
        if not ok:
            return CONN_FAILURE
        return self.test_connection(sif, sip, dif, d[0], proto, sport, dport)

    # -- testConnection (:394-471) via the C oracle ------------------------
    def _ref(self, acl):
        from . import AclRef, rules_to_c
        if acl is None:
            return AclRef(None, 0, 1), None
        cr = rules_to_c(acl.rules)
        return AclRef(cr.ptr(), cr.n, 0), cr

    def test_connection(self, src_if, src_ip, dst_if, dst_ip, proto, sport, dport):
        from . import lib
        s_in, s_out = self.by_if.get(src_if, [None, None])
        d_in, d_out = self.by_if.get(dst_if, [None, None])
        refs = [self._ref(a) for a in (s_in, s_out, d_in, d_out)]
        src_ip = src_ip or b""
        dst_ip = dst_ip or b""
        rc = lib().orc_test_connection(*[C.byref(r[0]) for r in refs],
                                       1 if src_if == dst_if else 0,
                                       src_ip, len(src_ip), dst_ip, len(dst_ip), proto,
                                       sport & 0xFFFF, dport & 0xFFFF)
        if rc < 0:
            raise RuntimeError("evalACL would panic")
        return rc
