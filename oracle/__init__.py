"""ORACLE -- test infrastructure only (see aclengine_ref.c header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product (vpp_amd/) never does.

Provides:
  * ``lib()``           -- the compiled C oracle (liborc.so, built by ``build()``)
  * ``rules_to_c``      -- vpp_acl model rules -> ``cls_rule`` ctypes array
  * ``eval_acl``        -- one evalACL evaluation (aclengine_mock.go:473-668)
  * ``classify_faithful`` / ``classify_fast`` -- batched CPU evaluation
  * ``gen_traffic_v4``  -- the synthetic packet stream (CPU reference)
  * ``OracleACLEngine`` -- MockACLEngine restated (aclengine_mock.go:94-471)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "liborc.so")


class ClsRule(C.Structure):
    _fields_ = [("flags", C.c_uint32), ("acl_action", C.c_int32),
                ("src_network", C.c_char_p), ("dst_network", C.c_char_p),
                ("tcp_src_lo", C.c_uint32), ("tcp_src_hi", C.c_uint32),
                ("tcp_dst_lo", C.c_uint32), ("tcp_dst_hi", C.c_uint32),
                ("udp_src_lo", C.c_uint32), ("udp_src_hi", C.c_uint32),
                ("udp_dst_lo", C.c_uint32), ("udp_dst_hi", C.c_uint32),
                ("icmp_code_first", C.c_uint32), ("icmp_code_last", C.c_uint32),
                ("icmp_type_first", C.c_uint32), ("icmp_type_last", C.c_uint32)]


class AclRef(C.Structure):
    _fields_ = [("rules", C.POINTER(ClsRule)), ("n", C.c_uint32), ("nil", C.c_int)]


class TrafficSpec(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("pct_pod_src", C.c_uint32), ("pct_rule_dst", C.c_uint32),
                ("pct_table_port", C.c_uint32), ("pct_icmp", C.c_uint32),
                ("pod_ips", C.POINTER(C.c_uint32)), ("n_pod_ips", C.c_uint32),
                ("dst_addrs", C.POINTER(C.c_uint32)), ("dst_lens", C.POINTER(C.c_uint8)),
                ("n_dst", C.c_uint32),
                ("ports", C.POINTER(C.c_uint16)), ("n_ports", C.c_uint32)]


# presence bits (include/contivcls.h)
R_MATCHES, R_MACIP, R_IPRULE, R_IP, R_OTHER = 1, 2, 4, 8, 16
R_TCP, R_TCP_SRC, R_TCP_DST = 32, 64, 128
R_UDP, R_UDP_SRC, R_UDP_DST = 256, 512, 1024
R_ICMP, R_ICMP_CODE, R_ICMP_TYPE, R_ICMPV6, R_ACTIONS = 2048, 4096, 8192, 16384, 32768


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liborc.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_eval_acl.restype = C.c_int
        L.orc_eval_acl.argtypes = [C.POINTER(ClsRule), C.c_uint32, C.c_int, C.c_char_p, C.c_int,
                                   C.c_char_p, C.c_int, C.c_int, C.c_uint16,
                                   C.POINTER(C.c_int32)]
        L.orc_test_connection.restype = C.c_int
        L.orc_test_connection.argtypes = [C.POINTER(AclRef)] * 4 + [
            C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, C.c_uint16, C.c_uint16]
        L.orc_test_connection_hits.restype = C.c_int
        L.orc_test_connection_hits.argtypes = [C.POINTER(AclRef)] * 4 + [
            C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, C.c_uint16, C.c_uint16,
            C.POINTER(C.c_int32)]
        L.orc_classify_faithful.restype = C.c_int
        L.orc_classify_faithful.argtypes = [C.POINTER(ClsRule), C.c_uint32, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                            C.c_void_p, C.c_void_p]
        L.orc_compile.restype = C.c_void_p
        L.orc_compile.argtypes = [C.POINTER(ClsRule), C.c_uint32]
        L.orc_ctable_free.argtypes = [C.c_void_p]
        L.orc_classify_fast_hits.restype = C.c_int
        L.orc_classify_fast_hits.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_classify_fast.restype = C.c_int
        L.orc_classify_fast.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_parse_cidr.restype = C.c_int
        L.orc_parse_cidr.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.c_char_p,
                                     C.POINTER(C.c_int)]
        L.orc_parse_ip.restype = C.c_int
        L.orc_parse_ip.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_int)]
        L.orc_cidr_contains.restype = C.c_int
        L.orc_cidr_contains.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        L.orc_connect_fast.restype = C.c_int
        L.orc_connect_fast.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                       C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_uint64, C.c_void_p, C.c_int]
        L.orc_gen_traffic_v16.restype = None
        L.orc_gen_traffic_v16.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64] + [C.c_void_p] * 5
        L.orc_gen_traffic_v4.restype = None
        L.orc_gen_traffic_v4.argtypes = [C.POINTER(TrafficSpec), C.c_uint64, C.c_uint64] + [C.c_void_p] * 5
        _LIB = L
    return _LIB


# ---------------------------------------------------------------------------
def _enc(s):
    return None if s is None else s.encode()


class CRules:
    """Owns a ``cls_rule`` array (and the CIDR string buffers it points to)."""

    def __init__(self, rules):
        self.n = len(rules)
        self.arr = (ClsRule * max(1, self.n))()
        self._keep = []
        for i, r in enumerate(rules):
            self._fill(self.arr[i], r)

    def _fill(self, c: ClsRule, r):
        f = 0
        if r.actions is not None:
            f |= R_ACTIONS
            c.acl_action = r.actions.acl_action
        m = r.matches
        if m is not None:
            f |= R_MATCHES
            if m.macip_rule is not None:
                f |= R_MACIP
            ipr = m.ip_rule
            if ipr is not None:
                f |= R_IPRULE
                if ipr.ip is not None:
                    f |= R_IP
                    s, d = _enc(ipr.ip.source_network), _enc(ipr.ip.destination_network)
                    self._keep += [s, d]
                    c.src_network, c.dst_network = s, d
                if ipr.other is not None:
                    f |= R_OTHER
                if ipr.tcp is not None:
                    f |= R_TCP
                    if ipr.tcp.source_port_range is not None:
                        f |= R_TCP_SRC
                        c.tcp_src_lo = ipr.tcp.source_port_range.lower_port
                        c.tcp_src_hi = ipr.tcp.source_port_range.upper_port
                    if ipr.tcp.destination_port_range is not None:
                        f |= R_TCP_DST
                        c.tcp_dst_lo = ipr.tcp.destination_port_range.lower_port
                        c.tcp_dst_hi = ipr.tcp.destination_port_range.upper_port
                if ipr.udp is not None:
                    f |= R_UDP
                    if ipr.udp.source_port_range is not None:
                        f |= R_UDP_SRC
                        c.udp_src_lo = ipr.udp.source_port_range.lower_port
                        c.udp_src_hi = ipr.udp.source_port_range.upper_port
                    if ipr.udp.destination_port_range is not None:
                        f |= R_UDP_DST
                        c.udp_dst_lo = ipr.udp.destination_port_range.lower_port
                        c.udp_dst_hi = ipr.udp.destination_port_range.upper_port
                if ipr.icmp is not None:
                    f |= R_ICMP
                    if ipr.icmp.icmpv6:
                        f |= R_ICMPV6
                    if ipr.icmp.icmp_code_range is not None:
                        f |= R_ICMP_CODE
                        c.icmp_code_first = ipr.icmp.icmp_code_range.first
                        c.icmp_code_last = ipr.icmp.icmp_code_range.last
                    if ipr.icmp.icmp_type_range is not None:
                        f |= R_ICMP_TYPE
                        c.icmp_type_first = ipr.icmp.icmp_type_range.first
                        c.icmp_type_last = ipr.icmp.icmp_type_range.last
        c.flags = f

    def ptr(self):
        return C.cast(self.arr, C.POINTER(ClsRule))


def rules_to_c(rules) -> CRules:
    return CRules(rules)


def ip_bytes(ip) -> bytes:
    """Go net.IP (bytes of len 0/4/16) or host-order uint32 -> bytes."""
    if isinstance(ip, (int, np.integer)):
        return int(ip).to_bytes(4, "big")
    return bytes(ip)


def eval_acl(crules, nil: bool, src: bytes, dst: bytes, proto: int, dport: int):
    """Returns (ACLAction, terminating rule index or n or -1)."""
    hit = C.c_int32(0)
    n = 0 if crules is None else crules.n
    ptr = None if crules is None else crules.ptr()
    a = lib().orc_eval_acl(ptr, n, 1 if nil else 0, src, len(src), dst, len(dst), proto,
                           dport & 0xFFFF, C.byref(hit))
    if a == -2:
        raise RuntimeError("evalACL would panic (rule.Matches == nil)")
    return a, hit.value


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def classify_faithful(crules, src, dst, dport, proto, af=4):
    n = len(dport)
    verdict = np.zeros(n, np.uint8)
    counters = np.zeros(crules.n + 1, np.uint64)
    rc = lib().orc_classify_faithful(crules.ptr(), crules.n, af, _p(src), _p(dst), _p(dport),
                                     _p(proto), n, _p(verdict), _p(counters))
    if rc != 0:
        raise RuntimeError("orc_classify_faithful rc=%d" % rc)
    return verdict, counters


class FastTable:
    def __init__(self, crules):
        self.crules = crules
        self.h = lib().orc_compile(crules.ptr(), crules.n)
        if not self.h:
            raise RuntimeError("rule with nil Matches")

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_ctable_free(self.h)
            self.h = None

    def classify(self, src, dst, dport, proto, af=4, nthreads=0):
        n = len(dport)
        verdict = np.zeros(n, np.uint8)
        counters = np.zeros(self.crules.n + 1, np.uint64)
        rc = lib().orc_classify_fast(self.h, af, _p(src), _p(dst), _p(dport), _p(proto), n,
                                     _p(verdict), _p(counters), nthreads)
        if rc != 0:
            raise RuntimeError("orc_classify_fast rc=%d" % rc)
        return verdict, counters


def classify_hits(crules, src, dst, dport, proto, af=4, nthreads=0):
    """Each packet's ACLAction and terminating rule index (n: the default
    DENY) on the fast port (orc_classify_fast_hits): (verdict, hits uint32)."""
    t = FastTable(crules)
    n = len(dport)
    verdict = np.zeros(n, np.uint8)
    hits = np.zeros(n, np.uint32)
    rc = lib().orc_classify_fast_hits(t.h, af, _p(src), _p(dst), _p(np.ascontiguousarray(dport, np.uint16)),
                                      _p(np.ascontiguousarray(proto, np.uint8)), n, _p(verdict), _p(hits), nthreads)
    if rc != 0:
        raise RuntimeError("orc_classify_fast_hits rc=%d" % rc)
    return verdict, hits


def connect_fast(tables, if_in, if_out, si, di, tr, af=4, nthreads=0):
    """testConnection over a batch on the fast port (orc_connect_fast,
    OpenMP): tables = [FastTable]; interface f binds tables[if_in[f]]
    inbound and tables[if_out[f]] outbound (-1: no ACL); connection i from
    interface si[i] to di[i], fields of tr (src, dst, proto, sport, dport)."""
    import numpy as np
    hs = (C.c_void_p * max(1, len(tables)))(*[t.h for t in tables])
    ii = np.ascontiguousarray(if_in, np.int32)
    io = np.ascontiguousarray(if_out, np.int32)
    a = np.ascontiguousarray(si, np.uint32)
    b = np.ascontiguousarray(di, np.uint32)
    adt = np.uint8 if af == 16 else np.uint32
    s = np.ascontiguousarray(tr["src"], adt)
    d = np.ascontiguousarray(tr["dst"], adt)
    pr = np.ascontiguousarray(tr["proto"], np.uint8)
    sp = np.ascontiguousarray(tr["sport"], np.uint16)
    dp = np.ascontiguousarray(tr["dport"], np.uint16)
    out = np.zeros(len(pr), np.uint8)
    rc = lib().orc_connect_fast(hs, _p(ii), _p(io), len(ii), _p(a), _p(b), af, _p(s), _p(d), _p(pr), _p(sp),
                                _p(dp), len(pr), _p(out), nthreads)
    if rc != 0:
        raise RuntimeError("orc_connect_fast rc=%d" % rc)
    return out


def classify_fast(crules, src, dst, dport, proto, af=4, nthreads=0):
    return FastTable(crules).classify(src, dst, dport, proto, af, nthreads)


def gen_traffic_v4(spec: dict, first: int, n: int):
    """CPU reference of the splitmix64 packet stream (DESIGN.md 'Traffic')."""
    pods = np.ascontiguousarray(spec.get("pod_ips", []), np.uint32)
    dsta = np.ascontiguousarray(spec.get("dst_addrs", []), np.uint32)
    dstl = np.ascontiguousarray(spec.get("dst_lens", []), np.uint8)
    ports = np.ascontiguousarray(spec.get("ports", []), np.uint16)
    ts = TrafficSpec(spec["seed"], spec.get("pct_pod_src", 60), spec.get("pct_rule_dst", 50),
                     spec.get("pct_table_port", 50), spec.get("pct_icmp", 0),
                     pods.ctypes.data_as(C.POINTER(C.c_uint32)), len(pods),
                     dsta.ctypes.data_as(C.POINTER(C.c_uint32)),
                     dstl.ctypes.data_as(C.POINTER(C.c_uint8)), len(dsta),
                     ports.ctypes.data_as(C.POINTER(C.c_uint16)), len(ports))
    out = dict(src=np.zeros(n, np.uint32), dst=np.zeros(n, np.uint32),
               sport=np.zeros(n, np.uint16), dport=np.zeros(n, np.uint16),
               proto=np.zeros(n, np.uint8))
    lib().orc_gen_traffic_v4(C.byref(ts), first, n, _p(out["src"]), _p(out["dst"]),
                             _p(out["sport"]), _p(out["dport"]), _p(out["proto"]))
    return out


class TrafficSpec16(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("pct_pod_src", C.c_uint32), ("pct_rule_dst", C.c_uint32),
                ("pct_table_port", C.c_uint32), ("pct_icmp", C.c_uint32),
                ("pod_ips", C.c_void_p), ("n_pod_ips", C.c_uint32),
                ("dst_addrs", C.c_void_p), ("dst_lens", C.c_void_p), ("n_dst", C.c_uint32),
                ("ports", C.c_void_p), ("n_ports", C.c_uint32)]


def gen_traffic_v16(spec: dict, first: int, n: int):
    """CPU reference of the 16-byte stream (include/contivcls.h cls_traffic_spec16)."""
    pods = np.ascontiguousarray(spec.get("pod_ips", np.zeros((0, 16))), np.uint8)
    da = np.ascontiguousarray(spec.get("dst_addrs", np.zeros((0, 16))), np.uint8)
    dl = np.ascontiguousarray(spec.get("dst_lens", []), np.uint8)
    ports = np.ascontiguousarray(spec.get("ports", []), np.uint16)
    ts = TrafficSpec16(spec["seed"], spec.get("pct_pod_src", 60), spec.get("pct_rule_dst", 50),
                       spec.get("pct_table_port", 50), spec.get("pct_icmp", 0),
                       pods.ctypes.data, len(pods), da.ctypes.data, dl.ctypes.data, len(da),
                       ports.ctypes.data, len(ports))
    out = dict(src=np.zeros((n, 16), np.uint8), dst=np.zeros((n, 16), np.uint8),
               sport=np.zeros(n, np.uint16), dport=np.zeros(n, np.uint16), proto=np.zeros(n, np.uint8))
    lib().orc_gen_traffic_v16(C.byref(ts), first, n, _p(out["src"]), _p(out["dst"]),
                              _p(out["sport"]), _p(out["dport"]), _p(out["proto"]))
    return out


from .aclengine import OracleACLEngine  # noqa: E402,F401
