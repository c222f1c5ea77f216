"""ctypes binding of libcontivcls.so (include/contivcls.h).

The Python host layer stands where the Go host layer of the north star would
(there is no Go toolchain in this image; INTEGRATION.md shows the cgo
binding of the same symbols).  Loading fails loudly if the gfx950 library is
missing -- there is no CPU fallback in the product.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CONTIVCLS_LIB: diagnostics only (A/B timing of kernel build variants)
LIB_PATH = os.environ.get("CONTIVCLS_LIB") or os.path.join(_HERE, "libcontivcls.so")

SOURCES = ("kernels.hip", "kernels_dev.hpp", "k4_ldsv.hip", "k4_rest.hip", "k4_pair.hip", "k16.hip", "kernels.hpp", "compile.cpp",
           "compile.hpp", "engine.cpp", "goparse.hpp", "engine_int.hpp", "fleet.cpp", "options.cpp", "options.hpp")


def source_hash() -> str:
    """Hash of the native sources (vpp_amd/csrc): ties a committed profile
    (profiles/pmc_*.json) to the kernels it measured."""
    h = hashlib.sha256()
    for f in SOURCES:
        with open(os.path.join(_HERE, "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


# status codes
OK, E_INVAL, E_NOMEM, E_HIP, E_RCCL, E_NOTFOUND, E_NODEV = 0, -1, -2, -3, -4, -5, -6
# flags
F_DEVICE, F_NO_VERDICT, F_ACCUMULATE, F_FORCE_LINEAR, F_TIMING, F_CONN_CLS, F_COUNT = 1, 2, 4, 8, 16, 32, 64
AF_V4, AF_V16 = 4, 16
# batch fields and flags (cls_batch_*)
BF_SRC, BF_DST, BF_SPORT, BF_DPORT, BF_PROTO, BF_VERDICT, BF_SRC_IF, BF_DST_IF = range(8)
BATCH_CONN, BATCH_MIRROR = 1, 2
ABI_VERSION = 5

R_MATCHES, R_MACIP, R_IPRULE, R_IP, R_OTHER = 1, 2, 4, 8, 16
R_TCP, R_TCP_SRC, R_TCP_DST = 32, 64, 128
R_UDP, R_UDP_SRC, R_UDP_DST = 256, 512, 1024
R_ICMP, R_ICMP_CODE, R_ICMP_TYPE, R_ICMPV6, R_ACTIONS = 2048, 4096, 8192, 16384, 32768

# the exported symbols (checked by tests/test_abi.py against include/contivcls.h)
SYMBOLS = ["cls_abi_version", "cls_engine_create", "cls_engine_destroy", "cls_last_error", "cls_engine_set_option",
           "cls_table_put", "cls_table_del", "cls_table_get_info", "cls_classify", "cls_classify_rules",
           "cls_last_kernel_ms", "cls_kernel_times", "cls_kernel_starts", "cls_kernel_times_reset", "cls_acl_put", "cls_acl_del", "cls_acl_table", "cls_acl_counts",
           "cls_if_id",
           "cls_if_acls", "cls_connect_batch", "cls_gen_traffic_v4", "cls_compile_v4", "cls_image_kernel",
           "cls_compile_v16", "cls_gen_traffic_v16", "cls_stream_floor", "cls_stream_floor_shapes", "cls_stream_floor_conn", "cls_conn_bitmap_eval", "cls_conn_counters",
           "cls_acl_stats", "cls_engine_devices", "cls_device_engine", "cls_shard_range", "cls_batch_create",
           "cls_batch_destroy", "cls_batch_shards", "cls_batch_shard", "cls_batch_field", "cls_batch_mirror",
           "cls_batch_upload", "cls_batch_download", "cls_batch_gen_traffic_v4", "cls_batch_gen_traffic_v16",
           "cls_classify_batch", "cls_batch_counters", "cls_batch_connect", "cls_batch_wait", "cls_comm_unique_id",
           "cls_comm_init", "cls_comm_info"]


class ClsRule(C.Structure):
    _fields_ = [("flags", C.c_uint32), ("acl_action", C.c_int32),
                ("src_network", C.c_char_p), ("dst_network", C.c_char_p),
                ("tcp_src_lo", C.c_uint32), ("tcp_src_hi", C.c_uint32),
                ("tcp_dst_lo", C.c_uint32), ("tcp_dst_hi", C.c_uint32),
                ("udp_src_lo", C.c_uint32), ("udp_src_hi", C.c_uint32),
                ("udp_dst_lo", C.c_uint32), ("udp_dst_hi", C.c_uint32),
                ("icmp_code_first", C.c_uint32), ("icmp_code_last", C.c_uint32),
                ("icmp_type_first", C.c_uint32), ("icmp_type_last", C.c_uint32)]


class PktSoa(C.Structure):
    _fields_ = [("af", C.c_uint32), ("src4", C.c_void_p), ("dst4", C.c_void_p),
                ("src16", C.c_void_p), ("dst16", C.c_void_p), ("sport", C.c_void_p),
                ("dport", C.c_void_p), ("proto", C.c_void_p)]


class ConnSoa(C.Structure):
    _fields_ = [("pkt", PktSoa), ("src_if", C.c_void_p), ("dst_if", C.c_void_p)]


class Config(C.Structure):
    _fields_ = [("device", C.c_int), ("n_devices", C.c_uint32), ("devices", C.POINTER(C.c_int)),
                ("reserved", C.c_uint32 * 4)]


class TableInfo(C.Structure):
    _fields_ = [("n_rules", C.c_uint32), ("kernel", C.c_uint32), ("lds_bytes", C.c_uint32),
                ("n_intervals", C.c_uint32), ("n_classes", C.c_uint32),
                ("n_templates", C.c_uint32), ("n_slots", C.c_uint32),
                ("lds_resident", C.c_uint32), ("has_v16", C.c_uint32), ("lds_bytes_v16", C.c_uint32),
                ("lds_resident_v16", C.c_uint32), ("n_lctr", C.c_uint32), ("ctr16", C.c_uint32),
                ("list_mode", C.c_uint32), ("swap", C.c_uint32), ("reserved", C.c_uint32 * 1)]


class TrafficSpec(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("pct_pod_src", C.c_uint32), ("pct_rule_dst", C.c_uint32),
                ("pct_table_port", C.c_uint32), ("pct_icmp", C.c_uint32),
                ("pod_ips", C.c_void_p), ("n_pod_ips", C.c_uint32),
                ("dst_addrs", C.c_void_p), ("dst_lens", C.c_void_p), ("n_dst", C.c_uint32),
                ("ports", C.c_void_p), ("n_ports", C.c_uint32)]


class TrafficSpec16(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("pct_pod_src", C.c_uint32), ("pct_rule_dst", C.c_uint32),
                ("pct_table_port", C.c_uint32), ("pct_icmp", C.c_uint32),
                ("pod_ips", C.c_void_p), ("n_pod_ips", C.c_uint32),
                ("dst_addrs", C.c_void_p), ("dst_lens", C.c_void_p), ("n_dst", C.c_uint32),
                ("ports", C.c_void_p), ("n_ports", C.c_uint32)]


class ImageHeader(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "magic", "version", "n_rules", "n_lin", "has_cls", "img_bytes", "off_bounds",
        "off_iclass", "off_cells", "off_lists", "off_tmpl", "n_bounds", "search_top",
        "n_classes", "n_tmpl", "n_list_entries", "n_ctr", "lds_bytes", "off_image",
        "off_ctr_rule", "off_lin", "total_bytes", "mode", "default_class", "n_hash")] + [
        ("hash_mask", C.c_uint32 * 3), ("hash_shift", C.c_uint32 * 3),
        ("hash_cap", C.c_uint32 * 3), ("off_hash", C.c_uint32 * 3),
        ("list_mode", C.c_uint32), ("off_bv", C.c_uint32), ("bv_steps_d", C.c_uint32),
        ("bv_steps_p", C.c_uint32), ("off_ptop", C.c_uint32), ("n_pclass", C.c_uint32),
        ("bv_wide", C.c_uint32), ("row_bytes", C.c_uint32), ("default_row", C.c_uint32),
        ("hash_mul", C.c_uint32 * 3), ("port_mul", C.c_uint32), ("port_mask4", C.c_uint32),
        ("port_dflt", C.c_uint32),
        ("n_hot", C.c_uint32), ("off_hot", C.c_uint32), ("n_lctr", C.c_uint32), ("ctr16", C.c_uint32),
        ("swap", C.c_uint32), ("off_other", C.c_uint32), ("off_trie", C.c_uint32), ("trie_depth", C.c_uint32),
        ("off_gcells", C.c_uint32), ("n_gcells", C.c_uint32)]


class Image16Header(C.Structure):
    """cls_image_v16_header: the core (rep-space) header, then the front end."""
    _fields_ = [("core", ImageHeader), ("fe_key", C.c_uint32 * 2), ("fe_val", C.c_uint32 * 2),
                ("fe_top", C.c_uint32 * 2), ("fe_n", C.c_uint32 * 2)] + [
        (n, C.c_uint32) for n in ("src_mode", "h4", "cap4", "mul4", "k6", "r6", "cap6", "mul6")] + [
        ("fold", C.c_uint32 * 3), ("dflt_row", C.c_uint32 * 2), ("off_src_search", C.c_uint32),
        ("src_search_val", C.c_uint32), ("fe_k8", C.c_uint32 * 2), ("src_search_top", C.c_uint32),
        ("src_search_k8", C.c_uint32)]


_lib = None


class ClsError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ClsError("libcontivcls.so not built (run __graft_entry__.build() or "
                       "make -C vpp_amd/csrc); the product has no CPU fallback")
    _lib = bind(LIB_PATH)
    return _lib


def bind(path: str, strict: bool = True):
    """Load a build of the library (RTLD_LOCAL: several builds may live in
    one process -- tools/ab_inproc.py) and declare its signatures (strict:
    every symbol of this ABI must be there)."""
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7.
    # Load it first so that our NEEDED libamdhip64.so.7 resolves to the same
    # already-loaded runtime (two runtimes in one process cannot share the
    # GPU).  CONTIVCLS_NO_TORCH=1: a torch-free host (the C ABI alone, as a
    # cgo host would use it -- tools/native_c3.py); the library then runs on
    # /opt/rocm's HIP runtime.
    if os.environ.get("CONTIVCLS_NO_TORCH") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = C.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    sig = {
        "cls_abi_version": (C.c_int, []),
        "cls_engine_create": (C.c_int, [C.POINTER(Config), C.POINTER(vp)]),
        "cls_engine_destroy": (None, [vp]),
        "cls_last_error": (C.c_char_p, [vp]),
        "cls_engine_set_option": (C.c_int, [vp, C.c_char_p, C.c_char_p]),
        "cls_table_put": (C.c_int, [vp, C.c_char_p, C.POINTER(ClsRule), u32, C.POINTER(u32)]),
        "cls_table_del": (C.c_int, [vp, u32]),
        "cls_table_get_info": (C.c_int, [vp, u32, C.POINTER(TableInfo)]),
        "cls_classify": (C.c_int, [vp, u32, C.POINTER(PktSoa), u64, vp, vp, u32, vp]),
        "cls_classify_rules": (C.c_int, [vp, u32, C.POINTER(PktSoa), u64, vp, vp, u32, vp]),
        "cls_last_kernel_ms": (C.c_int, [vp, C.POINTER(C.c_float)]),
        "cls_kernel_times": (C.c_int, [vp, C.POINTER(C.c_float), u32, C.POINTER(u32)]),
        "cls_kernel_starts": (C.c_int, [vp, C.POINTER(C.c_float), u32, C.POINTER(u32)]),
        "cls_kernel_times_reset": (C.c_int, [vp]),
        "cls_stream_floor": (C.c_int, [vp, C.POINTER(PktSoa), u64, vp, u32, C.POINTER(C.c_float), vp]),
        "cls_conn_bitmap_eval": (C.c_int, [C.POINTER(ClsRule), u32, vp, vp, vp, vp, u64, vp, vp]),
        "cls_stream_floor_shapes": (C.c_int, [vp, C.POINTER(PktSoa), u64, vp, u32, C.POINTER(C.c_float), u32,
                                              C.POINTER(C.c_uint32), vp]),
        "cls_stream_floor_conn": (C.c_int, [vp, C.POINTER(ConnSoa), u64, vp, u32, C.POINTER(C.c_float), vp]),
        "cls_acl_put": (C.c_int, [vp, C.c_char_p, C.POINTER(ClsRule), u32,
                                  C.POINTER(C.c_char_p), u32, C.POINTER(C.c_char_p), u32]),
        "cls_acl_del": (C.c_int, [vp, C.c_char_p]),
        "cls_acl_counts": (C.c_int, [vp, C.POINTER(u32), C.POINTER(u32)]),
        "cls_acl_table": (C.c_int, [vp, C.c_char_p, C.POINTER(u32)]),
        "cls_if_id": (C.c_int, [vp, C.c_char_p, C.POINTER(u32)]),
        "cls_if_acls": (C.c_int, [vp, u32, C.POINTER(i32), C.POINTER(i32)]),
        "cls_connect_batch": (C.c_int, [vp, C.POINTER(ConnSoa), u64, vp, u32, vp]),
        "cls_conn_counters": (C.c_int, [vp, u32, vp, u32]),
        "cls_acl_stats": (C.c_int, [vp, C.POINTER(u32), C.POINTER(u32)]),
        "cls_gen_traffic_v4": (C.c_int, [vp, C.POINTER(TrafficSpec), u64, u64, vp, vp, vp, vp,
                                         vp, vp]),
        "cls_compile_v4": (C.c_int, [C.POINTER(ClsRule), u32, vp, u64, C.POINTER(u64), C.c_char_p]),
        "cls_image_kernel": (C.c_int, [u32, u32, C.c_int, C.c_int]),
        "cls_compile_v16": (C.c_int, [C.POINTER(ClsRule), u32, vp, u64, C.POINTER(u64), C.c_char_p]),
        "cls_gen_traffic_v16": (C.c_int, [vp, C.POINTER(TrafficSpec16), u64, u64, vp, vp, vp, vp,
                                          vp, vp]),
        "cls_engine_devices": (C.c_int, [vp, C.POINTER(u32)]),
        "cls_device_engine": (C.c_int, [vp, u32, C.POINTER(vp)]),
        "cls_shard_range": (C.c_int, [u64, u32, u32, C.POINTER(u64), C.POINTER(u64)]),
        "cls_batch_create": (C.c_int, [vp, u32, u64, u32, C.POINTER(vp)]),
        "cls_batch_destroy": (None, [vp]),
        "cls_batch_shards": (C.c_int, [vp, C.POINTER(u32)]),
        "cls_batch_shard": (C.c_int, [vp, u32, C.POINTER(C.c_int), C.POINTER(u64), C.POINTER(u64)]),
        "cls_batch_field": (C.c_int, [vp, u32, u32, C.POINTER(vp)]),
        "cls_batch_mirror": (C.c_int, [vp, u32, C.POINTER(vp)]),
        "cls_batch_upload": (C.c_int, [vp, u32, u64, u64, vp]),
        "cls_batch_download": (C.c_int, [vp, u32, u64, u64, vp]),
        "cls_batch_gen_traffic_v4": (C.c_int, [vp, C.POINTER(TrafficSpec), u64]),
        "cls_batch_gen_traffic_v16": (C.c_int, [vp, C.POINTER(TrafficSpec16), u64]),
        "cls_classify_batch": (C.c_int, [vp, u32, vp, vp, u32]),
        "cls_batch_counters": (C.c_int, [vp, vp, u32]),
        "cls_batch_connect": (C.c_int, [vp, vp, u32]),
        "cls_batch_wait": (C.c_int, [vp]),
        "cls_comm_unique_id": (C.c_int, [vp]),
        "cls_comm_init": (C.c_int, [vp, u32, u32, vp]),
        "cls_comm_info": (C.c_int, [vp, C.POINTER(u32), C.POINTER(u32)]),
    }
    for name, (res, args) in sig.items():
        if not strict and not hasattr(L, name):      # an older build (A/B tools)
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


class CRules:
    """Owns a cls_rule array built from vpp_acl model rules."""

    def __init__(self, rules):
        self.n = len(rules)
        self.arr = (ClsRule * max(1, self.n))()
        self._keep = []
        for i, r in enumerate(rules):
            self._fill(self.arr[i], r)

    def _enc(self, s):
        b = s.encode()
        self._keep.append(b)
        return b

    def _fill(self, c, r):
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
                    c.src_network = self._enc(ipr.ip.source_network)
                    c.dst_network = self._enc(ipr.ip.destination_network)
                if ipr.other is not None:
                    f |= R_OTHER
                for sec, has, hs, hd, pre in ((ipr.tcp, R_TCP, R_TCP_SRC, R_TCP_DST, "tcp"),
                                              (ipr.udp, R_UDP, R_UDP_SRC, R_UDP_DST, "udp")):
                    if sec is None:
                        continue
                    f |= has
                    if sec.source_port_range is not None:
                        f |= hs
                        setattr(c, pre + "_src_lo", sec.source_port_range.lower_port)
                        setattr(c, pre + "_src_hi", sec.source_port_range.upper_port)
                    if sec.destination_port_range is not None:
                        f |= hd
                        setattr(c, pre + "_dst_lo", sec.destination_port_range.lower_port)
                        setattr(c, pre + "_dst_hi", sec.destination_port_range.upper_port)
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
