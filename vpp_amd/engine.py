"""Host layer of the GPU verdict backend (Python stand-in for the Go host).

``Engine`` wraps the C ABI (include/contivcls.h): compiled rule tables,
batched classification of packet batches resident in HBM (torch tensors) or
host memory (numpy), the device traffic generator.

``ACLEngine`` is the drop-in for the reference's MockACLEngine
(mock/aclengine/aclengine_mock.go:94-471) with the same method set:
RegisterPod, ApplyTxn, DumpACLs, GetNumOfACLs, GetInboundACL,
GetOutboundACL, GetACLByName, GetNumOfACLChanges and the three Connection*
entry points -- plus ``connection_batch`` which evaluates many connections in
one GPU launch.  ACL configuration (interfaces, replace-on-put, change
counting) lives in the C++ engine; this layer keeps only what the Go host
would: the protobuf ACLs by name, pods and interface names.
"""
from __future__ import annotations

import ctypes as C
import weakref
from typing import Optional

import numpy as np

from . import _abi, gonet
from ._abi import ClsError

ACL_KEY_PREFIX = "vpp/config/v1/acl/"
# ConnectionAction (aclengine_mock.go:46-60)
CONN_DENY_SYN, CONN_DENY_SYN_ACK, CONN_ALLOW, CONN_FAILURE = 0, 1, 2, 3
# ProtocolType (aclengine_mock.go:80-91)
TCP, UDP, ICMP = 0, 1, 2


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _ptr(x):
    if x is None:
        return None
    if _is_torch(x):
        return x.data_ptr()
    return x.ctypes.data


class Table:
    def __init__(self, engine: "Engine", tid: int, n_rules: int, name: str):
        self.engine = engine
        self.id = tid
        self.n_rules = n_rules
        self.name = name

    def info(self) -> dict:
        inf = _abi.TableInfo()
        self.engine._check(_abi.lib().cls_table_get_info(self.engine.h, self.id, C.byref(inf)))
        return {k: getattr(inf, k) for k, _ in _abi.TableInfo._fields_ if k != "reserved"}


class Engine:
    """One gfx950 device, or (``devices``) a multi-device engine: tables
    compiled once and replicated, batches sharded over the devices, hit
    counters merged by the library's RCCL all-reduce (include/contivcls.h)."""

    def __init__(self, device: int = -1, devices=None, options: Optional[dict] = None):
        L = _abi.lib()
        if devices:
            self._devs = (C.c_int * len(devices))(*devices)
            cfg = _abi.Config(-1, len(devices), C.cast(self._devs, C.POINTER(C.c_int)))
        else:
            cfg = _abi.Config(device, 0, None)
        h = C.c_void_p()
        rc = L.cls_engine_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise ClsError("cls_engine_create failed (rc=%d): %s" % (
                rc, "RCCL communicator" if rc == _abi.E_RCCL else "no usable gfx950 device"))
        self.h = h
        self._owned = True
        self._batches = weakref.WeakSet()       # closed before the engine (cls_engine_destroy)
        self._views = []                        # device_engine() views: invalid once the engine closes
        for k, v in (options or {}).items():
            self.set_option(k, v)

    @classmethod
    def _view(cls, handle) -> "Engine":
        v = cls.__new__(cls)
        v.h = handle
        v._owned = False
        v._batches = weakref.WeakSet()
        v._views = []
        return v

    def set_option(self, key: str, value=None):
        """cls_engine_set_option: a tuning / diagnostic switch of this engine
        (tests and measurements: forced list modes, counter tiers, launch
        plans; include/contivcls.h), ``None`` for its default.  The library
        never reads the environment."""
        v = None if value is None else str(value).encode()
        self._check(_abi.lib().cls_engine_set_option(self.h, key.encode(), v))

    def close(self):
        if getattr(self, "h", None) and getattr(self, "_owned", True):
            # the batches (and borrowed device views) hold this engine's handle
            for b in list(getattr(self, "_batches", ())):
                b.close()
            for v in getattr(self, "_views", ()):
                v.h = None
            _abi.lib().cls_engine_destroy(self.h)
        self.h = None

    # -- devices, batches, the counter all-reduce (ABI 4) -------------------
    def n_devices(self) -> int:
        n = C.c_uint32(0)
        self._check(_abi.lib().cls_engine_devices(self.h, C.byref(n)))
        return n.value

    def device_engine(self, index: int) -> "Engine":
        """Borrowed single-device view of device ``index`` (timing, stream
        floors, raw device pointers of that device)."""
        d = C.c_void_p()
        self._check(_abi.lib().cls_device_engine(self.h, index, C.byref(d)))
        v = Engine._view(d)
        self._views.append(v)
        return v

    def batch(self, n: int, af: int = _abi.AF_V4, conn: bool = False, mirror: bool = False) -> "Batch":
        return Batch(self, n, af, conn, mirror)

    def classify_batch(self, table: Table, batch: "Batch", counters: bool = True, timing: bool = False,
                       no_verdict: bool = False, force_linear: bool = False):
        """cls_classify_batch: verdicts stay in the batch (CLS_BF_VERDICT);
        returns the merged hit counters (uint64[R+1]) or, counters=False,
        None after only enqueueing the work."""
        flags = (_abi.F_TIMING if timing else 0) | (_abi.F_NO_VERDICT if no_verdict else 0) | \
            (_abi.F_FORCE_LINEAR if force_linear else 0)
        out = np.zeros(table.n_rules + 1, np.uint64) if counters else None
        self._check(_abi.lib().cls_classify_batch(self.h, table.id, batch.h, _ptr(out), flags))
        return out

    def connect_batch_b(self, batch: "Batch", mode: str = "auto", count: bool = False):
        """cls_batch_connect: ConnectionAction per connection into the batch."""
        flags = {"auto": 0, "classifier": _abi.F_CONN_CLS, "linear": _abi.F_FORCE_LINEAR}[mode]
        if count:
            flags |= _abi.F_COUNT
        self._check(_abi.lib().cls_batch_connect(self.h, batch.h, flags))

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        rc = _abi.lib().cls_comm_unique_id(buf)
        if rc != 0:
            raise ClsError("cls_comm_unique_id failed (rc=%d)" % rc)
        return bytes(buf)

    def comm_init(self, n_procs: int = 1, proc: int = 0, uid: Optional[bytes] = None):
        ib = (C.c_uint8 * 128).from_buffer_copy(uid) if uid is not None else None
        self._check(_abi.lib().cls_comm_init(self.h, n_procs, proc, ib))

    def comm_info(self):
        n, r = C.c_uint32(0), C.c_uint32(0)
        self._check(_abi.lib().cls_comm_info(self.h, C.byref(n), C.byref(r)))
        return n.value, r.value

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != 0:
            raise ClsError("rc=%d: %s" % (rc, _abi.lib().cls_last_error(self.h).decode()))

    # -- tables -----------------------------------------------------------
    def put_table(self, name: str, rules) -> Table:
        cr = rules if isinstance(rules, _abi.CRules) else _abi.CRules(rules)
        tid = C.c_uint32(0)
        self._check(_abi.lib().cls_table_put(self.h, name.encode(), cr.ptr(), cr.n, C.byref(tid)))
        return Table(self, tid.value, cr.n, name)

    def del_table(self, table: Table):
        self._check(_abi.lib().cls_table_del(self.h, table.id))

    # -- classify ---------------------------------------------------------
    def classify(self, table: Table, src, dst, dport, proto, verdict=None, counters=None,
                 force_linear=False, timing=False, accumulate=False, stream=None):
        """A packet batch: IPv4 (src, dst: uint32[n], host order) or the
        16-byte layout (src, dst: uint8[n, 16], network order; IPv4-mapped
        addresses are IPv4 packets).  numpy inputs: synchronous, returns
        (verdict, counters) as numpy arrays.  torch device tensors: enqueued on
        ``stream`` (a torch.cuda.Stream or raw handle; default torch's current
        stream); ``verdict`` (uint8[n]) and ``counters`` (int64[R+1]) are
        written."""
        n = int(len(dport))
        dev = _is_torch(src)
        v16 = (src.dim() if dev else np.ndim(src)) == 2

        def soa(s_, d_, dp_, pr_):
            if v16:
                return _abi.PktSoa(_abi.AF_V16, None, None, _ptr(s_), _ptr(d_), None, _ptr(dp_), _ptr(pr_))
            return _abi.PktSoa(_abi.AF_V4, _ptr(s_), _ptr(d_), None, None, None, _ptr(dp_), _ptr(pr_))
        flags = 0
        if force_linear:
            flags |= _abi.F_FORCE_LINEAR
        if timing:
            flags |= _abi.F_TIMING
        if accumulate:
            flags |= _abi.F_ACCUMULATE
        if dev:
            import torch
            flags |= _abi.F_DEVICE
            if verdict is None:
                flags |= _abi.F_NO_VERDICT
            if stream is None:
                stream = torch.cuda.current_stream()
            s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
            pk = soa(src, dst, dport, proto)
            self._check(_abi.lib().cls_classify(self.h, table.id, C.byref(pk), n, _ptr(verdict),
                                                _ptr(counters), flags, s))
            return verdict, counters
        adt = np.uint8 if v16 else np.uint32
        src = np.ascontiguousarray(src, adt)
        dst = np.ascontiguousarray(dst, adt)
        dport = np.ascontiguousarray(dport, np.uint16)
        proto = np.ascontiguousarray(proto, np.uint8)
        v = np.zeros(n, np.uint8) if verdict is None else verdict
        c = np.zeros(table.n_rules + 1, np.uint64) if counters is None else counters
        pk = soa(src, dst, dport, proto)
        self._check(_abi.lib().cls_classify(self.h, table.id, C.byref(pk), n, _ptr(v), _ptr(c),
                                            flags, None))
        return v, c

    def classify_rules(self, table: Table, src, dst, dport, proto, verdict=None, rules=None, stream=None):
        """Each packet's ACLAction and terminating rule index (R: the default
        DENY) -- cls_classify_rules, the batch form of the matched rule
        evalACL logs; no counters.  numpy inputs: synchronous, returns
        (verdict uint8[n], rules uint32[n]); torch device tensors: enqueued on
        ``stream``, ``rules`` (int32[n]) and ``verdict`` (uint8[n], optional)
        written and returned."""
        n = int(len(dport))
        dev = _is_torch(src)
        v16 = (src.dim() if dev else np.ndim(src)) == 2

        def soa(s_, d_, dp_, pr_):
            if v16:
                return _abi.PktSoa(_abi.AF_V16, None, None, _ptr(s_), _ptr(d_), None, _ptr(dp_), _ptr(pr_))
            return _abi.PktSoa(_abi.AF_V4, _ptr(s_), _ptr(d_), None, None, None, _ptr(dp_), _ptr(pr_))
        if dev:
            import torch
            if stream is None:
                stream = torch.cuda.current_stream()
            s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
            if rules is None:
                rules = torch.empty(n, dtype=torch.int32, device=src.device)
            pk = soa(src, dst, dport, proto)
            self._check(_abi.lib().cls_classify_rules(self.h, table.id, C.byref(pk), n, _ptr(verdict),
                                                      _ptr(rules), _abi.F_DEVICE, s))
            return verdict, rules
        adt = np.uint8 if v16 else np.uint32
        src = np.ascontiguousarray(src, adt)
        dst = np.ascontiguousarray(dst, adt)
        dport = np.ascontiguousarray(dport, np.uint16)
        proto = np.ascontiguousarray(proto, np.uint8)
        v = np.zeros(n, np.uint8) if verdict is None else verdict
        r = np.zeros(n, np.uint32) if rules is None else rules
        pk = soa(src, dst, dport, proto)
        self._check(_abi.lib().cls_classify_rules(self.h, table.id, C.byref(pk), n, _ptr(v), _ptr(r), 0, None))
        return v, r

    def stream_floor(self, src, dst, dport, proto, verdict, reps: int = 10, stream=None) -> float:
        """Average ms of the classify kernel's packet stream alone (same loads,
        stores and grid, no lookups) over a device batch: the measured floor
        the classify kernel is compared against (bench.py) -- the fastest
        stream shape."""
        return min(self.stream_floor_shapes(src, dst, dport, proto, verdict, reps, stream))

    def stream_floor_shapes(self, src, dst, dport, proto, verdict, reps: int = 10, stream=None):
        """Each stream shape's average ms (cls_stream_floor_shapes): index =
        variant << 1 | two workgroups per CU; IPv4 8 shapes, 16-byte 2."""
        import torch
        v16 = src.dim() == 2
        n = int(dport.numel())
        if v16:
            pk = _abi.PktSoa(_abi.AF_V16, None, None, _ptr(src), _ptr(dst), None, _ptr(dport), _ptr(proto))
            n -= n % 256
        else:
            pk = _abi.PktSoa(_abi.AF_V4, _ptr(src), _ptr(dst), None, None, None, _ptr(dport), _ptr(proto))
            n -= n % 4
        if stream is None:
            stream = torch.cuda.current_stream()
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        ms = (C.c_float * 8)()
        cnt = C.c_uint32(0)
        self._check(_abi.lib().cls_stream_floor_shapes(self.h, C.byref(pk), n, _ptr(verdict), reps, ms, 8,
                                                       C.byref(cnt), s))
        scale = int(dport.numel()) / n if n else 1.0
        return [ms[i] * scale for i in range(cnt.value)]

    def last_kernel_ms(self) -> float:
        ms = C.c_float(0)
        self._check(_abi.lib().cls_last_kernel_ms(self.h, C.byref(ms)))
        return ms.value

    def _timed(self, fn):
        n = C.c_uint32(0)
        self._check(fn(self.h, None, 0, C.byref(n)))
        buf = (C.c_float * max(1, n.value))()
        self._check(fn(self.h, buf, n.value, C.byref(n)))
        return [buf[i] for i in range(n.value)]

    def kernel_times(self, reset: bool = True, starts: bool = False):
        """Durations (ms) of every kernel timed since the last reset; with
        `starts`, (durations, start times in ms after the first one's)."""
        out = self._timed(_abi.lib().cls_kernel_times)
        if starts:
            out = (out, self._timed(_abi.lib().cls_kernel_starts))
        if reset:
            self._check(_abi.lib().cls_kernel_times_reset(self.h))
        return out

    # -- traffic ------------------------------------------------------------
    def gen_traffic_v4(self, spec: dict, first: int, out: dict, stream=None):
        """Generate packets [first, first+n) of the synthetic stream into the
        device tensors of ``out`` (src, dst, sport, dport, proto)."""
        pods = np.ascontiguousarray(spec.get("pod_ips", []), np.uint32)
        da = np.ascontiguousarray(spec.get("dst_addrs", []), np.uint32)
        dl = np.ascontiguousarray(spec.get("dst_lens", []), np.uint8)
        ports = np.ascontiguousarray(spec.get("ports", []), np.uint16)
        ts = _abi.TrafficSpec(spec["seed"], spec.get("pct_pod_src", 60), spec.get("pct_rule_dst", 50),
                              spec.get("pct_table_port", 50), spec.get("pct_icmp", 0),
                              pods.ctypes.data, len(pods), da.ctypes.data, dl.ctypes.data, len(da),
                              ports.ctypes.data, len(ports))
        n = int(len(out["dport"]))
        s = None
        if stream is not None:
            s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        self._check(_abi.lib().cls_gen_traffic_v4(
            self.h, C.byref(ts), first, n, _ptr(out.get("src")), _ptr(out.get("dst")),
            _ptr(out.get("sport")), _ptr(out.get("dport")), _ptr(out.get("proto")), s))

    def gen_traffic_v16(self, spec: dict, first: int, out: dict, stream=None):
        """The 16-byte stream (cls_traffic_spec16) into device tensors: src,
        dst uint8[n, 16] (16-B aligned), sport, dport, proto.  Pools:
        pod_ips / dst_addrs uint8[m, 16], dst_lens 0..128, ports."""
        pods = np.ascontiguousarray(spec.get("pod_ips", np.zeros((0, 16))), np.uint8)
        da = np.ascontiguousarray(spec.get("dst_addrs", np.zeros((0, 16))), np.uint8)
        dl = np.ascontiguousarray(spec.get("dst_lens", []), np.uint8)
        ports = np.ascontiguousarray(spec.get("ports", []), np.uint16)
        ts = _abi.TrafficSpec16(spec["seed"], spec.get("pct_pod_src", 60), spec.get("pct_rule_dst", 50),
                                spec.get("pct_table_port", 50), spec.get("pct_icmp", 0),
                                pods.ctypes.data, len(pods), da.ctypes.data, dl.ctypes.data, len(da),
                                ports.ctypes.data, len(ports))
        n = int(len(out["dport"]))
        s = None
        if stream is not None:
            s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        self._check(_abi.lib().cls_gen_traffic_v16(
            self.h, C.byref(ts), first, n, _ptr(out.get("src")), _ptr(out.get("dst")),
            _ptr(out.get("sport")), _ptr(out.get("dport")), _ptr(out.get("proto")), s))

    # -- ACL configuration (ACLConfig) ---------------------------------------
    def acl_put(self, name: str, rules, ingress, egress):
        cr = _abi.CRules(rules)
        ing = (C.c_char_p * max(1, len(ingress)))(*[x.encode() for x in ingress])
        eg = (C.c_char_p * max(1, len(egress)))(*[x.encode() for x in egress])
        return _abi.lib().cls_acl_put(self.h, name.encode(), cr.ptr(), cr.n, ing, len(ingress),
                                      eg, len(egress))

    def acl_del(self, name: str):
        return _abi.lib().cls_acl_del(self.h, name.encode())

    def acl_table(self, name: str) -> int:
        t = C.c_uint32(0)
        rc = _abi.lib().cls_acl_table(self.h, name.encode(), C.byref(t))
        return int(t.value) if rc == 0 else -1

    def acl_counts(self):
        a, c = C.c_uint32(0), C.c_uint32(0)
        self._check(_abi.lib().cls_acl_counts(self.h, C.byref(a), C.byref(c)))
        return a.value, c.value

    def acl_stats(self):
        """(tables compiled, puts that kept the installed table) by cls_acl_put."""
        a, c = C.c_uint32(0), C.c_uint32(0)
        self._check(_abi.lib().cls_acl_stats(self.h, C.byref(a), C.byref(c)))
        return a.value, c.value

    def if_id(self, name: str) -> int:
        i = C.c_uint32(0)
        self._check(_abi.lib().cls_if_id(self.h, name.encode(), C.byref(i)))
        return i.value

    def if_acls(self, if_id: int):
        a, b = C.c_int32(0), C.c_int32(0)
        self._check(_abi.lib().cls_if_acls(self.h, if_id, C.byref(a), C.byref(b)))
        return a.value, b.value

    def connect_batch(self, src_if, dst_if, src, dst, proto, sport, dport, mode: str = "auto",
                      count: bool = False, out=None) -> np.ndarray:
        """testConnection over a batch (cls_connect_batch).  Addresses: host-order
        u32 (IPv4) or n x 16 network-order bytes (IPv6, IPv4-mapped = IPv4).
        mode: "auto" (ACLs with a classifier image use it for batches >=
        65536), "classifier" (at any size) or "linear" (every ACL scanned).
        count: add every evalACL call's terminating rule to the tables'
        connection counters (conn_counters).  out (device batches): a
        contiguous uint8 GPU tensor of n verdicts to write instead of a new
        one."""
        flags = {"auto": 0, "classifier": _abi.F_CONN_CLS, "linear": _abi.F_FORCE_LINEAR}[mode]
        if count:
            flags |= _abi.F_COUNT
        if _is_torch(src):
            return self._connect_batch_device(src_if, dst_if, src, dst, proto, sport, dport, flags, out)
        v16 = np.asarray(src).ndim == 2
        if v16:
            s = np.ascontiguousarray(src, np.uint8).reshape(-1, 16)
            d = np.ascontiguousarray(dst, np.uint8).reshape(-1, 16)
        else:
            s, d = np.ascontiguousarray(src, np.uint32), np.ascontiguousarray(dst, np.uint32)
        si, di = np.ascontiguousarray(src_if, np.uint32), np.ascontiguousarray(dst_if, np.uint32)
        p, sp = np.ascontiguousarray(proto, np.uint8), np.ascontiguousarray(sport, np.uint16)
        dp = np.ascontiguousarray(dport, np.uint16)
        n = len(s)
        out = np.zeros(n, np.uint8)
        if v16:
            pk = _abi.PktSoa(_abi.AF_V16, None, None, _ptr(s), _ptr(d), _ptr(sp), _ptr(dp), _ptr(p))
        else:
            pk = _abi.PktSoa(_abi.AF_V4, _ptr(s), _ptr(d), None, None, _ptr(sp), _ptr(dp), _ptr(p))
        cs = _abi.ConnSoa(pk, _ptr(si), _ptr(di))
        self._check(_abi.lib().cls_connect_batch(self.h, C.byref(cs), n, _ptr(out), flags, None))
        return out

    def _connect_batch_device(self, src_if, dst_if, src, dst, proto, sport, dport, flags, out=None):
        """Device-resident batch (CLS_F_DEVICE): contiguous GPU tensors of 4-byte
        interface ids, 4-byte (or n x 16 uint8) addresses, 2-byte ports and
        1-byte protocols, already written (the call runs on the engine's
        stream).  Returns a uint8 tensor (`out` when given)."""
        import torch
        v16 = src.dim() == 2
        arrs = (src_if, dst_if, src, dst, sport, dport, proto)
        sizes = (4, 4, 1 if v16 else 4, 1 if v16 else 4, 2, 2, 1)
        n = src.shape[0]
        for x, sz in zip(arrs, sizes):
            if not (_is_torch(x) and x.is_cuda and x.is_contiguous() and x.element_size() == sz and x.shape[0] == n):
                raise ClsError("device connection batch: contiguous GPU tensors of element sizes %s" % (sizes,))
        if out is None:
            out = torch.empty(n, dtype=torch.uint8, device=src.device)
        elif not (_is_torch(out) and out.is_cuda and out.is_contiguous() and out.element_size() == 1 and
                  out.shape[0] == n):
            raise ClsError("device connection batch: out must be a contiguous uint8 GPU tensor of n elements")
        if v16:
            pk = _abi.PktSoa(_abi.AF_V16, None, None, _ptr(src), _ptr(dst), _ptr(sport), _ptr(dport), _ptr(proto))
        else:
            pk = _abi.PktSoa(_abi.AF_V4, _ptr(src), _ptr(dst), None, None, _ptr(sport), _ptr(dport), _ptr(proto))
        cs = _abi.ConnSoa(pk, _ptr(src_if), _ptr(dst_if))
        self._check(_abi.lib().cls_connect_batch(self.h, C.byref(cs), n, _ptr(out), flags | _abi.F_DEVICE, None))
        return out

    def stream_floor_conn(self, src_if, dst_if, src, dst, proto, sport, dport, reps: int = 20) -> float:
        """The connection path's HBM floor on a device batch (cls_stream_floor_conn):
        ms per launch of a kernel that reads the same 22 B per IPv4 connection
        and writes one byte, with no evaluation."""
        import torch
        n = src.shape[0]
        out = torch.empty(n, dtype=torch.uint8, device=src.device)
        pk = _abi.PktSoa(_abi.AF_V4, _ptr(src), _ptr(dst), None, None, _ptr(sport), _ptr(dport), _ptr(proto))
        cs = _abi.ConnSoa(pk, _ptr(src_if), _ptr(dst_if))
        ms = C.c_float()
        self._check(_abi.lib().cls_stream_floor_conn(self.h, C.byref(cs), n, _ptr(out), reps, C.byref(ms), None))
        return ms.value

    def conn_counters(self, table, reset: bool = False) -> np.ndarray:
        """Per-rule connection counters of a table (a Table, a table id or an
        installed ACL's name): R + 1 u64, [R] = default DENY."""
        if isinstance(table, str):
            table = self.acl_table(table)
        tid = table.id if isinstance(table, Table) else int(table)
        info = _abi.TableInfo()
        self._check(_abi.lib().cls_table_get_info(self.h, tid, C.byref(info)))
        out = np.zeros(info.n_rules + 1, np.uint64)
        self._check(_abi.lib().cls_conn_counters(self.h, tid, _ptr(out), 1 if reset else 0))
        return out


_BF_BYTES = {_abi.BF_SPORT: 2, _abi.BF_DPORT: 2, _abi.BF_PROTO: 1, _abi.BF_VERDICT: 1,
             _abi.BF_SRC_IF: 4, _abi.BF_DST_IF: 4}
_NP = {1: np.uint8, 2: np.uint16, 4: np.uint32}


def shard_range(n: int, n_shards: int, shard: int):
    """(first, count) of shard ``shard`` of n packets (cls_shard_range)."""
    a, b = C.c_uint64(0), C.c_uint64(0)
    rc = _abi.lib().cls_shard_range(n, n_shards, shard, C.byref(a), C.byref(b))
    if rc != 0:
        raise ClsError("cls_shard_range(%d, %d, %d): rc=%d" % (n, n_shards, shard, rc))
    return a.value, b.value


class Batch:
    """An engine-owned packet (or connection) batch in HBM, sharded over the
    engine's devices (cls_batch_*): no torch, no caller pointer kept."""

    def __init__(self, engine: Engine, n: int, af: int = _abi.AF_V4, conn: bool = False, mirror: bool = False):
        self.engine, self.n, self.af = engine, n, af
        flags = (_abi.BATCH_CONN if conn else 0) | (_abi.BATCH_MIRROR if mirror else 0)
        h = C.c_void_p()
        engine._check(_abi.lib().cls_batch_create(engine.h, af, n, flags, C.byref(h)))
        self.h = h
        engine._batches.add(self)

    def close(self):
        if getattr(self, "h", None):
            _abi.lib().cls_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _elem(self, field: int) -> int:
        return _BF_BYTES.get(field, 16 if self.af == _abi.AF_V16 else 4)

    def shards(self):
        """[(device, first, n)] per shard."""
        k = C.c_uint32(0)
        self.engine._check(_abi.lib().cls_batch_shards(self.h, C.byref(k)))
        out = []
        for g in range(k.value):
            d, a, b = C.c_int(0), C.c_uint64(0), C.c_uint64(0)
            self.engine._check(_abi.lib().cls_batch_shard(self.h, g, C.byref(d), C.byref(a), C.byref(b)))
            out.append((d.value, a.value, b.value))
        return out

    def field_ptr(self, shard: int, field: int) -> int:
        p = C.c_void_p()
        self.engine._check(_abi.lib().cls_batch_field(self.h, shard, field, C.byref(p)))
        return p.value

    def mirror(self, field: int) -> np.ndarray:
        """The pinned host mirror of a field (CLS_BATCH_MIRROR) as a numpy view."""
        p = C.c_void_p()
        self.engine._check(_abi.lib().cls_batch_mirror(self.h, field, C.byref(p)))
        eb = self._elem(field)
        buf = (C.c_uint8 * (self.n * eb)).from_address(p.value)
        a = np.frombuffer(buf, np.uint8)
        return a.reshape(-1, 16) if eb == 16 else a.view(_NP[eb])

    def upload(self, field: int, arr=None, first: int = 0, n: Optional[int] = None):
        """Packets [first, first+n) of a field from ``arr`` (None: the mirror)."""
        eb = self._elem(field)
        if arr is not None:
            arr = np.ascontiguousarray(arr, np.uint8 if eb == 16 else _NP[eb])
            n = len(arr) if n is None else n
        n = (self.n - first) if n is None else n
        self.engine._check(_abi.lib().cls_batch_upload(self.h, field, first, n, _ptr(arr)))

    def download(self, field: int, first: int = 0, n: Optional[int] = None, mirror: bool = False):
        n = (self.n - first) if n is None else n
        eb = self._elem(field)
        if mirror:
            self.engine._check(_abi.lib().cls_batch_download(self.h, field, first, n, None))
            return None
        out = np.zeros((n, 16) if eb == 16 else n, np.uint8 if eb == 16 else _NP[eb])
        self.engine._check(_abi.lib().cls_batch_download(self.h, field, first, n, _ptr(out)))
        return out

    def gen_traffic(self, spec: dict, stream_first: int = 0):
        """The synthetic stream generated on the devices: batch packet i =
        stream packet stream_first + i."""
        if self.af == _abi.AF_V16:
            ts, keep = _spec16(spec)
            self.engine._check(_abi.lib().cls_batch_gen_traffic_v16(self.h, C.byref(ts), stream_first))
        else:
            ts, keep = _spec4(spec)
            self.engine._check(_abi.lib().cls_batch_gen_traffic_v4(self.h, C.byref(ts), stream_first))
        del keep

    def counters(self, n_rules: int) -> np.ndarray:
        out = np.zeros(n_rules + 1, np.uint64)
        self.engine._check(_abi.lib().cls_batch_counters(self.h, _ptr(out), n_rules + 1))
        return out

    def wait(self):
        self.engine._check(_abi.lib().cls_batch_wait(self.h))


def _spec4(spec: dict):
    pods = np.ascontiguousarray(spec.get("pod_ips", []), np.uint32)
    da = np.ascontiguousarray(spec.get("dst_addrs", []), np.uint32)
    dl = np.ascontiguousarray(spec.get("dst_lens", []), np.uint8)
    ports = np.ascontiguousarray(spec.get("ports", []), np.uint16)
    ts = _abi.TrafficSpec(spec["seed"], spec.get("pct_pod_src", 60), spec.get("pct_rule_dst", 50),
                          spec.get("pct_table_port", 50), spec.get("pct_icmp", 0),
                          pods.ctypes.data, len(pods), da.ctypes.data, dl.ctypes.data, len(da),
                          ports.ctypes.data, len(ports))
    return ts, (pods, da, dl, ports)


def _spec16(spec: dict):
    pods = np.ascontiguousarray(spec.get("pod_ips", np.zeros((0, 16))), np.uint8)
    da = np.ascontiguousarray(spec.get("dst_addrs", np.zeros((0, 16))), np.uint8)
    dl = np.ascontiguousarray(spec.get("dst_lens", []), np.uint8)
    ports = np.ascontiguousarray(spec.get("ports", []), np.uint16)
    ts = _abi.TrafficSpec16(spec["seed"], spec.get("pct_pod_src", 60), spec.get("pct_rule_dst", 50),
                            spec.get("pct_table_port", 50), spec.get("pct_icmp", 0),
                            pods.ctypes.data, len(pods), da.ctypes.data, dl.ctypes.data, len(da),
                            ports.ctypes.data, len(ports))
    return ts, (pods, da, dl, ports)


def _ip16(ip: Optional[bytes]) -> Optional[bytes]:
    """net.IP as the 16-byte form (IPv4 as IPv4-mapped, like Go's To16)."""
    if ip is None or len(ip) not in (4, 16):
        return None
    return bytes(10) + b"\xff\xff" + bytes(ip) if len(ip) == 4 else bytes(ip)


def _ip4(ip: Optional[bytes]) -> Optional[int]:
    if ip is None:
        return None
    x = gonet.to4(ip)
    if x is None:
        return None
    return int.from_bytes(x, "big")


class ACLEngine:
    """MockACLEngine drop-in over the GPU engine (aclengine_mock.go:94-471)."""

    def __init__(self, contiv, engine: Optional[Engine] = None):
        self.contiv = contiv
        self.engine = engine or Engine()
        self.pods = {}              # PodID -> (net.IP bytes | None, another_node)
        self.by_name = {}           # ACL name -> Acl (the protobuf the host keeps)

    # RegisterPod (:144-148)
    def register_pod(self, pod, pod_ip: str, another_node: bool):
        self.pods[pod] = (gonet.parse_ip(pod_ip), another_node)

    # ApplyTxn (:151-198): returns an error string or None
    def apply_txn(self, ops):
        for key, value in ops:
            if not key.startswith(ACL_KEY_PREFIX):
                return "non-ACL changed in txn"
            name = key[len(ACL_KEY_PREFIX):]
            if value is not None:
                acl = value.clone()          # the engine keeps its own message (rules shared, never modified)
                ifs = acl.interfaces
                rc = self.engine.acl_put(acl.acl_name, acl.rules,
                                         ifs.ingress if ifs else [], ifs.egress if ifs else [])
                if rc != 0:
                    return _abi.lib().cls_last_error(self.engine.h).decode()
                self.by_name[acl.acl_name] = acl
            else:
                rc = self.engine.acl_del(name)
                if rc != 0:
                    return _abi.lib().cls_last_error(self.engine.h).decode()
                self.by_name.pop(name, None)
        return None

    def dump_acls(self):
        return list(self.by_name.values())

    def get_num_of_acls(self) -> int:
        return self.engine.acl_counts()[0]

    def get_num_of_acl_changes(self) -> int:
        return self.engine.acl_counts()[1]

    def _acl_of_table(self, tid: int):
        """The protobuf ACL whose compiled table the engine bound (-1: nil)."""
        if tid < 0:
            return None
        for name, acl in self.by_name.items():
            if self.engine.acl_table(name) == tid:
                return acl
        return None

    def get_inbound_acl(self, if_name: str):
        i, _ = self.engine.if_acls(self.engine.if_id(if_name))
        return self._acl_of_table(i)

    def get_outbound_acl(self, if_name: str):
        _, o = self.engine.if_acls(self.engine.if_id(if_name))
        return self._acl_of_table(o)

    def get_acl_by_name(self, name: str):
        return self.by_name.get(name)

    # -- Connection* (:243-390), resolved on the host, evaluated on the GPU --
    def _node_output_if(self):
        ifn = self.contiv.get_vxlan_bvi_if_name()
        return ifn if ifn != "" else self.contiv.get_main_physical_if_name()

    def _pod_if(self, pod, cfg):
        if cfg[1]:
            ifn = self._node_output_if()
            return ifn if ifn != "" else None
        ifn, ok = self.contiv.get_if_name(pod.namespace, pod.name)
        return ifn if ok else None

    def resolve(self, fn: str, args):
        """Returns (src_if, src_ip, dst_if, dst_ip, proto, sport, dport) or
        CONN_FAILURE when the reference fails before testConnection."""
        if fn == "ConnectionPodToPod":
            sp, dp, proto, sport, dport = args
            s, d = self.pods.get(sp), self.pods.get(dp)
            if s is None or d is None:
                return CONN_FAILURE
            sif, dif = self._pod_if(sp, s), self._pod_if(dp, d)
            if sif is None or dif is None:
                return CONN_FAILURE
            return sif, s[0], dif, d[0], proto, sport, dport
        if fn == "ConnectionPodToInternet":
            sp, dst_ip, proto, sport, dport = args
            s = self.pods.get(sp)
            if s is None or s[1]:
                return CONN_FAILURE
            sif, ok = self.contiv.get_if_name(sp.namespace, sp.name)
            dif = self._node_output_if()
            ip = gonet.parse_ip(dst_ip)
            if not ok or dif == "" or ip is None:
                return CONN_FAILURE
            return sif, s[0], dif, ip, proto, sport, dport
        src_ip, dp, proto, sport, dport = args
        d = self.pods.get(dp)
        if d is None or d[1]:
            return CONN_FAILURE
        sif = self._node_output_if()
        ip = gonet.parse_ip(src_ip)
        dif, ok = self.contiv.get_if_name(dp.namespace, dp.name)
        if sif == "" or ip is None or not ok:
            return CONN_FAILURE
        return sif, ip, dif, d[0], proto, sport, dport

    def connection_batch(self, calls, count: bool = False):
        """calls: list of (fn name, args).  One GPU launch for all of them: the
        IPv4 layout when every endpoint is IPv4, else the 16-byte layout."""
        out = [None] * len(calls)
        rows = []
        for i, (fn, args) in enumerate(calls):
            r = self.resolve(fn, args)
            if r == CONN_FAILURE:
                out[i] = CONN_FAILURE
                continue
            sif, sip, dif, dip, proto, sport, dport = r
            rows.append((i, self.engine.if_id(sif), self.engine.if_id(dif), sip, dip, proto, sport, dport))
        if not rows:
            return out
        four = [(_ip4(r[3]), _ip4(r[4])) for r in rows]
        meta = np.array([(r[1], r[2], r[5], r[6], r[7]) for r in rows], np.int64)
        if all(a is not None and b is not None for a, b in four):
            src = np.array([a for a, _ in four], np.uint32)
            dst = np.array([b for _, b in four], np.uint32)
        else:
            a16 = [(_ip16(r[3]), _ip16(r[4])) for r in rows]
            if any(a is None or b is None for a, b in a16):
                raise ClsError("connection endpoint is not an IPv4 or IPv6 address")
            src = np.frombuffer(b"".join(a for a, _ in a16), np.uint8).reshape(-1, 16)
            dst = np.frombuffer(b"".join(b for _, b in a16), np.uint8).reshape(-1, 16)
        res = self.engine.connect_batch(meta[:, 0], meta[:, 1], src, dst, meta[:, 2], meta[:, 3], meta[:, 4],
                                        count=count)
        for (i, *_), v in zip(rows, res):
            out[i] = int(v)
        return out

    def connection_pod_to_pod(self, src_pod, dst_pod, proto, sport, dport):
        return self.connection_batch([("ConnectionPodToPod", (src_pod, dst_pod, proto, sport, dport))])[0]

    def connection_pod_to_internet(self, src_pod, dst_ip, proto, sport, dport):
        return self.connection_batch([("ConnectionPodToInternet", (src_pod, dst_ip, proto, sport, dport))])[0]

    def connection_internet_to_pod(self, src_ip, dst_pod, proto, sport, dport):
        return self.connection_batch([("ConnectionInternetToPod", (src_ip, dst_pod, proto, sport, dport))])[0]
