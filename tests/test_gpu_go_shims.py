"""GPU: the Go binding's C shims (include/contivcls_go.h), as a Go 1.9 host
calls them (go/contivcls/contivcls.go), driven from C (go/shimtest, gcc) --
the image has no Go toolchain.

The program installs the config-2 global table (1003 rules, bound to if0/if1
inbound, if0/if2 outbound) and 12 random local ACLs through cls_acl_put,
classifies 1 Mi packets of the config-2 stream through clsg_classify_v4, the
same packets IPv4-mapped through clsg_classify_v16, and an engine-owned batch
filled through its pinned mirror (clsg_batch_mirror); then 20k connections
through clsg_connect_v4 with CLS_F_COUNT.  Verdicts, per-rule hit counters,
ConnectionActions and per-(ACL, rule) connection counters must equal the
oracle's (evalACL, aclengine_mock.go:473-668; testConnection, :394-471).
"""
import os
import subprocess

import numpy as np
import pytest

import oracle
from aclgen import random_traffic
from vpp_amd import _abi, workload

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "go", "shimtest", "shimtest")


class _Recorder:
    """Stands in for an engine in test_gpu_connect_scale.build: records the
    ACLs instead of installing them."""

    def __init__(self):
        self.acls = []

    def acl_put(self, name, rules, ing, eg):
        self.acls.append((name, rules, list(ing), list(eg)))
        return 0


def _net(b):
    return "-" if not b else "x" + b.hex()


def _write_acls(path, acls):
    with open(path, "w") as f:
        for name, rules, ing, eg in acls:
            f.write("acl %s %d %d %s %d %s\n" % (name, len(rules), len(ing), " ".join(ing), len(eg), " ".join(eg)))
            cr = _abi.CRules(rules)
            for k in range(cr.n):
                r = cr.arr[k]
                f.write("rule %d %d %d %d %d %d %d %d %d %d %d %d %d %d %s %s\n" % (
                    r.flags, r.acl_action, r.tcp_src_lo, r.tcp_src_hi, r.tcp_dst_lo, r.tcp_dst_hi, r.udp_src_lo,
                    r.udp_src_hi, r.udp_dst_lo, r.udp_dst_hi, r.icmp_code_first, r.icmp_code_last,
                    r.icmp_type_first, r.icmp_type_last, _net(r.src_network), _net(r.dst_network)))


def test_go_shims_on_gpu(tmp_path):
    from test_gpu_connect_scale import build, oracle_connections
    if not os.path.exists(SHIM):
        subprocess.run(["make", "-s", "-C", os.path.dirname(SHIM)], check=True)
    rec = _Recorder()
    ifs, bind, by_name, pool, spec = build(rec, 5, n_local=12, n_if=24, cfg=2)
    _write_acls(tmp_path / "acls.txt", rec.acls)
    (tmp_path / "ifs.txt").write_text("\n".join(ifs) + "\n")
    n = 1 << 20
    acl, spec2, _ = workload.config(2)
    tr = oracle.gen_traffic_v4(spec2, 0, n)
    with open(tmp_path / "pkt.bin", "wb") as f:
        f.write(np.uint64(n).tobytes())
        for k, dt in (("src", np.uint32), ("dst", np.uint32), ("dport", np.uint16), ("proto", np.uint8)):
            f.write(np.ascontiguousarray(tr[k], dt).tobytes())
    m = 20000
    rng = np.random.default_rng(5)
    ctr = random_traffic(55, m, pool, other_proto=True)
    mix = rng.random(m) < 0.4
    ctr["src"][mix] = rng.choice(spec["pod_ips"].astype(np.uint32), mix.sum())
    si = rng.integers(0, len(ifs), m).astype(np.uint32)
    di = np.where(rng.random(m) < 0.1, si, rng.integers(0, len(ifs), m)).astype(np.uint32)
    with open(tmp_path / "conn.bin", "wb") as f:
        f.write(np.uint64(m).tobytes())
        for a, dt in ((si, np.uint32), (di, np.uint32), (ctr["src"], np.uint32), (ctr["dst"], np.uint32),
                      (ctr["sport"], np.uint16), (ctr["dport"], np.uint16), (ctr["proto"], np.uint8)):
            f.write(np.ascontiguousarray(a, dt).tobytes())
    r = subprocess.run([SHIM, str(tmp_path)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]

    def out(name, dt):
        return np.fromfile(tmp_path / name, dt)

    ov, oc = oracle.classify_fast(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    for v, c in (("out_verdict.bin", "out_counters.bin"), ("out_verdict16.bin", "out_counters16.bin"),
                 ("out_bverdict.bin", "out_bcounters.bin")):
        got = out(v, np.uint8)
        bad = np.nonzero(got != ov)[0]
        assert bad.size == 0, (v, bad[:8])
        np.testing.assert_array_equal(out(c, np.uint64), oc.astype(np.uint64), err_msg=c)
    assert oc.sum() == n
    hv, hits = oracle.classify_hits(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    assert np.array_equal(out("out_rverdict.bin", np.uint8), hv)
    assert np.array_equal(out("out_rules.bin", np.uint32), hits)
    want, wcounts = oracle_connections(bind, by_name, ifs, si, di, ctr, 4)
    got = out("out_conn.bin", np.uint8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])
    assert len(set(want.tolist())) >= 3
    for k, (name, _rules, _i, _e) in enumerate(rec.acls):
        np.testing.assert_array_equal(out("out_conn_ctr_%d.bin" % k, np.uint64), wcounts[name], err_msg=name)
