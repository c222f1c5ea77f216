"""CPU: the bitmap form of connection-path ACLs (engine.cpp conn_bitmap4).

cls_connect_batch evaluates linear IPv4 ACLs through per-ACL interval tables
(source, destination, each protocol's destination port) with one rule bit
row per interval; the first match is the lowest bit set in all three rows.
cls_conn_bitmap_eval builds those tables from the rules and evaluates
packets on the host exactly as the connection kernel reads them.  Verdicts
and per-rule hit counts must equal the evalACL oracle's
(mock/aclengine/aclengine_mock.go:473-668) bit for bit; the GPU side is
tests/test_gpu_connect_scale.py::test_connections_bitmap_form_match_oracle.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from aclgen import long_list_acl, many_ports_acl, random_acl, random_traffic, single_port_acl
from vpp_amd import _abi


def _bitmap_eval(rules, tr):
    cr = _abi.CRules(rules)
    n = len(tr["src"])
    src = np.ascontiguousarray(tr["src"], np.uint32)
    dst = np.ascontiguousarray(tr["dst"], np.uint32)
    dport = np.ascontiguousarray(tr["dport"], np.uint16)
    proto = np.ascontiguousarray(tr["proto"], np.uint8)
    res = np.zeros(n, np.uint8)
    rule = np.zeros(n, np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    rc = _abi.lib().cls_conn_bitmap_eval(cr.ptr(), cr.n, p(src), p(dst), p(dport), p(proto), n, p(res), p(rule))
    assert rc == 0, rc
    return res, np.bincount(rule, minlength=len(rules) + 1).astype(np.uint64)


def _check(rules, tr):
    v, c = _bitmap_eval(rules, tr)
    ov, oc = oracle.classify_fast(oracle.rules_to_c(rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    bad = np.nonzero(v != ov)[0]
    assert len(bad) == 0, "verdict mismatch at %s" % bad[:8]
    np.testing.assert_array_equal(c, oc)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("weird", [0.0, 0.003, 0.15])
@pytest.mark.parametrize("size", [1, 12, 150, 300])
def test_random_acls(seed, weird, size):
    """The connection benchmark's local-ACL shapes (random_acl: nested and
    disjoint prefixes, every protocol section, port ranges, unconditional
    failures), every protocol in the traffic (protocols > 2 included)."""
    rules, pool = random_acl(1000 + 31 * seed + size, size, weird)
    _check(rules, random_traffic(seed, 6000, pool))


@pytest.mark.parametrize("seed", range(3))
def test_long_and_port_heavy_acls(seed):
    """Lists with no early catch-all (hundreds of live rules: rows of many
    words) and many distinct port ranges (many port intervals)."""
    rules, pool = long_list_acl(seed, 300)
    _check(rules, random_traffic(seed + 10, 8000, pool))
    rules, pool = many_ports_acl(seed, 400, host_src=bool(seed % 2))
    _check(rules, random_traffic(seed + 20, 8000, pool))


def test_edges():
    """Addresses and ports at the interval edges: 0, 255.255.255.255, port
    0 and 65535, /0 and /32 prefixes."""
    rules, pool = single_port_acl(5, 200, n_prefixes=4)
    tr = random_traffic(3, 4000, pool)
    n = len(tr["src"])
    tr["src"][: n // 8] = 0
    tr["dst"][n // 8: n // 4] = 0xFFFFFFFF
    tr["dport"][n // 4: n // 3] = 65535
    tr["dport"][n // 3: n // 2] = 0
    _check(rules, tr)
