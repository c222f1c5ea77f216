"""ACLConfig on the GPU engine (aclengine_mock.go:671-728) with the rebind
fast path: a PutACL whose rules equal the installed ACL's keeps the compiled
table (cls_acl_stats: no compilation) and only moves the interface bindings,
with the reference's change counting and last-writer-wins bindings; a put
with different rules compiles a new table.  The whole renderer chain sends
such puts when a local table's pod set changes (acl_renderer.go:186-190).
"""
import numpy as np
import pytest

from aclgen import random_acl

pytestmark = pytest.mark.gpu


def test_reput_equal_rules_rebinds_without_compiling():
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        rules, _ = random_acl(3, 40)
        other, _ = random_acl(4, 40)
        c0, r0 = eng.acl_stats()
        assert eng.acl_put("a", rules, ["if1"], ["if2"]) == 0
        tid = eng.acl_table("a")
        assert eng.acl_stats() == (c0 + 1, r0)
        # same rules, new interfaces: same table, bindings moved
        assert eng.acl_put("a", rules, ["if3"], []) == 0
        assert eng.acl_table("a") == tid
        assert eng.acl_stats() == (c0 + 1, r0 + 1)
        i1, i2, i3 = (eng.if_id(x) for x in ("if1", "if2", "if3"))
        assert eng.if_acls(i1) == (-1, -1) and eng.if_acls(i2) == (-1, -1)
        assert eng.if_acls(i3) == (tid, -1)
        assert eng.acl_counts() == (1, 2)                 # PutACL counts one change per put
        # different rules: compiled
        assert eng.acl_put("a", other, ["if3"], []) == 0
        assert eng.acl_stats() == (c0 + 2, r0 + 1)
        assert eng.acl_table("a") != tid
        assert eng.acl_counts() == (1, 3)
    finally:
        eng.close()


def test_rebound_table_restarts_connection_counters_keeps_verdicts():
    """Every put installs a new ACL (PutACL replaces the message,
    aclengine_mock.go:707-713): a rebind keeps the compiled table but its
    connection counters restart from zero, as after a compiling put."""
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        rules, pool = random_acl(5, 30, weird=0.0)
        assert eng.acl_put("a", rules, ["in0"], []) == 0
        n = 2000
        rng = np.random.default_rng(5)
        src = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        dst = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        proto = rng.integers(0, 3, n).astype(np.uint8)
        sport = rng.integers(1024, 65536, n).astype(np.uint16)
        dport = rng.integers(0, 65536, n).astype(np.uint16)
        i0, i9 = eng.if_id("in0"), eng.if_id("none")
        v1 = eng.connect_batch(np.full(n, i0), np.full(n, i9), src, dst, proto, sport, dport, count=True)
        c1 = eng.conn_counters("a")
        assert c1.sum() == n
        assert eng.acl_put("a", rules, ["in1"], []) == 0        # rebind
        i1 = eng.if_id("in1")
        v2 = eng.connect_batch(np.full(n, i1), np.full(n, i9), src, dst, proto, sport, dport, count=True)
        assert np.array_equal(v1, v2)
        assert np.array_equal(eng.conn_counters("a"), c1)      # only the batch after the put
        assert eng.acl_put("a", rules, ["in1"], []) == 0        # rebind with no batch after it
        assert not eng.conn_counters("a").any()
    finally:
        eng.close()
