"""GPU parity of the per-packet matched-rule trace (cls_classify_rules):
each packet's ACLAction and the index of the rule at which evalACL
terminated (R: the default DENY, aclengine_mock.go:667) -- the rule the
reference logs per call at Debug (:651-654) -- against the oracle's literal
first-match loop (orc_classify_fast_hits, pinned to orc_eval_acl's hit in
tests/test_oracle_pin_cpu.py).  Bar: bit-exact, and the rules' histogram
equals cls_classify's counters on the same batch.
"""
import numpy as np
import pytest

import oracle
from aclgen import random_acl, random_acl16, random_traffic, random_traffic16

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from vpp_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


def _check(eng, rules, tr, af=4, **opts):
    cr = oracle.rules_to_c(rules)
    ov, oh = oracle.classify_hits(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"], af=af)
    t = eng.put_table("r", rules)
    try:
        v, r = eng.classify_rules(t, tr["src"], tr["dst"], tr["dport"], tr["proto"])
        bad = np.nonzero((v != ov) | (r != oh))[0]
        assert len(bad) == 0, "mismatch at %s: got %s / %s want %s / %s" % (
            bad[:6], v[bad[:6]], r[bad[:6]], ov[bad[:6]], oh[bad[:6]])
        _, c = eng.classify(t, tr["src"], tr["dst"], tr["dport"], tr["proto"])
        np.testing.assert_array_equal(np.bincount(r, minlength=len(rules) + 1).astype(np.uint64), c)
        return t.info()
    finally:
        eng.del_table(t)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("n_rules,weird", [(5, 0.0), (7, 0.3), (80, 0.0), (400, 0.2)])
def test_rules_random_v4(eng, seed, n_rules, weird):
    """Small ACLs (no classifier image: the linear kernel) and imaged ones
    (slot mode, the OTHER image for protocols > 2), malformed rules
    included; an odd batch length."""
    rules, pool = random_acl(seed * 131 + n_rules, n_rules, weird)
    tr = random_traffic(seed + 7, 8191, pool, other_proto=True)
    _check(eng, rules, tr)


@pytest.mark.parametrize("orient", ["src", "dst"])
def test_rules_destination_keyed(eng, libopt, orient):
    """Both orientations of the image (a destination-keyed one swaps the
    packet's addresses into its frame)."""
    libopt.set("orient", orient, eng)
    rules, pool = random_acl(99, 300, 0.0)
    tr = random_traffic(5, 20011, pool, other_proto=True)
    info = _check(eng, rules, tr)
    assert info["kernel"] == 1 and info["swap"] == (1 if orient == "dst" else 0), info


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("n_rules", [6, 90, 350])
def test_rules_random_v16(eng, seed, n_rules):
    """The 16-byte layout (IPv6, IPv4-mapped, malformed rules)."""
    rules, pool = random_acl16(seed * 17 + n_rules, n_rules, 0.1)
    tr = random_traffic16(seed + 3, 6007, pool)
    _check(eng, rules, tr, af=16)


@pytest.mark.parametrize("cfg", [2, 3])
def test_rules_config_tables_on_device(eng, cfg):
    """The benchmark tables on 1 Mi + 3 device-generated packets (torch
    tensors, stream-ordered): rules against the oracle, and their histogram
    against cls_classify's device counters."""
    import torch
    from vpp_amd import workload
    acl, spec, _ = workload.config(cfg)
    n = (1 << 20) + 3
    out = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
           (("src", torch.int32), ("dst", torch.int32), ("sport", torch.int16), ("dport", torch.int16),
            ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, 1234, out)
    t = eng.put_table("cfg", acl.rules)
    try:
        v = torch.zeros(n, dtype=torch.uint8, device="cuda")
        vr, r = eng.classify_rules(t, out["src"], out["dst"], out["dport"], out["proto"], verdict=v)
        c = torch.zeros(len(acl.rules) + 1, dtype=torch.int64, device="cuda")
        eng.classify(t, out["src"], out["dst"], out["dport"], out["proto"], counters=c)
        torch.cuda.synchronize()
        tr = oracle.gen_traffic_v4(spec, 1234, n)
        ov, oh = oracle.classify_hits(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
        rr = r.cpu().numpy().view(np.uint32)
        assert np.array_equal(v.cpu().numpy(), ov)
        assert np.array_equal(rr, oh)
        np.testing.assert_array_equal(np.bincount(rr, minlength=len(acl.rules) + 1), c.cpu().numpy())
    finally:
        eng.del_table(t)


def test_rules_empty_batch_and_errors(eng):
    from vpp_amd import _abi
    rules, pool = random_acl(3, 40, 0.0)
    t = eng.put_table("e", rules)
    try:
        z = np.zeros(0, np.uint32)
        v, r = eng.classify_rules(t, z, z, np.zeros(0, np.uint16), np.zeros(0, np.uint8))
        assert len(v) == 0 and len(r) == 0
        tr = random_traffic(1, 10, pool)
        pk = _abi.PktSoa(_abi.AF_V4, tr["src"].ctypes.data, tr["dst"].ctypes.data, None, None, None,
                         tr["dport"].ctypes.data, tr["proto"].ctypes.data)
        import ctypes as C
        assert _abi.lib().cls_classify_rules(eng.h, t.id, C.byref(pk), 10, None, None, 0, None) == _abi.E_INVAL
        assert _abi.lib().cls_classify_rules(eng.h, 987654, C.byref(pk), 10, None, None, 0, None) != 0
    finally:
        eng.del_table(t)
