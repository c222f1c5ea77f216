"""GPU: counter tiers, per-stream counter scratch, the stream floor.

Counter tiers (vpp_amd/csrc/compile.hpp Cls4Image): the classifier image
stays in LDS whenever it fits; its per-slot hit counters are u32 LDS words,
else u16 LDS halves (a 0x8000 carry moved to the global slot counter), else
only the first n_lctr slots in LDS and the rest counted in global memory.
The lds_budget option shrinks the budget so small random ACLs exercise every
tier, and the global-image variant; verdicts and per-rule counters must equal
the evalACL oracle's (mock/aclengine/aclengine_mock.go:473-668) bit for bit.

Threading (include/contivcls.h): two device classifies of one table on two
streams have their own counter scratch; both counter vectors equal the
oracle's.
"""
import numpy as np
import pytest

import oracle
from aclgen import random_acl, random_traffic, single_port_acl

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from vpp_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


def _layout(rules, libopt):
    from cls_image import Image, compile_blob
    from vpp_amd import _abi
    libopt.set("orient", "src")
    return Image(compile_blob(_abi.CRules(rules))).h


def _budget(h, tier):
    """LDS budget that puts the image of header h in counter tier `tier`."""
    hot = h.n_hot * 256
    a16 = lambda x: (x + 15) & ~15
    if tier == "u32":
        return 160 * 1024
    if tier == "u16":
        return h.img_bytes + a16(2 * h.n_ctr) + hot
    if tier == "partial":
        return h.img_bytes + hot + a16(2 * max(h.n_hot, h.n_ctr // 3))
    return 256                                   # "global": no image of this table fits


def _check(eng, rules, tr, libopt, tier):
    h = _layout(rules, libopt)
    assert h.has_cls
    libopt.set("lds_budget", str(_budget(h, tier)), eng)
    libopt.set("list_mode", str(h.list_mode), eng)   # the layout the budget was sized on
    # and its source lookup: under a smaller budget the compiler would take
    # the smaller interval table instead of the trie, and its counters would
    # fit another tier
    libopt.set("trie", "1" if h.mode == 4 else "0", eng)
    libopt.set("orient", "src", eng)
    t = eng.put_table("tier", rules)
    try:
        info = t.info()
        if tier == "global":
            assert info["lds_resident"] == 0
        else:
            assert info["lds_resident"] == 1
            assert info["ctr16"] == (0 if tier == "u32" else 1)
            if tier == "partial":
                assert info["n_lctr"] < info["n_slots"]
            else:
                assert info["n_lctr"] == info["n_slots"]
        v, c = eng.classify(t, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    finally:
        eng.del_table(t)
    ov, oc = oracle.classify_fast(oracle.rules_to_c(rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    bad = np.nonzero(v != ov)[0]
    assert len(bad) == 0, "verdict mismatch at %s" % bad[:8]
    np.testing.assert_array_equal(c, oc)
    return info


@pytest.mark.parametrize("tier", ["u32", "u16", "partial", "global"])
@pytest.mark.parametrize("seed,weird", [(0, 0.05), (1, 0.0), (2, 0.02), (3, 0.0), (0, 0.0)])
def test_counter_tiers_random_acls(eng, libopt, seed, weird, tier):
    """List modes 4 (seeds 0, 2), 3 (seeds 1, 3) and 0 (seed 0 without weird rules)."""
    rules, pool = random_acl(seed * 101 + 17, 400, weird)
    tr = random_traffic(seed + 3, 40003, pool)      # ICMP and protocols > 2 included
    _check(eng, rules, tr, libopt, tier)


@pytest.mark.parametrize("tier", ["u16", "partial", "global"])
def test_counter_tiers_sublist_mode(eng, libopt, tier):
    """The rendered-table shape (list mode 4, hashed source classes)."""
    rules, pool = single_port_acl(7, 300, n_prefixes=3)
    tr = random_traffic(9, 65536 + 77, pool)
    info = _check(eng, rules, tr, libopt, tier)
    assert info["list_mode"] == 4 or tier == "global"


def test_u16_counter_carry(eng, libopt):
    """More than 0x8000 hits on one slot inside one workgroup: the u16
    counters carry to the global slot counters exactly."""
    rules, pool = single_port_acl(11, 120, n_prefixes=3)
    rng = np.random.default_rng(5)
    n = 1 << 25                                      # > 0x8000 packets per workgroup, all alike
    a = np.uint32(pool.v4[0][0])
    tr = dict(src=np.full(n, a, np.uint32), dst=np.full(n, a, np.uint32),
              dport=np.full(n, 80, np.uint16), proto=np.zeros(n, np.uint8))
    tr["proto"][rng.integers(0, n, 1000)] = 1
    _check(eng, rules, tr, libopt, "u16")
    _check(eng, rules, tr, libopt, "partial")


def test_two_streams_one_table(eng):
    """Device classifies of one table on two streams overlap; each call has
    its own counter scratch, so both results equal the oracle's."""
    import torch
    from vpp_amd import workload
    acl, spec, _ = workload.config(2)
    t = eng.put_table("streams", acl.rules)
    n = 1 << 21
    outs = []
    for first in (0, n):
        d = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
             (("src", torch.int32), ("dst", torch.int32), ("dport", torch.int16), ("proto", torch.uint8))}
        eng.gen_traffic_v4(spec, first, d)
        outs.append(d)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    res = []                                          # every buffer kept alive until checked
    for _ in range(3):                                # repeated: overlapping launches on both streams
        for k, (d, s) in enumerate(zip(outs, streams)):
            v = torch.empty(n, dtype=torch.uint8, device="cuda")
            c = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
            eng.classify(t, d["src"], d["dst"], d["dport"], d["proto"], verdict=v, counters=c, stream=s)
            res.append((k, v, c))
    torch.cuda.synchronize()
    cr = oracle.rules_to_c(acl.rules)
    want = []
    for first in (0, n):
        tr = oracle.gen_traffic_v4(spec, first, n)
        want.append(oracle.classify_fast(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"]))
    for k, v, c in res:
        ov, oc = want[k]
        np.testing.assert_array_equal(v.cpu().numpy(), ov)
        np.testing.assert_array_equal(c.cpu().numpy().astype(np.uint64), oc)
    # deleting the table while device work is queued waits for that work
    d = outs[0]
    c = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
    eng.classify(t, d["src"], d["dst"], d["dport"], d["proto"], counters=c, stream=streams[0])
    eng.del_table(t)
    torch.cuda.synchronize()
    assert int(c.sum()) == n


def test_stream_floor(eng):
    import torch
    n = 1 << 22
    d = {k: torch.zeros(n, dtype=dt, device="cuda") for k, dt in
         (("src", torch.int32), ("dst", torch.int32), ("dport", torch.int16), ("proto", torch.uint8))}
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    ms = eng.stream_floor(d["src"], d["dst"], d["dport"], d["proto"], v, reps=3)
    assert 0.0 < ms < 100.0
    d16 = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
    ms16 = eng.stream_floor(d16, d16, d["dport"], d["proto"], v, reps=3)
    assert 0.0 < ms16 < 100.0


@pytest.mark.parametrize("cap", [None, "0", "1000"])
@pytest.mark.parametrize("v16", [False, True])
@pytest.mark.parametrize("share", [0.3, 0.02])
def test_other_protocols_queue(eng, libopt, cap, v16, share):
    """Protocols outside ProtocolType (30 % or 2 % here): queued for the
    OTHER image and classified after the launch, or in place once the queue
    is full (option other_cap); every path equals the oracle."""
    from aclgen import random_acl16, random_traffic16
    if cap is not None:
        libopt.set("other_cap", cap, eng)
    if v16:
        rules, pool = random_acl16(23, 300, 0.0)
        tr = random_traffic16(4, 70001, pool)
    else:
        rules, pool = random_acl(23, 300, 0.0)
        tr = random_traffic(4, 70001, pool)
    rng = np.random.default_rng(9)
    tr["proto"][rng.random(len(tr["proto"])) < share] = 47
    t = eng.put_table("other", rules)
    try:
        v, c = eng.classify(t, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    finally:
        eng.del_table(t)
    ov, oc = oracle.classify_fast(oracle.rules_to_c(rules), tr["src"], tr["dst"], tr["dport"], tr["proto"],
                                  af=16 if v16 else 4)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(c, oc)


def test_other_protocols_many_rules(eng):
    """Protocol-47 packets whose terminating rules are more distinct rules
    than the finish launch's LDS rule histogram holds (6000 > 4096): counted
    with wave-aggregated atomics per rule instead; verdicts and counters
    equal the oracle's."""
    from vpp_amd import model as M
    rng = np.random.default_rng(11)
    hosts = rng.choice(1 << 24, 6000, replace=False) + (10 << 24)
    rules = [M.l4_rule(M.PERMIT if i % 3 else M.DENY, "%d.%d.%d.%d/32" % (h >> 24, (h >> 16) & 255, (h >> 8) & 255,
                                                                          h & 255), "", "tcp", 0, 65535, 80, 80)
             for i, h in enumerate(hosts.tolist())]
    n = 50000
    src = rng.choice(hosts, n).astype(np.uint32)
    miss = rng.random(n) < 0.2                   # some sources match no rule: default DENY
    src[miss] = rng.integers(0, 1 << 32, int(miss.sum()), dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    dport = rng.choice(np.array([80, 443], np.uint16), n)
    proto = rng.choice(np.array([0, 47, 47, 47], np.uint8), n)
    t = eng.put_table("other_many", rules)
    try:
        v, c = eng.classify(t, src, dst, dport, proto)
    finally:
        eng.del_table(t)
    ov, oc = oracle.classify_fast(oracle.rules_to_c(rules), src, dst, dport, proto)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(c, oc)
    assert (oc[:6000] > 0).sum() > 4096
