"""GPU parity: the gfx950 kernels, through the C ABI, against the CPU oracle.

Bit-exact bar (integer work): verdicts (ACLAction, aclengine_mock.go:63-77)
and per-rule hit counters must equal the oracle's on identical inputs.
"""
import numpy as np
import pytest

import oracle
from aclgen import random_acl, random_traffic
from scenario_replay import load_scenarios, replay

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _source_keyed(libopt, eng):
    """These tests pin list modes of the source-keyed layout; the compiler's
    choice of orientation (compile.cpp build_cls4) is tested on its own."""
    libopt.set("orient", "src", eng)


SCENARIOS = load_scenarios()


@pytest.fixture(scope="module")
def eng():
    from vpp_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


def _oracle(rules, tr, fast=False):
    cr = oracle.rules_to_c(rules)
    if fast:
        return oracle.classify_fast(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    return oracle.classify_faithful(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"])


def _gpu(eng, rules, tr, **kw):
    t = eng.put_table("t", rules)
    try:
        return eng.classify(t, tr["src"], tr["dst"], tr["dport"], tr["proto"], **kw)
    finally:
        eng.del_table(t)


def _assert_same(got, want):
    v, c = got
    ov, oc = want
    bad = np.nonzero(v != ov)[0]
    assert len(bad) == 0, "verdict mismatch at %s: got %s want %s" % (bad[:8], v[bad[:8]], ov[bad[:8]])
    np.testing.assert_array_equal(c, oc)


@pytest.mark.parametrize("test", SCENARIOS, ids=[t["name"] for t in SCENARIOS])
def test_reference_scenarios_on_gpu(eng, test):
    """The 221 Connection* KATs of acl_renderer_test.go, verdicts from the GPU
    connection kernel (one launch per phase)."""
    from vpp_amd.engine import ACLEngine, Engine

    # a fresh engine per scenario, as NewMockACLEngine is called per test
    checked, failures = replay(test, lambda contiv: ACLEngine(contiv, Engine()),
                               check_conn=lambda engine, calls: engine.connection_batch(calls))
    assert not failures, "\n".join(failures)
    assert checked > 0


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("n_rules,weird", [(5, 0.0), (60, 0.0), (60, 0.25), (400, 0.05)])
def test_random_acls_both_kernels(eng, seed, n_rules, weird):
    rules, pool = random_acl(seed * 7919 + n_rules, n_rules, weird)
    tr = random_traffic(seed, 20011, pool)           # odd length: vector body + scalar tail
    want = _oracle(rules, tr)
    _assert_same(_gpu(eng, rules, tr), want)
    _assert_same(_gpu(eng, rules, tr, force_linear=True), want)


VARIANTS = {  # kind -> (source lookup mode, list mode)
    "hash_sph": (1, 4), "search_sph": (0, 4),       # hash_*: several hashed prefix lengths
    "hash_cbv": (1, 3), "search_cbv": (0, 3),
    "host_sph": (1, 4), "host_cbv": (1, 3),         # /32 sources only: one hashed length (src kernel mode 2)
    "hrow_sph": (1, 4), "hrow_cbv": (1, 3),
    "hash_pc": (1, 2), "search_pc": (0, 2), "hash_bv": (1, 1), "search_bv": (0, 1),
    "hash_scan": (1, 0), "search_scan": (0, 0),
    "trie_sph": (4, 4), "trie_cbv": (4, 3)}


def _host_sources(rules, pool, seed):
    """Every source prefix of the rules (and the traffic pool) as a /32 host
    inside it: one hashed prefix length (the rendered global table's shape,
    the one-length hash kernels)."""
    import random
    from aclgen import _v4
    rng = random.Random(seed)
    host = {}
    for a, ln in pool.v4:
        host[(a, ln)] = (a | (rng.getrandbits(32) & ((1 << (32 - ln)) - 1) if ln < 32 else a), 32)
    pool.v4 = [host[x] for x in pool.v4]
    by_cidr = {"%s/%d" % (_v4(a), ln): "%s/32" % _v4(h[0]) for (a, ln), h in host.items()}
    for r in rules:
        ip = r.matches.ip_rule.ip if r.matches and r.matches.ip_rule else None
        if ip is not None and ip.source_network:
            ip.source_network = by_cidr.get(ip.source_network, ip.source_network.split("/")[0] + "/32")
    return rules, pool


def variant_acl(kind, seed):
    from aclgen import long_list_acl, many_ports_acl, single_port_acl
    if kind.startswith("host"):
        rules, pool = variant_acl("hrow" + kind[4:], seed)
        return _host_sources(rules, pool, seed)
    hashed = kind.startswith(("hash", "hrow"))       # trie_*: the search_* tables over the source trie
    if kind.endswith("_sph"):
        return single_port_acl(seed * 13 + 1, 90, n_prefixes=3 if hashed else 24)
    if kind.endswith("scan"):
        return long_list_acl(seed + 70, 300, n_src=3 if hashed else 30)
    if kind.endswith("_bv"):
        return many_ports_acl(seed + 5, 400, 40, host_src=hashed)
    return random_acl(seed * 31 + 7, 60 if kind.endswith("cbv") else 120, 0.0,
                      n_prefixes=4 if hashed else 24)


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("kind", sorted(VARIANTS))
def test_all_kernel_variants(eng, seed, kind, libopt):
    """The classifier variants (hash-LPM / interval-search source lookup x
    port-filtered sublists with hashed / radix port classes / bit vectors
    with global port classes / bit vectors with per-list port search /
    template scan; the source trie x both sublist forms) against the oracle."""
    if kind.endswith("_pc"):
        libopt.set("list_mode_max", "2", eng)
    # the interval search and the source trie each on the same tables
    libopt.set("trie", "1" if kind.startswith("trie") else "0", eng)
    libopt.set("src_search", "1" if kind.startswith(("search", "trie")) else "0", eng)
    from cls_image import Image, compile_blob
    from vpp_amd import _abi
    rules, pool = variant_acl(kind, seed)
    h = Image(compile_blob(_abi.CRules(rules))).h
    assert (h.mode, h.list_mode) == VARIANTS[kind], kind
    tr = random_traffic(seed + 11, 30000, pool)
    _assert_same(_gpu(eng, rules, tr), _oracle(rules, tr))


def test_misaligned_batch_uses_scalar_path(eng):
    rules, pool = random_acl(99, 200, 0.05)
    tr = random_traffic(5, 9001, pool)
    sl = {k: v[1:] for k, v in tr.items()}            # 4-byte offset: not 16-B aligned
    _assert_same(_gpu(eng, rules, sl), _oracle(rules, sl))


def test_empty_batch_and_empty_acl(eng):
    rules, pool = random_acl(3, 50)
    tr = random_traffic(1, 0, pool)
    v, c = _gpu(eng, rules, tr)
    assert len(v) == 0 and c.sum() == 0
    tr = random_traffic(2, 1000, pool)
    v, c = _gpu(eng, [], tr)
    assert (v == 0).all() and c[0] == 1000            # default DENY, counter R = 0


def test_device_generator_matches_cpu_stream(eng):
    import torch
    from vpp_amd import workload
    acl, spec, _ = workload.config(2)
    n = 1 << 20
    out = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
           (("src", torch.int32), ("dst", torch.int32), ("sport", torch.int16),
            ("dport", torch.int16), ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, 12345, out)
    torch.cuda.synchronize()
    ref = oracle.gen_traffic_v4(spec, 12345, n)
    for k in out:
        got = out[k].cpu().numpy().view(ref[k].dtype)
        np.testing.assert_array_equal(got, ref[k], err_msg=k)


@pytest.mark.parametrize("cfg,n", [(2, 1 << 20), (3, 1 << 20)])
def test_config_tables_device_path(eng, cfg, n):
    """Configs 2/3: device-generated traffic, device pointers, vs the oracle."""
    import torch
    from vpp_amd import workload
    acl, spec, _ = workload.config(cfg)
    t = eng.put_table("cfg%d" % cfg, acl.rules)
    info = t.info()
    assert info["kernel"] == 1 and info["lds_resident"] == 1
    out = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
           (("src", torch.int32), ("dst", torch.int32), ("sport", torch.int16),
            ("dport", torch.int16), ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, 0, out)
    verdict = torch.empty(n, dtype=torch.uint8, device="cuda")
    counters = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
    eng.classify(t, out["src"], out["dst"], out["dport"], out["proto"], verdict=verdict,
                 counters=counters)
    torch.cuda.synchronize()
    tr = oracle.gen_traffic_v4(spec, 0, n)
    ov, oc = _oracle(acl.rules, tr, fast=True)
    np.testing.assert_array_equal(verdict.cpu().numpy(), ov)
    np.testing.assert_array_equal(counters.cpu().numpy().astype(np.uint64), oc)
    # accumulate: a second identical pass doubles the counters
    eng.classify(t, out["src"], out["dst"], out["dport"], out["proto"], counters=counters,
                 accumulate=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(counters.cpu().numpy().astype(np.uint64), 2 * oc)
    eng.del_table(t)


def test_config3_full_size_properties(eng):
    """At the benchmark size (256 Mi packets): every packet counted exactly
    once, and the classifier agrees with the independent ballot kernel on a
    2 Mi-packet slice (size-independent GPU cross-check; the ballot kernel
    walks ~5k rules per wave at 10k rules, so the slice is kept small)."""
    import torch
    from vpp_amd import workload
    acl, spec, n = workload.config(3)
    t = eng.put_table("cfg3", acl.rules)
    out = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
           (("src", torch.int32), ("dst", torch.int32), ("dport", torch.int16),
            ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, 0, out)
    counters = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
    verdict = torch.empty(n, dtype=torch.uint8, device="cuda")
    eng.classify(t, out["src"], out["dst"], out["dport"], out["proto"], verdict=verdict,
                 counters=counters)
    torch.cuda.synchronize()
    assert int(counters.sum()) == n
    m = 2 << 20
    sl = {k: v[:m] for k, v in out.items()}
    v2 = torch.empty(m, dtype=torch.uint8, device="cuda")
    c2 = torch.zeros_like(counters)
    eng.classify(t, sl["src"], sl["dst"], sl["dport"], sl["proto"], verdict=v2, counters=c2,
                 force_linear=True)
    c1 = torch.zeros_like(counters)
    eng.classify(t, sl["src"], sl["dst"], sl["dport"], sl["proto"], counters=c1)
    torch.cuda.synchronize()
    assert torch.equal(v2, verdict[:m])
    assert torch.equal(c1, c2)
    # 64 windows of 4 Ki packets strided across the whole 256 Mi stream: the
    # full-batch verdicts, and each window classified on its own (counters),
    # equal the oracle's on the same stream positions
    cr = oracle.rules_to_c(acl.rules)
    w, stride = 4096, n // 64
    wc = torch.zeros_like(counters)
    for k in range(64):
        a = k * stride + (k * 7919 % (stride - w)) // 16 * 16
        tr = oracle.gen_traffic_v4(spec, a, w)
        ov, oc = oracle.classify_fast(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"])
        assert np.array_equal(verdict[a:a + w].cpu().numpy(), ov), "window %d at %d" % (k, a)
        eng.classify(t, out["src"][a:a + w], out["dst"][a:a + w], out["dport"][a:a + w],
                     out["proto"][a:a + w], counters=wc)
        torch.cuda.synchronize()
        assert np.array_equal(wc.cpu().numpy().astype(np.uint64), oc), "window %d counters" % k
    del out, verdict
    eng.del_table(t)


def test_batch_beyond_one_launch(eng):
    """A batch of 2^30 + 4099 packets (12.9 GB in HBM) takes two classify
    launches (32-bit packet offsets inside the kernel): the first launch's
    partials are folded without the remap, the last one's with it.  The
    whole batch in one call must equal the two pieces classified by separate
    calls (verdicts and counters), every packet counted once, and the pieces
    around the launch boundary equal the oracle."""
    import torch
    from vpp_amd import workload
    acl, spec, _ = workload.config(3)
    t = eng.put_table("chunks", acl.rules)
    n = (1 << 30) + 4099
    out = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
           (("src", torch.int32), ("dst", torch.int32), ("dport", torch.int16),
            ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, 0, out)
    verdict = torch.empty(n, dtype=torch.uint8, device="cuda")
    counters = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
    eng.classify(t, out["src"], out["dst"], out["dport"], out["proto"], verdict=verdict, counters=counters)
    torch.cuda.synchronize()
    assert int(counters.sum()) == n
    cut = 1 << 30
    parts = torch.zeros_like(counters)
    for a, b in ((0, cut), (cut, n)):
        v = torch.empty(b - a, dtype=torch.uint8, device="cuda")
        c = torch.zeros_like(counters)
        eng.classify(t, out["src"][a:b], out["dst"][a:b], out["dport"][a:b], out["proto"][a:b],
                     verdict=v, counters=c)
        torch.cuda.synchronize()
        assert torch.equal(v, verdict[a:b])
        parts += c
        del v
    assert torch.equal(parts, counters)
    cr = oracle.rules_to_c(acl.rules)
    for a in (0, cut - 4096, n - 4096):
        sl = {k: v[a:a + 4096].cpu().numpy() for k, v in out.items()}
        ov, _ = oracle.classify_fast(cr, sl["src"].view(np.uint32), sl["dst"].view(np.uint32),
                                     sl["dport"].view(np.uint16), sl["proto"])
        assert np.array_equal(verdict[a:a + 4096].cpu().numpy(), ov)
    del out, verdict
    torch.cuda.empty_cache()
    eng.del_table(t)


def test_kernel_timing(eng):
    import torch
    from vpp_amd import workload
    acl, spec, _ = workload.config(2)
    t = eng.put_table("cfg2", acl.rules)
    n = 1 << 22
    out = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
           (("src", torch.int32), ("dst", torch.int32), ("dport", torch.int16),
            ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, 0, out)
    eng.classify(t, out["src"], out["dst"], out["dport"], out["proto"], timing=True)
    ms = eng.last_kernel_ms()
    assert 0.0 < ms < 1000.0
    eng.del_table(t)
