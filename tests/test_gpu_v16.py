"""GPU parity of the 16-byte layout (CLS_AF_V16: IPv6 and IPv4-mapped
packets) through the C ABI, against the CPU oracle (af=16).

classify16_cls maps both addresses to 32-bit representatives (front end) and
runs the IPv4 classifier over the rules restated on them (compile.hpp
Cls16Image).  Bar: verdicts and per-rule counters bit-exact.  IPv6 matching is
pinned by the oracle's restatement of Go 1.9's net package, not by reference
fixtures (parity unpinned).
"""
import numpy as np
import pytest

import oracle
from aclgen import mix_families, random_acl16, random_traffic, random_traffic16
from test_gpu_parity import VARIANTS, _assert_same, _gpu, variant_acl

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from vpp_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


def _oracle16(rules, tr, fast=False):
    cr = oracle.rules_to_c(rules)
    f = oracle.classify_fast if fast else oracle.classify_faithful
    return f(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"], af=16)


@pytest.mark.parametrize("seed", range(5))
@pytest.mark.parametrize("n_rules,weird", [(5, 0.0), (60, 0.0), (60, 0.25), (300, 0.05)])
def test_v16_random_acls_both_kernels(eng, seed, n_rules, weird):
    rules, pool = random_acl16(seed * 7919 + n_rules, n_rules, weird)
    tr = random_traffic16(seed, 6007, pool)          # odd length: vector body + scalar tail
    want = _oracle16(rules, tr)
    _assert_same(_gpu(eng, rules, tr), want)
    _assert_same(_gpu(eng, rules, tr, force_linear=True), want)


@pytest.mark.parametrize("seed", range(2))
@pytest.mark.parametrize("kind", sorted(VARIANTS))
def test_v16_all_kernel_variants(eng, seed, kind, libopt):
    """Mixed-family twins of the IPv4 variant tables: every list mode and
    source lookup of the core behind the front end (the source trie for
    trie_*)."""
    if kind.endswith("_pc"):
        libopt.set("list_mode_max", "2", eng)
    libopt.set("trie", "1" if kind.startswith("trie") else "0", eng)
    rules, pool = variant_acl(kind, seed)
    rules, tr = mix_families(rules, random_traffic(seed + 11, 20000, pool), seed)
    _assert_same(_gpu(eng, rules, tr), _oracle16(rules, tr, fast=True))


def test_v16_misaligned_ports_use_scalar_path(eng):
    rules, pool = random_acl16(99, 200, 0.05)
    tr = random_traffic16(5, 9001, pool)
    sl = {k: v[1:] for k, v in tr.items()}           # dport / proto off their 8 / 4-B alignment
    _assert_same(_gpu(eng, rules, sl), _oracle16(rules, sl))


def test_v16_device_tensors_and_large_batch(eng):
    """torch device tensors (CLS_F_DEVICE) over 4 Mi + 3 packets, counters
    against the multi-threaded oracle."""
    import torch
    from aclgen import single_port_acl
    rules, pool = single_port_acl(17, 400, n_prefixes=40)
    tr = random_traffic(3, (4 << 20) + 3, pool)
    rules, tr = mix_families(rules, tr, 3)
    want = _oracle16(rules, tr, fast=True)
    t = eng.put_table("big16", rules)
    try:
        d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in tr.items()}
        v = torch.zeros(len(tr["dport"]), dtype=torch.uint8, device="cuda")
        c = torch.zeros(len(rules) + 1, dtype=torch.int64, device="cuda")
        eng.classify(t, d["src"], d["dst"], d["dport"], d["proto"], verdict=v, counters=c)
        torch.cuda.synchronize()
        _assert_same((v.cpu().numpy(), c.cpu().numpy().astype(np.uint64)), want)
    finally:
        eng.del_table(t)


def test_device_generator16_matches_cpu_stream(eng):
    import torch
    from vpp_amd import workload
    acl, spec, _ = workload.config(5)
    n = (1 << 18) + 5
    out = {k: torch.empty(shp, dtype=dt, device="cuda") for k, shp, dt in
           (("src", (n, 16), torch.uint8), ("dst", (n, 16), torch.uint8), ("sport", (n,), torch.int16),
            ("dport", (n,), torch.int16), ("proto", (n,), torch.uint8))}
    eng.gen_traffic_v16(spec, 777, out)
    torch.cuda.synchronize()
    ref = oracle.gen_traffic_v16(spec, 777, n)
    for k in ("src", "dst", "proto"):
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref[k], err_msg=k)
    for k in ("sport", "dport"):
        np.testing.assert_array_equal(out[k].cpu().numpy().view(np.uint16), ref[k], err_msg=k)
    pr = ref["proto"]
    assert 0.08 < (pr == 2).mean() < 0.12                     # 10% ICMP
    v4 = (ref["src"][:, :10] == 0).all(1) & (ref["src"][:, 10:12] == 255).all(1)
    assert 0.4 < v4.mean() < 0.6                              # half the sources IPv4(-mapped)


def test_config5_table_on_gpu(eng):
    """The config 5 render (mixed families, dst port ranges) on a device-
    generated batch: verdicts and counters against the oracle's fast port."""
    import torch
    from vpp_amd import workload
    acl, spec, _ = workload.config(5)
    n = (1 << 20) + 1
    out = {k: torch.empty(shp, dtype=dt, device="cuda") for k, shp, dt in
           (("src", (n, 16), torch.uint8), ("dst", (n, 16), torch.uint8),
            ("dport", (n,), torch.int16), ("proto", (n,), torch.uint8))}
    eng.gen_traffic_v16(spec, 0, out)
    t = eng.put_table("cfg5", acl.rules)
    try:
        v = torch.zeros(n, dtype=torch.uint8, device="cuda")
        c = torch.zeros(len(acl.rules) + 1, dtype=torch.int64, device="cuda")
        eng.classify(t, out["src"], out["dst"], out["dport"], out["proto"], verdict=v, counters=c)
        torch.cuda.synchronize()
        tr = oracle.gen_traffic_v16(spec, 0, n)
        want = _oracle16(acl.rules, tr, fast=True)
        _assert_same((v.cpu().numpy(), c.cpu().numpy().astype(np.uint64)), want)
    finally:
        eng.del_table(t)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("kind", ["v4", "mixed", "v16"])
def test_v16_source_trie_on_gpu(eng, seed, kind, libopt):
    """src_mode 2 (forced): IPv4-mapped sources through the trie over their
    IPv4 word, the others through the non-IPv4 search, protocols > 2 through
    the global table -- classify16_cls and the linear cross-check against the
    oracle, verdicts and counters."""
    from aclgen import random_acl
    libopt.set("v16_src_trie", "1", eng)
    if kind == "v16":
        rules, pool = random_acl16(seed * 101 + 7, 150, 0.1, n_prefixes=60)
        tr = random_traffic16(seed + 40, 20000, pool)
    else:
        rules, pool = random_acl(seed * 101 + 5, 150, 0.1, n_prefixes=80)
        rules, tr = mix_families(rules, random_traffic(seed + 40, 20000, pool), seed, 0.0 if kind == "v4" else 0.5)
    want = _oracle16(rules, tr, fast=True)
    _assert_same(_gpu(eng, rules, tr), want)
    _assert_same(_gpu(eng, rules, tr, force_linear=True), want)
