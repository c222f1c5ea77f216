"""The rule compiler, checked on CPU against the oracle.

cls_compile_v4 (the same compiler cls_table_put runs) emits the device
layouts; tests/cls_image.py interprets them exactly as the kernels do.
Verdicts and per-rule counters must be bit-exact against the faithful oracle
(evalACL restated, aclengine_mock.go:473-668) on adversarial random ACLs.
"""
import numpy as np
import pytest

import oracle
from aclgen import random_acl, random_traffic
from cls_image import Image, compile_blob
from vpp_amd import _abi


@pytest.fixture(autouse=True)
def _source_keyed(libopt):
    """These tests pin list modes of the source-keyed layout; the compiler's
    choice of orientation (compile.cpp build_cls4) is tested on its own."""
    libopt.set("orient", "src")


def _check(rules, traffic):
    img = Image(compile_blob(_abi.CRules(rules)))
    v, c = img.classify(traffic["src"], traffic["dst"], traffic["dport"], traffic["proto"])
    ov, oc = oracle.classify_faithful(oracle.rules_to_c(rules), traffic["src"], traffic["dst"],
                                      traffic["dport"], traffic["proto"])
    bad = np.nonzero(v != ov)[0]
    assert len(bad) == 0, "verdict mismatch at %s: got %s want %s" % (bad[:5], v[bad[:5]], ov[bad[:5]])
    np.testing.assert_array_equal(c, oc)
    return img


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("n_rules,weird", [(6, 0.0), (40, 0.0), (40, 0.2), (150, 0.05)])
def test_compiler_matches_oracle(seed, n_rules, weird):
    rules, pool = random_acl(seed * 1000 + n_rules, n_rules, weird)
    tr = random_traffic(seed, 3000, pool)
    _check(rules, tr)


@pytest.mark.parametrize("lens", [(32,), (32, 24), (32, 24, 16), (32, 0), (8, 16, 24, 32)])
@pytest.mark.parametrize("seed", range(4))
def test_hash_lpm_and_search_modes(seed, lens):
    """Few distinct source prefix lengths -> cuckoo-hash LPM (mode 1); more ->
    interval search (mode 0).  Both must be exact, incl. /0 and nesting."""
    import random
    from aclgen import PrefixPool, random_rule
    rng = random.Random(seed)
    pool = PrefixPool(rng, 40)
    base = [rng.getrandbits(32) for _ in range(6)]
    pool.v4 = []
    for i in range(60):
        ln = lens[i % len(lens)]
        m = (0xFFFFFFFF << (32 - ln)) & 0xFFFFFFFF if ln else 0
        pool.v4.append(((rng.choice(base) ^ (rng.getrandbits(12) << 4)) & m, ln))
    rules = [random_rule(rng, pool, 0.0) for _ in range(120)]
    img = _check(rules, random_traffic(seed, 4000, pool))
    assert img.has_cls
    assert img.h.mode in ((1, 6) if len([x for x in lens if x]) <= 3 else (0, 4))


@pytest.mark.parametrize("seed", range(4))
def test_long_candidate_lists_use_scan_mode(seed):
    """> 32 candidates in a cell: the template-scan list mode (list_mode 0)."""
    from aclgen import long_list_acl
    rules, pool = long_list_acl(seed + 500)
    img = _check(rules, random_traffic(seed, 4000, pool))
    assert img.has_cls and img.h.list_mode == 0


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("host_src", [True, False])
def test_many_port_ranges_use_per_list_port_search(seed, host_src):
    """> 256 global port classes: bit vectors with per-list port search
    (list_mode 1); few port ranges: global port classes (list_mode 2)."""
    from aclgen import many_ports_acl
    rules, pool = many_ports_acl(seed + 900, 400, 40, host_src=host_src)
    img = _check(rules, random_traffic(seed, 6000, pool))
    assert img.has_cls and img.h.list_mode == 1
    assert img.h.mode == (1 if host_src else 0)
    rules, pool = random_acl(seed + 77, 150, 0.0)
    img = _check(rules, random_traffic(seed, 6000, pool))
    assert img.has_cls and img.h.list_mode in (2, 3) and img.h.n_pclass <= 256


@pytest.mark.parametrize("max_mode", [2, 3])
def test_port_class_radix_edges(libopt, max_mode):
    """Port classes at chunk edges (255/256, 65535) and ranges inside one
    256-port chunk: every port of every boundary checked against the oracle."""
    from vpp_amd import model as M
    edges = [(0, 0), (255, 256), (256, 511), (300, 300), (301, 302), (1023, 1024),
             (65534, 65535), (65535, 65535), (80, 80), (8080, 8081)]
    rules = [M.l4_rule(M.PERMIT if i % 2 else M.REFLECT, "10.0.%d.0/24" % i, "", "tcp", 0, 65535,
                       lo, hi) for i, (lo, hi) in enumerate(edges)]
    rules += [M.l4_rule(M.DENY, "10.0.0.0/16", "", "udp", 0, 65535, lo, hi) for lo, hi in edges]
    ports = sorted({x for lo, hi in edges for x in (lo - 1, lo, hi, hi + 1) if 0 <= x <= 65535})
    n = len(ports) * 40
    rng = np.random.default_rng(5)
    tr = dict(src=(np.uint32(0x0A000000) + rng.integers(0, 12 << 8, n)).astype(np.uint32),
              dst=rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
              dport=np.tile(np.array(ports, np.uint16), 40),
              proto=rng.choice(np.array([0, 1, 2], np.uint8), n))
    libopt.set("list_mode_max", str(max_mode))
    img = _check(rules, tr)
    assert img.h.list_mode <= max_mode


def test_compiler_uses_classifier_for_larger_tables():
    rules, pool = random_acl(7, 120, 0.0)
    img = _check(rules, random_traffic(7, 2000, pool))
    assert img.has_cls


def test_empty_acl_denies_everything():
    img = _check([], random_traffic(1, 100, random_acl(1, 1)[1]))
    assert not img.has_cls


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("max_mode", [1, 2])
def test_capped_list_modes_match_oracle(libopt, seed, max_mode):
    """The lower bit-vector list modes (what tables with > 16-entry lists or
    too many port classes get) stay exact when selected explicitly."""
    libopt.set("list_mode_max", str(max_mode))
    rules, pool = random_acl(seed * 7 + 3, 150, 0.0, n_prefixes=4 if seed % 2 else 24)
    img = _check(rules, random_traffic(seed, 5000, pool))
    assert img.h.list_mode <= max_mode


@pytest.mark.parametrize("seed", range(6))
def test_compact_lists_edge_addresses(seed):
    """List mode 3 at the address-space edges (0.0.0.0, 255.255.255.255 hit the
    padding of shallow lists) and /32 sources outside the probe filter."""
    rules, pool = random_acl(seed * 11 + 5, 60, 0.0, n_prefixes=6)
    tr = random_traffic(seed, 4000, pool)
    n = len(tr["dst"])
    tr["dst"][: n // 4] = np.uint32(0xFFFFFFFF)
    tr["dst"][n // 4: n // 2] = np.uint32(0)
    tr["src"][::7] = np.uint32(0xFFFFFFFF)
    img = _check(rules, tr)
    assert img.h.list_mode in (2, 3)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("max_mode", [3, 4])
def test_single_port_tables_hash_port_classes(libopt, seed, max_mode):
    """Rendered-shape tables (single dst ports): merged port classes, the
    perfect-hash port lookup (list mode 4) and, capped, the radix (mode 3)."""
    from aclgen import single_port_acl
    libopt.set("list_mode_max", str(max_mode))
    rules, pool = single_port_acl(seed + 31, 70, n_prefixes=6 if seed % 2 else 20)
    tr = random_traffic(seed, 5000, pool)
    img = _check(rules, tr)
    assert img.h.list_mode == max_mode
    assert img.h.n_pclass <= 10


def test_image_without_kernel_is_refused():
    """cls_image_kernel (the check cls_table_put runs before any launch, and
    the launchers again): combinations no classify kernel implements are
    CLS_E_INVAL -- the removed inline-cell source mode 6, the source trie or
    wide cells outside LDS, front-end rows (mode 3) on the IPv4 path, list
    modes past 6 -- and the implemented ones are CLS_OK."""
    L = _abi.lib()
    INVAL = -1
    for mode, lm, lds, rep16 in [(6, 3, 1, 0), (6, 4, 1, 1), (4, 3, 0, 0), (4, 2, 1, 0), (1, 5, 0, 0),
                                 (0, 6, 0, 1), (3, 4, 1, 0), (0, 7, 1, 0), (2, 0, 1, 0)]:
        assert L.cls_image_kernel(mode, lm, lds, rep16) == INVAL, (mode, lm, lds, rep16)
    for mode, lm, lds, rep16 in [(0, 0, 0, 0), (1, 4, 1, 0), (1, 2, 0, 0), (4, 3, 1, 0), (4, 6, 1, 1),
                                 (3, 5, 1, 1), (3, 0, 0, 1), (0, 5, 1, 0)]:
        assert L.cls_image_kernel(mode, lm, lds, rep16) == 0, (mode, lm, lds, rep16)


@pytest.mark.parametrize("seed", range(4))
def test_compiled_images_have_kernels(seed):
    """Every image the compiler emits for random ACLs has a kernel at its
    own residency (lds_bytes within the workgroup's LDS)."""
    from aclgen import many_ports_acl, single_port_acl
    for rules, _ in [random_acl(seed, 200, 0.1), single_port_acl(seed, 90), many_ports_acl(seed, 300, 30)]:
        h = Image(compile_blob(_abi.CRules(rules))).h
        if not h.has_cls:
            continue
        lds = h.lds_bytes + 16 <= 160 * 1024
        assert _abi.lib().cls_image_kernel(h.mode, h.list_mode, int(lds), 0) == 0, (h.mode, h.list_mode)
