"""The 16-byte layout's compiler (cls_compile_v16: representatives + the IPv4
classifier over them), checked on CPU against the oracle.

tests/cls_image.py Image16 evaluates the blob exactly as classify16_cls does
(front-end binary search over 128-bit interval starts, then the core image).
Verdicts and counters must be bit-exact against the faithful evalACL
restatement (oracle, af=16: Go 1.9 To4 / networkNumberAndMask semantics,
aclengine_mock.go:499-524).  IPv6 and IPv4-mapped matching is not covered by
the reference's own tests: parity here is against the
oracle's restatement of the Go 1.9 net package, "parity unpinned" by
reference fixtures.
"""
import numpy as np
import pytest

import oracle
from aclgen import (mix_families, random_acl, random_acl16, random_traffic, random_traffic16)
from cls_image import Image, Image16, compile_blob
from vpp_amd import _abi


@pytest.fixture(autouse=True)
def _source_keyed(libopt):
    """These tests pin list modes of the source-keyed layout; the compiler's
    choice of orientation (compile.cpp build_cls4) is tested on its own."""
    libopt.set("orient", "src")


def _img16(rules):
    return Image16(compile_blob(_abi.CRules(rules), "cls_compile_v16"))


def _check16(rules, tr):
    img = _img16(rules)
    v, c = img.classify(tr["src"], tr["dst"], tr["dport"], tr["proto"])
    ov, oc = oracle.classify_faithful(oracle.rules_to_c(rules), tr["src"], tr["dst"], tr["dport"],
                                      tr["proto"], af=16)
    bad = np.nonzero(v != ov)[0]
    assert len(bad) == 0, "verdict mismatch at %s: got %s want %s" % (bad[:5], v[bad[:5]], ov[bad[:5]])
    np.testing.assert_array_equal(c, oc)
    return img


@pytest.mark.parametrize("seed", range(10))
@pytest.mark.parametrize("n_rules,weird", [(5, 0.0), (40, 0.0), (40, 0.2), (150, 0.05)])
def test_v16_compiler_matches_oracle(seed, n_rules, weird):
    rules, pool = random_acl16(seed * 1000 + n_rules, n_rules, weird)
    _check16(rules, random_traffic16(seed, 1500, pool))


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("cap", [0, 1, 2, 3, 4])
def test_v16_list_modes(seed, cap, libopt):
    """Every list mode of the core, over mixed-family twins of IPv4 tables."""
    from aclgen import long_list_acl, many_ports_acl, single_port_acl
    libopt.set("list_mode_max", str(cap))
    gen = [single_port_acl(seed + 3, 120), random_acl(seed + 9, 120, 0.0), many_ports_acl(seed, 300, 30),
           long_list_acl(seed + 1, 200)][seed % 4]
    rules, pool = gen
    rules, tr = mix_families(rules, random_traffic(seed, 2500, pool), seed)
    img = _check16(rules, tr)
    assert img.core.h.list_mode <= cap


@pytest.mark.parametrize("seed", range(4))
def test_v4_mapped_batch_equals_ipv4_batch(seed):
    """An IPv4 batch spelled as IPv4-mapped 16-byte addresses (Go's To4)
    classifies exactly as the 4-byte batch does."""
    rules, pool = random_acl(seed + 40, 120, 0.1)
    tr = random_traffic(seed, 3000, pool)
    _, tr16 = mix_families(rules, tr, seed, frac=0.0)
    v4, c4 = Image(compile_blob(_abi.CRules(rules))).classify(tr["src"], tr["dst"], tr["dport"], tr["proto"])
    v16, c16 = _img16(rules).classify(tr16["src"], tr16["dst"], tr16["dport"], tr16["proto"])
    np.testing.assert_array_equal(v4, v16)
    np.testing.assert_array_equal(c4, c16)


def test_v16_empty_and_any_tables():
    import vpp_amd.model as M
    pool_rules, pool = random_acl16(5, 10)
    tr = random_traffic16(2, 500, pool)
    _check16([], tr)
    _check16([M.l4_rule(M.PERMIT, "", "", "tcp", 0, 65535, 0, 65535)], tr)
    _check16([M.l4_rule(M.DENY, "::/0", "", "udp", 0, 65535, 53, 53),
              M.l4_rule(M.REFLECT, "0.0.0.0/0", "::ffff:0:0/96", "tcp", 0, 65535, 0, 65535)], tr)


def test_v16_representatives_preserve_containment():
    """Nested IPv6 prefixes, IPv4 prefixes and the v4-mapped block's edges:
    the interval table's reps must separate exactly what Contains separates."""
    import vpp_amd.model as M
    nets = ["fd00:10::/32", "fd00:10:1::/48", "fd00:10:1:2::/64", "fd00:10:1:2::7/128", "::ffff:0:0/95",
            "::/80", "10.0.0.0/8", "10.1.0.0/16", "::ffff:10.1.2.0/120", "::/0", "0.0.0.0/0"]
    rules = []
    for k, a in enumerate(nets):
        for b in nets[::-1]:
            rules.append(M.l4_rule([M.DENY, M.PERMIT, M.REFLECT][k % 3], a, b, "tcp", 0, 65535, 0, 65535))
    from aclgen import PrefixPool16, to16
    import random
    pool = PrefixPool16(random.Random(1), 8)
    rng = np.random.default_rng(3)
    tr = random_traffic16(4, 2000, pool)
    edge = to16(pool.addr16(rng, 500) + [0xFD000010 << 96, (0xFD000010 << 96) - 1, (0xFD000011 << 96) - 1,
                                         0xFFFF << 32, (0xFFFF << 32) - 1, 0x0A010203 | (0xFFFF << 32)])
    n = len(edge)
    tr = dict(src=edge, dst=edge[::-1].copy(), dport=np.full(n, 80, np.uint16), proto=np.zeros(n, np.uint8))
    _check16(rules, tr)


def test_oracle_fast_matches_faithful_v16():
    rules, pool = random_acl16(77, 200, 0.1)
    tr = random_traffic16(8, 3000, pool)
    cr = oracle.rules_to_c(rules)
    fv, fc = oracle.classify_fast(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"], af=16)
    ov, oc = oracle.classify_faithful(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"], af=16)
    np.testing.assert_array_equal(fv, ov)
    np.testing.assert_array_equal(fc, oc)


def _host_src_acl(seed, n_rules=200):
    """Rules whose sources are all host routes (/32 and, as twins, /128): the
    rendered global table's shape -> the source hashes (src_mode 1)."""
    import random
    import vpp_amd.model as M
    from aclgen import PrefixPool, _v4
    rng = random.Random(seed)
    pool = PrefixPool(rng, 24)
    hosts = [rng.getrandbits(32) for _ in range(40)] + [a for a, _ in pool.v4[:8]]
    rules = []
    for _ in range(n_rules):
        src = "%s/32" % _v4(rng.choice(hosts)) if rng.random() < 0.85 else ""
        da, dl = rng.choice(pool.v4)
        dst = "%s/%d" % (_v4(da), dl) if rng.random() < 0.7 else ""
        p = rng.choice([22, 53, 80, 443, 0])
        rules.append(M.l4_rule(rng.choice([M.DENY, M.PERMIT, M.REFLECT]), src, dst,
                               rng.choice(["tcp", "udp"]), 0, 65535, p, p if p else 65535))
    pool.v4 = [(h, 32) for h in hosts] + pool.v4
    return rules, pool


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("forced_search", [False, True])
def test_v16_source_host_hashes(seed, forced_search, libopt):
    if forced_search:
        libopt.set("v16_src_search", "1")
    rules, pool = _host_src_acl(seed)
    rules, tr = mix_families(rules, random_traffic(seed, 4000, pool), seed)
    img = _check16(rules, tr)
    assert img.h.src_mode == (0 if forced_search else 1)


def test_config5_table_cpu():
    """The config 5 render (vpp_amd/workload.py) on a prefix of its 16-byte
    stream, against the oracle's fast port."""
    from vpp_amd import workload
    acl, spec, _ = workload.config(5)
    tr = oracle.gen_traffic_v16(spec, 0, 20000)
    img = _img16(acl.rules)
    assert img.h.src_mode == 1
    v, c = img.classify(tr["src"], tr["dst"], tr["dport"], tr["proto"])
    ov, oc = oracle.classify_fast(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"],
                                  tr["proto"], af=16)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(c, oc)


# ---- src_mode 2: the IPv4 source trie of the 16-byte layout ----------------

@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("kind", ["v4", "mixed", "v16"])
def test_v16_source_trie_matches_oracle(seed, kind, libopt):
    """src_mode 2 (forced): IPv4-mapped sources through the trie over their
    IPv4 word, the others through the non-IPv4 search (rows), protocols > 2
    through the global table's reps -- against the faithful oracle on IPv4
    tables widened to 16 bytes, their mixed-family twins and random
    mixed-family ACLs with malformed rules."""
    libopt.set("v16_src_trie", "1")
    if kind == "v16":
        rules, pool = random_acl16(seed * 101 + 7, 150, 0.1, n_prefixes=60)
        tr = random_traffic16(seed + 40, 3000, pool)
    else:
        rules, pool = random_acl(seed * 101 + 5, 150, 0.1, n_prefixes=80)
        rules, tr = mix_families(rules, random_traffic(seed + 40, 3000, pool), seed, 0.0 if kind == "v4" else 0.5)
    img = _check16(rules, tr)
    if img.core.has_cls:                       # (all-host-route sources keep the hashes, src_mode 1)
        assert img.h.src_mode in (1, 2)


def test_v16_source_trie_edges(libopt):
    """Addresses at the trie's chunk and /8 boundaries and at the edges of the
    IPv4-mapped block (::ffff:0.0.0.0, ::ffff:255.255.255.255 and their IPv6
    neighbours), prefixes ending at those edges, host routes among blocks."""
    import vpp_amd.model as M
    libopt.set("v16_src_trie", "1")
    nets = ["10.0.0.0/8", "10.1.0.0/16", "10.1.255.0/24", "10.2.0.0/15", "10.1.2.3/32", "0.0.0.0/1",
            "128.0.0.0/1", "255.255.255.255/32", "0.0.0.0/32", "10.255.255.0/24", "11.0.0.0/16",
            "fd00::/16", "::ffff:0:0/97", "::fffe:0:0/96"]
    rules = []
    for k, a in enumerate(nets * 3):
        d = "" if k % 3 else "192.168.%d.0/24" % k
        rules.append(M.l4_rule([M.DENY, M.PERMIT, M.REFLECT][k % 3], a, d, ["tcp", "udp"][k % 2],
                               0, 65535, 0, 65535 if k % 4 else 80))
    edges = [0x0A000000, 0x0A00FFFF, 0x0A010000, 0x0A01FFFF, 0x0A01FF00, 0x0A0100FF, 0x0A010203, 0x0A010204,
             0x0AFFFFFF, 0x0B000000, 0x09FFFFFF, 0, 1, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFE, 0xFFFFFFFF,
             0x0A020000, 0x0A03FFFF, 0x0A040000, 0x0B00FFFF, 0x0B010000]
    addrs = [(0xFFFF << 32) | a for a in edges] + [(0xFFFF << 32) - 1, (0xFFFF << 32) + (1 << 32),
                                                  0xFD00 << 112, (0xFFFE << 32) | 5, 0x0A010203]
    src = np.array([list(a.to_bytes(16, "big")) for a in addrs], np.uint8)
    n = len(src)
    dst = np.array([list(((0xFFFF << 32) | 0xC0A80000 | (i * 7)).to_bytes(16, "big")) for i in range(n)], np.uint8)
    for proto in (0, 1, 2, 47):
        tr = dict(src=src, dst=dst, dport=np.full(n, 80, np.uint16), proto=np.full(n, proto, np.uint8))
        img = _check16(rules, tr)
        assert img.h.src_mode == 2


@pytest.mark.parametrize("blocks", [20, 200])
def test_gen_policy_lists_v16_source_trie(blocks):
    """The gen-policy.py lists (tests/policy/perf/gen-policy.py:8-65) in the
    16-byte layout take the source trie by themselves and stay LDS-resident
    (sublist list mode, like their IPv4 images); 4000 packets -- IPv4-mapped
    inside and around the blocks, IPv6, protocol 47 -- against the fast
    oracle, both orientations."""
    import random
    from vpp_amd import configurator as C
    from vpp_amd.renderer.api import PodID
    from vpp_amd.renderer.traffic import compile_rules
    pol = C.gen_policy(random.Random(blocks), num_cidrs=blocks)
    txn = C.PolicyConfigurator({PodID("db", "default"): "10.1.1.1"}).new_txn(False)
    g = np.random.default_rng(blocks)
    n = 4000
    for match in (C.MATCH_INGRESS, C.MATCH_EGRESS):
        acl = compile_rules(txn.generate_rules(match, [pol]))
        import libopts
        keyed = libopts.CURRENT.pop("orient")      # the compiler's own orientation here
        img = Image16(compile_blob(_abi.CRules(acl), "cls_compile_v16"))
        libopts.CURRENT["orient"] = keyed
        assert img.h.src_mode == 2 and img.core.h.list_mode in (3, 4, 5, 6)
        assert img.core.h.lds_bytes <= 160 * 1024
        blk = g.integers(0, blocks + blocks // 10 + 1, n).astype(np.uint64)
        inblk = (((blk + 0x100) << 16) | g.integers(0, 1 << 16, n).astype(np.uint64)).astype(np.uint64)
        other = g.integers(0, 1 << 32, n).astype(np.uint64)
        a, b = (inblk, other) if match == C.MATCH_INGRESS else (other, inblk)

        def wide(x, v6):
            hi = np.where(v6, np.uint64(0xFD000000 << 32), np.uint64(0))
            lo = np.where(v6, x, np.uint64(0xFFFF << 32) | x)
            out = np.empty((n, 16), np.uint8)
            out[:, :8] = hi.astype(">u8").view(np.uint8).reshape(n, 8)
            out[:, 8:] = lo.astype(">u8").view(np.uint8).reshape(n, 8)
            return out
        v6 = g.random(n) < 0.1
        src, dst = wide(a, v6), wide(b, g.random(n) < 0.1)
        ports = np.array([p.number for p in pol.matches[0].ports], np.uint16)
        dport = np.where(g.random(n) < 0.5, g.choice(ports, n), g.integers(0, 65536, n)).astype(np.uint16)
        proto = g.choice(np.array([0, 1, 2, 47], np.uint8), n, p=[0.445, 0.445, 0.1, 0.01])
        v, c = img.classify(src, dst, dport, proto)
        ov, oc = oracle.classify_fast(oracle.rules_to_c(acl), src, dst, dport, proto, af=16)
        np.testing.assert_array_equal(v, ov)
        np.testing.assert_array_equal(c, oc)
