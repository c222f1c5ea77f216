"""The source trie (src mode 4) and the wide global cells (list modes 5, 6),
checked on CPU against the oracle through the compiled blob
(tests/cls_image.py interprets it as the kernels do).

The trie replaces the interval search of tables with many source prefixes
(gen-policy.py's IP blocks minus excepts); wide cells carry 32-bit counter
bases, so lists with more than 2^18 counter slots (gen-policy.py at its
1000-block default) keep the LDS sublist form instead of the template scan.
Verdicts and per-rule counters must equal the faithful evalACL oracle
(aclengine_mock.go:473-668) bit for bit.
"""
import random

import numpy as np
import pytest

import oracle
from aclgen import random_acl, random_traffic, single_port_acl
from cls_image import Image, compile_blob
from vpp_amd import _abi


def _check(rules, traffic, fast=False):
    img = Image(compile_blob(_abi.CRules(rules)))
    v, c = img.classify(traffic["src"], traffic["dst"], traffic["dport"], traffic["proto"])
    f = oracle.classify_fast if fast else oracle.classify_faithful
    ov, oc = f(oracle.rules_to_c(rules), traffic["src"], traffic["dst"], traffic["dport"], traffic["proto"])
    bad = np.nonzero(v != ov)[0]
    assert len(bad) == 0, "verdict mismatch at %s: got %s want %s" % (bad[:5], v[bad[:5]], ov[bad[:5]])
    np.testing.assert_array_equal(c, oc)
    return img


def _chunk_edges(pool, n, seed):
    """Sources on /16 and /8 chunk boundaries and prefix edges (the trie's
    leaf and node boundaries)."""
    rng = np.random.default_rng(seed)
    base = np.array([a for a, _ in pool.v4], np.uint64)
    size = np.array([1 << (32 - ln) for _, ln in pool.v4], np.uint64)
    i = rng.integers(0, len(base), n)
    cand = np.stack([base[i], base[i] - 1, base[i] + size[i], base[i] + size[i] - 1,
                     base[i] & 0xFFFF0000, (base[i] & 0xFFFF0000) - 1, base[i] | 0xFFFF,
                     (base[i] | 0xFFFF) + 1, base[i] & 0xFF000000, base[i] | 0xFFFFFF]) & 0xFFFFFFFF
    return cand[rng.integers(0, cand.shape[0], n), np.arange(n)].astype(np.uint32)


@pytest.mark.parametrize("seed", range(10))
@pytest.mark.parametrize("n_prefixes", [24, 120])
def test_trie_matches_oracle(libopt, seed, n_prefixes):
    libopt.set("orient", "src")
    libopt.set("trie", "1")
    rules, pool = single_port_acl(seed * 7 + 3, 160, n_prefixes=n_prefixes)
    tr = random_traffic(seed, 4000, pool)
    tr["src"][::3] = _chunk_edges(pool, len(tr["src"][::3]), seed)
    tr["src"][:4] = np.array([0, 0xFFFFFFFF, 0xFFFF, 0xFFFF0000], np.uint32)
    img = _check(rules, tr)
    if img.h.list_mode >= 3 and img.h.mode != 1:
        assert img.h.mode == 4


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("trie", ["0", "1"])
def test_wide_cells_match_oracle(libopt, seed, trie):
    """Wide cells forced (option wide=1), with the trie or the interval
    search behind them."""
    libopt.set("orient", "src")
    libopt.set("wide", "1")
    libopt.set("trie", trie)
    rules, pool = single_port_acl(seed * 13 + 1, 140, n_prefixes=40)
    tr = random_traffic(seed + 100, 4000, pool)
    img = _check(rules, tr)
    assert img.h.list_mode in (5, 6)
    assert img.h.mode == (4 if trie == "1" else 0)
    assert img.h.n_gcells == 2 * 3 * img.h.n_classes


@pytest.mark.parametrize("seed", range(4))
def test_wide_cells_hash_sources(libopt, seed):
    """Wide cells behind the hash LPM (rendered global tables: pod /32s)."""
    from vpp_amd import workload
    libopt.set("orient", "src")
    libopt.set("wide", "1")
    acl, spec, _ = workload.config(2)
    tr = oracle.gen_traffic_v4(spec, seed * 5000, 5000)
    img = _check(acl.rules, tr, fast=True)
    assert img.h.list_mode in (5, 6) and img.h.mode == 1


@pytest.mark.parametrize("seed", range(6))
def test_trie_with_random_weird_rules(libopt, seed):
    """Adversarial rules (parse failures, nil sections, reversed ranges) over a
    trie image when the compiler picks one."""
    libopt.set("trie", "1")
    rules, pool = random_acl(seed * 31 + 9, 120, 0.1, n_prefixes=60)
    tr = random_traffic(seed, 3000, pool)
    tr["src"][::4] = _chunk_edges(pool, len(tr["src"][::4]), seed)
    _check(rules, tr)


def _gen_policy_list(blocks, match):
    from vpp_amd import configurator as C
    from vpp_amd.renderer.api import PodID
    from vpp_amd.renderer.traffic import compile_rules
    pol = C.gen_policy(random.Random(blocks), num_cidrs=blocks)
    txn = C.PolicyConfigurator({PodID("db", "default"): "10.1.1.1"}).new_txn(False)
    return compile_rules(txn.generate_rules(C.MATCH_INGRESS if match == "ingress" else C.MATCH_EGRESS, [pol]))


def _gen_policy_traffic(blocks, n, seed, match):
    g = np.random.default_rng(seed)
    blk = g.integers(0, blocks + blocks // 10 + 1, n, dtype=np.uint64)
    inblk = (((blk + 0x100) << 16) | g.integers(0, 1 << 16, n, dtype=np.uint64)).astype(np.uint32)
    other = g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    src, dst = (inblk, other) if match == "ingress" else (other, inblk)
    dport = np.where(g.random(n) < 0.5, g.choice(np.array([22, 53, 80, 443], np.uint16), n),
                     g.integers(0, 65536, n)).astype(np.uint16)
    proto = g.choice(np.array([0, 1, 2, 47], np.uint8), n, p=(0.445, 0.445, 0.1, 0.01))
    return dict(src=src, dst=dst, dport=dport, proto=proto)


@pytest.mark.parametrize("match", ["ingress", "egress"])
def test_gen_policy_200_blocks_trie(match):
    """200 blocks (~95k rules): LDS-resident sublists over the source trie."""
    rules = _gen_policy_list(200, match)
    img = _check(rules, _gen_policy_traffic(200, 20000, 7, match), fast=True)
    assert img.h.mode == 4 and img.h.list_mode == 4


@pytest.mark.parametrize("match", ["ingress", "egress"])
def test_gen_policy_default_1000_blocks_wide(match):
    """gen-policy.py's default (1000 blocks, ~480k rules, > 2^18 counter
    slots): LDS-resident trie + sublists with wide global cells, not the
    template scan."""
    rules = _gen_policy_list(1000, match)
    img = _check(rules, _gen_policy_traffic(1000, 6000, 11, match), fast=True)
    assert img.h.mode == 4 and img.h.list_mode == 5
    assert img.h.n_ctr > 1 << 18
