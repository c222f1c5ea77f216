"""The connection pair launch's four-cell image (CPU).

classify4_pair (vpp_amd/csrc/k4_pair.hip) classifies both tuples of every
connection on an image with a fourth cell per source class for protocols > 2
(compile.hpp Cls4Opts::with_other; cls_compile_v4 option pair4), instead of
the main image plus the OTHER image.  Here that compile is checked without a
GPU: every index the image hands the kernels is in range
(test_image_ranges_cpu's walk), and the image decoded as the kernels read it
(tests/cls_image.py: min(protocol, 3) picks the cell) gives evalACL's verdict
and terminating rule for TCP, UDP, ICMP and other protocol values -- which
match on networks alone (aclengine_mock.go:527-643 has no case for them) --
against the oracle's first-match loop (orc_classify_fast, pinned to the
literal evalACL in test_oracle_pin_cpu.py).  Bit-exact verdicts and per-rule
counts.
"""
import numpy as np
import pytest

import oracle
from aclgen import long_list_acl, many_ports_acl, random_acl, random_traffic, single_port_acl
from cls_image import Image, compile_blob
from test_image_ranges_cpu import check_image
from vpp_amd import _abi


def _pair_image(rules, **opts):
    return Image(compile_blob(_abi.CRules(rules), options=dict(opts, pair4=1)))


def _check(rules, tr, **opts):
    im = _pair_image(rules, **opts)
    if not im.has_cls:                          # no classifier for this ACL at all (the main compile agrees)
        assert not Image(compile_blob(_abi.CRules(rules), options=opts)).has_cls
        return im
    assert im.other is None and im.ncell == 4, im.ncell
    check_image(im, len(rules))
    v, c = im.classify(tr["src"], tr["dst"], tr["dport"], tr["proto"])
    ov, oc = oracle.classify_fast(oracle.rules_to_c(rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    bad = np.nonzero(v != ov)[0]
    assert bad.size == 0, (bad[:8], v[bad[:8]], ov[bad[:8]], tr["proto"][bad[:8]])
    np.testing.assert_array_equal(c, oc)
    return im


def _with_other_protocols(tr, seed, frac=0.2):
    rng = np.random.default_rng(seed)
    other = rng.random(len(tr["proto"])) < frac
    tr["proto"] = np.where(other, rng.choice(np.array([3, 6, 17, 47, 255], np.uint8), len(other)),
                           tr["proto"]).astype(np.uint8)
    return tr


@pytest.mark.parametrize("cfg", [2, 3])
def test_pair_image_config_tables(cfg):
    """The benchmark tables (the config-3 one is the connection bench's global
    ACL): traffic of the configs' generator with a fifth of the packets on
    other protocols."""
    from vpp_amd import workload
    acl, spec, _ = workload.config(cfg)
    tr = _with_other_protocols(oracle.gen_traffic_v4(spec, 5, 60000), cfg)
    im = _check(acl.rules, tr)
    assert im.h.list_mode >= 3                  # the sublist modes of the main image


@pytest.mark.parametrize("seed", range(4))
def test_pair_image_random_acls_every_list_mode(seed):
    """Random ACLs with malformed rules under every list-mode cap and with and
    without the source trie."""
    gens = [random_acl(seed, 300, 0.1), single_port_acl(seed + 3, 200), many_ports_acl(seed, 300, 30),
            long_list_acl(seed + 1, 250)]
    for k, (rules, pool) in enumerate(gens):
        tr = _with_other_protocols(random_traffic(seed * 7 + k, 6000, pool, other_proto=True), seed + k)
        for cap in (0, 1, 2, 3, 4, 6):
            for trie in (0, 1):
                _check(rules, tr, list_mode_max=cap, trie=trie)


def test_pair_image_follows_the_main_orientation():
    """A destination-keyed main image gives a destination-keyed pair image
    (the pair launch frames the tuples once for both)."""
    rules, pool = random_acl(99, 300, 0.0)
    tr = _with_other_protocols(random_traffic(5, 8000, pool, other_proto=True), 5)
    for orient, swap in (("dst", 1), ("src", 0)):
        im = _check(rules, tr, orient=orient)
        assert im.has_cls and im.h.swap == swap
