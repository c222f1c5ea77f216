"""Orientation of the classifier (compile.cpp build_cls4 / build_cls16): the
classes may be keyed on the packet's destination instead of its source.
evalACL tests both networks the same way (aclengine_mock.go:499-524; a dst
parse error is a FAIL term once the src matched, which the semantic rules
state as dst ANY + FAIL), so the rules with src and dst exchanged, run on
packets with src and dst exchanged, give the same first match and the same
terminating rule.  Checked on CPU against the faithful oracle, through the
interpreter of the compiled layouts (tests/cls_image.py).
"""
import random

import numpy as np
import pytest

import oracle
from aclgen import random_acl, random_acl16, random_traffic, random_traffic16
from cls_image import Image, Image16, compile_blob
from vpp_amd import _abi


def _img(rules, fn="cls_compile_v4"):
    blob = compile_blob(_abi.CRules(rules), fn)
    return Image16(blob) if fn == "cls_compile_v16" else Image(blob)


def _same(got, want):
    v, c = got
    ov, oc = want
    bad = np.nonzero(v != ov)[0]
    assert len(bad) == 0, "verdict mismatch at %s" % bad[:5]
    np.testing.assert_array_equal(c, oc)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("n_rules,weird", [(60, 0.0), (200, 0.01), (400, 0.0)])
def test_destination_keyed_v4(seed, n_rules, weird, libopt):
    libopt.set("orient", "dst")
    rules, pool = random_acl(seed * 31 + n_rules, n_rules, weird)
    img = _img(rules)
    if not img.has_cls:
        pytest.skip("an early unconditional terminator: no classifier")
    assert img.h.swap == 1
    tr = random_traffic(seed, 6001, pool)
    _same(img.classify(tr["src"], tr["dst"], tr["dport"], tr["proto"]),
          oracle.classify_faithful(oracle.rules_to_c(rules), tr["src"], tr["dst"], tr["dport"], tr["proto"]))


@pytest.mark.parametrize("seed", range(4))
def test_destination_keyed_v16(seed, libopt):
    libopt.set("orient", "dst")
    rules, pool = random_acl16(seed + 40, 150, 0.02)
    img = _img(rules, "cls_compile_v16")
    assert img.h.core.swap == 1
    tr = random_traffic16(seed, 3001, pool)
    _same(img.classify(tr["src"], tr["dst"], tr["dport"], tr["proto"]),
          oracle.classify_faithful(oracle.rules_to_c(rules), tr["src"], tr["dst"], tr["dport"], tr["proto"], af=16))


def _gen_policy_list(blocks, match):
    from vpp_amd import configurator as C
    from vpp_amd.renderer.api import PodID
    from vpp_amd.renderer.traffic import compile_rules
    pol = C.gen_policy(random.Random(blocks), num_cidrs=blocks)
    txn = C.PolicyConfigurator({PodID("db", "default"): "10.1.1.1"}).new_txn(False)
    return compile_rules(txn.generate_rules(match, [pol]))


@pytest.mark.parametrize("fn", ["cls_compile_v4", "cls_compile_v16"])
def test_gen_policy_lists_pick_their_orientation(fn):
    """gen-policy.py's pod lists: the list keyed on sources (IP blocks as
    peers' sources) stays source-keyed; the list keyed on destinations gets a
    destination-keyed, LDS-resident sublist classifier instead of one
    ~10k-entry template scan."""
    from configurator_replay import gen_policy_packets
    from vpp_amd import configurator as C
    for match, want_swap in ((C.MATCH_INGRESS, 0), (C.MATCH_EGRESS, 1)):
        acl = _gen_policy_list(20, match)
        img = _img(acl, fn)
        h = img.h.core if fn == "cls_compile_v16" else img.h
        assert h.swap == want_swap and h.list_mode >= 3, (match, h.swap, h.list_mode)
        assert h.lds_bytes <= 160 * 1024
        src, dst, proto, dport, s16, d16 = gen_policy_packets(random.Random(3), 3000, 20)
        p8, dp16 = np.array(proto, np.uint8), np.array(dport, np.uint16)
        cr = oracle.rules_to_c(acl)
        if fn == "cls_compile_v16":
            _same(img.classify(s16, d16, dp16, p8), oracle.classify_faithful(cr, s16, d16, dp16, p8, af=16))
        else:
            s4 = np.array([int.from_bytes(x, "big") for x in src], np.uint32)
            d4 = np.array([int.from_bytes(x, "big") for x in dst], np.uint32)
            _same(img.classify(s4, d4, dp16, p8), oracle.classify_faithful(cr, s4, d4, dp16, p8))


def test_rendered_global_table_stays_source_keyed():
    from vpp_amd import workload
    acl, _, _ = workload.config(2)
    assert _img(acl.rules).h.swap == 0
