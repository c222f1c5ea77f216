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


def test_compiler_uses_classifier_for_larger_tables():
    rules, pool = random_acl(7, 120, 0.0)
    img = _check(rules, random_traffic(7, 2000, pool))
    assert img.has_cls


def test_empty_acl_denies_everything():
    img = _check([], random_traffic(1, 100, random_acl(1, 1)[1]))
    assert not img.has_cls
