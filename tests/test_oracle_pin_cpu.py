"""The fast oracle pinned to the faithful one on IPv4 (CPU).

Every config-scale GPU check compares the device with ``oracle.classify_fast``
(the precompiled-rule port, ``oracle/aclengine_ref.c`` orc_compile /
orc_classify_fast).  ``classify_faithful`` restates ``evalACL`` literally
(``mock/aclengine/aclengine_mock.go:473-668``: every CIDR string re-parsed per
rule per packet).  This pins the first to the second -- verdicts and per-rule
hit counters -- on the benchmark tables' own streams and on random ACLs with
malformed rules, so the config-scale GPU tests inherit the literal oracle's
pinning to the reference's KATs.
"""
import numpy as np
import pytest

import oracle
from aclgen import random_acl, random_traffic


def _pin(rules, tr):
    cr = oracle.rules_to_c(rules)
    fv, fc = oracle.classify_fast(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    ov, oc = oracle.classify_faithful(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    np.testing.assert_array_equal(fv, ov)
    np.testing.assert_array_equal(fc, oc)
    return ov, oc


@pytest.mark.parametrize("cfg", [2, 3])
def test_fast_matches_faithful_on_benchmark_stream(cfg):
    """4096 packets of the config-2 / config-3 stream (the bench's first
    packets and a window deep in the 256 Mi config-3 stream)."""
    from vpp_amd import workload
    acl, spec, _ = workload.config(cfg)
    for first in (0, (1 << 28) - 2048 if cfg == 3 else (1 << 24) - 2048):
        tr = oracle.gen_traffic_v4(spec, first, 2048)
        v, c = _pin(acl.rules, tr)
        assert c.sum() == 2048
        # the window exercises more than the default rule
        assert np.count_nonzero(c[:-1]) > 10


@pytest.mark.parametrize("seed", range(6))
def test_fast_matches_faithful_weird_random_v4(seed):
    """Random IPv4 ACLs with malformed networks, missing sections, reversed
    and truncated port ranges (tests/aclgen.py), protocols > 2 in the stream."""
    rules, pool = random_acl(seed * 7 + 1, [20, 120, 400][seed % 3], 0.25)
    tr = random_traffic(seed + 100, 4096, pool, other_proto=True)
    _pin(rules, tr)


@pytest.mark.parametrize("seed", [0, 3])
def test_fast_connections_match_faithful(seed):
    """orc_connect_fast (the connection line's OpenMP CPU baseline) against
    orc_test_connection_hits (testConnection restated literally,
    aclengine_mock.go:394-471) on the connection-scale layout: the config-2
    global table and 12 random local ACLs with malformed rules, 4000
    connections with same-interface pairs and protocol 47."""
    from test_gpu_connect_scale import build, oracle_connections

    class Rec:
        def __init__(self):
            self.acls = []

        def acl_put(self, name, rules, ing, eg):
            self.acls.append((name, rules, ing, eg))
            return 0

    rec = Rec()
    ifs, bind, by_name, pool, spec = build(rec, seed, n_local=12, n_if=24, cfg=2)
    names = [a[0] for a in rec.acls]
    tabs = [oracle.FastTable(oracle.rules_to_c(by_name[x])) for x in names]
    if_in = [names.index(bind[f][0]) if bind[f][0] else -1 for f in ifs]
    if_out = [names.index(bind[f][1]) if bind[f][1] else -1 for f in ifs]
    m = 4000
    rng = np.random.default_rng(seed)
    tr = random_traffic(seed + 7, m, pool, other_proto=True)
    mix = rng.random(m) < 0.4
    tr["src"][mix] = rng.choice(spec["pod_ips"].astype(np.uint32), mix.sum())
    si = rng.integers(0, len(ifs), m)
    di = np.where(rng.random(m) < 0.1, si, rng.integers(0, len(ifs), m))
    got = oracle.connect_fast(tabs, if_in, if_out, si, di, tr, nthreads=4)
    want, _ = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
    np.testing.assert_array_equal(got, want)
    assert len(set(want.tolist())) >= 3


@pytest.mark.parametrize("seed", range(3))
def test_fast_hits_match_literal_eval_acl(seed):
    """orc_classify_fast_hits (the checker of cls_classify_rules) against
    evalACL restated literally (orc_eval_acl, its *hit: the terminating rule,
    n for the default DENY) packet by packet, on random IPv4 ACLs with
    malformed rules and protocols > 2; their histogram is the counters."""
    rules, pool = random_acl(seed * 11 + 3, [30, 150, 300][seed], 0.25)
    tr = random_traffic(seed + 40, 600, pool, other_proto=True)
    cr = oracle.rules_to_c(rules)
    v, hits = oracle.classify_hits(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    for i in range(len(v)):
        a, h = oracle.eval_acl(cr, False, int(tr["src"][i]).to_bytes(4, "big"), int(tr["dst"][i]).to_bytes(4, "big"),
                               int(tr["proto"][i]), int(tr["dport"][i]))
        assert (int(v[i]), int(hits[i])) == (a, h), i
    _, c = oracle.classify_faithful(cr, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    np.testing.assert_array_equal(np.bincount(hits, minlength=cr.n + 1), c)
