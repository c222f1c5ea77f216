"""GPU: the source trie (src mode 4) and wide global cells (list modes 5, 6).

classify4_cls over trie images, wide-cell images (forced on small tables with
options wide / trie, in every counter tier the LDS budget leaves),
and the gen-policy.py lists at 200 blocks (trie, LDS cells) and at the
1000-block default (trie, wide cells, > 2^18 counter slots) -- verdicts and
per-rule counters equal the evalACL oracle (aclengine_mock.go:473-668) on
oracle-sized batches, and the CPU interpreter of the same blob
(tests/cls_image.py, pinned to the oracle in test_trie_wide_cpu.py) on
device-resident batches of millions of packets.  The slot mode of connection
batches runs the same images.
"""
import numpy as np
import pytest

import oracle
from aclgen import random_traffic, single_port_acl
from test_trie_wide_cpu import _gen_policy_list, _gen_policy_traffic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from vpp_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


def _oracle(rules, tr):
    return oracle.classify_fast(oracle.rules_to_c(rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("trie,wide", [("1", "0"), ("1", "1"), ("0", "1")])
def test_forced_trie_wide_match_oracle(eng, libopt, seed, trie, wide):
    libopt.set("orient", "src", eng)
    libopt.set("trie", trie, eng)
    libopt.set("wide", wide, eng)
    rules, pool = single_port_acl(seed * 17 + 5, 200, n_prefixes=60)
    tr = random_traffic(seed, 50000, pool)
    t = eng.put_table("tw", rules)
    try:
        info = t.info()
        assert info["lds_resident"] == 1
        if wide == "1":
            assert info["list_mode"] in (5, 6)
        v, c = eng.classify(t, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    finally:
        eng.del_table(t)
    ov, oc = _oracle(rules, tr)
    bad = np.nonzero(v != ov)[0]
    assert len(bad) == 0, "verdict mismatch at %s" % bad[:8]
    np.testing.assert_array_equal(c, oc)


@pytest.mark.parametrize("partial", [False, True])
def test_wide_cells_counter_tiers(eng, libopt, partial):
    """Wide cells with every slot in LDS, and with a budget that leaves two
    thirds of the slots to the global counters."""
    from cls_image import Image, compile_blob
    from vpp_amd import _abi
    libopt.set("orient", "src", eng)
    libopt.set("wide", "1", eng)
    rules, pool = single_port_acl(77, 400, n_prefixes=120)
    if partial:
        h = Image(compile_blob(_abi.CRules(rules))).h
        a16 = lambda x: (x + 15) & ~15
        budget = h.img_bytes + h.n_hot * 256 + a16(2 * max(h.n_hot, h.n_ctr // 3))
        libopt.set("lds_budget", str(budget), eng)
    tr = random_traffic(5, 200000, pool)
    t = eng.put_table("tiers", rules)
    try:
        info = t.info()
        assert info["list_mode"] in (5, 6) and info["lds_resident"] == 1
        if partial:
            assert info["n_lctr"] < info["n_slots"]
        v, c = eng.classify(t, tr["src"], tr["dst"], tr["dport"], tr["proto"])
    finally:
        eng.del_table(t)
    ov, oc = _oracle(rules, tr)
    assert np.array_equal(v, ov)
    np.testing.assert_array_equal(c, oc)


def _device(tr):
    import torch
    return {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else
                                v.view(np.int16) if v.dtype == np.uint16 else v).to("cuda")
            for k, v in tr.items() if k in ("src", "dst", "dport", "proto")}


@pytest.mark.parametrize("blocks,n_oracle", [(200, 60000), (1000, 12000)])
@pytest.mark.parametrize("match", ["ingress", "egress"])
def test_gen_policy_trie_wide_on_gpu(eng, blocks, n_oracle, match):
    """gen-policy.py lists on the IPv4 path: a batch the oracle checks
    directly, and 4 Mi device-resident packets against the CPU interpreter of
    the same compiled blob."""
    import torch
    from cls_image import Image, compile_blob
    from vpp_amd import _abi
    rules = _gen_policy_list(blocks, match)
    t = eng.put_table("gp%d" % blocks, rules)
    try:
        info = t.info()
        assert info["lds_resident"] == 1 and info["list_mode"] == (4 if blocks == 200 else 5)
        small = _gen_policy_traffic(blocks, n_oracle, 3, match)
        v, c = eng.classify(t, small["src"], small["dst"], small["dport"], small["proto"])
        ov, oc = _oracle(rules, small)
        assert np.array_equal(v, ov)
        np.testing.assert_array_equal(c, oc)
        big = _gen_policy_traffic(blocks, 4 << 20, 4, match)
        d = _device(big)
        verdict = torch.empty(4 << 20, dtype=torch.uint8, device="cuda")
        counters = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
        eng.classify(t, d["src"], d["dst"], d["dport"], d["proto"], verdict=verdict, counters=counters)
        torch.cuda.synchronize()
        img = Image(compile_blob(_abi.CRules(rules)))
        iv, ic = img.classify(big["src"], big["dst"], big["dport"], big["proto"])
        assert np.array_equal(verdict.cpu().numpy(), iv)
        np.testing.assert_array_equal(counters.cpu().numpy().astype(np.uint64), ic)
    finally:
        eng.del_table(t)


@pytest.mark.parametrize("trie,wide", [("1", "1"), ("0", "1")])
def test_connection_slot_mode_over_trie_wide(trie, wide):
    """Connection batches (the config-3 global ACL and 64 local ACLs, every
    imaged one compiled with wide cells, with / without the trie) evaluate
    them with the classifier's slot mode: equal to orc_test_connection,
    counters included."""
    from test_gpu_connect_scale import _run
    from vpp_amd.engine import Engine
    e = Engine(options={"orient": "src", "trie": trie, "wide": wide})
    try:
        _run(e, 3, "classifier", 4, True)
    finally:
        e.close()
