"""GPU parity of the configurator -> renderer -> classifier chain
(configurator_impl.go:129-479 feeding renderer_mock.go TestTraffic, SURVEY
8(f) rank 4 on top of 8(a10)).

1. The reference's configurator_test.go scenarios (115 TestTraffic verdicts)
   replayed with every TestTraffic evaluated by the gfx950 classifier.
2. Random policy sets (pod peers, IP blocks with excepts, IPv6 pods, ports)
   committed to the GPU renderer and the literal oracle renderer at once;
   per-pod packet batches must give bit-identical verdicts and per-rule hit
   counts on the device.
"""
import random

import numpy as np
import pytest

from configurator_replay import load, mismatches, random_packets, random_policy_set, replay
from oracle import traffic as otraffic
from vpp_amd import configurator as C
from vpp_amd import gonet
from vpp_amd.renderer import traffic as T

pytestmark = pytest.mark.gpu

SCENARIOS = load()["scenarios"]


@pytest.fixture(scope="module")
def eng():
    from vpp_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


@pytest.mark.parametrize("scn", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_reference_scenarios_on_gpu(eng, scn):
    renderers, checks = replay(scn, lambda name: T.TrafficRenderer(name, eng))
    try:
        assert checks and not mismatches(checks)
    finally:
        for r in renderers.values():
            r.close()


def _rows(ips):
    return np.frombuffer(b"".join(gonet.V4_IN_V6_PREFIX + x if len(x) == 4 else x for x in ips),
                         np.uint8).reshape(-1, 16)


@pytest.mark.parametrize("seed", range(3))
def test_random_policy_sets_on_gpu(eng, seed):
    rng = random.Random(1000 + seed)
    cache, assign = random_policy_set(rng, n_pods=120, n_policies=40)
    r = T.TrafficRenderer("gpu", eng)
    conf = C.PolicyConfigurator(cache)
    conf.register_renderer(r)
    txn = conf.new_txn(True)
    for pod, pols in assign.items():
        txn.configure(pod, pols)
    txn.commit()
    src, dst, proto, sport, dport = random_packets(rng, cache, 4000)
    s16, d16 = _rows(src), _rows(dst)
    p8, dp16 = np.array(proto, np.uint8), np.array(dport, np.uint16)
    checked = 0
    try:
        for pod in list(r.config)[:16]:
            for d in (T.INGRESS_TRAFFIC, T.EGRESS_TRAFFIC):
                cfg = r.config[pod]
                rules = cfg.ingress if d == T.INGRESS_TRAFFIC else cfg.egress
                if not rules:
                    continue
                want, want_c, want_u = otraffic.test_traffic_batch(rules, src, dst, proto, sport, dport)
                v, c, u = r.test_traffic_batch(pod, d, s16, d16, p8, dp16)
                assert list(v) == want, (pod, d)
                assert [int(x) for x in c] == want_c and u == want_u, (pod, d)
                checked += 1
    finally:
        r.close()
    assert checked >= 8


@pytest.mark.parametrize("num_cidrs", [20, 60, 200])
def test_gen_policy_scale_on_gpu(eng, num_cidrs):
    """gen-policy.py's NetworkPolicy (1 policy, num_cidrs blocks x 5 excepts,
    20 ports per direction) through the configurator: ~10k-95k rules per
    list, compiled onto the classifier (LDS counter tiers from 60 blocks on,
    the global-memory image at 200).  The expectation comes from the C
    evalACL oracle over the same translation, which test_traffic_cpu.py pins
    to the literal TestTraffic oracle."""
    import oracle
    from configurator_replay import gen_policy_packets
    from vpp_amd.renderer.api import PodID
    rng = random.Random(num_cidrs)
    pol = C.gen_policy(rng, num_cidrs=num_cidrs)
    pod = PodID("db", "default")
    conf = C.PolicyConfigurator({pod: "10.1.1.1"})
    r = T.TrafficRenderer("gen", eng)
    conf.register_renderer(r)
    conf.new_txn(False).configure(pod, [pol]).commit()
    try:
        # give a share of packets the policy's ports so PERMITs are exercised
        src, dst, proto, dport, s16, d16 = gen_policy_packets(rng, 8000, num_cidrs)
        ports = [p.number for m in pol.matches for p in m.ports]
        dport = [rng.choice(ports) if rng.random() < 0.5 else p for p in dport]
        p8, dp16 = np.array(proto, np.uint8), np.array(dport, np.uint16)
        for d in (T.INGRESS_TRAFFIC, T.EGRESS_TRAFFIC):
            rules = r.config[pod].ingress if d == T.INGRESS_TRAFFIC else r.config[pod].egress
            assert len(rules) > 400 * num_cidrs
            cr = oracle.rules_to_c(T.compile_rules(rules))
            if num_cidrs <= 60:
                want_v, want_c = oracle.classify_faithful(cr, s16, d16, dp16, p8, af=16)
            else:                                      # ~95k rules: the pre-parsed oracle
                want_v, want_c = oracle.classify_fast(cr, s16, d16, dp16, p8, af=16)
            v, c, u = r.test_traffic_batch(pod, d, s16, d16, p8, dp16)
            assert np.array_equal(v, want_v), d
            per_rule, unmatched = T.rule_counters(want_c, len(rules))
            assert np.array_equal(np.asarray(c), np.asarray(per_rule)) and u == unmatched
            assert len(set(want_v.tolist())) >= 2
    finally:
        r.close()


def test_gen_policy_default_scale_on_gpu(eng):
    """gen-policy.py at its defaults (tests/policy/perf/gen-policy.py:8-11:
    1000 blocks x 5 excepts x 20 ports): the pod's ingress list has ~477k
    rules.  In the 16-byte layout it compiles to an LDS-resident image (the
    IPv4 source trie of src_mode 2, wide cells; tests/test_cls16_cpu.py and
    test_gen_policy_lists_v16_on_gpu check the blob at scale).  2000 packets
    through the host path against the pre-parsed C evalACL oracle, verdicts
    and per-rule counts."""
    import oracle
    from configurator_replay import gen_policy_packets
    from vpp_amd.renderer.api import PodID
    rng = random.Random(1000)
    pol = C.gen_policy(rng, num_cidrs=1000)
    pod = PodID("db", "default")
    rules = C.PolicyConfigurator({pod: "10.1.1.1"}).new_txn(False).generate_rules(C.MATCH_INGRESS, [pol])
    assert len(rules) > 400_000
    src, dst, proto, dport, s16, d16 = gen_policy_packets(rng, 2000, 1000)
    ports = [p.number for m in pol.matches for p in m.ports]
    dport = [rng.choice(ports) if rng.random() < 0.5 else p for p in dport]
    p8, dp16 = np.array(proto, np.uint8), np.array(dport, np.uint16)
    acl_rules = T.compile_rules(rules)
    want_v, want_c = oracle.classify_fast(oracle.rules_to_c(acl_rules), s16, d16, dp16, p8, af=16)
    t = eng.put_table("gen1000", acl_rules)
    try:
        v, c = eng.classify(t, s16, d16, dp16, p8)
        assert np.array_equal(v, want_v)
        assert np.array_equal(c, want_c)
        assert len(set(want_v.tolist())) >= 2
    finally:
        eng.del_table(t)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("blocks", [200, 1000])
def test_gen_policy_lists_v16_on_gpu(eng, blocks):
    """The gen-policy.py lists in the 16-byte layout (IPv4-mapped packets in
    and around the blocks, 10 % IPv6, ICMP, protocol 47), ingress and egress:
    the image is LDS-resident (src_mode 2: the IPv4 source trie), 1 Mi
    device-resident packets bit-exact against the blob interpreter
    (tests/cls_image.py Image16, verdicts and counters), and a 16 Ki sample
    against the pre-parsed C evalACL oracle."""
    import torch

    import oracle
    from cls_image import Image16, compile_blob
    from vpp_amd import _abi
    from vpp_amd.renderer.api import PodID
    pol = C.gen_policy(random.Random(blocks), num_cidrs=blocks)
    txn = C.PolicyConfigurator({PodID("db", "default"): "10.1.1.1"}).new_txn(False)
    g = np.random.default_rng(blocks)
    n = 1 << 20
    ports = np.array([p.number for p in pol.matches[0].ports], np.uint16)
    # (1000 blocks: the ingress list only -- each ~480k-rule list compiles for
    # tens of seconds on the host, three times here)
    for match in (C.MATCH_INGRESS, C.MATCH_EGRESS) if blocks <= 200 else (C.MATCH_INGRESS,):
        acl = T.compile_rules(txn.generate_rules(match, [pol]))
        img = Image16(compile_blob(_abi.CRules(acl), "cls_compile_v16"))
        t = eng.put_table("gp16", acl)
        try:
            info = t.info()
            assert info["lds_resident_v16"] == 1 and img.h.src_mode == 2
            blk = g.integers(0, blocks + blocks // 10 + 1, n).astype(np.uint64)
            inblk = ((blk + 0x100) << np.uint64(16)) | g.integers(0, 1 << 16, n).astype(np.uint64)
            other = g.integers(0, 1 << 32, n).astype(np.uint64)
            a, b = (inblk, other) if match == C.MATCH_INGRESS else (other, inblk)

            def wide(x, v6):
                hi = np.where(v6, np.uint64(0xFD000000 << 32), np.uint64(0))
                lo = np.where(v6, x, np.uint64(0xFFFF << 32) | x)
                out = np.empty((n, 16), np.uint8)
                out[:, :8] = hi.astype(">u8").view(np.uint8).reshape(n, 8)
                out[:, 8:] = lo.astype(">u8").view(np.uint8).reshape(n, 8)
                return out
            src, dst = wide(a, g.random(n) < 0.1), wide(b, g.random(n) < 0.1)
            dport = np.where(g.random(n) < 0.5, g.choice(ports, n), g.integers(0, 65536, n)).astype(np.uint16)
            proto = g.choice(np.array([0, 1, 2, 47], np.uint8), n, p=[0.445, 0.445, 0.1, 0.01])
            d = {k: torch.from_numpy(v.view(np.int16) if v.dtype == np.uint16 else v).to("cuda")
                 for k, v in dict(src=src, dst=dst, dport=dport, proto=proto).items()}
            verdict = torch.empty(n, dtype=torch.uint8, device="cuda")
            counters = torch.zeros(len(acl) + 1, dtype=torch.int64, device="cuda")
            eng.classify(t, d["src"], d["dst"], d["dport"], d["proto"], verdict, counters)
            torch.cuda.synchronize()
            v, c = verdict.cpu().numpy(), counters.cpu().numpy().astype(np.uint64)
            wv, wc = img.classify(src, dst, dport, proto)
            assert np.array_equal(v, wv), match
            assert np.array_equal(c, wc), match
            k = 1 << 14
            ov, _ = oracle.classify_fast(oracle.rules_to_c(acl), src[:k], dst[:k], dport[:k], proto[:k], af=16)
            assert np.array_equal(v[:k], ov), match
            assert len(set(ov.tolist())) >= 2
        finally:
            eng.del_table(t)
