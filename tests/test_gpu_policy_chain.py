"""The whole Contiv policy chain on the GPU, end to end:

  ContivPolicy sets -> PolicyConfigurator (configurator_impl.go:129-479)
  -> ACL Renderer + renderer cache (acl_renderer.go, cache_impl.go)
  -> TxnTracker -> ACLEngine.ApplyTxn (aclengine_mock.go:94-242)
  -> Connection* batches on the gfx950 connection + classifier kernels.

The same chain with the oracle MockACLEngine restatement (OracleACLEngine)
gives the expected ConnectionAction for every connection: pod to pod, pod to
internet and internet to pod, between 150 pods with random policies.  With
IPv6 pods among them the batch goes through the 16-byte connection path
(CLS_AF_V16: IPv4 endpoints IPv4-mapped, as Go's To4/To16 see them).
"""
import random

import pytest

import oracle
from configurator_replay import random_policy_set
from vpp_amd import configurator as C
from vpp_amd.renderer.acl import ContivIfs, Renderer, TxnTracker

pytestmark = pytest.mark.gpu


def chain(engine_factory, cache, assign, contiv):
    engine = engine_factory(contiv)
    for pod, ip in cache.items():
        engine.register_pod(pod, ip, False)
    tracker = TxnTracker(engine.apply_txn)
    renderer = Renderer(contiv, tracker.new_linux_data_change_txn).init()
    conf = C.PolicyConfigurator(cache)
    conf.register_renderer(renderer)
    txn = conf.new_txn(True)
    for pod, pols in assign.items():
        txn.configure(pod, pols)
    txn.commit()
    return engine


@pytest.mark.parametrize("families", ["v4", "mixed"])
@pytest.mark.parametrize("seed", range(2))
def test_policy_chain_connections_on_gpu(seed, families):
    from vpp_amd.engine import ACLEngine, Engine
    rng = random.Random(seed)
    cache, assign = random_policy_set(rng, n_pods=150, n_policies=50)
    if families == "v4":
        cache = {p: ip for p, ip in cache.items() if ":" not in ip}
    else:
        assert any(":" in ip for ip in cache.values())
    contiv = ContivIfs(main_if="GbE", vxlan_bvi="VXLAN-BVI", host_interconnect="VPP-Host")
    for k, pod in enumerate(cache):
        contiv.set_pod_if_name(pod, "tap%d" % k)
    want_eng = chain(oracle.OracleACLEngine, cache, assign, contiv)
    eng = Engine()
    try:
        got_eng = chain(lambda c: ACLEngine(c, eng), cache, assign, contiv)
        pods = list(cache)
        calls = []
        for _ in range(3000):
            k = rng.random()
            proto, sport = rng.randrange(2), rng.randrange(1024, 65536)
            dport = rng.choice([22, 53, 80, 443, 8080, rng.randrange(65536)])
            ext = "10.%d.%d.%d" % (rng.randrange(4), rng.randrange(256), rng.randrange(256))
            if families == "mixed" and rng.random() < 0.3:
                ext = "fd00:10::%x" % rng.randrange(1 << 16)
            if k < 0.6:
                calls.append(("ConnectionPodToPod", (rng.choice(pods), rng.choice(pods), proto, sport, dport)))
            elif k < 0.8:
                calls.append(("ConnectionPodToInternet", (rng.choice(pods), ext, proto, sport, dport)))
            else:
                calls.append(("ConnectionInternetToPod", (ext, rng.choice(pods), proto, sport, dport)))
        fn = {"ConnectionPodToPod": want_eng.connection_pod_to_pod,
              "ConnectionPodToInternet": want_eng.connection_pod_to_internet,
              "ConnectionInternetToPod": want_eng.connection_internet_to_pod}
        want = [fn[f](*a) for f, a in calls]
        got = got_eng.connection_batch(calls)
        bad = [(c, g, w) for c, g, w in zip(calls, got, want) if g != w]
        assert not bad, bad[:5]
        assert len(set(want)) >= 2
        assert got_eng.get_num_of_acls() == want_eng.get_num_of_acls()
    finally:
        eng.close()
