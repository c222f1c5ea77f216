"""The keyed table construction of the renderer cache (cache.py _LocalCtx and
_rebuild_global_table: one sort by a Compare-consistent key) against the
literal path (sorted InsertRule / RemoveByPredicate, cache_impl.go:418-673).

Random pod configurations in both orientations -- egress and ingress rules
whose networks include other pods' host routes (the rules installAllowedPorts
removes), IPv6 pods, duplicate rules, deny-all rules, pods removed and
re-added across transactions -- must give identical local and global tables
(every field of every rule, in order) and identical change lists.
"""
import random

import pytest

from vpp_amd import gonet
from vpp_amd.renderer import api, cache as C
from vpp_amd.renderer.api import ContivRule, PodID


def _pods(rng, n):
    pods = [PodID("ns%d" % (i % 3), "pod%d" % i) for i in range(n)]
    ips = {}
    for i, p in enumerate(pods):
        if i % 5 == 4:
            ips[p] = gonet.one_host_subnet("fd00::%x" % (i + 1))
        else:
            ips[p] = gonet.one_host_subnet("10.%d.%d.%d" % (i % 3, i // 250, 1 + i % 250))
    return pods, ips


def _rule(rng, ips):
    def net():
        k = rng.random()
        if k < 0.3:
            return gonet.IPNet()
        if k < 0.65:
            return rng.choice(list(ips.values()))          # another pod's host route
        if k < 0.85:
            return gonet.ip_network("10.%d.%d.0/%d" % (rng.randrange(3), rng.randrange(4), rng.choice([8, 16, 24, 28])))
        return gonet.ip_network(rng.choice(["fd00::/64", "fd00::/112", "::/0", "0.0.0.0/0"]))
    action = api.ACTION_DENY if rng.random() < 0.3 else api.ACTION_PERMIT
    port = rng.choice([0, 0, 22, 53, 80, 443, 8080])
    return ContivRule(action, net(), net(), rng.choice([api.TCP, api.UDP]), 0, port)


def _cfg(rng, ips, pod):
    ing = [_rule(rng, ips) for _ in range(rng.randrange(0, 6))]
    eg = [_rule(rng, ips) for _ in range(rng.randrange(0, 6))]
    if rng.random() < 0.3 and ing:
        ing.append(ing[0].copy())                          # duplicate
    if rng.random() < 0.4:
        ing.append(api.deny_all_tcp())
    if rng.random() < 0.3:
        eg.append(api.deny_all_udp())
    return C.PodConfig(ips[pod], ing, eg)


def _dump_rule(r):
    return (r.action, r.protocol, r.src_port, r.dest_port, bytes(r.src_network.ip), bytes(r.src_network.mask),
            bytes(r.dest_network.ip), bytes(r.dest_network.mask))


def _state(cache, pods):
    local = {}
    for p in pods:
        t = cache.get_local_table_by_pod(p)
        local[p] = None if t is None else [_dump_rule(r) for r in t.rules]
    return local, [_dump_rule(r) for r in cache.get_global_table().rules]


def _changes(txn):
    return sorted((c.table.type, len(c.table.pods), sorted(map(tuple, c.table.pods)),
                   sorted(map(tuple, c.previous_pods)), [_dump_rule(r) for r in c.table.rules])
                  for c in txn.get_changes())


def _run(seed, orientation, keyed, monkeypatch):
    monkeypatch.setattr(C, "KEYED", keyed)
    rng = random.Random(seed)
    pods, ips = _pods(rng, 24)
    cache = C.RendererCache()
    cache.init(orientation)
    out = []
    live = set()
    for step in range(10):   # refreshes share the renderer cache's content caches
        txn = cache.new_txn()
        for p in rng.sample(pods, rng.randrange(1, 12) if step else len(pods)):
            if p in live and rng.random() < 0.15:
                txn.update(p, C.PodConfig(removed=True))
                live.discard(p)
            else:
                txn.update(p, _cfg(rng, ips, p))
                live.add(p)
        out.append(_changes(txn))
        txn.commit()
        out.append(_state(cache, pods))
    return out


@pytest.mark.parametrize("orientation", [C.EGRESS_ORIENTATION, C.INGRESS_ORIENTATION])
@pytest.mark.parametrize("seed", range(6))
def test_keyed_tables_equal_literal_tables(seed, orientation, monkeypatch):
    assert _run(seed, orientation, True, monkeypatch) == _run(seed, orientation, False, monkeypatch)


def test_keyed_path_is_taken(monkeypatch):
    """The random sets above are inside the keyed form (host-route pod
    addresses, canonical masks): the fast path is what they compare."""
    rng = random.Random(1)
    pods, ips = _pods(rng, 10)
    cache = C.RendererCache()
    cache.init(C.EGRESS_ORIENTATION)
    txn = cache.new_txn()
    for p in pods:
        txn.update(p, _cfg(rng, ips, p))
    ctx = C._LocalCtx(txn)
    assert ctx.ok


def test_rule_key_orders_like_compare():
    rng = random.Random(7)
    _, ips = _pods(rng, 30)
    rules = [_rule(rng, ips) for _ in range(400)]
    for a, b in zip(rules, rules[1:] + rules[:1]):
        ka, kb = api.rule_key(a), api.rule_key(b)
        c = a.compare(b)
        assert (ka < kb) == (c < 0) and (ka == kb) == (c == 0), (a, b)
