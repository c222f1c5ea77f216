"""The sort-based global table (renderer/cache.py build_global_table, used to
render the config 2-4 tables) equals the renderer cache's own construction:
rebuildGlobalTable inserting every pod's ingress rule with the pod's /32 as
source, one InsertRule each, then allow-all TCP and UDP
(plugins/policy/renderer/cache/cache_impl.go:638-673, cache_api.go:250-265).
Config 2 goes through a whole RendererCache transaction (local tables
included); config 3's 1000 pods through InsertRule alone (the transaction's
local tables are O(pods^2) in Python)."""
import random

import pytest

from vpp_amd import gonet, workload
from vpp_amd.renderer import cache as CA
from vpp_amd.renderer.api import PodID, allow_all_tcp, allow_all_udp


def _pods(cfg):
    c = workload.CONFIGS[cfg]
    rng = random.Random(c.get("table", cfg))        # workload.render_global's stream
    cidrs = workload.service_cidrs(rng)
    apps = [workload.app_rules(rng, cidrs, c["rules_per_pod"]) for _ in range(c["n_apps"])]
    return [(gonet.one_host_subnet(workload._v4(workload.pod_ip(k))), apps[k % c["n_apps"]])
            for k in range(c["n_pods"])]


def _same(a, b):
    assert len(a.rules) == len(b.rules)
    for i, (x, y) in enumerate(zip(a.rules, b.rules)):
        assert x.compare(y) == 0, (i, x, y)


def test_config2_global_table_equals_renderer_cache_txn():
    pods = _pods(2)
    rc = CA.RendererCache()
    rc.init(CA.EGRESS_ORIENTATION)
    txn = rc.new_txn()
    for k, (ip, ingress) in enumerate(pods):
        txn.update(PodID("pod%d" % k, "default"), CA.PodConfig(ip, ingress, []))
    txn.commit()
    _same(rc.get_global_table(), CA.build_global_table(pods))


@pytest.mark.parametrize("cfg", [2, 3])
def test_global_table_equals_insert_rule(cfg):
    pods = _pods(cfg)
    table = CA.ContivRuleTable(CA.GLOBAL_TABLE_ID)
    for ip, ingress in pods:
        for r in ingress:
            c = r.copy()
            c.src_network = ip
            table.insert_rule(c)
    table.insert_rule(allow_all_tcp())
    table.insert_rule(allow_all_udp())
    fast = CA.build_global_table(pods)
    _same(table, fast)
    acl, _, _ = workload.config(cfg)
    assert len(acl.rules) == len(fast.rules) + 1       # renderACL appends the ICMP rule
