"""Commit latency of the policy data path (incremental
renderer txns -> table puts).

A node with N pods (config 3's synthetic policy: per app a list of ingress
ContivRules, acl_renderer.go's global table ~10 rules per pod) is rendered
once; then single-pod changes are committed and timed:
  * rules:  one pod gains an ingress rule -> the global table changes (one
            recompile of the ~10k-rule table);
  * pods:   a new pod joins an app -> the renderer re-puts tables whose pod
            sets changed with equal rules (cls_acl_put keeps the compiled
            table: a rebind) plus the changed global table;
  * nochange: re-render a pod with its current config (no txn at all).
Each commit is split into the renderer's own time (cache txn, renderACL,
acl_renderer.go:124-264 / cache_impl.go:229-343) and ApplyTxn (the engine:
compile + upload of the changed tables only).

usage: python tools/commit_bench.py [--pods 1000] [--engine gpu|oracle]
prints one JSON line.
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from vpp_amd import gonet, workload  # noqa: E402
from vpp_amd.renderer import api  # noqa: E402
from vpp_amd.renderer.acl import ContivIfs, Renderer, TxnTracker  # noqa: E402
from vpp_amd.renderer.api import PodID  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1000)
    ap.add_argument("--apps", type=int, default=100)
    ap.add_argument("--rules-per-pod", type=int, default=10)
    ap.add_argument("--engine", default="gpu")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()

    rng = random.Random(3)
    cidrs = workload.service_cidrs(rng)
    apps = [workload.app_rules(rng, cidrs, a.rules_per_pod) for _ in range(a.apps)]
    pods = [PodID("default", "pod%d" % k) for k in range(a.pods + a.reps)]
    contiv = ContivIfs(main_if="GbE", vxlan_bvi="VXLAN-BVI", host_interconnect="VPP-Host")
    for k, p in enumerate(pods):
        contiv.set_pod_if_name(p, "tap%d" % k)
    if a.engine == "gpu":
        from vpp_amd.engine import ACLEngine, Engine
        eng = ACLEngine(contiv, Engine())
    else:
        sys.path.insert(0, ROOT)
        import oracle
        eng = oracle.OracleACLEngine(contiv)
    apply_s = [0.0]

    def on_commit(ops):
        t = time.perf_counter()
        err = eng.apply_txn(ops)
        apply_s[0] += time.perf_counter() - t
        return err

    tracker = TxnTracker(on_commit)
    r = Renderer(contiv, tracker.new_linux_data_change_txn).init()
    ip = [gonet.one_host_subnet(workload._v4(workload.pod_ip(k))) for k in range(len(pods))]

    def commit(items, resync=False):
        apply_s[0] = 0.0
        ops0 = len(tracker.committed)
        t = time.perf_counter()
        txn = r.new_txn(resync)
        for k, ingress in items:
            txn.render(pods[k], ip[k], ingress, [], False)
        txn.commit()
        total = time.perf_counter() - t
        ops = sum(len(o) for o in tracker.committed[ops0:])
        return dict(total_ms=round(1e3 * total, 2), renderer_ms=round(1e3 * (total - apply_s[0]), 2),
                    apply_ms=round(1e3 * apply_s[0], 2), acl_ops=ops)

    stats0 = eng.engine.acl_stats() if a.engine == "gpu" else None
    full = commit([(k, apps[k % a.apps]) for k in range(a.pods)], resync=True)
    res = dict(pods=a.pods, engine=a.engine, full_render=full)
    gt = r.cache.get_global_table()
    res["global_rules"] = gt.num_of_rules
    out = {"rules": [], "pods": [], "nochange": []}
    for i in range(a.reps):
        k = rng.randrange(a.pods)
        extra = api.ContivRule(api.ACTION_PERMIT, gonet.IPNet(), gonet.ip_network("192.168.%d.0/24" % i),
                               api.TCP, 0, 9000 + i)
        apps_k = list(apps[k % a.apps])
        out["rules"].append(commit([(k, [extra] + apps_k)]))
        out["pods"].append(commit([(a.pods + i, apps[(a.pods + i) % a.apps])]))
        out["nochange"].append(commit([(k, [extra] + apps_k)]))
    for key, v in out.items():
        med = sorted(v, key=lambda x: x["total_ms"])[len(v) // 2]
        res[key] = dict(median=med, all_total_ms=[x["total_ms"] for x in v])
    if a.engine == "gpu":
        s1 = eng.engine.acl_stats()
        res["engine_puts"] = dict(compiles=s1[0] - stats0[0], rebinds=s1[1] - stats0[1])
        eng.engine.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
