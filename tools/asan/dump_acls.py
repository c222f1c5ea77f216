#!/usr/bin/env python3
"""Write the ACLs of the sanitizer run (tools/asan/asan_main.cpp): one rule
per line (cls_rule fields; '-' for a NULL network, '""' spelled as '-'
too), '=' after each ACL."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main(out):
    from aclgen import random_acl, random_acl16
    from vpp_amd import _abi, configurator as C, workload
    from vpp_amd.renderer.api import PodID
    from vpp_amd.renderer.traffic import compile_rules
    acls = []
    for seed in range(24):
        acls.append(random_acl(seed, [5, 40, 200, 600][seed % 4], [0.0, 0.05, 0.3][seed % 3])[0])
        acls.append(random_acl16(seed + 100, [20, 150][seed % 2], [0.0, 0.1][seed % 2])[0])
    for cfg in (2, 3, 5):
        acls.append(workload.config(cfg)[0].rules)
    pol = C.gen_policy(random.Random(60), num_cidrs=60)
    txn = C.PolicyConfigurator({PodID("db", "default"): "10.1.1.1"}).new_txn(False)
    for m in (C.MATCH_INGRESS, C.MATCH_EGRESS):
        acls.append(compile_rules(txn.generate_rules(m, [pol])))
    with open(out, "w") as f:
        for rules in acls:
            cr = _abi.CRules(rules)
            for i in range(cr.n):
                r = cr.arr[i]
                net = lambda x: (x.decode() or "-") if x else "-"
                f.write("%d %d %s %s %s\n" % (r.flags, r.acl_action, net(r.src_network), net(r.dst_network),
                                               " ".join(str(getattr(r, k)) for k in (
                                                   "tcp_src_lo", "tcp_src_hi", "tcp_dst_lo", "tcp_dst_hi",
                                                   "udp_src_lo", "udp_src_hi", "udp_dst_lo", "udp_dst_hi",
                                                   "icmp_code_first", "icmp_code_last", "icmp_type_first",
                                                   "icmp_type_last"))))
            f.write("=\n")
    print("wrote %d ACLs to %s" % (len(acls), out))


if __name__ == "__main__":
    main(sys.argv[1])
