"""Connection path at scale on the GPU (testConnection, aclengine_mock.go:394-471;
SURVEY 8(a5) / 8(f) rank 1).

Many ACLs bound to many interfaces -- a 1003-rule rendered global table
(config 2), 64 random local ACLs of 1-300 rules with REFLECT, DENY and
PERMIT actions and odd protocols, interfaces with no ACL -- and 20k random
connections between them, including same-interface pairs (the REFLECT
short-cuts of :412-421).  Every ConnectionAction must equal the C oracle's
orc_test_connection (aclengine_ref.c), bit for bit -- with the large ACLs
evaluated by the classifier kernel (cls_connect_batch's precomputed SYN /
SYN-ACK verdicts), by the linear scan, and in the automatic mode.
"""
import ctypes as C
import random

import numpy as np
import pytest

import oracle
from aclgen import random_acl, random_traffic
from vpp_amd import workload

pytestmark = pytest.mark.gpu


def _b4(a: int) -> bytes:
    return int(a).to_bytes(4, "big")


def build(eng, seed=0, n_local=64, n_if=80, cfg=2):
    rng = random.Random(seed)
    glob, spec, _ = workload.config(cfg)
    ifs = ["if%d" % i for i in range(n_if)]
    bind = {name: [None, None] for name in ifs}          # name -> [in rules, out rules]
    acls = [("global", glob.rules, ["if0", "if1"], ["if0", "if2"])]
    pool = None
    for k in range(n_local):
        rules, pool = random_acl(1000 + k, rng.choice([1, 3, 12, 40, 150, 300]),
                                 weird=rng.choice([0.0, 0.003, 0.15]))
        ing = rng.sample(ifs[3:], rng.randrange(1, 3))
        eg = rng.sample(ifs[3:], rng.randrange(0, 3))
        acls.append(("local%d" % k, rules, ing, eg))
    for name, rules, ing, eg in acls:
        assert eng.acl_put(name, rules, ing, eg) == 0
        for i in ing:
            bind[i][0] = rules
        for e in eg:
            bind[e][1] = rules
    return ifs, bind, pool, spec


def oracle_connections(bind, ifs, si, di, src, dst, proto, sport, dport):
    crs = {}

    def ref(rules):
        if rules is None:
            return oracle.AclRef(None, 0, 1)
        key = id(rules)
        if key not in crs:
            crs[key] = oracle.rules_to_c(rules)
        cr = crs[key]
        return oracle.AclRef(cr.ptr(), cr.n, 0)

    L = oracle.lib()
    out = np.zeros(len(src), np.uint8)
    for i in range(len(src)):
        a, b = ifs[si[i]], ifs[di[i]]
        refs = [ref(bind[a][0]), ref(bind[a][1]), ref(bind[b][0]), ref(bind[b][1])]
        s, d = _b4(src[i]), _b4(dst[i])
        rc = L.orc_test_connection(*[C.byref(r) for r in refs], 1 if a == b else 0, s, 4, d, 4,
                                   int(proto[i]), int(sport[i]), int(dport[i]))
        assert rc >= 0
        out[i] = rc
    return out


@pytest.mark.parametrize("mode", ["classifier", "linear", "auto", "device"])
@pytest.mark.parametrize("seed", [0, 1])
def test_connections_at_scale_match_oracle(seed, mode):
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        ifs, bind, pool, spec = build(eng, seed)
        n = 20000
        tr = random_traffic(50 + seed, n, pool)
        rng = np.random.default_rng(seed)
        # a third of the endpoints from the global table's pod addresses
        pods = spec["pod_ips"].astype(np.uint32)
        mix = rng.random(n) < 0.33
        tr["src"][mix] = rng.choice(pods, mix.sum())
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        si = rng.integers(0, len(ifs), n)
        di = np.where(rng.random(n) < 0.1, si, rng.integers(0, len(ifs), n))
        args = [ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"]]
        if mode == "device":                      # CLS_F_DEVICE batch: every ACL >= 64 rules on the classifier
            import torch
            dv = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
                  .to("cuda") for x in args]
            torch.cuda.synchronize()
            got = eng.connect_batch(*dv, mode="classifier").cpu().numpy()
        else:
            got = eng.connect_batch(*args, mode=mode)
        want = oracle_connections(bind, ifs, si, di, tr["src"], tr["dst"], tr["proto"], tr["sport"],
                                  tr["dport"])
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (bad[:10], got[bad[:10]], want[bad[:10]])
        assert len(set(want.tolist())) >= 3              # allowed, denied, reflected/failure all seen
    finally:
        eng.close()
