"""Connection path at scale on the GPU (testConnection, aclengine_mock.go:394-471;
SURVEY 8(a5) / 8(f) rank 1).

Many ACLs bound to many interfaces -- a rendered global table (config 2,
1003 rules), random local ACLs of 1-300 rules with REFLECT, DENY and PERMIT
actions and odd protocols, interfaces with no ACL -- and 20k random
connections between them, including same-interface pairs (the REFLECT
short-cuts of :412-421).  Every ConnectionAction must equal the C oracle's
orc_test_connection (aclengine_ref.c), bit for bit -- with the large ACLs
evaluated by the classifier kernel (cls_connect_batch's slot-mode SYN /
SYN-ACK passes), by the linear scan, and in the automatic mode; for IPv4
(CLS_AF_V4) and mixed-family (CLS_AF_V16: IPv4-mapped and IPv6 endpoints,
IPv6 and IPv4 networks in the ACLs) batches.

Counters (CLS_F_COUNT): the per-(ACL, rule) connection counters must equal
the oracle's -- the terminating rule of every evalACL call testConnection
makes (orc_test_connection_hits), summed per ACL -- with the rule pool in LDS
or global memory and the counters in LDS or global memory.  The reference
has no counters (parity unpinned; the definition is the oracle's).
"""
import ctypes as C
import random

import numpy as np
import pytest

import oracle
from aclgen import mix_families, random_acl, random_acl16, random_traffic, random_traffic16
from vpp_amd import workload

pytestmark = pytest.mark.gpu

V6_TWIN = 0xFD000030 << 96


def build(eng, seed=0, n_local=64, n_if=80, cfg=2, fam=4):
    """ACLs installed on `eng`; returns (interface names, binding: if -> [in
    ACL name, out ACL name], rules by ACL name, prefix pool, traffic spec)."""
    rng = random.Random(seed)
    glob, spec, _ = workload.config(cfg)
    grules = glob.rules
    if fam == 16:
        tr0 = random_traffic(1, 4, random_acl(1, 1)[1])
        grules, _ = mix_families(grules, tr0, seed)
    ifs = ["if%d" % i for i in range(n_if)]
    bind = {name: [None, None] for name in ifs}
    acls = [("global", grules, ["if0", "if1"], ["if0", "if2"])]
    pool = None
    for k in range(n_local):
        size = rng.choice([1, 3, 12, 40, 150, 300])
        weird = rng.choice([0.0, 0.003, 0.15])
        rules, pool = (random_acl16 if fam == 16 else random_acl)(1000 + k, size, weird=weird)
        ing = rng.sample(ifs[3:], rng.randrange(1, 3))
        eg = rng.sample(ifs[3:], rng.randrange(0, 3))
        acls.append(("local%d" % k, rules, ing, eg))
    by_name = {}
    for name, rules, ing, eg in acls:
        assert eng.acl_put(name, rules, ing, eg) == 0
        by_name[name] = rules
        for i in ing:
            bind[i][0] = name
        for e in eg:
            bind[e][1] = name
    return ifs, bind, by_name, pool, spec


def traffic(seed, n, pool, spec, fam):
    rng = np.random.default_rng(seed)
    pods = spec["pod_ips"].astype(np.uint32)
    mix = rng.random(n) < 0.33                       # a third of the sources are the global table's pods
    if fam == 4:
        tr = random_traffic(50 + seed, n, pool)
        tr["src"][mix] = rng.choice(pods, mix.sum())
        return tr
    tr = random_traffic16(50 + seed, n, pool)
    p = rng.choice(pods, mix.sum()).astype(np.uint64)
    twin = rng.random(mix.sum()) < 0.5
    hi = np.where(twin, np.uint64(V6_TWIN >> 64), np.uint64(0))
    lo = np.where(twin, np.uint64(0), np.uint64(0xFFFF << 32)) | p
    b = np.empty((mix.sum(), 16), np.uint8)
    b[:, :8] = hi.astype(">u8").view(np.uint8).reshape(-1, 8)
    b[:, 8:] = lo.astype(">u8").view(np.uint8).reshape(-1, 8)
    tr["src"][mix] = b
    return tr


def _addr(a, fam) -> bytes:
    return int(a).to_bytes(4, "big") if fam == 4 else bytes(a)


def oracle_connections(bind, by_name, ifs, si, di, tr, fam):
    """Verdicts and per-ACL hit counters (name -> R + 1 counts)."""
    crs = {name: oracle.rules_to_c(rules) for name, rules in by_name.items()}
    counts = {name: np.zeros(len(rules) + 1, np.uint64) for name, rules in by_name.items()}

    def ref(name):
        if name is None:
            return oracle.AclRef(None, 0, 1)
        return oracle.AclRef(crs[name].ptr(), crs[name].n, 0)

    L = oracle.lib()
    n = len(tr["proto"])
    out = np.zeros(n, np.uint8)
    hits = (C.c_int32 * 4)()
    alen = 4 if fam == 4 else 16
    for i in range(n):
        a, b = ifs[si[i]], ifs[di[i]]
        names = [bind[a][0], bind[a][1], bind[b][0], bind[b][1]]
        s, d = _addr(tr["src"][i], fam), _addr(tr["dst"][i], fam)
        rc = L.orc_test_connection_hits(*[C.byref(ref(x)) for x in names], 1 if a == b else 0, s, alen, d, alen,
                                        int(tr["proto"][i]), int(tr["sport"][i]), int(tr["dport"][i]), hits)
        assert rc >= 0
        out[i] = rc
        # call order: src inbound, dst outbound, dst inbound, src outbound
        for k, name in zip(range(4), (names[0], names[3], names[2], names[1])):
            if hits[k] >= 0:
                counts[name][hits[k]] += 1
    return out, counts


def _run(eng, seed, mode, fam, count, n=20000, n_local=64, cfg=2):
    ifs, bind, by_name, pool, spec = build(eng, seed, fam=fam, n_local=n_local, cfg=cfg)
    tr = traffic(seed, n, pool, spec, fam)
    rng = np.random.default_rng(seed)
    ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
    si = rng.integers(0, len(ifs), n)
    di = np.where(rng.random(n) < 0.1, si, rng.integers(0, len(ifs), n))
    args = [ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"]]
    if mode in ("device", "device_auto"):     # CLS_F_DEVICE batch: every ACL >= 64 rules on the classifier
        import torch

        def dev(x):
            x = np.ascontiguousarray(x)
            if x.ndim == 2:
                return torch.from_numpy(x).to("cuda")
            return torch.from_numpy(x.view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize])).to("cuda")
        dv = [dev(x) for x in args]
        torch.cuda.synchronize()
        # device_auto: the default selection (ACLs of >= 2048 rules on the
        # classifier, the others in the bitmap form or scanned)
        got = eng.connect_batch(*dv, mode="classifier" if mode == "device" else "auto",
                                count=count).cpu().numpy()
    else:
        got = eng.connect_batch(*args, mode=mode, count=count)
    want, wcounts = oracle_connections(bind, by_name, ifs, si, di, tr, fam)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:10], got[bad[:10]], want[bad[:10]])
    assert len(set(want.tolist())) >= 3              # allowed, denied, reflected/failure all seen
    if count:
        for name in by_name:
            c = eng.conn_counters(name, reset=True)
            d = np.nonzero(c != wcounts[name])[0]
            assert d.size == 0, (name, d[:10], c[d[:10]], wcounts[name][d[:10]])
        assert sum(int(v.sum()) for v in wcounts.values()) > n // 4   # counted calls seen
        assert not eng.conn_counters("global").any()    # reset
    return want


@pytest.mark.parametrize("mode", ["classifier", "linear", "auto", "device", "device_auto"])
@pytest.mark.parametrize("seed", [0, 1])
def test_connections_at_scale_match_oracle(seed, mode):
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        _run(eng, seed, mode, 4, count=False)
    finally:
        eng.close()


@pytest.mark.parametrize("no_lds", [0, 1, 6])
@pytest.mark.parametrize("bitmap", ["1", "0"])
def test_connections_bitmap_form_match_oracle(bitmap, no_lds):
    """Device batches with the default selection: the linear IPv4 ACLs (1-300
    random rules) in the bitmap form (engine.cpp conn_bitmap4) or scanned
    (option conn_bitmap=0), the pool in LDS or (no_lds 1) global memory,
    the counters and tables in global memory (no_lds 6); verdicts and per-(ACL, rule) counters against orc_test_connection."""
    from vpp_amd.engine import Engine
    eng = Engine(options={"conn_bitmap": bitmap, "conn_no_lds": no_lds})
    try:
        _run(eng, 11 + no_lds, "device_auto", 4, count=True, n=16000, n_local=24)
    finally:
        eng.close()


@pytest.mark.parametrize("mode", ["classifier", "linear", "device"])
def test_connections16_mixed_families_match_oracle(mode):
    """CLS_AF_V16 batches: IPv4-mapped and IPv6 endpoints, both families of
    networks, counters included."""
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        _run(eng, 3, mode, 16, count=True, n=12000)
    finally:
        eng.close()


@pytest.mark.parametrize("fam", [4, 16])
@pytest.mark.parametrize("no_lds", [0, 1, 2, 3, 7])
def test_connection_counters_match_oracle(fam, no_lds):
    """Per-(ACL, rule) counters with the rule pool in LDS (few locals: the
    pool fits) or in global memory, the counters in LDS or global memory,
    the descriptor and interface tables in LDS or (bit 2) global memory."""
    from vpp_amd.engine import Engine
    eng = Engine(options={"conn_no_lds": no_lds})
    try:
        _run(eng, 7 + no_lds, "classifier", fam, count=True, n=8000, n_local=12)
    finally:
        eng.close()


def test_connection_counters_accumulate_over_calls():
    """Counters add up over batches until read with reset; nil ACLs are not counted."""
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        ifs, bind, by_name, pool, spec = build(eng, 5, n_local=8, n_if=20)
        tr = traffic(5, 3000, pool, spec, 4)
        rng = np.random.default_rng(5)
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        si, di = rng.integers(0, len(ifs), 3000), rng.integers(0, len(ifs), 3000)
        args = [ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"]]
        eng.connect_batch(*args, count=True)
        eng.connect_batch(*args, count=True)
        eng.connect_batch(*args)                     # not counted
        _, want = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
        for name in by_name:
            assert np.array_equal(eng.conn_counters(name), 2 * want[name]), name
    finally:
        eng.close()


def test_device_batch_unknown_interface_is_failure():
    """A device batch cannot be checked on the host: an interface id outside
    the engine's ids is a Failure verdict for that connection (never a read
    out of bounds)."""
    import torch
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        ifs, bind, by_name, pool, spec = build(eng, 2, n_local=4, n_if=10)
        n = 4096
        tr = traffic(2, n, pool, spec, 4)
        rng = np.random.default_rng(2)
        si = rng.integers(0, 10, n).astype(np.uint32)
        di = rng.integers(0, 10, n).astype(np.uint32)
        bad = rng.random(n) < 0.1
        si[bad] = 1 << 20
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        si_ok = np.where(bad, 0, si)
        dv = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
              .to("cuda") for x in [np.where(bad, si, ids[si_ok]).astype(np.uint32), ids[di], tr["src"], tr["dst"],
                                    tr["proto"], tr["sport"], tr["dport"]]]
        got = eng.connect_batch(*dv).cpu().numpy()
        assert (got[bad] == 3).all()
        want, _ = oracle_connections(bind, by_name, ifs, si_ok[~bad], di[~bad],
                                     {k: v[~bad] for k, v in tr.items()}, 4)
        assert np.array_equal(got[~bad], want)
    finally:
        eng.close()


@pytest.mark.parametrize("fam", [4, 16])
@pytest.mark.parametrize("count", [False, True])
def test_global_tables_match_oracle(fam, count):
    """The connection kernel with its descriptor and interface tables read
    from global memory (option conn_no_lds bit 2; the default stages them
    in LDS): the same verdicts and counters."""
    from vpp_amd.engine import Engine
    eng = Engine(options={"conn_no_lds": 4})
    try:
        _run(eng, 11, "linear", fam, count=count, n=8000, n_local=12)
    finally:
        eng.close()


@pytest.mark.parametrize("count", [False, True])
def test_device_plan_follows_binding_changes(count):
    """A device batch keeps its plan (descriptors, interface table, rule pool)
    until a table or binding changes (engine.cpp ConnPlan / conn_gen): after
    a replaced ACL, a deleted one, a re-put of equal rules on other
    interfaces (the rebind path) and a new interface, the same device batch
    must follow the new bindings -- verdicts and counters against the
    oracle, before and after."""
    import torch
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        ifs, bind, by_name, pool, spec = build(eng, 3, n_local=16, n_if=40)
        n = 20000
        tr = traffic(3, n, pool, spec, 4)
        rng = np.random.default_rng(3)
        ifs.append("if_new")                               # bound below; its id exists from now on
        bind["if_new"] = [None, None]
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        si = rng.integers(0, len(ifs), n)
        di = np.where(rng.random(n) < 0.1, si, rng.integers(0, len(ifs), n))
        host = [ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"]]
        dv = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
              .to("cuda") for x in host]
        torch.cuda.synchronize()

        def check():
            got = eng.connect_batch(*dv, count=count).cpu().numpy()
            want, wcounts = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (bad[:10], got[bad[:10]], want[bad[:10]])
            if count:
                for name in by_name:
                    c = eng.conn_counters(name, reset=True)
                    assert np.array_equal(c, wcounts[name]), name

        check()
        check()                                            # the kept plan, nothing uploaded
        # replace local0 with other rules on other interfaces
        for i in ifs:
            bind[i] = [None if x == "local0" else x for x in bind[i]]
        rules0, _ = random_acl(7777, 150, weird=0.0)
        assert eng.acl_put("local0", rules0, ["if5", "if_new"], ["if6"]) == 0
        by_name["local0"] = rules0
        bind["if5"][0] = bind["if_new"][0] = "local0"
        bind["if6"][1] = "local0"
        # delete local1
        assert eng.acl_del("local1") == 0
        for i in ifs:
            bind[i] = [None if x == "local1" else x for x in bind[i]]
        del by_name["local1"]
        # re-put local2's rules on other interfaces (same table, new bindings)
        for i in ifs:
            bind[i] = [None if x == "local2" else x for x in bind[i]]
        assert eng.acl_put("local2", by_name["local2"], ["if7"], ["if8", "if_new"]) == 0
        bind["if7"][0] = "local2"
        bind["if8"][1] = bind["if_new"][1] = "local2"
        check()
    finally:
        eng.close()


_Q = {"pair_o4": 0}      # the OTHER queue path, not the four-cell pair image


@pytest.mark.parametrize("opts,cfg", [({}, 2), ({}, 3), ({"conn_pre_rules": 0}, 3), ({"pair_map_lds": 0}, 3),
                                      (_Q, 2), (dict(_Q, pair_other_global=1), 2), (dict(_Q, pair_qcap=3), 2),
                                      (dict(_Q, pair_other_global=1, pair_qcap=0), 2),
                                      (dict(_Q, pair_lq=0), 2), (dict(_Q, pair_lq=2, pair_qcap=4), 2),
                                      (dict(_Q, pair_lq=3), 2),
                                      (_Q, 3), (dict(_Q, pair_other_late=2), 2), (dict(_Q, pair_other_late=2), 3),
                                      (dict(_Q, pair_other_late=2, pair_qcap=3), 3),
                                      (dict(_Q, pair_other_late=2, pair_lq=0), 3), (dict(_Q, pair_class=0), 3),
                                      (dict(_Q, pair_class=0, pair_other_late=2), 3),
                                      (dict(_Q, pair_other_global=1), 3)])
def test_pair_launch_tail_and_other_protocols(opts, cfg, capfd):
    """classify4_pair (k4_pair.hip) on a batch of 4k + 3 connections with
    protocol-47 connections everywhere, the last three included (the scalar
    tail): on the pair image (four cells per class, protocols > 2 with the
    others: the default where it fits and the batch does not count by slot),
    or with the OTHER queue (option pair_o4=0, or a counting batch without
    counter-index words): the OTHER image beside the main one in LDS,
    read from global memory (o_at = 0), or staged over the main image for
    the drain (o_late: the plan when it does not fit beside the main one;
    option pair_other_late=2 forces it), the queued connections carrying
    their source classes (the OTHER image's classes are the main image's)
    or (option pair_class=0) searched again, the OTHER queue roomy or nearly
    full / empty so that connections overflow to in-place classification,
    its entries in LDS, in global memory (option pair_lq=0) or in both.
    Verdicts and counters against orc_test_connection."""
    from vpp_amd.engine import Engine
    eng = Engine(options=dict(opts, debug_conn=1))
    try:
        ifs, bind, by_name, pool, spec = build(eng, 21, n_local=6, n_if=16, cfg=cfg)
        n = 4 * 4000 + 3
        tr = traffic(21, n, pool, spec, 4)
        rng = np.random.default_rng(21)
        other = rng.random(n) < 0.05
        other[-3:] = True
        tr["proto"] = np.where(other, 47, tr["proto"]).astype(np.uint8)
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        si = rng.integers(0, 3, n)                      # the global ACL's interfaces: the pair launch
        di = rng.integers(0, len(ifs), n)
        args = [ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"]]
        got = eng.connect_batch(*args, mode="classifier", count=True)
        want, wcounts = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (bad[:10], got[bad[:10]], want[bad[:10]])
        for name in by_name:
            assert np.array_equal(eng.conn_counters(name, reset=True), wcounts[name]), name
    finally:
        eng.close()
    lines = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("pair:")]
    pimg = [ln for ln in lines if ln.startswith("pair: pimg")]
    pairs = [ln for ln in lines if " o_at " in ln]
    if opts.get("pair_o4", 1) and opts.get("conn_pre_rules", 1):
        assert pimg, lines
        # (counting: the slot -> rule map staged in LDS unless pair_map_lds=0)
        assert any((" map 0 " in ln) == (opts.get("pair_map_lds") == 0) for ln in pimg), pimg
        return
    assert pairs and not pimg, lines
    if opts.get("pair_other_late") == 2:
        assert all(" o_at 0 o_late 1 " in ln for ln in pairs), pairs
    if opts.get("pair_class") == 0:
        assert all(" cdiv 0" in ln for ln in pairs), pairs
    else:
        assert any(" cdiv 0" not in ln for ln in pairs), pairs


def test_conn_counters_do_not_wait_for_other_streams():
    """cls_conn_counters waits for the table's last counting batch (an event),
    not for the device: a long torch kernel on another stream is still
    running when the counters come back, bit-exact."""
    import time

    import torch
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        ifs, bind, by_name, pool, spec = build(eng, 8, n_local=6, n_if=16)
        n = 6000
        tr = traffic(8, n, pool, spec, 4)
        rng = np.random.default_rng(8)
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        si, di = rng.integers(0, len(ifs), n), rng.integers(0, len(ifs), n)
        eng.connect_batch(ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"], count=True)
        _, want = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
        side = torch.cuda.Stream()
        done = torch.cuda.Event()
        with torch.cuda.stream(side):
            torch.cuda._sleep(int(3e9))                 # ~1 s of spinning on `side`
            done.record(side)
        t0 = time.perf_counter()
        got = {name: eng.conn_counters(name) for name in by_name}
        dt = time.perf_counter() - t0
        still = not done.query()
        side.synchronize()
        assert still, "the sleep kernel finished before the counters were read"
        assert dt < 0.5, dt
        for name in by_name:
            assert np.array_equal(got[name], want[name]), name
    finally:
        eng.close()


@pytest.mark.parametrize("no_jobs", ["0", "1"])
@pytest.mark.parametrize("count", [False, True])
def test_ipv4_job_lists_and_shuffles(no_jobs, count):
    """The connection kernel's two ways to hand a wave's jobs to its lanes
    (IPv4): the per-wave job lists in LDS (the default where they fit) and
    the owner search with shuffles (option conn_jobs=0, and launches
    whose LDS is full) -- verdicts and counters against the oracle."""
    from vpp_amd.engine import Engine
    eng = Engine(options={"conn_jobs": 0} if no_jobs == "1" else None)
    try:
        _run(eng, 31, "device_auto", 4, count=count, n=16000, n_local=24)
    finally:
        eng.close()


@pytest.mark.parametrize("words", ["u16", "u32", "slots"])
def test_counted_large_acl_words(words):
    """Counting batches: the pair launch writes each large-ACL word's counter
    index (descriptor base + rule) as u16 words (indices below 2^14) or
    (option conn_pre_narrow=0) u32 words, and the connection kernel adds it
    directly, or (option conn_pre_rules=0) writes slots the kernel maps to
    rules -- per-(ACL, rule) counters against the oracle, protocol-47
    connections included (their OTHER-image slots).  Uncounted batches of the
    same connections (one result byte per connection, or u32 words) give the
    same verdicts."""
    from vpp_amd.engine import Engine
    eng = Engine(options={"u16": {}, "u32": {"conn_pre_narrow": 0}, "slots": {"conn_pre_rules": 0}}[words])
    try:
        ifs, bind, by_name, pool, spec = build(eng, 41, n_local=10, n_if=24)
        n = 4 * 6000 + 1
        tr = traffic(41, n, pool, spec, 4)
        rng = np.random.default_rng(41)
        tr["proto"] = np.where(rng.random(n) < 0.04, 47, tr["proto"]).astype(np.uint8)
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        si = np.where(rng.random(n) < 0.5, rng.integers(0, 3, n), rng.integers(0, len(ifs), n))
        di = rng.integers(0, len(ifs), n)
        got = eng.connect_batch(ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"],
                                mode="classifier", count=True)
        want, wcounts = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
        assert np.array_equal(got, want)
        for name in by_name:
            assert np.array_equal(eng.conn_counters(name, reset=True), wcounts[name]), name
        plain = eng.connect_batch(ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"],
                                  mode="classifier")
        assert np.array_equal(plain, want)
    finally:
        eng.close()


@pytest.mark.parametrize("same_if", [False, True])
def test_counted_batch_beyond_workgroup_bound(same_if):
    """u16 LDS call counters (kConnWgConns connections per workgroup): a
    counted batch of 12 Mi connections -- more than the resident workgroups
    may take, so the launch grows its grid -- counts exactly what the same
    connections count in 4 Mi pieces (counters are linear in the batch).
    same_if: one connection, repeated, from if0 to if0 (inbound and outbound
    ACL the global one): its calls pile onto one or two counters, far past a
    u16 per workgroup without the bound."""
    import torch
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        ifs, bind, by_name, pool, spec = build(eng, 9, n_local=12, cfg=3)
        n, piece = 12 << 20, 4 << 20
        tr = traffic(9, n, pool, spec, 4)
        rng = np.random.default_rng(9)
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        if same_if:
            si = di = np.zeros(n, np.int64)
            tr = {f: np.repeat(v[:1], n, axis=0) for f, v in tr.items()}
        else:
            si, di = rng.integers(0, len(ifs), n), rng.integers(0, len(ifs), n)
        args = [ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"]]
        dv = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
              .to("cuda") for x in args]
        whole = eng.connect_batch(*dv, count=True).cpu().numpy()
        got = {name: eng.conn_counters(name, reset=True) for name in by_name}
        parts = np.concatenate([eng.connect_batch(*[x[a:a + piece] for x in dv], count=True).cpu().numpy()
                                for a in range(0, n, piece)])
        assert np.array_equal(whole, parts)
        total = 0
        for name in by_name:
            want = eng.conn_counters(name, reset=True)
            assert np.array_equal(got[name], want), name
            total += int(want.sum())
        assert total > n // 2
        if same_if:
            assert got["global"].max() >= n              # the first call (src inbound) is always made
    finally:
        eng.close()


@pytest.mark.parametrize("flush", ["rows", "atomic"])
@pytest.mark.parametrize("plan", ["32j", "16j", "32s", "16s"])
def test_counter_widths_and_flush_paths(flush, plan):
    """LDS call counters as u32 or u16 pairs, with job lists (two workgroups
    per CU, the 128-VGPR kernel) or shuffles, leaving the launch as
    per-workgroup rows (summed by the rows launch) or by device atomics into
    the copies of the call counters: per-(ACL, rule) counters against
    orc_test_connection."""
    from vpp_amd.engine import Engine
    eng = Engine(options={"conn_plan": plan, "conn_flush_atomic": int(flush == "atomic")})
    try:
        _run(eng, 21, "device_auto", 4, count=True, n=20000, n_local=12)
    finally:
        eng.close()


@pytest.mark.parametrize("wg768", [1, 0])
def test_counted_768_thread_workgroups(wg768, capfd):
    """The bench's counted plan (config-3 global ACL, 12 local ACLs, seed 0):
    three 512-thread workgroups do not fit the LDS, two 768-thread ones do
    (24 waves per CU, u16 counters, job lists); option conn_wg768=0 keeps the
    512-thread shape.  Verdicts and per-(ACL, rule) counters against
    orc_test_connection either way."""
    from vpp_amd.engine import Engine
    eng = Engine(options={"conn_wg768": wg768, "debug_conn": 1})
    try:
        # (>= kConnClsMinBatch connections: the global ACL on the classifier)
        _run(eng, 0, "device_auto", 4, count=True, n=70000, n_local=12, cfg=3)
    finally:
        eng.close()
    plans = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("connect:") and "cmode 1" in ln]
    assert plans and all(("block 768" in ln) == bool(wg768) for ln in plans), plans


def test_pair_launch_partial_last_step_matches_linear():
    """classify4_pair with two steps per lane, the second taken by a prefix
    of the grid's lanes only, and 5 % protocol-47 connections: the wave's
    OTHER queue fill must come from lane 0 (the lanes past the prefix keep
    stale copies).  Every connection against the pure-scan mode (mode
    "linear", no classifier)."""
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        ifs, bind, by_name, pool, spec = build(eng, 31, n_local=4, n_if=12)
        n = 4 * 256 * 1024 + 4 * 700 + 3
        tr = traffic(31, n, pool, spec, 4)
        rng = np.random.default_rng(31)
        tr["proto"] = np.where(rng.random(n) < 0.05, 47, tr["proto"]).astype(np.uint8)
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        si = rng.integers(0, 3, n)                      # the global ACL's interfaces: the pair launch
        di = rng.integers(0, len(ifs), n)
        args = [ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"]]
        got = eng.connect_batch(*args, mode="classifier")
        want = eng.connect_batch(*args, mode="linear")
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (bad[:10], got[bad[:10]], want[bad[:10]])
    finally:
        eng.close()


@pytest.mark.parametrize("count", [False, True])
def test_two_large_acls(count):
    """Two large ACLs (the config-3 global table and a 3,000-rule random one,
    bound on interfaces of their own, most connections through them): two
    pair-launch blocks, both loaded with the connection's fields (the early
    words, kConnEarlyBlocks), result bytes or counter-index words; verdicts
    and per-(ACL, rule) counters against orc_test_connection."""
    import torch
    from vpp_amd.engine import Engine
    eng = Engine()
    try:
        ifs, bind, by_name, pool, spec = build(eng, 13, n_local=6, n_if=20, cfg=3)
        big2, _ = random_acl(4242, 3000, 0.0)
        assert eng.acl_put("big2", big2, ["bx0", "bx1"], ["bx1", "bx2"]) == 0
        by_name["big2"] = big2
        ifs = ifs + ["bx0", "bx1", "bx2"]
        bind.update({"bx0": ["big2", None], "bx1": ["big2", "big2"], "bx2": [None, "big2"]})
        n = 24000
        tr = traffic(13, n, pool, spec, 4)
        rng = np.random.default_rng(13)
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        hot = np.array([0, 1, 2, len(ifs) - 3, len(ifs) - 2, len(ifs) - 1])   # the two large ACLs' interfaces
        si = np.where(rng.random(n) < 0.6, rng.choice(hot, n), rng.integers(0, len(ifs), n))
        di = np.where(rng.random(n) < 0.6, rng.choice(hot, n), rng.integers(0, len(ifs), n))
        args = [ids[si], ids[di], tr["src"], tr["dst"], tr["proto"], tr["sport"], tr["dport"]]
        dv = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
              .to("cuda") for x in args]
        got = eng.connect_batch(*dv, count=count).cpu().numpy()
        want, wcounts = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
        assert np.array_equal(got, want)
        if count:
            for name in by_name:
                assert np.array_equal(eng.conn_counters(name, reset=True), wcounts[name]), name
            assert wcounts["big2"].sum() > 1000 and wcounts["global"].sum() > 1000
    finally:
        eng.close()


def test_device_batch_out_tensor():
    """connect_batch(out=...) writes the verdicts into the caller's tensor
    (the same values as a fresh one) and refuses a wrong one."""
    import torch
    from vpp_amd.engine import Engine
    from vpp_amd._abi import ClsError
    eng = Engine()
    try:
        ifs, bind, by_name, pool, spec = build(eng, 17, n_local=4, n_if=10)
        n = 9001
        tr = traffic(17, n, pool, spec, 4)
        rng = np.random.default_rng(17)
        ids = np.array([eng.if_id(x) for x in ifs], np.uint32)
        args = [ids[rng.integers(0, len(ifs), n)], ids[rng.integers(0, len(ifs), n)], tr["src"], tr["dst"],
                tr["proto"], tr["sport"], tr["dport"]]
        dv = [torch.from_numpy(np.ascontiguousarray(x).view({4: np.int32, 2: np.int16, 1: np.uint8}[x.dtype.itemsize]))
              .to("cuda") for x in args]
        fresh = eng.connect_batch(*dv)
        out = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        got = eng.connect_batch(*dv, out=out)
        assert got.data_ptr() == out.data_ptr()
        assert torch.equal(out, fresh)
        with pytest.raises(ClsError):
            eng.connect_batch(*dv, out=torch.empty(n - 1, dtype=torch.uint8, device="cuda"))
    finally:
        eng.close()
