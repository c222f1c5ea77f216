"""The HBM-resident path through the C ABI alone: engine-owned batches,
multi-device engines and the in-library RCCL counter all-reduce
(include/contivcls.h ABI 4; SURVEY 8(b) ownership, 8(e) sharding).

- tools/native_c3.py runs config 3 at 256 Mi packets in a child process that
  never imports torch (the cgo host's view of the library): 64 verdict
  windows bit-exact against the oracle, the batch path's kernel time within
  2 % of the raw-pointer cls_classify on the same arrays, the counters sum to
  the batch.
- A one-device engine with cls_comm_init (an RCCL group of one): counters
  merged by ncclAllReduce, bit-exact against the oracle.
- Eight shards on the one GPU of the box (a device list repeating device 0:
  eight peer engines, no communicator, host-summed counters): tables compiled
  once and replicated to every shard's engine, verdicts and counters equal to
  one device's and to the oracle's, on a ragged batch.
- Uploads (pinned mirror, staged from pageable memory in several 32 MiB
  chunks) and downloads round-trip; connection batches sharded over eight
  shards equal the oracle's testConnection, and their counters the oracle's.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from vpp_amd import _abi, workload
from vpp_amd.engine import Engine

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle(acl, tr, af=4):
    return oracle.classify_fast(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"], af=af)


def test_config3_256mi_through_the_abi_alone_without_torch():
    env = dict(os.environ, CONTIVCLS_NO_TORCH="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "native_c3.py"), "--steps", "20",
                        "--warmup", "10", "--windows", "64"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    print(out)
    assert out["torch_imported"] is False
    assert out["packets"] == 1 << 28 and out["rules"] > 9000
    assert out["windows"] == 64 and out["window_mismatches"] == 0
    assert out["counter_sum"] == out["packets"]
    k, raw = out["ab_batch_kernel_ms_avg"], out["raw_kernel_ms_avg"]
    assert abs(k - raw) <= 0.02 * raw, (k, raw)


def test_rccl_group_of_one_counters_bit_exact():
    acl, spec, _ = workload.config(2)
    n = (1 << 20) + 7
    eng = Engine(0)
    eng.comm_init()
    assert eng.comm_info() == (1, 0)
    t = eng.put_table("c2", acl.rules)
    b = eng.batch(n)
    b.gen_traffic(spec, 5)
    c1 = eng.classify_batch(t, b)
    c2 = eng.classify_batch(t, b)           # the other counter buffer
    tr = oracle.gen_traffic_v4(spec, 5, n)
    ov, oc = _oracle(acl, tr)
    assert np.array_equal(c1, oc) and np.array_equal(c2, oc)
    assert np.array_equal(b.download(_abi.BF_VERDICT), ov)
    # async calls: counters of the last one, read later
    for _ in range(5):
        assert eng.classify_batch(t, b, counters=False) is None
    assert np.array_equal(b.counters(t.n_rules), oc)
    b.close()
    eng.close()


def test_eight_shards_replicate_tables_and_merge_counters():
    acl, spec, _ = workload.config(2)
    n = 3 * (1 << 20) + 13                 # ragged: shards of unequal size, tails not multiples of 4
    multi = Engine(devices=[0] * 8)
    assert multi.n_devices() == 8
    assert multi.comm_info() == (0, 0)      # a repeated device: no communicator, host-summed counters
    t = multi.put_table("c2", acl.rules)
    infos = [multi.device_engine(g) for g in range(8)]
    from vpp_amd.engine import Table
    ref_info = t.info()
    for v in infos:                          # the same table id on every shard's engine, same compiled form
        assert Table(v, t.id, t.n_rules, "c2").info() == ref_info
    # configuration goes through the primary only
    with pytest.raises(_abi.ClsError):
        infos[3].put_table("x", acl.rules[:3])
    b = multi.batch(n)
    sh = b.shards()
    assert [s[1] for s in sh] == [g * n // 8 for g in range(8)] and sum(s[2] for s in sh) == n
    b.gen_traffic(spec, 0)
    cm = multi.classify_batch(t, b)
    single = Engine(0)
    ts = single.put_table("c2", acl.rules)
    bs = single.batch(n)
    bs.gen_traffic(spec, 0)
    cs = single.classify_batch(ts, bs)
    assert np.array_equal(cm, cs)
    vm = b.download(_abi.BF_VERDICT)
    assert np.array_equal(vm, bs.download(_abi.BF_VERDICT))
    sample = np.arange(0, n, 97)
    tr = oracle.gen_traffic_v4(spec, 0, n)
    ov, oc = _oracle(acl, tr)
    assert np.array_equal(cm, oc)
    assert np.array_equal(vm[sample], ov[sample]) and np.array_equal(vm, ov)
    # a table deleted on the primary is gone from every shard
    multi.del_table(t)
    for v in infos:
        with pytest.raises(_abi.ClsError):
            Table(v, t.id, t.n_rules, "c2").info()
    for x in (b, bs):
        x.close()
    multi.close()
    single.close()


def test_mirror_and_staged_upload_round_trip():
    acl, spec, _ = workload.config(2)
    n = (9 << 20) + 3                      # 36 MiB of addresses: two staging chunks
    tr = oracle.gen_traffic_v4(spec, 11, n)
    ov, oc = _oracle(acl, tr)
    eng = Engine(devices=[0, 0])
    t = eng.put_table("c2", acl.rules)
    # staged from pageable numpy
    b = eng.batch(n)
    for f, k in ((_abi.BF_SRC, "src"), (_abi.BF_DST, "dst"), (_abi.BF_DPORT, "dport"), (_abi.BF_PROTO, "proto")):
        b.upload(f, tr[k])
    assert np.array_equal(eng.classify_batch(t, b), oc)
    assert np.array_equal(b.download(_abi.BF_VERDICT), ov)
    assert np.array_equal(b.download(_abi.BF_SRC, 1000, 5000), tr["src"][1000:6000])
    # the pinned mirror: fill in place, upload, classify, download into it
    m = eng.batch(n, mirror=True)
    for f, k in ((_abi.BF_SRC, "src"), (_abi.BF_DST, "dst"), (_abi.BF_DPORT, "dport"), (_abi.BF_PROTO, "proto")):
        m.mirror(f)[:] = tr[k]
        m.upload(f)
    assert np.array_equal(eng.classify_batch(t, m), oc)
    m.download(_abi.BF_VERDICT, mirror=True)
    assert np.array_equal(m.mirror(_abi.BF_VERDICT), ov)
    for x in (b, m):
        x.close()
    eng.close()


def test_sharded_connection_batch_matches_oracle():
    from test_gpu_connect_scale import build, oracle_connections, traffic
    multi = Engine(devices=[0] * 4)
    ifs, bind, by_name, pool, spec = build(multi, seed=3, n_local=24, n_if=40)
    n = 20003
    rng = np.random.default_rng(9)
    tr = traffic(3, n, pool, spec, 4)
    si = rng.integers(0, len(ifs), n).astype(np.uint32)
    di = np.where(rng.random(n) < 0.1, si, rng.integers(0, len(ifs), n)).astype(np.uint32)
    ids = np.array([multi.if_id(x) for x in ifs], np.uint32)
    b = multi.batch(n, conn=True)
    for f, v in ((_abi.BF_SRC, tr["src"]), (_abi.BF_DST, tr["dst"]), (_abi.BF_SPORT, tr["sport"]),
                 (_abi.BF_DPORT, tr["dport"]), (_abi.BF_PROTO, tr["proto"]), (_abi.BF_SRC_IF, ids[si]),
                 (_abi.BF_DST_IF, ids[di])):
        b.upload(f, v)
    want, counts = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
    for mode in ("auto", "classifier", "linear"):
        multi.connect_batch_b(b, mode=mode, count=(mode == "classifier"))
        assert np.array_equal(b.download(_abi.BF_VERDICT), want), mode
    for name in by_name:                     # counted once (classifier mode): summed over the four shards
        got = multi.conn_counters(name)
        assert np.array_equal(got, counts[name]), name
    b.close()
    multi.close()


def _gpu_count():
    import torch                            # counting devices does not initialise HIP on this image
    return torch.cuda.device_count()


@pytest.mark.skipif(_gpu_count() < 2, reason="needs two GPUs (distinct devices: an RCCL communicator)")
def test_two_distinct_devices_all_reduce_counters():
    """Two distinct devices: the engine builds an ncclCommInitAll
    communicator (comm_info == (2, 0)), replicates the table, shards the
    batch, and the RCCL all-reduce of the hit counters equals the oracle's,
    as do the verdicts of both shards and a sharded connection batch."""
    acl, spec, _ = workload.config(2)
    n = (2 << 20) + 5
    multi = Engine(devices=[0, 1])
    assert multi.n_devices() == 2
    assert multi.comm_info() == (2, 0), multi.comm_info()
    t = multi.put_table("c2", acl.rules)
    b = multi.batch(n)
    b.gen_traffic(spec, 11)
    c = multi.classify_batch(t, b)
    tr = oracle.gen_traffic_v4(spec, 11, n)
    ov, oc = _oracle(acl, tr)
    assert np.array_equal(c, oc)
    assert np.array_equal(b.download(_abi.BF_VERDICT), ov)
    # async: counters of the last call, read later (the all-reduce on its side stream)
    for _ in range(3):
        assert multi.classify_batch(t, b, counters=False) is None
    assert np.array_equal(b.counters(t.n_rules), oc)
    b.close()
    multi.close()


@pytest.mark.skipif(_gpu_count() < 2, reason="needs two GPUs (distinct devices: peer table uploads)")
def test_two_distinct_devices_connection_batch_counted():
    """A counted connection batch sharded over two distinct devices: the
    tables uploaded to the second GPU, both shards' verdicts and the
    per-(ACL, rule) counters summed over the devices equal the oracle's."""
    from test_gpu_connect_scale import build, oracle_connections, traffic
    multi = Engine(devices=[0, 1])
    ifs, bind, by_name, pool, spec = build(multi, seed=5, n_local=16, n_if=32)
    n = 30011
    rng = np.random.default_rng(13)
    tr = traffic(5, n, pool, spec, 4)
    si = rng.integers(0, len(ifs), n).astype(np.uint32)
    di = np.where(rng.random(n) < 0.1, si, rng.integers(0, len(ifs), n)).astype(np.uint32)
    ids = np.array([multi.if_id(x) for x in ifs], np.uint32)
    b = multi.batch(n, conn=True)
    for f, v in ((_abi.BF_SRC, tr["src"]), (_abi.BF_DST, tr["dst"]), (_abi.BF_SPORT, tr["sport"]),
                 (_abi.BF_DPORT, tr["dport"]), (_abi.BF_PROTO, tr["proto"]), (_abi.BF_SRC_IF, ids[si]),
                 (_abi.BF_DST_IF, ids[di])):
        b.upload(f, v)
    want, counts = oracle_connections(bind, by_name, ifs, si, di, tr, 4)
    multi.connect_batch_b(b, count=True)
    assert np.array_equal(b.download(_abi.BF_VERDICT), want)
    for name in by_name:
        assert np.array_equal(multi.conn_counters(name), counts[name]), name
    b.close()
    multi.close()
