"""N>1 on the GPU: two ranks on the box's GPU, each running the HIP engine on
its contiguous shard of the config-3 stream; the counters are
merged with the same vpp_amd.dist code bench.py uses (gloo here: RCCL refuses
two ranks on one device, and the driver's 8-GPU run uses RCCL).  The merged
counters and the per-shard verdicts must equal the oracle's over the whole
stream.  Also: bench.py --gpus 2 launches its own ranks and reports n_gpus 2,
on the product path (the C ABI alone; two ranks sharing the box's GPU sum
their counters over gloo) and on the torch harness (--torch).
"""
import json
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

WORKER = textwrap.dedent("""
    import os, sys
    sys.path[:0] = [%(root)r]
    import numpy as np, torch
    import torch.distributed as dist
    from vpp_amd import dist as D, workload
    from vpp_amd.engine import Engine
    D.init("gloo")
    rank, size, local = D.world()
    torch.cuda.set_device(D.device_index(local))
    acl, spec, _ = workload.config(3)
    eng = Engine(torch.cuda.current_device())
    t = eng.put_table("g", acl.rules)
    n = %(n)d
    first, _ = D.shard(rank, n)
    pk = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
          (("src", torch.int32), ("dst", torch.int32), ("dport", torch.int16), ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, first, pk)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    c = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
    eng.classify(t, pk["src"], pk["dst"], pk["dport"], pk["proto"], verdict=v, counters=c)
    D.merge_counters(c)
    torch.cuda.synchronize()
    parts = [torch.empty(n, dtype=torch.uint8) for _ in range(size)]
    dist.all_gather(parts, v.cpu())
    if rank == 0:
        np.save(%(out)r + ".c.npy", c.cpu().numpy())
        np.save(%(out)r + ".v.npy", torch.cat(parts).numpy())
    eng.close()
    dist.destroy_process_group()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_hip_engine(tmp_path):
    import oracle
    from vpp_amd import workload
    n = 1 << 20
    out = str(tmp_path / "r")
    script = tmp_path / "w.py"
    script.write_text(WORKER % {"root": ROOT, "out": out, "n": n})
    env = dict(os.environ, VPP_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), str(script)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    merged, verdict = np.load(out + ".c.npy"), np.load(out + ".v.npy")
    acl, spec, _ = workload.config(3)
    tr = oracle.gen_traffic_v4(spec, 0, 2 * n)
    ov, oc = oracle.classify_fast(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    np.testing.assert_array_equal(verdict, ov)
    np.testing.assert_array_equal(merged, oc.astype(np.int64))
    assert merged.sum() == 2 * n


def test_bench_native_two_ranks_one_gpu(tmp_path):
    """bench.py --gpus 2 (the product path, its default): the launcher, the
    ranks' stream offsets (rank r classifies packets [r n, (r+1) n)), one
    engine-owned batch per rank, and the counters merged over the ranks --
    here summed over gloo, because both ranks share the box's one GPU (RCCL
    needs one rank per device; the driver's 8-GPU run takes cls_comm_init and
    the library's ncclAllReduce).  Every rank's verdicts and the merged
    counters equal the oracle's over the whole 2 n-packet stream."""
    import oracle
    from vpp_amd import workload
    n = 1 << 20
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    d = str(tmp_path / "dump")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--settle-ms", "20", "--packets", str(n), "--cpu-sample", "0", "--no-stream-floor", "--dump", d]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["counters_sum_ok"] is True
    assert line["config"]["path"].startswith("native")
    assert "gloo" in line["config"]["collective"]
    acl, spec, _ = workload.config(3)
    tr = oracle.gen_traffic_v4(spec, 0, 2 * n)
    ov, oc = oracle.classify_fast(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    verdict = np.concatenate([np.load(os.path.join(d, "verdict_r%d.npy" % k)) for k in range(2)])
    np.testing.assert_array_equal(verdict, ov)
    np.testing.assert_array_equal(np.load(os.path.join(d, "counters.npy")), oc.astype(np.uint64))


def test_bench_launches_its_ranks():
    env = dict(os.environ, VPP_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--packets", str(1 << 22), "--cpu-sample", "0", "--no-stream-floor", "--torch"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["packets_per_gpu"] == 1 << 22
    assert line["roofline"]["allreduce_ms_avg_max_rank"] is not None


RCCL_WORKER = textwrap.dedent("""
    import os, sys
    sys.path[:0] = [%(root)r]
    import numpy as np, torch
    import torch.distributed as dist
    from vpp_amd import dist as D, workload
    from vpp_amd.engine import Engine
    D.init("nccl")                      # RCCL; a 1-rank group under torch.distributed.run
    assert D.backend() == "nccl", D.backend()
    rank, size, local = D.world()
    torch.cuda.set_device(D.device_index(local))
    acl, spec, _ = workload.config(3)
    eng = Engine(torch.cuda.current_device())
    t = eng.put_table("g", acl.rules)
    n = %(n)d
    first, _ = D.shard(rank, n)
    pk = {k: torch.empty(n, dtype=dt, device="cuda") for k, dt in
          (("src", torch.int32), ("dst", torch.int32), ("dport", torch.int16), ("proto", torch.uint8))}
    eng.gen_traffic_v4(spec, first, pk)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    c = torch.zeros(t.n_rules + 1, dtype=torch.int64, device="cuda")
    eng.classify(t, pk["src"], pk["dst"], pk["dport"], pk["proto"], verdict=v, counters=c)
    side = torch.cuda.Stream()
    done = torch.cuda.Event()
    done.record()
    with torch.cuda.stream(side):       # the overlapped form bench.py uses
        side.wait_event(done)
        D.merge_counters(c)             # int64 SUM in HBM over RCCL
    torch.cuda.synchronize()
    mx = D.max_over_ranks([1.5 + rank, -2.0], torch.device("cuda", torch.cuda.current_device()))
    assert mx == [1.5 + size - 1, -2.0], mx
    np.save(%(out)r + ".c.npy", c.cpu().numpy())
    np.save(%(out)r + ".v.npy", v.cpu().numpy())
    eng.close()
    dist.destroy_process_group()
""")


def test_rccl_counter_allreduce_one_rank(tmp_path):
    """The RCCL branch itself: a 1-rank nccl group (torch.distributed.run
    --nproc-per-node 1), counters merged on device (int64 SUM) from a side
    stream, max_over_ranks on device float64; counters equal the oracle's."""
    import oracle
    from vpp_amd import workload
    n = 1 << 20
    out = str(tmp_path / "r")
    script = tmp_path / "w.py"
    script.write_text(RCCL_WORKER % {"root": ROOT, "out": out, "n": n})
    env = dict(os.environ)
    env.pop("VPP_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), str(script)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    merged, verdict = np.load(out + ".c.npy"), np.load(out + ".v.npy")
    acl, spec, _ = workload.config(3)
    tr = oracle.gen_traffic_v4(spec, 0, n)
    ov, oc = oracle.classify_fast(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    np.testing.assert_array_equal(verdict, ov)
    np.testing.assert_array_equal(merged, oc.astype(np.int64))


def test_bench_rccl_overlapped_allreduce_one_rank():
    """bench.py under torch.distributed.run with one rank: the counter
    all-reduce runs over RCCL on the side stream and is timed."""
    env = dict(os.environ)
    env.pop("VPP_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "8", "--warmup", "2", "--settle-ms", "20", "--packets", str(1 << 24),
           "--cpu-sample", "0", "--no-stream-floor", "--torch"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert "nccl" in line["config"]["collective"]
    assert line["roofline"]["allreduce_ms_avg_max_rank"] > 0
    assert line["roofline"]["allreduce_ms_median_max_rank"] > 0
    assert line["settle_ms"] >= 20


def test_bench_native_rccl_one_rank():
    """bench.py (the product path) under torch.distributed.run with one rank:
    the rank joins an RCCL communicator through cls_comm_init (rank 0's
    unique id over gloo) and every step's counters are merged by the
    library's ncclAllReduce on its side stream -- the path an 8-GPU run
    takes, at one rank."""
    env = dict(os.environ)
    env.pop("VPP_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "8", "--warmup", "2", "--settle-ms", "20", "--packets", str(1 << 24),
           "--cpu-sample", "0", "--no-stream-floor"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert "ncclAllReduce" in line["config"]["collective"] and line["counters_sum_ok"] is True
