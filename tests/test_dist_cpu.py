"""N>1 path on CPU (gloo, world_size 2): contiguous packet shards per rank and
the integer all-reduce of hit counters reproduce the single-process counters
of the whole stream.  The per-rank classifier here is the oracle (no GPU on
the CPU runner); the GPU ranks run the same vpp_amd.dist code with RCCL."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import os, sys
    sys.path[:0] = [%(root)r]
    import numpy as np, torch
    import oracle
    from vpp_amd import dist as D, workload
    D.init("gloo")
    rank, size, _ = D.world()
    acl, spec, _ = workload.config(2)
    first, n = D.shard(rank, 3000)
    tr = oracle.gen_traffic_v4(spec, first, n)
    _, c = oracle.classify_fast(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    t = torch.from_numpy(c.astype(np.int64))
    D.merge_counters(t)
    if rank == 0:
        np.save(%(out)r, t.numpy())
    torch.distributed.destroy_process_group()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_counter_allreduce(tmp_path):
    import oracle
    from vpp_amd import workload
    out = str(tmp_path / "c.npy")
    script = tmp_path / "w.py"
    script.write_text(WORKER % {"root": ROOT, "out": out})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), str(script)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    merged = np.load(out)
    acl, spec, _ = workload.config(2)
    tr = oracle.gen_traffic_v4(spec, 0, 6000)
    _, full = oracle.classify_fast(oracle.rules_to_c(acl.rules), tr["src"], tr["dst"], tr["dport"], tr["proto"])
    np.testing.assert_array_equal(merged, full.astype(np.int64))
    assert merged.sum() == 6000
