#!/usr/bin/env python3
"""Benchmark: Mpps classified at 10k ACL rules per MI355X, and % of HBM roofline.

Workload (BASELINE.json configs[2]): the ~10k-rule
global ACL of a 1000-pod render (vpp_amd/workload.py), 256 Mi synthetic IPv4
TCP/UDP packets per GPU generated in HBM by the splitmix64 stream (seed
0xC0175EED03, rank r generates packets [r*N, (r+1)*N)).  A step = one
classify pass over the batch (verdict per packet + per-rule hit counters),
plus, at N>1 GPUs, the RCCL all-reduce of the hit counters (the only
collective: packets shard across ranks, the table is replicated).

Config 4 (--config 4): the config 3 table over a fixed 2 Gi-packet batch,
sharded contiguously over the ranks (strong scaling, 2 Gi / N per GPU).  The
default run is weak: 256 Mi packets per GPU, so N = 8 classifies config 4's
2 Gi packets.

The measured path is the product's (main_native): the C ABI alone -- an
engine-owned batch in HBM, cls_classify_batch, and at N>1 the library's own
ncclAllReduce of the hit counters (cls_comm_init) -- with torch only as the
launcher's control plane (a gloo group for the RCCL id, barriers and
max-over-ranks), never on the GPU.  --torch runs the same step through the
torch harness instead (torch tensors and streams, torch.distributed's
all-reduce).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
N>1: one rank per GPU.  Under torch.distributed.run (WORLD_SIZE set) the
ranks run directly; otherwise bench.py starts torch.distributed.run itself as
a child process, before anything touches the GPU, and exits with its status.
Ranks sharing a GPU (fewer devices than ranks: a rehearsal on a one-GPU box)
run without an RCCL communicator -- RCCL needs one rank per device -- and
sum their counters over the gloo group.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_PKT = {4: 12,         # src 4 + dst 4 + dport 2 + proto 1 + verdict 1
                 16: 36}        # 16-byte layout (config 5): src 16 + dst 16 + 2 + 1 + 1


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=25, help="untimed steps after the settle phase")
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed steps first, for at least this much wall time: the GPU clocks settle "
                         "over the first ~10 ms of work, whatever --warmup is")
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 4, 5])
    ap.add_argument("--packets", type=int, default=0, help="packets per GPU (default: config's)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 21,
                    help="packets timed on the host for the CPU baseline (0: skip)")
    ap.add_argument("--faithful-sample", type=int, default=4096)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: every core this process may use)")
    ap.add_argument("--no-stream-floor", action="store_true", help="skip the live stream-floor measurement")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option key=value (cls_engine_set_option; A/B measurements)")
    ap.add_argument("--torch", action="store_true",
                    help="the torch harness instead of the product path: torch tensors and streams on the GPU, "
                         "counters merged by torch.distributed (the default, main_native, is the C ABI alone: "
                         "cls_batch_*, cls_classify_batch and the library's RCCL all-reduce)")
    ap.add_argument("--native", action="store_true", help="(the default) the product path through the C ABI")
    ap.add_argument("--dump", default="",
                    help="tests: directory for every rank's verdicts (verdict_r<rank>.npy) and the merged "
                         "counters (counters.npy, rank 0)")
    ap.add_argument("--events", type=int, default=1, choices=[0, 1, 2],
                    help="1 (the reported line): the classify kernels stamp their own start/end events "
                         "(hipExtLaunchKernel; the step period is start-to-start); diagnostics: 2 adds an "
                         "event record at each step boundary, 0 times nothing (wall time only)")
    ap.add_argument("--event-every", type=int, default=4,
                    help="native path: the timing events on every n-th step of the timed region (a timed "
                         "launch costs the stream ~4 us: config 2 0.0437 against 0.0397 ms per step with none)")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """--gpus N > 1 without a launcher: run torch.distributed.run as a child
    (this process has not touched the GPU) and return its exit status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def cpu_share() -> int:
    """Cores this process may use: its affinity mask, capped by a cgroup CPU
    quota (a GPU box shows every host core but grants a share of them)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def host_cpu():
    """(logical cores, model name) of the host (lscpu's 'Model name')."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count() or 1, model


def cpu_baseline(acl, spec, sample: int, faithful_sample: int, threads: int = 0):
    """Oracle CPU port on the host cores (OpenMP over every core this process
    may use -- affinity and cgroup quota -- unless --cpu-threads says
    otherwise), and the faithful Go-style evaluator (string re-parse per rule,
    one thread) on a smaller prefix."""
    import oracle
    nproc, model = host_cpu()
    threads = threads or cpu_share()
    af = spec.get("layout", 4)
    tr = (oracle.gen_traffic_v16 if af == 16 else oracle.gen_traffic_v4)(spec, 0, sample)
    cr = oracle.rules_to_c(acl.rules)
    ft = oracle.FastTable(cr)
    ft.classify(tr["src"][:1024], tr["dst"][:1024], tr["dport"][:1024], tr["proto"][:1024],
                af=af, nthreads=threads)
    t0 = time.perf_counter()
    ft.classify(tr["src"], tr["dst"], tr["dport"], tr["proto"], af=af, nthreads=threads)
    dt = time.perf_counter() - t0
    out = {"value": round(sample / dt / 1e6, 4), "unit": "Mpps", "cores": threads, "kind": "port",
           "nproc": nproc, "cpu_share": cpu_share(), "cpu_model": model,
           "sample": "%d packets of the same config stream (oracle/aclengine_ref.c orc_classify_fast, "
                     "rules pre-parsed, OpenMP %d threads), %.1f s" % (sample, threads, dt)}
    if faithful_sample:
        f = {k: v[:faithful_sample] for k, v in tr.items()}
        t0 = time.perf_counter()
        oracle.classify_faithful(cr, f["src"], f["dst"], f["dport"], f["proto"], af=af)
        dt2 = time.perf_counter() - t0
        out["faithful"] = {"value": round(faithful_sample / dt2 / 1e6, 6), "unit": "Mpps", "cores": 1,
                           "sample": "%d packets, evalACL restated literally (CIDR strings re-parsed "
                                     "per rule per packet, aclengine_mock.go:500,514), %.1f s"
                                     % (faithful_sample, dt2)}
    return out


def pmc_traffic(cfg: int, n: int):
    """Per-launch HBM bytes of the classify kernel from the committed rocprofv3
    PMC summary (profiles/pmc_*.json, written by tools/pmc_traffic.py on the
    GPU box).  Only a summary measured on the current kernel sources counts:
    each records the hash of vpp_amd/csrc, and a stale one is dropped.
    Returns (bytes or None, source note)."""
    import glob
    from vpp_amd._abi import source_hash
    h = source_hash()
    best, stale = None, None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("config") == cfg and d.get("packets") == n:
            if d.get("source_hash") == h:
                best = (d, os.path.relpath(p, ROOT))
            else:
                stale = os.path.relpath(p, ROOT)
    if best is None:
        return None, ("no PMC summary for these kernel sources (stale: %s)" % stale) if stale else "not measured"
    d, p = best
    return d.get("hbm_bytes_per_launch"), "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, %s" % p


def main():
    args = parse()
    rank, world, local = (int(os.environ.get(k, d)) for k, d in
                          (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))          # nothing has touched the GPU in this process
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if not args.torch:
        return main_native(args, rank, world, local)
    # under torch.distributed.run (also with one rank) the counters are merged
    # by a real collective; a plain N=1 run has no process group
    import torch
    import torch.distributed as dist

    from vpp_amd import dist as D
    from vpp_amd import workload
    D.init("nccl")
    torch.cuda.set_device(D.device_index(local))
    from vpp_amd.engine import Engine

    acl, spec, n_default = workload.config(args.config)
    strong = args.config == 4
    if args.packets:
        n = args.packets
    elif strong:
        n = -(-n_default // world)            # config 4: the fixed batch over the ranks
    else:
        n = n_default
    eng = Engine(torch.cuda.current_device(), options=dict(o.split("=", 1) for o in args.opt))
    table = eng.put_table("contiv/vpp-policy-GLOBAL", acl.rules)
    info = table.info()
    R = table.n_rules

    dev = torch.device("cuda", torch.cuda.current_device())
    af = spec.get("layout", 4)
    shape = (n, 16) if af == 16 else (n,)
    adt = torch.uint8 if af == 16 else torch.int32
    pk = {k: torch.empty(shape if k in ("src", "dst") else (n,), dtype=dt, device=dev) for k, dt in
          (("src", adt), ("dst", adt), ("dport", torch.int16), ("proto", torch.uint8))}
    first, _ = D.shard(rank, n)
    (eng.gen_traffic_v16 if af == 16 else eng.gen_traffic_v4)(spec, first, pk)
    verdict = torch.empty(n, dtype=torch.uint8, device=dev)
    # The counter all-reduce (the only collective, whenever a process group
    # exists -- also a 1-rank RCCL group under torch.distributed.run) runs on
    # a side stream behind an event, so step i's all-reduce overlaps step
    # i+1's classify; the counter buffers alternate, and a buffer is written
    # again only after its previous all-reduce (event) has finished.
    coll = dist.is_initialized()
    nbuf = 2 if coll else 1
    counters = [torch.zeros(R + 1, dtype=torch.int64, device=dev) for _ in range(nbuf)]
    side = torch.cuda.Stream(device=dev) if coll else None
    reduced = [None] * nbuf                   # event after the last all-reduce of each buffer
    ev = []                                   # (before, after) the counter all-reduce, per timed step
    sev = []                                  # one event at the start of each timed step (and one after the last)
    torch.cuda.synchronize()

    # Every step runs on one explicit stream (`main`): the engine launches on
    # torch's current stream, so the step events and the all-reduce's wait
    # event bracket the classify itself.
    main = torch.cuda.Stream(device=dev)
    sev_pool = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]

    def step(i, timing):
        b = i % nbuf
        if timing and args.events >= 2:
            # step boundaries: one event per step (step i = boundary i to i + 1),
            # each event record costs the stream a few microseconds; the events
            # are created before the timed loop (no allocation inside it)
            s0 = sev_pool[len(sev)]
            s0.record(main)
            sev.append(s0)
        if reduced[b] is not None:
            main.wait_event(reduced[b])
        eng.classify(table, pk["src"], pk["dst"], pk["dport"], pk["proto"], verdict=verdict,
                     counters=counters[b], timing=timing and args.events >= 1, stream=main)
        if coll:
            done = torch.cuda.Event()
            done.record(main)
            with torch.cuda.stream(side):
                side.wait_event(done)
                if timing:
                    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(side)
                D.merge_counters(counters[b])     # RCCL over xGMI: merge per-rule hit counters
                if timing:
                    z.record(side)
                    ev.append((a, z))
                r = torch.cuda.Event()
                r.record(side)
                reduced[b] = r

    # Settle the clocks independently of --warmup: untimed steps for at least
    # --settle-ms of wall time with the GPU busy (the first ~10 ms of work run
    # at lower clocks), then the counted warm-up steps.  Steps go in rounds
    # of 8, and every rank runs the same rounds (each step may hold a
    # collective): another round while any rank is short of the time.
    i = 0
    t_settle = time.perf_counter()
    while True:
        for _ in range(8):
            step(i, False)
            i += 1
        torch.cuda.synchronize()
        short = (time.perf_counter() - t_settle) * 1e3 < args.settle_ms
        if not D.max_over_ranks(1.0 if short else 0.0, dev):
            break
    settle_ms = (time.perf_counter() - t_settle) * 1e3
    for _ in range(args.warmup):
        step(i, False)
        i += 1
    torch.cuda.synchronize()
    eng.kernel_times(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(i, True)
        i += 1
    t_submit = time.perf_counter() - t0      # host time to enqueue the timed steps
    if sev:
        last = sev_pool[len(sev)]
        last.record(main)
        sev.append(last)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    kms, starts = eng.kernel_times(reset=True, starts=True)
    avg_k = float(np.mean(kms)) if kms else float("nan")
    med_k = float(np.median(kms)) if kms else float("nan")
    # the step period: between step-boundary events (--events 2), else between
    # the classify kernels' own start stamps
    periods = ([a.elapsed_time(b) for a, b in zip(sev, sev[1:])] if len(sev) > 1
               else list(np.diff(starts)) if len(starts) > 1 else [])
    med_step = float(np.median(periods)) if periods else float("nan")
    ar = [a.elapsed_time(b) for a, b in ev]
    ar_ms = float(np.mean(ar)) if ar else 0.0
    ar_med = float(np.median(ar)) if ar else 0.0
    floor_ms = shape_ms = None
    shapes = []
    lds = info["lds_bytes"] if af == 4 else info["lds_bytes_v16"]
    resident = info["lds_resident"] if af == 4 else info["lds_resident_v16"]
    two_per_cu = not resident or 2 * (lds + 16) <= 160 * 1024     # the classify launch's workgroups per CU
    if not args.no_stream_floor:
        # one launch covers at most 2^30 packets (the kernels' 32-bit offsets):
        # time the floor on that prefix and scale to the batch
        m = min(n, 1 << 30)
        shapes = [t * (n / m) for t in eng.stream_floor_shapes(pk["src"][:m], pk["dst"][:m], pk["dport"][:m],
                                                              pk["proto"][:m], verdict[:m])]
        floor_ms = min(shapes)
        # the fastest shape with the classify launch's workgroups per CU (the
        # kernel cannot take the other: its LDS image allows one per CU)
        shape_ms = min(t for i, t in enumerate(shapes) if (i & 1) == int(two_per_cu) or len(shapes) < 2)
    wall, k_max, kmed_max, ar_max, armed_max = D.max_over_ranks([wall, avg_k, med_k, ar_ms, ar_med], dev)
    if floor_ms is not None:
        floor_ms, shape_ms = D.max_over_ranks([floor_ms, shape_ms], dev)

    if rank == 0:
        total = n * world * args.steps
        mpps = total / wall / 1e6
        alg_bytes = n * BYTES_PER_PKT[af] + (R + 1) * 8
        achieved = alg_bytes / (avg_k / 1e3) / 1e9
        traffic, traffic_src = pmc_traffic(args.config, n)
        cpu = None
        if world == 1 and args.cpu_sample:
            cpu = cpu_baseline(acl, spec, args.cpu_sample, args.faithful_sample, args.cpu_threads)
        if af == 4:
            wl = "config%d: %d-rule global ACL (%d pods), %d IPv4 TCP/UDP packets per GPU" % (
                args.config, R, len(spec["pod_ips"]), n)
            if strong:
                wl += " (%d-packet batch sharded over %d GPU%s)" % (n * world, world, "s" if world > 1 else "")
        else:
            wl = ("config%d: %d-rule global ACL (%d pods, half IPv6, dst port ranges), %d mixed IPv4/IPv6 "
                  "packets per GPU (10%% ICMP)" % (args.config, R, len(spec["pod_ips"]), n))
        line = {
            "metric": "Mpps classified at 10k ACL rules, 1/8 GPU; % of HBM roofline",
            "value": round(mpps, 2),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 stream generated in HBM, seed %#x; rules rendered from a "
                    "synthetic 1000-pod policy set)" % spec["seed"],
            "config": {"workload": wl, **({"options": args.opt} if args.opt else {}),
                       "rules": R, "packets_per_gpu": n,
                       "layout": "IPv4 SoA, 12 B/packet" if af == 4 else "16-byte address SoA, 36 B/packet",
                       "kernel": "classifier" if info["kernel"] == 1 else "linear",
                       "lds_bytes": info["lds_bytes"] if af == 4 else info["lds_bytes_v16"],
                       "lds_resident": info["lds_resident"] if af == 4 else info["lds_resident_v16"],
                       "parallelism": "dp%d" % world,
                       "collective": ("counter all-reduce, %s, %d B, side stream overlapping the next "
                                      "step's classify" % (D.backend(), (R + 1) * 8)) if coll else None},
            "settle_ms": round(settle_ms, 1),
            "step_ms_median": round(med_step, 4),
            # host time to enqueue a step (Python, ctypes, launches, events):
            # when it reaches ms_per_step the GPU waits for the host
            "host_submit_ms_per_step": round(t_submit * 1e3 / max(1, args.steps), 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel_ms_avg": round(avg_k, 4),
                         "kernel_ms_median": round(med_k, 4),
                         "kernel_ms_avg_max_rank": round(k_max, 4),
                         "kernel_ms_median_max_rank": round(kmed_max, 4),
                         "allreduce_ms_avg_max_rank": round(ar_max, 4) if coll else None,
                         "allreduce_ms_median_max_rank": round(armed_max, 4) if coll else None,
                         "stream_floor_ms": round(floor_ms, 4) if floor_ms is not None else None,
                         "frac_of_stream_floor": round(floor_ms / avg_k, 4) if floor_ms else None,
                         "frac_of_stream_floor_median": round(floor_ms / med_k, 4) if floor_ms else None,
                         "stream_floor_launch_shape_ms": round(shape_ms, 4) if shape_ms else None,
                         # every stream shape, index = variant << 1 | two workgroups per CU (rank 0)
                         "stream_floor_shapes_ms": [round(t, 4) for t in shapes],
                         "launch_shape": "%d x 1024-thread workgroups per CU" % (2 if two_per_cu else 1),
                         "frac_of_launch_shape_floor": round(shape_ms / avg_k, 4) if shape_ms else None,
                         "algorithmic_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_native(args, rank, world, local):
    """--native: the measured path as a cgo host runs it -- no torch tensor,
    stream or collective touches the GPU.  Per rank: one engine on its GPU,
    the table compiled and uploaded (cls_table_put), an engine-owned batch
    generated in HBM (cls_batch_gen_traffic_v4, rank r's packets [r N,
    (r+1) N) of the stream), and per step one cls_classify_batch: the
    classify kernels on the engine stream, then the library's ncclAllReduce
    of the hit counters on its side stream, overlapping the next step (two
    counter buffers alternate).  Under torch.distributed.run the ranks join
    one RCCL communicator (cls_comm_init with rank 0's id, exchanged over a
    gloo group that also carries the barriers and max-over-ranks); a plain
    N=1 run has no communicator.  Ranks that share a GPU (fewer devices
    than ranks: a rehearsal on a one-GPU box) have no communicator either --
    RCCL needs one rank per device -- and sum their counters over gloo."""
    import ctypes as C

    dist = None
    device, shared = local, False
    if "WORLD_SIZE" in os.environ:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        n_dev = torch.cuda.device_count()      # (counting devices does not initialise the GPU)
        if n_dev and world > n_dev:
            device, shared = local % n_dev, True
    else:
        os.environ["CONTIVCLS_NO_TORCH"] = "1"     # a plain N=1 run: torch is never imported
    from vpp_amd import _abi, workload
    from vpp_amd.engine import Engine

    def max_over(vals):
        if dist is None:
            return vals
        import torch
        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(x) for x in t]

    def barrier():
        if dist is not None:
            dist.barrier()

    acl, spec, n_default = workload.config(args.config)
    strong = args.config == 4
    n = args.packets or (-(-n_default // world) if strong else n_default)
    af = spec.get("layout", 4)
    eng = Engine(device, options=dict(o.split("=", 1) for o in args.opt))   # one rank per GPU (RCCL: one per device)
    comm_err = None
    if dist is not None and not shared:
        uid = [Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        try:
            eng.comm_init(world, rank, uid[0])
            ok = 1.0
        except Exception as ex:                # (reported in the line; every rank takes the same path)
            comm_err, ok = str(ex), 0.0
        t = __import__("torch").tensor([ok], dtype=__import__("torch").float64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if t.item() < 1.0:                     # no RCCL group: counters summed over gloo after the steps
            shared = True
            comm_err = comm_err or "another rank's cls_comm_init failed"
            eng.close()                        # (a rank whose init succeeded must not all-reduce alone)
            eng = Engine(device, options=dict(o.split("=", 1) for o in args.opt))
    table = eng.put_table("contiv/vpp-policy-GLOBAL", acl.rules)
    info = table.info()
    R = table.n_rules
    b = eng.batch(n, af=af)
    b.gen_traffic(spec, rank * n)
    b.wait()

    def step(timing):
        eng.classify_batch(table, b, counters=False, timing=timing)

    i = 0
    t_settle = time.perf_counter()
    while True:
        for _ in range(8):
            step(False)
            i += 1
        b.wait()
        short = (time.perf_counter() - t_settle) * 1e3 < args.settle_ms
        if not max_over([1.0 if short else 0.0])[0]:
            break
    settle_ms = (time.perf_counter() - t_settle) * 1e3
    for _ in range(args.warmup):
        step(False)
    b.wait()
    eng.kernel_times(reset=True)
    barrier()
    b.wait()
    t0 = time.perf_counter()
    every = max(1, args.event_every)
    for j in range(args.steps):
        step(args.events >= 1 and j % every == 0)
    t_submit = time.perf_counter() - t0
    b.wait()                                   # every kernel and the last all-reduce
    barrier()
    wall = time.perf_counter() - t0
    kms, starts = eng.kernel_times(reset=True, starts=True)
    counters = b.counters(R)
    if shared:
        # no communicator: the ranks' counters summed over the gloo group
        import torch
        t = torch.from_numpy(counters.astype(np.int64))
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        counters = t.numpy().astype(np.uint64)
    if args.dump:
        os.makedirs(args.dump, exist_ok=True)
        np.save(os.path.join(args.dump, "verdict_r%d.npy" % rank), b.download(_abi.BF_VERDICT))
        if rank == 0:
            np.save(os.path.join(args.dump, "counters.npy"), counters)
    avg_k = float(np.mean(kms)) if kms else float("nan")
    med_k = float(np.median(kms)) if kms else float("nan")
    periods = list(np.diff(starts) / every) if len(starts) > 1 else []      # timed steps `every` apart
    med_step = float(np.median(periods)) if periods else float("nan")
    # the stream floor over the batch's own device arrays
    shapes = []
    lds = info["lds_bytes"] if af == 4 else info["lds_bytes_v16"]
    resident = info["lds_resident"] if af == 4 else info["lds_resident_v16"]
    two_per_cu = not resident or 2 * (lds + 16) <= 160 * 1024
    floor_ms = shape_ms = None
    if not args.no_stream_floor:
        m = min(n, 1 << 30)
        m -= m % (256 if af == 16 else 4)
        p = lambda f: b.field_ptr(0, f)  # noqa: E731
        if af == 16:
            pk = _abi.PktSoa(_abi.AF_V16, None, None, p(_abi.BF_SRC), p(_abi.BF_DST), None, p(_abi.BF_DPORT),
                             p(_abi.BF_PROTO))
        else:
            pk = _abi.PktSoa(_abi.AF_V4, p(_abi.BF_SRC), p(_abi.BF_DST), None, None, None, p(_abi.BF_DPORT),
                             p(_abi.BF_PROTO))
        ms = (C.c_float * 8)()
        cnt = C.c_uint32(0)
        eng._check(_abi.lib().cls_stream_floor_shapes(eng.h, C.byref(pk), m, p(_abi.BF_VERDICT), 10, ms, 8,
                                                       C.byref(cnt), None))
        shapes = [ms[k] * (n / m) for k in range(cnt.value)]
        floor_ms = min(shapes)
        shape_ms = min(t for k, t in enumerate(shapes) if (k & 1) == int(two_per_cu) or len(shapes) < 2)
    wall, k_max, kmed_max = max_over([wall, avg_k, med_k])
    if floor_ms is not None:
        floor_ms, shape_ms = max_over([floor_ms, shape_ms])
    ok_sum = int(counters.sum()) == n * world
    if rank == 0:
        total = n * world * args.steps
        mpps = total / wall / 1e6
        alg_bytes = n * BYTES_PER_PKT[af] + (R + 1) * 8
        achieved = alg_bytes / (avg_k / 1e3) / 1e9
        traffic, traffic_src = pmc_traffic(args.config, n)
        cpu = None
        if world == 1 and args.cpu_sample:
            cpu = cpu_baseline(acl, spec, args.cpu_sample, args.faithful_sample, args.cpu_threads)
        if af == 4:
            wl = "config%d: %d-rule global ACL (%d pods), %d IPv4 TCP/UDP packets per GPU" % (
                args.config, R, len(spec["pod_ips"]), n)
            if strong:
                wl += " (%d-packet batch sharded over %d GPU%s)" % (n * world, world, "s" if world > 1 else "")
        else:
            wl = ("config%d: %d-rule global ACL (%d pods, half IPv6, dst port ranges), %d mixed IPv4/IPv6 "
                  "packets per GPU (10%% ICMP)" % (args.config, R, len(spec["pod_ips"]), n))
        comm = eng.comm_info()
        line = {
            "metric": "Mpps classified at 10k ACL rules, 1/8 GPU; % of HBM roofline",
            "value": round(mpps, 2),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 stream generated in HBM, seed %#x; rules rendered from a "
                    "synthetic 1000-pod policy set)" % spec["seed"],
            "config": {"workload": wl, **({"options": args.opt} if args.opt else {}),
                       "rules": R, "packets_per_gpu": n,
                       "layout": "IPv4 SoA, 12 B/packet" if af == 4 else "16-byte address SoA, 36 B/packet",
                       "kernel": "classifier" if info["kernel"] == 1 else "linear",
                       "lds_bytes": lds, "lds_resident": resident,
                       "parallelism": "dp%d" % world,
                       "path": "native: C ABI only (cls_batch_*, cls_classify_batch), no torch on the GPU",
                       "collective": ("counter all-reduce in the library: ncclAllReduce u64 sum over %d RCCL "
                                      "ranks (cls_comm_init), %d B, side stream overlapping the next step's "
                                      "classify" % (comm[0], (R + 1) * 8)) if comm[0] else
                                     ("counters summed over gloo after the timed steps (%s)" % (
                                         "cls_comm_init failed: %s" % comm_err if comm_err else
                                         "%d ranks share a GPU: RCCL needs one rank per device; rehearsal, "
                                         "not a scaling number" % world))
                                     if shared else None},
            "counters_sum_ok": ok_sum,
            "settle_ms": round(settle_ms, 1),
            "step_ms_median": round(med_step, 4),
            "timed_every": every,
            "host_submit_ms_per_step": round(t_submit * 1e3 / max(1, args.steps), 4),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel_ms_avg": round(avg_k, 4),
                         "kernel_ms_median": round(med_k, 4),
                         "kernel_ms_avg_max_rank": round(k_max, 4),
                         "kernel_ms_median_max_rank": round(kmed_max, 4),
                         "stream_floor_ms": round(floor_ms, 4) if floor_ms is not None else None,
                         "frac_of_stream_floor": round(floor_ms / avg_k, 4) if floor_ms else None,
                         "stream_floor_launch_shape_ms": round(shape_ms, 4) if shape_ms else None,
                         "stream_floor_shapes_ms": [round(t, 4) for t in shapes],
                         "launch_shape": "%d x 1024-thread workgroups per CU" % (2 if two_per_cu else 1),
                         "frac_of_launch_shape_floor": round(shape_ms / avg_k, 4) if shape_ms else None,
                         "algorithmic_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    b.close()
    eng.close()
    if dist is not None:
        dist.destroy_process_group()
    if not ok_sum:
        sys.exit("bench.py --native: the merged counters do not sum to the packets of all ranks")


if __name__ == "__main__":
    main()
