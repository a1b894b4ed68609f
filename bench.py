"""Benchmark: points clustered/s on MI355X (BASELINE.json metric), one JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W]
        (N > 1 without a launcher: bench.py starts the N ranks below as a child process and
        relays rank 0's line; fewer than N visible GPUs: exit 2, nothing measured)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workloads (BASELINE.json configs, SURVEY.md §8d generator G(n, noise, dense, seed), eps = 2.55
(k_bar ~ 49), minPoints = 10, LocalDBSCANNaive semantics, visit order = generation order):
  N = 1  config 2: G(10^7, no noise, seed 1), one local fit per step
         (dbscan_fit_device_async; the K steps are enqueued back to back, one sync at the end).
  N > 1  config 3 weak-scaled: G(1.25*10^7 x N, 20% uniform noise, seed 2) -- exactly config 3
         (10^8 points) at N = 8 -- through the slab-sharded node path (dbscan_amd/node.py): per-
         GPU slab fits with eps halos + RCCL all-gathers of the boundary records + global
         union-find + relabel; per-GPU work fixed (weak scaling).
A step is one pass of the hot path over the resident points (HBM in -> labels in HBM): `value`.
`end_to_end` times host SoA -> host labels on the same data (PCIe included; N = 1:
dbscan_fit_h; N > 1: each rank's H2D of its 1/N chunk of the input, an all_to_all routing the
points to their slabs, the node step, an all_to_all returning the labels to the chunk owners,
D2H); it is reported beside `value`, never as it.

roofline: the dominant kernel of the timed region, timed with HIP events on the library's own
stream, carried on the kernels' own dispatch packets (hipExtLaunchKernelGGL: no idle gaps);
achieved = algorithmic bytes per launch (SURVEY §8d per-point figure x points) / the kernel's
average launch duration.  `traffic` (HBM bytes per launch from rocprofv3 PMC) and `valu`
(fp32/fp64 lane-ops from SQ counters) come from profiles/pmc_traffic.json, used only when its
entry was measured on this workload size AND from the same kernel sources (src_sha).
cpu_baseline (rank 0, N = 1): the reference's whole DBSCAN.train path restated in C
(oracle/reference_pipeline.c: EvenSplitPartitioner with maxPointsPerPartition = 8192, eps
halos, LocalDBSCANNaive.fit O(m^2) per partition on a thread pool, the margin merge and
relabel) on the same points, on the host cores this process may use; plus the strong CPU
comparator (the closed form on an eps grid, oracle_fit_grid) on the same threads.
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dbscan-on-spark_amd"))

METRIC = "points clustered/sec (whole node) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU peaks in lane-operations per second (one lane of one VALU instruction; an FMA is ONE
# lane-op here): fp64 vector 78.6 TFLOP/s counting FMA as 2 -> 39.3e12; fp32 157.3 -> 78.6e12.
VALU_PEAK = {"f64": 39.3e12, "f32": 78.65e12}
SIMD_CLOCK_HZ = 2.4e9  # MI355X peak engine clock
# Algorithmic bytes per point and launch, by kernel (SURVEY.md §8d's per-phase figures; each
# array crosses HBM once).  count = 21: the count kernel also builds the quarter
# records and the tile-local quarter union (fused), so it carries §8d's count (sorted x,y 16 +
# core 1) and union (parent 4; the union's x,y read is the count's, already in LDS).
# edge_union and quarter_root touch tile-edge strips and quarter reps only.  The §8d output 30
# is carried by final (13), the rank scan and label_sorted/permute_out.  Radix passes: each
# reads key+perm 8 and writes 8.
ALG_BYTES = {
    "bbox_partial": 16, "bin": 20, "radix_upsweep": 4, "radix_downsweep": 16, "inverse": 8,
    "scatter_xy": 36, "heads_reduce": 4, "heads_down": 16, "count": 21, "count_wave": 21,
    "count_tiny": 21,
    "count32": 21, "big_count": 21, "edge_union": 0, "quarter_root": 0, "final": 13,
    "label_sorted": 13, "permute_out": 13,
    # bucketed sort (fits of >= 2^23 points): the MSD pass reads key + x,y and
    # writes key, the 32-B place record and pos; an LSD pass reads and writes key + place;
    # the gather reads place + record and writes perm + sorted x,y
    "bucket_msd": 60, "bucket_lsd": 16, "gather_bucket": 56,
}
# The clique-grid count kernels each process one class of tiles: their per-launch algorithmic
# bytes count that class's points only (dbscan_last_stats [11..13]).
CLASS_PTS = {"count_wave": "pts_small", "count32": "pts_medium", "big_count": "pts_big"}
PIPELINE_ALG_BYTES = 132  # whole pipeline, B_alg per point


def src_stamp() -> str:
    """Content hash of the sources libdbscan_hip.so is built from (the GPU box has no .git):
    PMC entries are used only when they were measured on these exact sources."""
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "dbscan-on-spark_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + [os.path.join(csrc, "internal.h"),
                   os.path.join(csrc, "Makefile"), os.path.join(ROOT, "include", "dbscan_hip.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def host_threads() -> int:
    """Host threads this process may use: its CPU affinity, capped by OMP_NUM_THREADS when set
    (the GPU box exports its per-GPU CPU share there; its affinity shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--points-per-gpu", type=int, default=None,
                    help="default: 10^7 at N = 1 (config 2), 1.25*10^7 at N > 1 (config 3)")
    ap.add_argument("--eps", type=float, default=2.55)
    ap.add_argument("--min-points", type=int, default=10)
    ap.add_argument("--noise", type=float, default=None, help="default 0 (N = 1), 0.2 (N > 1)")
    ap.add_argument("--dense", type=float, default=None, help="default 1")
    ap.add_argument("--config", type=int, choices=sorted(CONFIGS), default=None,
                    help="BASELINE config shape (points per GPU, noise, dense, seed)")
    ap.add_argument("--seed", type=int, default=None, help="default 1 (N = 1), 2 (N > 1)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: host_threads()")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-steps", type=int, default=3, help="end-to-end steps (0: skip)")
    ap.add_argument("--no-profile", action="store_true", help="no kernel timing events")
    ap.add_argument("--profile-steps", type=int, default=3,
                    help="untimed steps with every kernel timed (the breakdown)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--force-collectives", action="store_true",
                    help="rehearse the N > 1 node path on one GPU: a one-rank process group and "
                         "the node exchange's collectives run anyway (not a measurement)")
    ap.add_argument("--node", action="store_true", help="use the node path even at N = 1")
    ap.add_argument("--no-seam", action="store_true",
                    help="skip the seam leg (partition-sized fits and batches, N = 1)")
    ap.add_argument("--seam-only", action="store_true", help="only the seam leg (no timed fit)")
    ap.add_argument("--launch-probe", action="store_true",
                    help="test hook: the ranks join the process group and report their devices")
    return ap.parse_args(argv)


# BASELINE.json configs as G(n, noise, dense, seed) shapes: (points per GPU at
# the config's own GPU count, noise, dense, seed, GPUs the config names).  --config C runs that
# shape with the per-GPU share fixed (weak scaling): exactly the config at its own GPU count,
# its per-GPU share on one GPU.
CONFIGS = {
    2: (10_000_000, 0.0, 1.0, 1, 1),
    3: (12_500_000, 0.2, 1.0, 2, 8),
    4: (50_000_000, 0.0, 8.0, 3, 1),
    5: (125_000_000, 0.2, 1.0, 4, 8),
}


def workload_name(n_total, per_gpu, noise, dense, seed, world):
    """Which BASELINE config this run is (or is the per-GPU share / weak-scaled form of)."""
    for c, (pg, nz, dn, sd, ngpu) in CONFIGS.items():
        if (per_gpu, float(noise), float(dense), int(seed)) != (pg, nz, dn, sd):
            continue
        if world == ngpu:
            return f"config {c}"
        if world == 1:
            return f"config {c}'s per-GPU share (config {c} is {ngpu} GPUs x {pg})"
        return (f"config {c} shape weak-scaled to {world} GPUs ({pg} points per GPU; config {c} "
                f"itself at {ngpu} GPU{'s' if ngpu > 1 else ''})")
    return "custom"


def workload_defaults(args, world):
    """Fill the unset workload flags: --config C (BASELINE config C's shape, per-GPU share
    fixed); else config 2 at N = 1 (G(10^7, no noise, seed 1)) and config 3 weak-scaled at
    N > 1 (1.25*10^7 points per GPU, 20% noise, seed 2: G(10^8) at N = 8), also for the one-GPU
    rehearsal of that path (--force-collectives)."""
    if getattr(args, "force_collectives", False):
        world = max(world, 2)
    if getattr(args, "config", None):
        pg, nz, dn, sd, _ = CONFIGS[args.config]
        args.points_per_gpu = args.points_per_gpu or pg
        args.noise = nz if args.noise is None else args.noise
        args.dense = dn if args.dense is None else args.dense
        args.seed = sd if args.seed is None else args.seed
    if args.dense is None:
        args.dense = 1.0
    if args.points_per_gpu is None:
        args.points_per_gpu = 12_500_000 if world > 1 else 10_000_000
    if args.noise is None:
        args.noise = 0.2 if world > 1 else 0.0
    if args.seed is None:
        args.seed = 2 if world > 1 else 1
    return args


def load_pmc(stage, n_points, stamp):
    """The committed rocprofv3 summary for `stage` (tools/pmc_summary.py), or (None, reason)
    unless it was measured on this workload size and these kernel sources."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/pmc_traffic.json"
    e = d.get("stages", {}).get(stage)
    if e is None:
        return None, f"{stage} not profiled"
    if d.get("src_sha") != stamp:
        return None, f"stale: profiled on sources {d.get('src_sha')}, running {stamp}"
    if d.get("n_points") != n_points:
        return None, f"profiled at n = {d.get('n_points')}, running n = {n_points}"
    return e, d.get("source")


def _limiter(pmc):
    """What actually bounds the roofline kernel, from its SQ counters (the contract's `bound`
    names the ceiling it is priced against): the waves' cycle split."""
    sq = (pmc or {}).get("sq") or {}
    wc = sq.get("SQ_WAVE_CYCLES")
    if not wc:
        return None
    parked, stalled = sq.get("SQ_WAIT_ANY", 0) / wc, sq.get("SQ_WAIT_INST_ANY", 0) / wc
    kind = "latency" if parked > 0.5 else ("issue" if stalled > 0.3 else "mixed")
    return (f"{kind}: {parked:.0%} of wave cycles parked on waitcnt/barriers, {stalled:.0%} "
            f"issue-stalled, {sq.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0%} issuing (SQ counters)")


def _affinity() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_baseline(x, y, eps, min_points, threads, sample_s=None, h=None):
    """The reference path on the host cores.  sample_s = None: the whole restated DBSCAN.train
    (partitioner, halos, per-partition LocalDBSCANNaive.fit O(m^2), merge) over every point, plus
    the strong comparator.  sample_s = S (N > 1: 10^8+ points): the same per-partition fits on
    the reference's partitions of the same points, stopped after S seconds; value = the
    partitions' own points / the time they took (the partitioner and merge are not timed)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle as O  # CPU baseline leg only

    if sample_s is not None:
        import dbscan_amd

        parts = dbscan_amd.partition.partition_points(x, y, eps, 8192, h)
        rects = np.array([r for r, _ in parts])
        counts = np.array([c for _, c in parts], np.int64)
        r = O.ref_fit_partitions_timed(x, y, eps, min_points, rects, counts, threads, sample_s)
        return {
            "value": r["main_points"] / max(r["seconds"], 1e-9), "unit": "points/s",
            "cores": threads, "kind": "port", "seconds": round(r["seconds"], 3),
            "sample": (f"bounded sample: LocalDBSCANNaive.fit O(m^2) restated in C "
                       f"(oracle/reference_pipeline.c) on {r['parts']} of the {len(counts)} "
                       f"partitions the reference's EvenSplitPartitioner(maxPointsPerPartition="
                       f"8192) makes of the same {x.size} points ({r['outer_points']} points with "
                       f"eps halos), {threads} threads, {sample_s:.0f} s budget; value = those "
                       f"partitions' own points / seconds (partitioner and merge not timed)")}

    t0 = time.perf_counter()
    r = O.ref_train(x, y, eps, min_points, 8192, threads)
    t_ref = time.perf_counter() - t0
    lost = int((r["records"] == 0).sum())
    t0 = time.perf_counter()
    g = O.fit_grid(x, y, eps, min_points, 0, threads)
    t_grid = time.perf_counter() - t0
    # the GPU result on the same points equals the grid closed form (tests/test_gpu_configs.py)
    return {
        "value": x.size / t_ref,
        "unit": "points/s",
        "cores": threads,
        "kind": "port",
        "seconds": round(t_ref, 3),
        "sample": (f"the reference's whole DBSCAN.train path restated in C "
                   f"(oracle/reference_pipeline.c) over the same {x.size} points: "
                   f"EvenSplitPartitioner(maxPointsPerPartition=8192) -> {len(r['rects'])} "
                   f"partitions, eps halos, LocalDBSCANNaive.fit O(m^2) per partition on "
                   f"{threads} threads, margin merge + relabel, in {t_ref:.2f} s; value = input "
                   f"points / s (the restated partitioner's split-line defect, SURVEY §8f-2, "
                   f"drops {lost} points; the reference's own O(#cells) partitioner scan and "
                   f"O(points x partitions) margin scan are replaced by indexed forms with the "
                   f"same decisions)"),
        "strong_comparator": {
            "value": x.size / t_grid, "unit": "points/s", "cores": threads,
            "seconds": round(t_grid, 3), "n_clusters": g[2],
            "what": "closed form on an eps grid (oracle_fit_grid, pthreads), same points"},
    }


def visible_devices() -> int:
    """GPUs this process can see.  torch.cuda.device_count() does not initialise HIP on this
    image, so a launcher may still start children after it."""
    import torch

    return torch.cuda.device_count()


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) started without a launcher (no WORLD_SIZE in the environment): start
    the N ranks as ONE child process -- python -m torch.distributed.run --nproc-per-node N on
    127.0.0.1 running this script with the same arguments -- relay its output (rank 0 prints
    the JSON line) and return its exit code.  Fewer than N visible GPUs: a clear error, exit 2,
    nothing measured.  Called before anything touches the GPU (no exec: the child is a
    separate process).  Returns None when this process should run the bench itself."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    ndev = visible_devices()
    if ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this process sees "
              f"{ndev}; refusing to measure fewer GPUs than asked", file=sys.stderr, flush=True)
        return 2
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    print(f"bench.py: no launcher in the environment; starting {args.gpus} ranks: "
          + " ".join(cmd[1:]), file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def rank_devices(dist, backend):
    """(world size, the device each rank runs on) as the process group sees them: every rank's
    (rank, local device index, PCI bus id) all-gathered."""
    import torch

    if torch.cuda.is_available() and backend == "nccl":
        d = torch.cuda.current_device()
        bus = getattr(torch.cuda.get_device_properties(d), "pci_bus_id", -1)
    else:
        d, bus = -1, -1
    mine = [dist.get_rank(), d, int(bus)]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, mine)
    return dist.get_world_size(), [{"rank": r, "device": dv, "pci_bus_id": b}
                                   for r, dv, b in sorted(out)]


def launch_probe(args):
    """--launch-probe (test hook for the launcher): each rank joins the process group and
    reports where it runs; rank 0 prints one JSON line.  No fit, no GPU work with gloo."""
    import torch.distributed as dist

    dist.init_process_group(args.backend)
    world, devs = rank_devices(dist, args.backend)
    if dist.get_rank() == 0:
        print(json.dumps({"probe": True, "n_gpus": world, "devices": devs}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    rc = launch_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if args.launch_probe:
        launch_probe(args)
        return
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and (world > 1 or "WORLD_SIZE" in os.environ):
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    node_path = world > 1 or args.node or args.force_collectives
    workload_defaults(args, world)
    ndev = torch.cuda.device_count()
    if world > 1 and local_rank >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK={local_rank} but only {ndev} visible GPUs "
                         "(one rank per GPU; ranks never share a device)")
    dev = local_rank % max(1, ndev)
    torch.cuda.set_device(dev)
    import dbscan_amd
    from dbscan_amd import device as D

    h = dbscan_amd.Handle(dev)
    if args.seam_only:
        print(json.dumps({"seam": seam(args, h, args.cpu_threads or host_threads())}), flush=True)
        return
    dist = None
    if world > 1 or args.force_collectives:
        import torch.distributed as dist

        if world == 1:  # rehearsal: a process group of one rank (no launcher)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29400 + os.getpid() % 1000))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.backend)
        pg_world, pg_devices = rank_devices(dist, args.backend)
        if pg_world != world:
            raise SystemExit(f"WORLD_SIZE={world} but the process group has {pg_world} ranks")
        if args.backend == "nccl" and len({d["pci_bus_id"] for d in pg_devices}) != pg_world:
            raise SystemExit(f"ranks share GPUs: {pg_devices}")
    else:
        pg_devices = [{"rank": 0, "device": dev,
                       "pci_bus_id": getattr(torch.cuda.get_device_properties(dev),
                                             "pci_bus_id", -1)}]

    n_total = args.points_per_gpu * world
    if not node_path:
        x, y = D.generate_blobs(n_total, args.noise, args.dense, args.seed, h)
        cl = torch.empty(n_total, dtype=torch.int32, device="cuda")
        fl = torch.empty(n_total, dtype=torch.uint8, device="cuda")

        nk = torch.zeros(1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()

        def step():  # enqueue only: no host synchronization inside a fit
            D.fit_tensors_async(x, y, args.eps, args.min_points, 0, h, cl, fl, nk)
            return nk
    else:
        from dbscan_amd import node

        torch.cuda.synchronize()
        ts0 = time.perf_counter()
        job = node.NodeJob.synthetic(n_total, args.noise, args.dense, args.seed, args.eps,
                                     args.min_points, h, dist, force=args.force_collectives)
        torch.cuda.synchronize()
        setup_s = time.perf_counter() - ts0  # (generation + cuts + zones + halo routing)

        def step():
            return job.run()

    for _ in range(args.warmup):
        k = step()
    h.sync()
    kernels, dom = {}, None
    if not args.no_profile:
        # Per-kernel breakdown from a short profiled pass outside the timed region: events on
        # every launch cost ~0.2 ms per fit of extra GPU time, so the timed region
        # carries events on the dominant kernel's launches only.
        h.profile(True, kernels=True)
        h.profile_only(None)
        h.profile_reset()
        for _ in range(args.profile_steps):
            step()
        h.sync()
        torch.cuda.synchronize()
        kprof = h.profile_read()
        kernels = {k2: v["ms"] / max(1, args.profile_steps) for k2, v in kprof.items()}
        dom = max(kprof, key=lambda s: kprof[s]["ms"]) if kprof else None
        h.profile_only(dom)
        h.profile_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        k = step()
    h.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0

    def max_over_ranks(v):
        if not dist:
            return v
        t = torch.tensor([v], dtype=torch.float64,
                         device="cuda" if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    el = max_over_ranks(el)
    setup_ms = round(max_over_ranks(setup_s) * 1e3, 3) if node_path else None
    if isinstance(k, torch.Tensor):
        k = int(k.item())
    prof = h.profile_read() if not args.no_profile else {}
    h.profile(False)
    stats = h.stats()

    ms_per_step = el / args.steps * 1e3
    value = n_total * args.steps / el
    roof, valu = None, None
    if prof and dom in prof:
        avg_ms = prof[dom]["ms"] / max(1, prof[dom]["launches"])  # live, in the timed region
        pts = stats.get("n", args.points_per_gpu)
        unit_pts = stats.get(CLASS_PTS[dom], pts) if dom in CLASS_PTS else pts
        alg = ALG_BYTES.get(dom.split("<")[0], 0) * unit_pts  # per launch
        achieved = alg / (avg_ms * 1e-3) / 1e9
        pmc, pmc_src = load_pmc(dom, pts, src_stamp()) if not node_path else (None, "node path")
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                "traffic_source": pmc_src,
                "kernel": dom, "avg_launch_ms": round(avg_ms, 4),
                "alg_bytes_per_point": ALG_BYTES.get(dom.split("<")[0], 0),
                "points_per_launch": unit_pts,
                "limiter": _limiter(pmc),
                "pipeline_frac": round(PIPELINE_ALG_BYTES * pts / (ms_per_step * 1e-3) / 1e9
                                       / HBM_PEAK_GBS, 5)}
        if pmc and pmc.get("valu_insts_per_launch"):
            vi = pmc["valu_insts_per_launch"]  # wave-instructions by type, per launch
            lanes = {t: 64.0 * sum(v for kk, v in vi.items() if kk.endswith(t.upper()))
                     for t in ("f32", "f64")}
            rate = {t: lanes[t] / (avg_ms * 1e-3) for t in lanes}
            frac = sum(rate[t] / VALU_PEAK[t] for t in rate)
            sq = pmc.get("sq") or {}
            # every VALU wave-instruction (float, integer, moves) holds its SIMD >= 2 cycles
            # (64 lanes over SIMD-32): issue share of 1024 SIMDs x 2.4 GHz x launch time
            issue = (2.0 * sq.get("SQ_INSTS_VALU", 0.0) /
                     (1024 * SIMD_CLOCK_HZ * avg_ms * 1e-3)) if sq else None
            valu = {"bound": "valu", "kernel": dom, "unit": "T lane-ops/s",
                    "achieved": {t: round(rate[t] / 1e12, 3) for t in rate},
                    "peak": {t: VALU_PEAK[t] / 1e12 for t in VALU_PEAK},
                    "frac": round(frac, 5),
                    "lane_ops_per_launch": {t: lanes[t] for t in lanes},
                    "int32_lane_ops_per_launch": 64.0 * sq.get("SQ_INSTS_VALU_INT32", 0.0),
                    "valu_issue_frac": round(issue, 4) if issue is not None else None,
                    "wave_time": ({k: round(sq[k] / sq["SQ_WAVE_CYCLES"], 4) for k in
                                   ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
                                  if sq.get("SQ_WAVE_CYCLES") else None),
                    "note": ("lane-ops = 64 x VALU wave-instructions (SQ_INSTS_VALU_{ADD,MUL,FMA,"
                             "TRANS}_F32/F64, full exec mask assumed: an upper bound) over the "
                             "live average launch time; frac = f32/peak_f32 + f64/peak_f64 "
                             "(both share the VALU); valu_issue_frac = every VALU instruction "
                             "(integer included) x 2 cycles over the 1024 SIMDs' cycles; "
                             "wave_time = share of wave cycles parked / issue-stalled / issuing"),
                    "source": pmc_src}

    e2e = None
    if args.e2e_steps > 0:
        e2e = end_to_end(args, h, dist, world, rank, n_total, node_path, max_over_ranks,
                         x if not node_path else None, y if not node_path else None)

    seam_out = None
    if world == 1 and not node_path and not args.no_seam:
        seam_out = seam(args, h, args.cpu_threads or host_threads())

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        if world == 1 and not node_path:
            sx, sy = x.cpu().numpy(), y.cpu().numpy()
            threads = args.cpu_threads or host_threads()
            cpu = cpu_baseline(sx, sy, args.eps, args.min_points, threads)
        else:
            # the node's CPU share for this job (the other ranks idle meanwhile): the per-GPU
            # share times the ranks, capped by this process's affinity; a bounded sample of the
            # reference's per-partition fits over the same G(n_total)
            from dbscan_amd import device as D

            threads = args.cpu_threads or min(host_threads() * world, _affinity())
            gx, gy = D.generate_blobs(n_total, args.noise, args.dense, args.seed, h)
            sx, sy = gx.cpu().numpy(), gy.cpu().numpy()
            del gx, gy
            torch.cuda.empty_cache()
            cpu = cpu_baseline(sx, sy, args.eps, args.min_points, threads, sample_s=12.0, h=h)
            del sx, sy
        if cpu is not None:
            cpu["nproc"] = os.cpu_count()
            cpu["gpu_over_cpu"] = round(value / cpu["value"], 1)

    if node_path:
        job.close()
    if rank == 0:
        name = workload_name(n_total, args.points_per_gpu, args.noise, args.dense, args.seed,
                             world)
        workload = (f"{name}: G({n_total} points" +
                    (f" = {args.points_per_gpu} per GPU x {world}" if world > 1 else "") +
                    f", 32 Gaussian blobs, noise={args.noise}, dense={args.dense}, "
                    f"seed={args.seed})")
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "points/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "value_basis": ("device-resident: coordinates already in HBM when the timed region "
                            "starts, labels left in HBM (the bench contract); the PCIe-inclusive "
                            "host-array rate is end_to_end, and vs_baseline stays null because "
                            "BASELINE.md holds no published number (GPU/CPU ratio: "
                            "cpu_baseline.gpu_over_cpu)"),
            "data": "synthetic (device generator G(n, noise, dense, seed), SURVEY §8d)",
            "config": {
                "workload": workload + f", eps={args.eps}, minPoints={args.min_points}, "
                                       "LocalDBSCANNaive semantics",
                "n_points": n_total, "eps": args.eps, "min_points": args.min_points,
                "parallelism": ("single GPU, one local fit" if not node_path else
                                f"x-slabs x{world} with eps halos" +
                                (f" + {'RCCL' if args.backend == 'nccl' else args.backend} "
                                 "all-gathers + global union-find" +
                                 (" (one-rank rehearsal)" if world == 1 else "")
                                 if world > 1 or args.force_collectives else
                                 " (one slab: no exchange)") +
                                f"; per-job setup outside the timed steps (synthetic data, "
                                f"slab cuts, zones, halo routing): {setup_ms} ms"),
                "node_setup_ms": setup_ms,
                "world_size": world,
                "devices": pg_devices,
                "node_step_note": (None if not node_path else
                                   "a timed step re-fits every slab and exchanges the b-side "
                                   "records; the cuts, zones and the a-side records are fixed "
                                   "at setup (node_setup_ms), as the reference partitions once "
                                   "per train() call"),
                "clusters": k, "core_points": stats.get("core"),
                "occupied_cells": stats.get("cells"), "occupied_tiles": stats.get("tiles")},
            "roofline": roof,
            "valu": valu,
            "end_to_end": e2e,
            "seam": seam_out,
            "cpu_baseline": cpu,
            "kernels_ms_per_step": {k2: round(v, 4) for k2, v in
                                    sorted(kernels.items(), key=lambda kv: -kv[1])},
            "kernels_ms_note": (f"per-kernel event times from {args.profile_steps} untimed "
                                "profiled steps; the timed steps carry events only on the "
                                "roofline kernel"),
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def seam(args, h, threads):
    """The seam's real call pattern (DBSCAN.scala:150-155: one LocalDBSCANNaive.fit per spatial
    partition of <= maxPointsPerPartition points + eps halo).
      per_call   one fit of m points per call, m in 250 / 2k / 8k / 64k: dbscan_fit_h (host
                 arrays, PCIe included) and dbscan_fit_device (device-resident, synchronous),
                 median of repeated calls, and capi_us: the dbscan_fit_device call alone as a JNI
                 caller makes it (no torch stream sync); the plain columns are the LDS kernels
                 (small.hip): up to 8192 points the whole partition in each workgroup, from
                 DBSCAN_SPREAD_DEFAULT_POINTS (512) over several workgroups, above 8192 (to
                 DBSCAN_BAND_DEFAULT_POINTS, 65536) the band form; 'tiled' is the same call
                 through the tiled pipeline (dbscan_set_small_max 0)
      train      G(10^7) (config 2) cut by the reference's EvenSplitPartitioner with
                 maxPointsPerPartition 8192 and duplicated into eps-grown partitions
                 (DBSCAN.scala:105-137): every partition fitted (a) by one dbscan_fit_h call each
                 (one executor thread calling the seam per partition), (b) as ONE
                 dbscan_fit_batch call (host arrays), (c) device-resident
                 (dbscan_fit_batch_device_async, back to back), against (d) the reference's
                 LocalDBSCANNaive.fit O(m^2) restated in C on the same partitions, `threads`
                 host threads, for a bounded sample of partitions."""
    import ctypes

    import numpy as np
    import torch

    import dbscan_amd
    from dbscan_amd import device as D

    out = {"per_call": {}}
    eps, mp = args.eps, args.min_points
    default_small = h.set_small_max(8192)  # (restored below: the handle's default cap)
    for m in (250, 2000, 8192, 65536):
        tx, ty = D.generate_blobs(m, 0.0, 1.0, 5, h)
        hx, hy = tx.cpu().numpy(), ty.cpu().numpy()
        cl = np.ones(m, np.int32)
        fl = np.ones(m, np.uint8)
        dcl = torch.empty(m, dtype=torch.int32, device="cuda")
        dfl = torch.empty(m, dtype=torch.uint8, device="cuda")
        row = {}
        lib = dbscan_amd.load()
        kk = ctypes.c_int32(0)
        capi_args = (h.ptr, ctypes.c_void_p(tx.data_ptr()), ctypes.c_void_p(ty.data_ptr()), m,
                     float(eps), int(mp), 0, ctypes.c_void_p(dcl.data_ptr()),
                     ctypes.c_void_p(dfl.data_ptr()), ctypes.byref(kk))
        torch.cuda.synchronize()
        for tag, small in (("", 8192), ("tiled_", 0)):
            h.set_small_max(small)
            reps = 30 if m <= 8192 else 10
            for kind in ("host", "device", "capi"):
                ts = []
                for i in range(reps + 2):
                    t0 = time.perf_counter()
                    if kind == "host":
                        dbscan_amd.fit_arrays(hx, hy, eps, mp, 0, handle=h, cluster_out=cl,
                                              flag_out=fl)
                    elif kind == "device":
                        D.fit_tensors(tx, ty, eps, mp, 0, h, dcl, dfl)
                    else:  # the C-ABI call alone, as a JNI caller makes it (inputs resident)
                        lib.dbscan_fit_device(*capi_args)
                    if i >= 2:
                        ts.append(time.perf_counter() - t0)
                row[f"{tag}{kind}_us"] = round(float(np.median(ts)) * 1e6, 1)
        h.set_small_max(default_small)
        out["per_call"][str(m)] = row

    n = 10_000_000
    tx, ty = D.generate_blobs(n, 0.0, 1.0, 1, h)
    x, y = tx.cpu().numpy(), ty.cpu().numpy()
    del tx, ty
    parts = dbscan_amd.partition.partition_points(x, y, eps, 8192, h)
    rects = np.array([r for r, _ in parts])
    counts = np.array([c for _, c in parts], np.int64)
    offs, idx = dbscan_amd.duplicate(x, y, rects, eps)
    px, py = x[idx], y[idx]
    sizes = np.diff(offs)
    npart, total = len(sizes), int(offs[-1])
    cl = np.ones(total, np.int32)
    fl = np.ones(total, np.uint8)
    # (a) one seam call per partition, one thread (recalls: partitions whose band fit
    # overflowed its staging or whose grid barrier gave up, re-run through the tiled pipeline)
    rec0 = h.spread_fallbacks()
    t0 = time.perf_counter()
    for p in range(npart):
        a, b = offs[p], offs[p + 1]
        dbscan_amd.fit_arrays(px[a:b], py[a:b], eps, mp, 0, handle=h, cluster_out=cl[a:b],
                              flag_out=fl[a:b])
    t_calls = time.perf_counter() - t0
    recalls = h.spread_fallbacks() - rec0
    # (a'') the same calls as a JNI caller makes them: dbscan_fit_h straight through the C-ABI
    # (ctypes with precomputed addresses: no numpy views or argument checks per call)
    lib = dbscan_amd.load()
    fit_h = lib.dbscan_fit_h
    vp = ctypes.c_void_p
    ax, ay, acl, afl = (int(a.ctypes.data) for a in (px, py, cl, fl))
    kk = ctypes.c_int32(0)
    pk = ctypes.byref(kk)
    hp = h.ptr
    calls = [(vp(ax + 8 * int(offs[p])), vp(ay + 8 * int(offs[p])), int(offs[p + 1] - offs[p]),
              vp(acl + 4 * int(offs[p])), vp(afl + int(offs[p]))) for p in range(npart)]
    t0 = time.perf_counter()
    for cx_, cy_, m_, ccl, cfl in calls:
        fit_h(hp, cx_, cy_, m_, float(eps), int(mp), 0, ccl, cfl, pk)
    t_capi = time.perf_counter() - t0
    # (a') the same calls from 4 executor threads with a handle each (Spark local[4]: the box
    # gives a process 4 hardware queues), partitions dealt round-robin
    import threading

    hs = [dbscan_amd.Handle(h.device) for _ in range(4)]

    def worker(t):
        for p in range(t, npart, 4):
            a, b = offs[p], offs[p + 1]
            dbscan_amd.fit_arrays(px[a:b], py[a:b], eps, mp, 0, handle=hs[t], cluster_out=cl[a:b],
                                  flag_out=fl[a:b])

    for hh in hs:  # (each handle's workspace allocated before the clock starts)
        dbscan_amd.fit_arrays(px[:1000], py[:1000], eps, mp, 0, handle=hh)
    rec4 = sum(hh.spread_fallbacks() for hh in hs)
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    t_calls4 = time.perf_counter() - t0
    recalls4 = sum(hh.spread_fallbacks() for hh in hs) - rec4
    for hh in hs:
        hh.close()
    # (b) one batch call, host arrays
    ts = []
    for i in range(4):
        t0 = time.perf_counter()
        dbscan_amd.fit_batch(px, py, offs, eps, mp, 0, handle=h, cluster_out=cl, flag_out=fl)
        if i:
            ts.append(time.perf_counter() - t0)
    t_batch = float(np.median(ts))
    # (c) device-resident batches, back to back
    dx, dy = torch.from_numpy(px).cuda(), torch.from_numpy(py).cuda()
    dcl = torch.empty(total, dtype=torch.int32, device="cuda")
    dfl = torch.empty(total, dtype=torch.uint8, device="cuda")
    dnk = torch.empty(npart, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    D.fit_batch_tensors_async(dx, dy, offs, eps, mp, 0, h, dcl, dfl, dnk)
    h.sync()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        D.fit_batch_tensors_async(dx, dy, offs, eps, mp, 0, h, dcl, dfl, dnk)
    h.sync()
    t_dev = (time.perf_counter() - t0) / reps
    same = bool(np.array_equal(dcl.cpu().numpy(), cl) and np.array_equal(dfl.cpu().numpy(), fl))
    del dx, dy, dcl, dfl
    torch.cuda.empty_cache()
    out["train"] = {
        "workload": (f"G(10^7) config 2 -> EvenSplitPartitioner(maxPointsPerPartition=8192): "
                     f"{npart} partitions, {total} points with eps halos (max {int(sizes.max())}, "
                     f"{int((sizes > 8192).sum())} over the one-workgroup capacity)"),
        "partitions": npart, "points_with_halos": total,
        "per_partition_calls": {"seconds": round(t_calls, 4),
                                "us_per_partition": round(t_calls / npart * 1e6, 2),
                                "recalled_partitions": int(recalls)},
        "per_partition_capi_calls": {"seconds": round(t_capi, 4),
                                     "us_per_partition": round(t_capi / npart * 1e6, 2),
                                     "what": "dbscan_fit_h per partition through ctypes with "
                                             "precomputed addresses, one thread"},
        "per_partition_calls_4_threads": {"seconds": round(t_calls4, 4),
                                          "us_per_partition": round(t_calls4 / npart * 1e6, 2),
                                          "points_per_s": round(total / t_calls4, 1),
                                          "recalled_partitions": int(recalls4)},
        "batch_host": {"seconds": round(t_batch, 4),
                       "us_per_partition": round(t_batch / npart * 1e6, 3),
                       "points_per_s": round(total / t_batch, 1)},
        "batch_device": {"ms": round(t_dev * 1e3, 4),
                         "us_per_partition": round(t_dev / npart * 1e6, 3),
                         "points_per_s": round(total / t_dev, 1), "equals_host_batch": same},
    }
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg only

        r = O.ref_fit_partitions_timed(x, y, eps, mp, rects, counts, threads, 8.0)
        out["train"]["cpu_reference_fits"] = {
            "threads": threads, "seconds": round(r["seconds"], 3), "partitions": r["parts"],
            "points_with_halos": r["outer_points"],
            "us_per_partition": round(r["seconds"] / max(1, r["parts"]) * 1e6, 1),
            "points_per_s": round(r["outer_points"] / max(r["seconds"], 1e-9), 1),
            "what": ("LocalDBSCANNaive.fit O(m^2) restated in C (oracle/reference_pipeline.c) on "
                     "the same partitions, a thread pool of `threads`, stopped after an 8 s "
                     "budget (a sample of the partitions)")}
    return out


def end_to_end(args, h, dist, world, rank, n_total, node_path, max_over_ranks, x, y):
    """Host SoA -> host labels on the same data (PCIe included), median over e2e_steps after one
    untimed step.  N = 1: dbscan_fit_h from pageable numpy arrays (the JNI case: Java arrays are
    pageable) and from pinned host memory.  Node path: each rank copies the global arrays to its
    GPU, selects its slab (zones), runs the node step and copies its owned labels back."""
    import numpy as np
    import torch

    import dbscan_amd
    from dbscan_amd import device as D

    out = {"steps": args.e2e_steps}
    if not node_path:
        hx, hy = x.cpu().numpy(), y.cpu().numpy()
        px = torch.empty(n_total, dtype=torch.float64, pin_memory=True)
        py = torch.empty(n_total, dtype=torch.float64, pin_memory=True)
        px.numpy()[:] = hx
        py.numpy()[:] = hy
        # output arrays allocated and touched once, reused by every step (a JNI caller's Java
        # arrays are resident); "fresh_outputs" allocates them per call (np.zeros: the copy back
        # then faults in 50 MB of new pages)
        ocl = np.zeros(n_total, np.int32)
        ofl = np.zeros(n_total, np.uint8)
        ocl[:] = 1
        ofl[:] = 1
        for tag, ax, ay, fresh in (("pageable", hx, hy, False), ("pinned", px.numpy(), py.numpy(),
                                   False), ("fresh_outputs", hx, hy, True)):
            ts = []
            for i in range(args.e2e_steps + 1):
                t0 = time.perf_counter()
                if fresh:
                    dbscan_amd.fit_arrays(ax, ay, args.eps, args.min_points, 0, handle=h)
                else:
                    dbscan_amd.fit_arrays(ax, ay, args.eps, args.min_points, 0, handle=h,
                                          cluster_out=ocl, flag_out=ofl)
                if i:
                    ts.append(time.perf_counter() - t0)
            t = float(np.median(ts))
            out[tag] = {"value": round(n_total / t, 1), "ms_per_step": round(t * 1e3, 3)}
        # two executor threads, one handle (stream) each, fitting back to back on the one GPU
        # (Spark local[N] runs N concurrent fits): one fit's transfers overlap the other's
        # kernels; value = points of all fits / wall time
        import threading

        h2 = dbscan_amd.Handle(h.device)
        outs = [(np.ones(n_total, np.int32), np.ones(n_total, np.uint8)) for _ in range(2)]
        reps = max(2, args.e2e_steps)

        def worker(hh, o, bar):
            dbscan_amd.fit_arrays(hx, hy, args.eps, args.min_points, 0, handle=hh,
                                  cluster_out=o[0], flag_out=o[1])  # warm
            bar.wait()
            for _ in range(reps):
                dbscan_amd.fit_arrays(hx, hy, args.eps, args.min_points, 0, handle=hh,
                                      cluster_out=o[0], flag_out=o[1])

        bar = threading.Barrier(3)
        th = [threading.Thread(target=worker, args=(hh, o, bar)) for hh, o in zip((h, h2), outs)]
        for t_ in th:
            t_.start()
        bar.wait()
        t0 = time.perf_counter()
        for t_ in th:
            t_.join()
        t = time.perf_counter() - t0
        h2.close()
        out["pipelined_2_handles"] = {"value": round(2 * reps * n_total / t, 1),
                                      "ms_per_fit": round(t / (2 * reps) * 1e3, 3)}
        out["value"] = out["pageable"]["value"]
        out["path"] = ("dbscan_fit_h: host x,y (16 B/point, pageable) -> H2D -> fit -> D2H "
                       "cluster,flag (5 B/point) into resident caller arrays, synchronous; "
                       "pipelined_2_handles: two threads with a handle each, fits back to back")
        return out
    from dbscan_amd import node

    xa, ya = D.generate_blobs(n_total, args.noise, args.dense, args.seed, h)
    comm = node.Comm(dist)
    comm.force = args.force_collectives
    bounds = node.NodeJob.chunk_bounds(n_total, comm.world)
    c0, c1 = bounds[comm.rank], bounds[comm.rank + 1]
    # this rank's chunk of the global input in host memory (pageable, as a caller's arrays),
    # and resident host output arrays for its labels
    hx, hy = xa[c0:c1].cpu().numpy(), ya[c0:c1].cpu().numpy()
    del xa, ya
    torch.cuda.empty_cache()
    ocl = np.ones(c1 - c0, np.int32)
    ofl = np.ones(c1 - c0, np.uint8)
    ops = node.HipSlabOps(h)
    ts = []
    for i in range(args.e2e_steps + 1):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tx = torch.from_numpy(hx).cuda()
        ty = torch.from_numpy(hy).cuda()
        job = node.NodeJob.from_chunk(tx, ty, c0, n_total, args.eps, args.min_points, 0, comm,
                                      ops)
        del tx, ty
        job.run()
        cl, fl = job.chunk_labels(c0, c1 - c0, bounds)
        torch.from_numpy(ocl).copy_(cl)
        torch.from_numpy(ofl).copy_(fl)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el = max_over_ranks(time.perf_counter() - t0)
        if i:
            ts.append(el)
        del job
    ops.close()
    t = float(np.median(ts))
    out.update({"value": round(n_total / t, 1), "ms_per_step": round(t * 1e3, 3),
                "path": ("each rank: H2D of its 1/N chunk of the host input (pageable), one "
                         "all_to_all routing every point to the slabs holding it (cuts from an "
                         "all-gathered sample), the node step, one all_to_all returning the "
                         "labels to the chunk owners, D2H into resident host arrays; max over "
                         "ranks")})
    return out


if __name__ == "__main__":
    main()
