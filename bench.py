"""Benchmark: points clustered/s on MI355X (BASELINE.json metric), one JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): G(n = 10^7 x N, 32 Gaussian blobs, no noise,
seed 1), eps = 2.55 (k_bar ~ 49), minPoints = 10, LocalDBSCANNaive semantics, visit order =
generation order (i.i.d. draws).  A step = one full local fit of the resident points (HBM in ->
labels in HBM).  N = 1: one dbscan_fit_device_async per step (the fit never synchronizes with
the host; the K steps are enqueued back to back and the timed region ends with one sync).  N > 1: the slab-sharded node path
(dbscan_amd/node.py): per-GPU slab fits with 2*eps halos + RCCL all-gathers of the boundary
records + global union-find + relabel; per-GPU work is fixed (weak scaling).

roofline: the dominant kernel of the timed region, timed with HIP events on the library's own
stream -- carried on the kernels' own dispatch packets (hipExtLaunchKernelGGL), so timing adds
no idle gaps between kernels; achieved = algorithmic bytes per launch (SURVEY §8d per-point
figure x points) / the kernel's average launch duration.
cpu_baseline (rank 0, N = 1): the oracle's restatement of the reference path -- the
EvenSplitPartitioner (maxPointsPerPartition = 8192) + LocalDBSCANNaive.fit O(m^2) per partition
(oracle/reference_pipeline.c), on host threads, for a bounded time on the same points.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dbscan-on-spark_amd"))

METRIC = "points clustered/sec (whole node) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Algorithmic bytes per point and launch, by kernel (SURVEY.md §8d's per-phase figures; each
# array crosses HBM once).  count = 21: the count kernel also builds the quarter
# records and the tile-local quarter union (fused), so it carries §8d's count (sorted x,y 16 +
# core 1) and union (parent 4; the union's x,y read is the count's, already in LDS).
# edge_union and quarter_root touch tile-edge strips and quarter reps only.  The §8d output 30
# is carried by final (13), the rank scan and label_sorted/permute_out.  Radix passes: 4
# launches per fit, each reading key+perm 8 and writing 8.
ALG_BYTES = {
    "bbox_partial": 16, "bin": 20, "radix_upsweep": 4, "radix_downsweep": 16, "inverse": 8,
    "scatter_xy": 36, "heads_reduce": 4, "heads_down": 16, "count": 21, "count_wave": 21,
    "count32": 21, "big_count": 21, "edge_union": 0, "quarter_root": 0, "final": 13,
    "label_sorted": 13, "permute_out": 13,
}
# The clique-grid count kernels each process one class of tiles: their per-launch algorithmic
# bytes count that class's points only (dbscan_last_stats [11..13]).
CLASS_PTS = {"count_wave": "pts_small", "count32": "pts_medium", "big_count": "pts_big"}
PIPELINE_ALG_BYTES = 132  # whole pipeline, B_alg per point

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--points-per-gpu", type=int, default=10_000_000)
    ap.add_argument("--eps", type=float, default=2.55)
    ap.add_argument("--min-points", type=int, default=10)
    ap.add_argument("--noise", type=float, default=0.0)
    ap.add_argument("--dense", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU baseline work")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="no kernel timing events")
    ap.add_argument("--profile-steps", type=int, default=3,
                    help="untimed steps with every kernel timed (the breakdown)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--node", action="store_true", help="use the node path even at N = 1")
    return ap.parse_args()


def load_traffic(kernel, n_points):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (tools/profile.sh + tools/pmc_summary.py), only if it was measured on this workload size."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(kernel, {})
        if e.get("n_points", 10_000_000) != n_points:
            return None
        return e.get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(x, y, eps, min_points, budget, threads):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # CPU baseline leg only

    rects, counts = O.ref_partition(x, y, eps, 8192)
    r = O.ref_fit_partitions_timed(x, y, eps, min_points, rects, counts, threads, budget)
    return {
        "value": r["main_points"] / r["seconds"] if r["seconds"] > 0 else None,
        "unit": "points/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"reference path restated in C (oracle/reference_pipeline.c): "
                   f"EvenSplitPartitioner(maxPointsPerPartition=8192) over the same {x.size} "
                   f"points -> {len(counts)} partitions; LocalDBSCANNaive.fit O(m^2) on the first "
                   f"{r['parts']} partitions ({r['main_points']} main / {r['outer_points']} "
                   f"points incl. eps halos) in {r['seconds']:.2f} s on {threads} threads; "
                   f"merge not timed"),
    }


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    import dbscan_amd
    from dbscan_amd import device as D

    h = dbscan_amd.Handle(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.backend)

    n_total = args.points_per_gpu * world
    if world == 1 and not args.node:
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

        job = node.NodeJob.synthetic(n_total, args.noise, args.dense, args.seed, args.eps,
                                     args.min_points, h, dist)

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
    if dist:
        t = torch.tensor([el], dtype=torch.float64,
                         device="cuda" if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if isinstance(k, torch.Tensor):
        k = int(k.item())
    prof = h.profile_read() if not args.no_profile else {}
    h.profile(False)
    stats = h.stats()

    ms_per_step = el / args.steps * 1e3
    value = n_total * args.steps / el
    roof = None
    if prof and dom in prof:
        avg_ms = prof[dom]["ms"] / max(1, prof[dom]["launches"])  # live, in the timed region
        pts = stats.get("n", args.points_per_gpu)
        unit_pts = stats.get(CLASS_PTS[dom], pts) if dom in CLASS_PTS else pts
        alg = ALG_BYTES.get(dom, 0) * unit_pts  # per launch
        achieved = alg / (avg_ms * 1e-3) / 1e9
        traffic = load_traffic(dom, pts) if (world == 1 and not args.node) else None
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "kernel": dom, "avg_launch_ms": round(avg_ms, 4),
                "alg_bytes_per_point": ALG_BYTES.get(dom, 0), "points_per_launch": unit_pts,
                "pipeline_frac": round(PIPELINE_ALG_BYTES * pts / (ms_per_step * 1e-3) / 1e9
                                       / HBM_PEAK_GBS, 5)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.node:
        sx, sy = x.cpu().numpy(), y.cpu().numpy()
        cpu = cpu_baseline(sx, sy, args.eps, args.min_points, args.cpu_budget, args.cpu_threads)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "points/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (device generator G(n, noise, dense, seed), SURVEY §8d)",
            "config": {
                "workload": (f"G({n_total} points, 32 Gaussian blobs, noise={args.noise}, "
                             f"dense={args.dense}, seed={args.seed}), eps={args.eps}, "
                             f"minPoints={args.min_points}, LocalDBSCANNaive semantics"),
                "n_points": n_total, "eps": args.eps, "min_points": args.min_points,
                "parallelism": ("single GPU" if world == 1 and not args.node else
                                f"slab x{world} + {'RCCL' if args.backend == 'nccl' else args.backend} merge"),
                "clusters": k, "core_points": stats.get("core"),
                "occupied_cells": stats.get("cells"), "occupied_tiles": stats.get("tiles")},
            "roofline": roof,
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


if __name__ == "__main__":
    main()
