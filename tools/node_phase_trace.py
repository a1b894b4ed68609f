"""Phase trace of the node path (dbscan_amd/node.py) on config 3's per-GPU share, with the
collectives of a one-rank RCCL process group forced (the N > 1 code path on one GPU):

  setup   NodeJob.synthetic: generation, cuts, zones, slab selection, the job's shared points,
          a-side all-gather and merge arrays -- twice (the first call pays the one-time costs:
          torch kernels loaded, allocator growth, RCCL communicator warm-up)
  e2e     bench.py's end_to_end step: H2D of the host chunk, NodeJob.from_chunk (sample + cuts,
          routing, all_to_all, columns, job setup), the node step (NodeJob.run's phases),
          chunk_labels (owned points, records, all_to_all, scatter), D2H; median of 5 steps

Every phase is synchronized (torch.cuda.synchronize) and timed on the host.
    python tools/node_phase_trace.py [--no-force] [--points N]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D, node  # noqa: E402


class Ticker:
    def __init__(self):
        self.rows = []
        self.t = None

    def start(self):
        torch.cuda.synchronize()
        self.t = time.perf_counter()

    def __call__(self, name):
        torch.cuda.synchronize()
        now = time.perf_counter()
        self.rows.append((name, (now - self.t) * 1e3))
        self.t = now


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-force", action="store_true")
    ap.add_argument("--points", type=int, default=12_500_000)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    force = not a.no_force
    n = a.points
    torch.cuda.set_device(0)
    h = dbscan_amd.Handle(0)
    if force:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    out = {"points": n, "forced_collectives": force, "setup": [], "e2e": {}}
    for rep in range(2):
        tk = Ticker()
        tk.start()
        job = node.NodeJob.synthetic(n, 0.2, 1.0, 2, 2.55, 10, h, dist if force else None,
                                     force=force, tick=tk)
        job.run()
        tk("first step")
        out["setup"].append({k: round(v, 3) for k, v in tk.rows})
        job.close()
        del job
        torch.cuda.empty_cache()
    xa, ya = D.generate_blobs(n, 0.2, 1.0, 2, h)
    hx, hy = xa.cpu().numpy(), ya.cpu().numpy()
    del xa, ya
    torch.cuda.empty_cache()
    ocl, ofl = np.ones(n, np.int32), np.ones(n, np.uint8)
    comm = node.Comm(dist if force else None)
    comm.force = force
    ops = node.HipSlabOps(h)
    runs = []
    for i in range(a.steps + 1):
        tk = Ticker()
        tk.start()
        tx = torch.from_numpy(hx).cuda()
        ty = torch.from_numpy(hy).cuda()
        tk("h2d")
        job = node.NodeJob.from_chunk(tx, ty, 0, n, 2.55, 10, 0, comm, ops, tick=tk)
        del tx, ty
        job.run(tick=lambda name: tk("step: " + name))
        cl, fl = job.chunk_labels(0, n, [0, n], tick=tk)
        torch.from_numpy(ocl).copy_(cl)
        torch.from_numpy(ofl).copy_(fl)
        tk("d2h")
        if i:
            runs.append(tk.rows)
        del job
    ops.close()
    names = [k for k, _ in runs[0]]
    med = {k: round(float(np.median([r[j][1] for r in runs])), 3) for j, k in enumerate(names)}
    med["total"] = round(sum(med.values()), 3)
    out["e2e"] = med
    print(json.dumps(out, indent=1), flush=True)
    if force:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
