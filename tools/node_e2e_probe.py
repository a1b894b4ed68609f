"""Phase times of the node path's end-to-end step at N = 1 (bench.py --node end_to_end):
    python tools/node_e2e_probe.py [config]
H2D of the host chunk, NodeJob.from_chunk (cuts + routing), the node step, chunk_labels,
D2H -- each phase synchronized and timed, median of 5 steps."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D, node  # noqa: E402


def main():
    n = 12_500_000
    h = dbscan_amd.Handle(0)
    xa, ya = D.generate_blobs(n, 0.2, 1.0, 2, h)
    hx, hy = xa.cpu().numpy(), ya.cpu().numpy()
    del xa, ya
    torch.cuda.empty_cache()
    ocl = np.ones(n, np.int32)
    ofl = np.ones(n, np.uint8)
    comm = node.Comm(None)
    ops = node.HipSlabOps(h)
    rows = []
    for i in range(6):
        t = [time.perf_counter()]

        def tick():
            torch.cuda.synchronize()
            t.append(time.perf_counter())
        tx = torch.from_numpy(hx).cuda()
        ty = torch.from_numpy(hy).cuda()
        tick()
        job = node.NodeJob.from_chunk(tx, ty, 0, n, 2.55, 10, 0, comm, ops)
        tick()
        job.run()
        tick()
        cl, fl = job.chunk_labels(0, n, [0, n])
        tick()
        torch.from_numpy(ocl).copy_(cl)
        torch.from_numpy(ofl).copy_(fl)
        tick()
        if i:
            rows.append(np.diff(t) * 1e3)
        del job, tx, ty
    ops.close()
    med = np.median(np.array(rows), axis=0)
    for name, v in zip(["h2d", "from_chunk", "step", "chunk_labels", "d2h"], med):
        print(f"{name:14s} {v:8.3f} ms")
    print(f"{'total':14s} {med.sum():8.3f} ms")


if __name__ == "__main__":
    main()
