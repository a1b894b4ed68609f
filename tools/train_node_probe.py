"""Phase times of the one-process whole-node entry dbscan_train_node on config 5's data.

    DBSCAN_NODE_TRACE=1 python tools/train_node_probe.py [n] [shards]

G(n, 20% noise, seed 4) from the device generator, copied to host arrays, then
dbscan_train_node with `shards` x-slabs (default 8) on the visible GPUs; the library prints
each phase's wall time on stderr (DBSCAN_NODE_TRACE=1)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dbscan-on-spark_amd"))

import torch  # noqa: E402

import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    shards = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    h = dbscan_amd.Handle(0)
    t0 = time.time()
    tx, ty = D.generate_blobs(n, 0.2, 1.0, 4, h)
    hx, hy = tx.cpu().numpy(), ty.cpu().numpy()
    del tx, ty
    h.close()
    torch.cuda.empty_cache()
    print(f"generated + copied {n} points: {time.time() - t0:.1f} s", flush=True)
    t0 = time.time()
    cl, fl, k = dbscan_amd.train_node(hx, hy, 2.55, 10, 0, shards)
    print(f"train_node {shards} slabs: {time.time() - t0:.1f} s, {k} clusters, "
          f"{int((fl == 1).sum())} core", flush=True)


if __name__ == "__main__":
    main()
