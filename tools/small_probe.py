"""Kernel durations of partition-sized fits (run under rocprofv3 --kernel-trace --stats):
the one-workgroup kernel (small.hip) and the tiled pipeline at m = 250 / 2000 / 8192, and a
tiled batch of the reference's partitions of G(10^6)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dbscan-on-spark_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402

h = dbscan_amd.Handle(0)
for m in (250, 2000, 8192):
    tx, ty = D.generate_blobs(m, 0.0, 1.0, 5, h)
    cl = torch.empty(m, dtype=torch.int32, device="cuda")
    fl = torch.empty(m, dtype=torch.uint8, device="cuda")
    for small in (8192, 0):
        h.set_small_max(small)
        for _ in range(20):
            D.fit_tensors(tx, ty, 2.55, 10, 0, h, cl, fl)
h.set_small_max(8192)
print("probe done", flush=True)
