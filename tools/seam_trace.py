"""Kernel timeline of single tiled fits at partition sizes (run under rocprofv3 --kernel-trace):
    rocprofv3 --kernel-trace -d gpurun_out/st -o st -- python tools/seam_trace.py
then python tools/trace_fit.py <the kernel_trace.csv> prints the last fit's timeline."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dbscan-on-spark_amd"))
import torch  # noqa: E402

import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 19273
h = dbscan_amd.Handle(0)
h.set_small_max(0)
tx, ty = D.generate_blobs(m, 0.0, 1.0, 5, h)
cl = torch.empty(m, dtype=torch.int32, device="cuda")
fl = torch.empty(m, dtype=torch.uint8, device="cuda")
for _ in range(12):
    D.fit_tensors(tx, ty, 2.55, 10, 0, h, cl, fl)
print("done", m, flush=True)
