"""Phase times of the one-workgroup fit (small.hip) from a DBSCAN_AB_STAMPS=1 timing build:
    ABFLAGS=-DDBSCAN_AB_STAMPS=1 tools/build_ab.sh stamps WORKTREE
    DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/stamps/libdbscan_hip.so python tools/small_stamps.py
Thread 0 of the workgroup stamps the 100 MHz clock at the phase boundaries."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402

PH = ["load + bbox + grid", "counting sort", "count", "union", "roots + numbering", "labels"]
lib = dbscan_amd.load()
f = lib.dbscan_ab_small_stamps
f.argtypes = [ctypes.c_void_p]
h = dbscan_amd.Handle(0)
h.set_small_max(8192)  # every size through the one-workgroup kernel
buf = (ctypes.c_longlong * 24)()
for m in (250, 2000, 8192):
    tx, ty = D.generate_blobs(m, 0.0, 1.0, 5, h)
    cl = torch.empty(m, dtype=torch.int32, device="cuda")
    fl = torch.empty(m, dtype=torch.uint8, device="cuda")
    rows = []
    for _ in range(5):
        D.fit_tensors(tx, ty, 2.55, 10, 0, h, cl, fl)
        f(buf)
        st = np.array(buf[:7], dtype=np.int64)
        rows.append(np.diff(st) / 100.0)  # us
    r = np.median(np.array(rows), axis=0)
    print(f"m={m}: " + ", ".join(f"{p} {v:.1f}" for p, v in zip(PH, r)) + f"  total {r.sum():.1f} us",
          flush=True)
