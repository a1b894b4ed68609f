"""Phase times of the spread (multi-workgroup) LDS fit from a DBSCAN_AB_STAMPS=1 timing build:
    ABFLAGS=-DDBSCAN_AB_STAMPS=1 tools/build_ab.sh stamps WORKTREE
    DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/stamps/libdbscan_hip.so python tools/spread_stamps.py
Thread 0 of workgroup 0 stamps the 100 MHz clock at the phase boundaries (its barrier waits hold
the other workgroups' lag)."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402

IDX = [0, 2, 7, 8, 9, 10, 11, 12, 13, 14]
PH = ["stage", "count", "barrier1", "union walks", "publish", "barrier2", "merge", "numbering",
      "labels"]
lib = dbscan_amd.load()
f = getattr(lib, "dbscan_ab_small_stamps", None)  # (absent from non-timing builds: walls only)
if f is not None:
    f.argtypes = [ctypes.c_void_p]
h = dbscan_amd.Handle(0)
h.set_small_max(8192)
h.set_spread_min(0)
buf = (ctypes.c_longlong * 24)()
for m in [int(a) for a in (sys.argv[1:] or ["2000", "8192"])]:
    tx, ty = D.generate_blobs(m, 0.0, 1.0, 5, h)
    cl = torch.empty(m, dtype=torch.int32, device="cuda")
    fl = torch.empty(m, dtype=torch.uint8, device="cuda")
    rows, walls, raws = [], [], []
    k = ctypes.c_int32(0)
    args = (h.ptr, ctypes.c_void_p(tx.data_ptr()), ctypes.c_void_p(ty.data_ptr()), m, 2.55, 10, 0,
            ctypes.c_void_p(cl.data_ptr()), ctypes.c_void_p(fl.data_ptr()), ctypes.byref(k))
    for _ in range(7):
        t0 = time.perf_counter()
        D.fit_tensors(tx, ty, 2.55, 10, 0, h, cl, fl)
        walls.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        lib.dbscan_fit_device(*args)  # the C-ABI call alone (inputs already synchronized)
        raws.append(time.perf_counter() - t0)
        if f is not None:
            f(buf)
        st = np.array([buf[i] for i in IDX], dtype=np.int64)
        rows.append(np.diff(st) / 100.0)  # us
    r = np.median(np.array(rows), axis=0)
    print(f"m={m}: " + ", ".join(f"{p} {v:.1f}" for p, v in zip(PH, r)) +
          f"  kernel {r.sum():.1f} us, call {np.median(walls) * 1e6:.1f} us, C-ABI call alone "
          f"{np.median(raws) * 1e6:.1f} us", flush=True)
