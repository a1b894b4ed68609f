"""Per-call latency of partition-sized fits (the seam's one call per partition) around and
above the LDS fits' capacity: the C-ABI call dbscan_fit_device (synchronous, inputs resident),
the asynchronous form's host enqueue time alone, and back-to-back asynchronous fits (GPU time
per fit once the host is out of the way); median of 20 calls."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402

h = dbscan_amd.Handle(0)
L = dbscan_amd.load()
for m in (8192, 12000, 20000, 40000, 65536):
    x, y = D.generate_blobs(m, 0.0, 1.0, 5, h)
    cl = torch.empty(m, dtype=torch.int32, device="cuda")
    fl = torch.empty(m, dtype=torch.uint8, device="cuda")
    kk = ctypes.c_int32(0)
    args = (h.ptr, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), m, 2.55, 10, 0,
            ctypes.c_void_p(cl.data_ptr()), ctypes.c_void_p(fl.data_ptr()), ctypes.byref(kk))
    torch.cuda.synchronize()
    for _ in range(3):
        L.dbscan_fit_device(*args)
    ts, enq = [], []
    for _ in range(20):
        t0 = time.perf_counter()
        assert L.dbscan_fit_device(*args) == 0
        ts.append(time.perf_counter() - t0)
    nk = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl, nk)
        enq.append(time.perf_counter() - t0)
        h.sync()
    t0 = time.perf_counter()
    for _ in range(20):
        D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl, nk)
    h.sync()
    b2b = (time.perf_counter() - t0) / 20
    print(f"m={m}: call {1e6 * np.median(ts):.1f} us, enqueue {1e6 * np.median(enq):.1f} us, "
          f"back-to-back {1e6 * b2b:.1f} us/fit (k={kk.value})", flush=True)
