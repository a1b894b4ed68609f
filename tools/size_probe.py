"""Per-call latency (dbscan_fit_device, inputs resident; median of 20 calls after 3) over
partition sizes, for comparing the LDS fit forms:
    [DBSCAN_LIB_PATH=...] [BAND_MIN=n] python tools/size_probe.py [m ...]
(BAND_MIN: the handle's dbscan_set_band_min, to time the band form below its default)"""
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
if os.environ.get("BAND_MIN"):
    h.set_band_min(int(os.environ["BAND_MIN"]))
L = dbscan_amd.load()
sizes = [int(a) for a in sys.argv[1:]] or [600, 1200, 2000, 3000, 4096, 6000, 8192, 12000, 16000]
out = []
for m in sizes:
    x, y = D.generate_blobs(m, 0.0, 1.0, 5, h)
    cl = torch.empty(m, dtype=torch.int32, device="cuda")
    fl = torch.empty(m, dtype=torch.uint8, device="cuda")
    kk = ctypes.c_int32(0)
    args = (h.ptr, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), m, 2.55, 10, 0,
            ctypes.c_void_p(cl.data_ptr()), ctypes.c_void_p(fl.data_ptr()), ctypes.byref(kk))
    torch.cuda.synchronize()
    for _ in range(3):
        L.dbscan_fit_device(*args)
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        assert L.dbscan_fit_device(*args) == 0
        ts.append(time.perf_counter() - t0)
    out.append(f"{m}: {np.median(ts) * 1e6:.1f}")
print("call us  " + ", ".join(out), flush=True)
