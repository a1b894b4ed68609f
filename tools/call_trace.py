"""Repeated single seam calls, for a rocprofv3 HIP-API + kernel + copy trace of where one call's
time goes (host work before the launch, launch-to-start, the kernels, end-to-return):
    rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv \
        -d gpurun_out/ct -o run -- python3 tools/call_trace.py
    python3 tools/call_timeline.py gpurun_out/ct
Each block (size x {device, host}) runs 40 calls after 5 warm ones; blocks are separated by
20 ms of idle so the timeline tool can cut them apart.  Also prints the wall time per call."""
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
sizes = [int(a) for a in sys.argv[1:]] or [250, 2000, 8192, 65536]
for m in sizes:
    x, y = D.generate_blobs(m, 0.0, 1.0, 5, h)
    hx, hy = x.cpu().numpy(), y.cpu().numpy()
    cl = torch.empty(m, dtype=torch.int32, device="cuda")
    fl = torch.empty(m, dtype=torch.uint8, device="cuda")
    hcl = np.ones(m, np.int32)
    hfl = np.ones(m, np.uint8)
    kk = ctypes.c_int32(0)
    vp = ctypes.c_void_p
    dargs = (h.ptr, vp(x.data_ptr()), vp(y.data_ptr()), m, 2.55, 10, 0, vp(cl.data_ptr()),
             vp(fl.data_ptr()), ctypes.byref(kk))
    hargs = (h.ptr, vp(hx.ctypes.data), vp(hy.ctypes.data), m, 2.55, 10, 0,
             vp(hcl.ctypes.data), vp(hfl.ctypes.data), ctypes.byref(kk))
    torch.cuda.synchronize()
    for kind, fn, args in (("device", L.dbscan_fit_device, dargs), ("host", L.dbscan_fit_h, hargs)):
        time.sleep(0.02)
        for _ in range(5):
            fn(*args)
        ts = []
        for _ in range(40):
            t0 = time.perf_counter()
            assert fn(*args) == 0
            ts.append(time.perf_counter() - t0)
        print(f"{m} {kind}: {np.median(ts) * 1e6:.1f} us per call (median of 40)", flush=True)
time.sleep(0.02)
h.close()
