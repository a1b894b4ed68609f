"""Host<->device transfer rates on the GPU box for the end-to-end path (dbscan_fit_h): 10^7
points = x, y 160 MB in, cluster + flag 50 MB out.  Pageable vs pinned, one stream vs two."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "dbscan-on-spark_amd")
import dbscan_amd  # noqa: E402

n = 10_000_000
dev = torch.device("cuda", 0)
hx = np.random.default_rng(1).normal(size=n) * 1000
hy = np.random.default_rng(2).normal(size=n) * 1000
px = torch.from_numpy(hx).pin_memory()
py = torch.from_numpy(hy).pin_memory()
dx = torch.empty(n, dtype=torch.float64, device=dev)
dy = torch.empty(n, dtype=torch.float64, device=dev)


def timeit(f, reps=5):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def pageable_one():
    dx.copy_(torch.from_numpy(hx))
    dy.copy_(torch.from_numpy(hy))


def pinned_one():
    dx.copy_(px, non_blocking=True)
    dy.copy_(py, non_blocking=True)


s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def pinned_two():
    with torch.cuda.stream(s1):
        dx.copy_(px, non_blocking=True)
    with torch.cuda.stream(s2):
        dy.copy_(py, non_blocking=True)


cl = torch.empty(n, dtype=torch.int32, device=dev)
fl = torch.empty(n, dtype=torch.uint8, device=dev)
pcl = torch.empty(n, dtype=torch.int32).pin_memory()
pfl = torch.empty(n, dtype=torch.uint8).pin_memory()


def d2h_pinned():
    pcl.copy_(cl, non_blocking=True)
    pfl.copy_(fl, non_blocking=True)


def d2h_pageable():
    cl.cpu()
    fl.cpu()


h = dbscan_amd.Handle(0)
from dbscan_amd import device as D  # noqa: E402

gx, gy = D.generate_blobs(n, 0.0, 1.0, 1, h)
hgx, hgy = gx.cpu().numpy(), gy.cpu().numpy()
out = {
    "h2d_pageable_ms": timeit(pageable_one),
    "h2d_pinned_one_stream_ms": timeit(pinned_one),
    "h2d_pinned_two_streams_ms": timeit(pinned_two),
    "d2h_pinned_ms": timeit(d2h_pinned),
    "d2h_pageable_ms": timeit(d2h_pageable),
    "fit_device_ms": timeit(lambda: D.fit_tensors(gx, gy, 2.55, 10, 0, h)),
    "fit_h_ms": timeit(lambda: dbscan_amd.fit_arrays(hgx, hgy, 2.55, 10, 0, handle=h)),
}
print({k: round(v, 3) for k, v in out.items()})
