"""Host-side cost of enqueueing one step (no synchronization inside), for the direct fit and the
node step at N = 1: is the host or the GPU the bottleneck?"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "dbscan-on-spark_amd"))
import torch  # noqa: E402

import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402
from dbscan_amd import node  # noqa: E402

n, eps, mp = 10_000_000, 2.55, 10
h = dbscan_amd.Handle(0)
x, y = D.generate_blobs(n, 0.0, 1.0, 1, h)
cl = torch.empty(n, dtype=torch.int32, device="cuda")
fl = torch.empty(n, dtype=torch.uint8, device="cuda")
nk = torch.zeros(1, dtype=torch.int32, device="cuda")
for _ in range(3):
    D.fit_tensors_async(x, y, eps, mp, 0, h, cl, fl, nk)
h.sync()
enq, tot = [], []
for _ in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    D.fit_tensors_async(x, y, eps, mp, 0, h, cl, fl, nk)
    t1 = time.perf_counter()
    h.sync()
    t2 = time.perf_counter()
    enq.append(t1 - t0)
    tot.append(t2 - t0)
print(f"direct fit: enqueue {1e3 * min(enq):.3f} ms (median {1e3 * sorted(enq)[5]:.3f}), "
      f"enqueue+sync {1e3 * min(tot):.3f} ms")
del x, y
job = node.NodeJob.synthetic(n, 0.0, 1.0, 1, eps, mp, h, None)
for _ in range(3):
    job.run()
torch.cuda.synchronize()
marks = {}


def tick(name):
    marks.setdefault(name, []).append(time.perf_counter())


for _ in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    marks.setdefault("start", []).append(t0)
    job.run(tick)
    torch.cuda.synchronize()
    marks.setdefault("end", []).append(time.perf_counter())
names = list(marks)
for a, b in zip(names, names[1:]):
    d = sorted(1e3 * (q - p) for p, q in zip(marks[a], marks[b]))
    print(f"node {a:>10} -> {b:<10} host {d[5]:.3f} ms")
