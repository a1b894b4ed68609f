import os, sys, time
sys.path.insert(0, "dbscan-on-spark_amd")
import torch, dbscan_amd
from dbscan_amd import node
h = dbscan_amd.Handle(0)
ops = node.HipSlabOps(h)
n = 10_000_000
core = (torch.rand(n, device="cuda") < 0.88).to(torch.uint8)
root = torch.where(torch.rand(n, device="cuda") < 0.0015, torch.arange(n, device="cuda"), torch.zeros(n, dtype=torch.int64, device="cuda")).to(torch.int32)
zone = torch.zeros(n, dtype=torch.uint8, device="cuda")
gid = torch.arange(n, dtype=torch.int64, device="cuda")
par = torch.full((n,), -1, dtype=torch.int32, device="cuda")
gs = torch.zeros(n, dtype=torch.int64, device="cuda")
for it in range(5):
    torch.cuda.synchronize(); t = time.perf_counter()
    lr, own = ops.merge_roots(zone, gid, core, root, par, gs)
    torch.cuda.synchronize(); print("merge_roots ms", (time.perf_counter() - t) * 1e3, lr.numel())
for it in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    m = (core != 0) & (root == torch.arange(n, device="cuda", dtype=torch.int32))
    k = int(m.sum())
    torch.cuda.synchronize(); print("torch ms", (time.perf_counter() - t) * 1e3, k)
