import sys, time, os
sys.path.insert(0, "dbscan-on-spark_amd")
import torch, dbscan_amd
from dbscan_amd import device as D
h = dbscan_amd.Handle(0)
x, y = D.generate_blobs(10_000_000, 0.0, 1.0, 1, h)
cl = torch.empty(x.numel(), dtype=torch.int32, device="cuda"); fl = torch.empty(x.numel(), dtype=torch.uint8, device="cuda")
def run(K):
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(K): D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl)
    h.sync(); torch.cuda.synchronize(); return (time.perf_counter() - t) / K * 1e3
run(3)
for rep in range(2):
    h.profile(False); print("off", run(20))
    h.profile(True, kernels=True); h.profile_only(None); h.profile_reset(); print("kernels-all", run(20))
    h.profile_only("count"); h.profile_reset(); print("count-only", run(20), h.profile_read())
    h.profile(True); h.profile_only(None); h.profile_reset(); print("stages", run(20))
