import os, sys
sys.path.insert(0, os.path.join(os.getcwd(), "dbscan-on-spark_amd"))
import dbscan_amd
from dbscan_amd import device as D
h = dbscan_amd.Handle(0)
for cfg, (n, noise, dense, seed) in {"2": (10**7, 0.0, 1.0, 1), "3share": (12_500_000, 0.2, 1.0, 2)}.items():
    x, y = D.generate_blobs(n, noise, dense, seed, h)
    D.fit_tensors(x, y, 2.55, 10, 0, h)
    print(cfg, h.stats(), flush=True)
