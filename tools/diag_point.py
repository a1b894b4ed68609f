"""Debug helper: one point's GPU vs oracle labels on the golden csv, with its neighbourhood."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dbscan-on-spark_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import dbscan_amd  # noqa: E402
import oracle as O  # noqa: E402

x, y, lab = O.load_labeled_csv(os.path.join(ROOT, "tests", "golden", "labeled_data.csv"))
eps = float(np.float32(0.3))
h = dbscan_amd.Handle(0)
cl, fl, k = dbscan_amd.fit_arrays(x, y, eps, 10, 0, handle=h)
rc, rf, rk = O.fit_sequential(x, y, eps, 10, 0)
print("stats", h.stats())
bad = np.flatnonzero((cl != rc) | (fl != rf))
for i in bad[:5]:
    d2 = (x - x[i]) ** 2 + (y - y[i]) ** 2
    nb = np.flatnonzero(d2 <= eps * eps)
    print(f"point {i}: gpu ({cl[i]},{fl[i]}) oracle ({rc[i]},{rf[i]}) |N|={nb.size} "
          f"xy=({x[i]:.6f},{y[i]:.6f})")
    print("  neighbours", nb.tolist(), "oracle flags", rf[nb].tolist(), "gpu flags", fl[nb].tolist())
h.close()
