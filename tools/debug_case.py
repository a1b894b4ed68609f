"""Run one edge fixture through the GPU fit and print where it differs from the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "dbscan-on-spark_amd"))
from conftest import load_edge_cases  # noqa: E402
import oracle as O  # noqa: E402
import dbscan_amd  # noqa: E402

name = sys.argv[1]
c = [c for c in load_edge_cases() if c["name"] == name][0]
x, y = c["x"], c["y"]
h = dbscan_amd.Handle(0)
cl, fl, k = dbscan_amd.fit_arrays(x, y, c["eps"], c["min_points"], c["mode"], handle=h)
rc, rf, rk = O.fit_grid(x, y, c["eps"], c["min_points"], c["mode"])
fin = np.isfinite(x) & np.isfinite(y)
print("k", k, "ref", rk, "stats", h.stats())
for part, m in (("finite", fin), ("nonfinite", ~fin)):
    bad = np.flatnonzero(m & ((cl != rc) | (fl != rf)))
    print(part, "n", m.sum(), "mismatch", bad.size, "gpu clusters", np.unique(cl[m])[:20],
          "ref clusters", np.unique(rc[m])[:20])
    for i in bad[:5]:
        print("  ", i, x[i], y[i], "gpu", cl[i], fl[i], "ref", rc[i], rf[i])
