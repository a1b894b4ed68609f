"""edge_union's pair-test outcomes over one config-2 fit, from a DBSCAN_AB_EDGE_COUNT=1 build:
    ABFLAGS=-DDBSCAN_AB_EDGE_COUNT=1 tools/build_ab.sh ecount WORKTREE
    DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/ecount/libdbscan_hip.so python tools/edge_probe.py
Counters (fit.hip EDGE_CNT): trips (tile sides with cores), pairs tested at quarter distance 1
and 2 (not yet joined in LDS), full tests through registers / the generic loop (rep pair not
within eps), pairs found, global unions, trips over 64 nodes."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402

NAMES = ["trips", "pairs d1", "pairs d2", "full (regs)", "full (generic)", "found",
         "global unions", "trips > 64 nodes"]


def main():
    n = int(os.environ.get("N", 10_000_000))
    noise = float(os.environ.get("NOISE", 0.0))
    lib = dbscan_amd.load()
    f = lib.dbscan_ab_edge_counts
    f.argtypes = [ctypes.c_void_p]
    f.restype = ctypes.c_int
    h = dbscan_amd.Handle(0)
    x, y = D.generate_blobs(n, noise, 1.0, 1, h)
    cl = torch.empty(n, dtype=torch.int32, device="cuda")
    fl = torch.empty(n, dtype=torch.uint8, device="cuda")
    nk = torch.zeros(1, dtype=torch.int32, device="cuda")
    D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl, nk)
    h.sync()
    out = (ctypes.c_ulonglong * 8)()
    assert f(out) == 0
    D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl, nk)
    h.sync()
    assert f(out) == 0
    for name, v in zip(NAMES, out):
        print(f"{name:18s} {v}")
    h.close()


if __name__ == "__main__":
    main()
