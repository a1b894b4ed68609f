"""count32's scan divergence over one config-2 fit, from a DBSCAN_AB_COUNTDIV=1 build:
    ABFLAGS=-DDBSCAN_AB_COUNTDIV=1 tools/build_ab.sh cdiv WORKTREE
    DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/cdiv/libdbscan_hip.so python tools/countdiv_probe.py
Per wave iteration of count32's count loop (64 own points): the longest lane's candidate batches
(what the wave executes) against the sum over its lanes (what they need)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402


def main():
    n = int(os.environ.get("N", 10_000_000))
    lib = dbscan_amd.load()
    f = lib.dbscan_ab_countdiv
    f.argtypes = [ctypes.c_void_p]
    f.restype = ctypes.c_int
    h = dbscan_amd.Handle(0)
    x, y = D.generate_blobs(n, float(os.environ.get("NOISE", 0.0)), 1.0, 1, h)
    cl = torch.empty(n, dtype=torch.int32, device="cuda")
    fl = torch.empty(n, dtype=torch.uint8, device="cuda")
    nk = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = (ctypes.c_ulonglong * 8)()
    D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl, nk)
    h.sync()
    assert f(out) == 0
    D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl, nk)
    h.sync()
    assert f(out) == 0
    mx, sm, lanes, cores, its = (int(out[k]) for k in range(5))
    print(f"wave iterations {its}, lanes {lanes} ({lanes / its:.1f} per iteration), cores {cores}")
    print(f"batches: executed (wave max) {mx}, needed (lane sum) {sm}: "
          f"lane utilization {sm / (64 * mx):.3f} of 64, {sm / (lanes / its * mx):.3f} of the active")
    print(f"mean batches per wave iteration {mx / its:.2f}, per point {sm / lanes:.2f}")
    h.close()


if __name__ == "__main__":
    main()
