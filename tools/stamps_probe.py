"""Per-phase latency of count_tile32's tiles from a DBSCAN_AB_STAMPS=1 timing build:
    ABFLAGS=-DDBSCAN_AB_STAMPS=1 tools/build_ab.sh stamps WORKTREE
    DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/stamps/libdbscan_hip.so python tools/stamps_probe.py
One fit of the bench's config-2 data (device generator); wave 0 of each workgroup stamped the
100 MHz clock at the phase boundaries (fit.hip AB_STAMP).  Prints the phase durations (us) over
the workgroups that counted a tile, and how many tiles were in flight over the kernel's span."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402

K_STAMPS, K_GRID = 12, 8192
PHASES = [("stage (meta + xy loads)", 0, 1), ("rowoff + barrier", 1, 2),
          ("count (wave 0)", 2, 3), ("count barrier", 3, 4), ("union init", 4, 5),
          ("sweep 0", 5, 6), ("sweep 1 + cmin", 6, 8), ("writes + barrier", 8, 9)]
# KERNEL=edge: a build whose edge_union_kernel stamps instead (slots 0, 1, 2, 9; 10 = nodes)
EDGE_PHASES = [("strip loads", 0, 1), ("pre-join", 1, 2), ("pair tests + unions", 2, 9)]


def main():
    n = int(os.environ.get("N", 10_000_000))
    noise = float(os.environ.get("NOISE", 0.0))
    lib = dbscan_amd.load()
    f = lib.dbscan_ab_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    f.restype = ctypes.c_int
    h = dbscan_amd.Handle(0)
    x, y = D.generate_blobs(n, noise, 1.0, 1, h)
    cl = torch.empty(n, dtype=torch.int32, device="cuda")
    fl = torch.empty(n, dtype=torch.uint8, device="cuda")
    nk = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(3):
        D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl, nk)
    h.sync()
    assert f(None, 0) == 0
    D.fit_tensors_async(x, y, 2.55, 10, 0, h, cl, fl, nk)
    h.sync()
    buf = np.zeros(K_GRID * K_STAMPS, dtype=np.int64)
    assert f(buf.ctypes.data, buf.size) == 0
    s = buf.reshape(K_GRID, K_STAMPS).astype(np.float64)
    live = s[(s[:, 0] > 0) & (s[:, 9] > 0)]
    phases = PHASES
    if os.environ.get("KERNEL") == "edge":
        phases = EDGE_PHASES
    else:
        s7 = np.where(live[:, 7] > 0, live[:, 7], live[:, 6])
        live[:, 7] = s7
    print(f"tiles stamped: {len(live)}  staged points mean {live[:, 10].mean():.0f}, own mean "
          f"{live[:, 11].mean():.0f}")
    tot = (live[:, 9] - live[:, 0]) / 100.0
    print(f"per tile total: mean {tot.mean():.2f} us  p50 {np.median(tot):.2f}  p90 "
          f"{np.percentile(tot, 90):.2f}")
    for name, a, b in phases:
        d = (live[:, b] - live[:, a]) / 100.0
        print(f"  {name:26s} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  p90 "
              f"{np.percentile(d, 90):7.2f}  share {d.sum() / ((live[:, 9] - live[:, 0]) / 100.0).sum():.2f}")
    t0, t1 = live[:, 0].min(), live[:, 9].max()
    span = (t1 - t0) / 100.0
    grid = np.linspace(t0, t1, 200)
    inflight = [((live[:, 0] <= t) & (live[:, 9] > t)).sum() for t in grid]
    print(f"kernel span (stamped) {span:.1f} us; tiles in flight: mean {np.mean(inflight):.0f} "
          f"max {np.max(inflight)}; sum of tile time / span = {tot.sum() / span:.0f}")
    starts = np.sort((live[:, 0] - t0) / 100.0)
    print("tile start quantiles (us):", np.round(np.percentile(starts, [0, 10, 25, 50, 75, 90, 100]), 1))
    big = live[:, 11] > np.percentile(live[:, 11], 75)
    print(f"largest quartile of tiles (own > {np.percentile(live[:, 11], 75):.0f}): total mean "
          f"{tot[big].mean():.2f} us")
    h.close()


if __name__ == "__main__":
    main()
