"""Phase times of the band LDS fit (small.hip band_fit_kernel) from a DBSCAN_AB_STAMPS=1
timing build:
    ABFLAGS=-DDBSCAN_AB_STAMPS=1 tools/build_ab.sh stamps WORKTREE
    DBSCAN_LIB_PATH=dbscan-on-spark_amd/lib_ab/stamps/libdbscan_hip.so python tools/band_stamps.py
Thread 0 of workgroup 0 stamps the 100 MHz clock at the phase boundaries (its barrier waits
hold the other workgroups' lag); every workgroup records its count + union-walk time (stage end
to barrier 2), own and staged points: the slowest and the spread are printed."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "dbscan-on-spark_amd"))
import dbscan_amd  # noqa: E402
from dbscan_amd import device as D  # noqa: E402

PH = ["slice", "barrierA", "grid+rows", "barrierB", "bands+scatter", "barrierC", "stage",
      "count", "barrier1", "union walks", "publish", "barrier2", "merge", "barrier3", "roots",
      "barrier4", "numbering", "labels"]
lib = dbscan_amd.load()
f = lib.dbscan_ab_small_stamps
f.argtypes = [ctypes.c_void_p]
h = dbscan_amd.Handle(0)
buf = (ctypes.c_longlong * 24)()
fw = lib.dbscan_ab_band_wg
fw.argtypes = [ctypes.c_void_p]
wg = (ctypes.c_longlong * 768)()
for m in [int(a) for a in (sys.argv[1:] or ["12000", "20000", "40000", "65536"])]:
    tx, ty = D.generate_blobs(m, 0.0, 1.0, 5, h)
    rows = []
    for _ in range(7):
        D.fit_tensors(tx, ty, 2.55, 10, 0, h)
        f(buf)
        fw(wg)
        rows.append(np.diff(np.array([buf[i] for i in range(19)], dtype=np.int64)) / 100.0)
    r = np.median(np.array(rows), axis=0)
    print(f"m={m}: " + ", ".join(f"{p} {v:.1f}" for p, v in zip(PH, r)) +
          f"  kernel {r.sum():.1f} us", flush=True)
    a = np.array(list(wg), dtype=np.int64).reshape(64, 12)
    gw = int((a[:, 4] > 0).sum())  # (workgroups of this launch: the rest are stale rows)
    a = a[:max(gw, 1)]
    tc = (a[:, 1] - a[:, 0]) / 100.0
    tw = (a[:, 3] - a[:, 2]) / 100.0
    tl = (a[:, 6] - a[:, 2]) / 100.0
    tu = (a[:, 7] - a[:, 6]) / 100.0
    tp = (a[:, 3] - a[:, 7]) / 100.0
    tq = (a[:, 8] - a[:, 6]) / 100.0
    t0 = (a[:, 9] - a[:, 8]) / 100.0
    t1 = (a[:, 11] - a[:, 9]) / 100.0
    for name, t in (("count", tc), ("core load + walks + publish", tw), ("core load", tl),
                    ("walks alone", tu), ("publish", tp), ("chains + quarter list", tq),
                    ("adjacent pass", t0), ("distance-2 pass", t1)):
        k = int(np.argmax(t))
        print(f"  {name} per workgroup: max {t.max():.1f} us (wg {k}: own {a[k, 4]}, staged "
              f"{a[k, 5]}), median {np.median(t):.1f}; slowest 5: " +
              ", ".join(f"wg{j} {t[j]:.0f}us/{a[j, 4]}" for j in np.argsort(-t)[:5]), flush=True)
    print(f"  own points max {a[:, 4].max()} median {int(np.median(a[:, 4]))}; staged max "
          f"{a[:, 5].max()}", flush=True)
