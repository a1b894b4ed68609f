"""CPU ORACLE for the local DBSCAN fit -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product path
(``dbscan-on-spark_amd``, ``libdbscan_hip.so``) never imports it and fails loudly when its HIP
library is missing.

The reference (Scala 2.10 / Spark 2.1.0 / archery 0.3.0) cannot be built or run here (no JVM,
no Scala toolchain, no jars, no network).  Parity is pinned by the reference's
own fixture ``src/test/resources/labeled_data.csv`` (copied to ``tests/golden/``).

Two independent restatements live here:

* ``liboracle.so`` (``dbscan_oracle.c`` + ``reference_pipeline.c``) -- C, ``-ffp-contract=off``:
  the literal sequential BFS (``fit_sequential``), the order-parametrised closed form with
  all-pairs scans (``fit_bruteforce``) and on an eps grid (``fit_grid``), plus the reference's
  partitioner / merge (``ref_partition``, ``ref_train``) and the timed per-partition fits used as
  the CPU baseline.
* ``py_fit_sequential`` -- a pure-Python loop restatement of
  ``LocalDBSCANNaive.scala:37-118`` / ``LocalDBSCANArchery.scala:36-112`` for small inputs,
  written separately from the C code so the two can check each other.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

import jvm  # noqa: E402  (oracle/jvm.py: JDK 7/8 Double.toString, Scala 2.10 hashing)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

BORDER, CORE, NOISE, NOT_FLAGGED = 0, 1, 2, 3  # DBSCANLabeledPoint.scala:30
NAIVE, ARCHERY, ARCHERY_F32BOX = 0, 1, 2

_lib = None


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def scala_range_count(start: float, end: float, step: float, inclusive: bool = False) -> int:
    """Scala 2.10 NumericRange.count(start, end, step, isInclusive) for Double ranges
    (`start until end by step`, EvenSplitPartitioner.scala:150-152), restated with Python's
    decimal module: diff = end - start in double arithmetic; quot = (BigDecimal(diff) /
    BigDecimal(step)) at DECIMAL128 (34 digits, HALF_EVEN), doubleValue, toLong; rem =
    BigDecimal remainder (zero iff the decimals divide exactly); BigDecimal(d) is the decimal
    of Double.toString(d) as JDK 7/8 print it (oracle/jvm.py jdk8_double_string; longer than
    the shortest round-trip digits for ~0.3% of doubles)."""
    import decimal
    from fractions import Fraction

    if step == 0.0:
        raise ValueError("step cannot be 0.")
    if start == end:
        return 1 if inclusive else 0
    if (start < end) != (step > 0.0):
        return 0
    start, end, step = float(start), float(end), float(step)
    diff = end - start
    d = decimal.Decimal(jvm.jdk8_double_string(diff))
    s = decimal.Decimal(jvm.jdk8_double_string(step))
    ctx = decimal.Context(prec=34, rounding=decimal.ROUND_HALF_EVEN)
    q = float(ctx.divide(d, s))  # float(Decimal) is correctly rounded
    jumps = int(q) if q == q else 0
    exact = (Fraction(d) / Fraction(s)).denominator == 1
    count = jumps + (0 if (not inclusive and exact) else 1)
    if count > 2 ** 31 - 1 or count < 0:
        raise ValueError("seqs cannot contain more than Int.MaxValue elements.")
    return count


_RANGE_COUNT_FN = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double)


def _range_count_py(a, b, c):
    try:
        return scala_range_count(a, b, c)
    except ValueError:
        return -1


_range_count_cb = _RANGE_COUNT_FN(_range_count_py)

_SPLIT_KEY_FN = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double)
_split_key_cb = _SPLIT_KEY_FN(lambda a, b, c, d: jvm.split_order_key(a, b, c, d))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        dp, i64, i32, vp = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.oracle_fit_sequential.argtypes = [dp, dp, i64, ctypes.c_double, i32, i32, vp, vp]
        L.oracle_fit_sequential.restype = i32
        L.oracle_fit_bruteforce.argtypes = [dp, dp, i64, ctypes.c_double, i32, i32, vp, vp, vp]
        L.oracle_fit_bruteforce.restype = i32
        L.oracle_fit_grid.argtypes = [dp, dp, i64, ctypes.c_double, i32, i32, i32, vp, vp, vp]
        L.oracle_fit_grid.restype = i32
        L.oracle_fit_bfs_grid.argtypes = [dp, dp, i64, ctypes.c_double, i32, i32, vp, vp]
        L.oracle_fit_bfs_grid.restype = i32
        L.ref_partition.argtypes = [dp, dp, i64, ctypes.c_double, i64, vp, vp, i64]
        L.ref_partition.restype = i64
        L.ref_partition_cells.argtypes = [dp, dp, dp, i64, i64, ctypes.c_double, vp, vp, i64]
        L.ref_partition_cells.restype = i64
        L.ref_fit_partitions_timed.argtypes = [dp, dp, i64, ctypes.c_double, i32, dp, dp, i64,
                                               i32, ctypes.c_double, vp, vp, vp]
        L.ref_fit_partitions_timed.restype = ctypes.c_double
        L.ref_train.argtypes = [dp, dp, i64, ctypes.c_double, i32, i64, i32, vp, vp, vp, vp,
                                vp, i64]
        L.ref_train.restype = i64
        L.oracle_slab_fit.argtypes = [dp, dp, vp, i64, ctypes.c_double, i32, i32, vp, vp]
        L.oracle_slab_fit.restype = i32
        L.oracle_slab_label.argtypes = [dp, dp, vp, i64, ctypes.c_double, vp, vp, vp, vp, vp,
                                        i32, vp, vp]
        L.oracle_slab_label.restype = i32
        L.oracle_set_range_count.argtypes = [_RANGE_COUNT_FN]
        L.oracle_set_range_count.restype = None
        L.oracle_set_range_count(_range_count_cb)
        L.oracle_set_split_key.argtypes = [_SPLIT_KEY_FN]
        L.oracle_set_split_key.restype = None
        L.oracle_set_split_key(_split_key_cb)
        _lib = L
    return _lib


def _xy(x, y):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    assert x.shape == y.shape and x.ndim == 1
    return x, y


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def default_threads() -> int:
    """Host threads for the pthreads formulations: the cores this process may run on, at most
    16 (the GPU box's CPU share per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def fit_sequential(x, y, eps, min_points, mode=NAIVE):
    """Literal BFS restatement. Returns (cluster int32[n], flag uint8[n], n_clusters)."""
    x, y = _xy(x, y)
    n = x.size
    cl = np.zeros(n, np.int32)
    fl = np.zeros(n, np.uint8)
    k = lib().oracle_fit_sequential(_ptr(x), _ptr(y), n, float(eps), int(min_points), int(mode),
                                    _ptr(cl), _ptr(fl))
    return cl, fl, int(k)


def fit_bfs_grid(x, y, eps, min_points, mode=NAIVE):
    """The literal BFS with neighbour queries on the eps grid (every mode, incl. ARCHERY_F32BOX:
    archery's float32 search box).  Returns (cluster int32[n], flag uint8[n], n_clusters)."""
    x, y = _xy(x, y)
    n = x.size
    cl = np.zeros(n, np.int32)
    fl = np.zeros(n, np.uint8)
    k = lib().oracle_fit_bfs_grid(_ptr(x), _ptr(y), n, float(eps), int(min_points), int(mode),
                                  _ptr(cl), _ptr(fl))
    return cl, fl, int(k)


def fit_bruteforce(x, y, eps, min_points, mode=NAIVE, with_counts=False):
    x, y = _xy(x, y)
    n = x.size
    cl = np.zeros(n, np.int32)
    fl = np.zeros(n, np.uint8)
    cnt = np.zeros(n, np.int64) if with_counts else None
    k = lib().oracle_fit_bruteforce(_ptr(x), _ptr(y), n, float(eps), int(min_points), int(mode),
                                    _ptr(cl), _ptr(fl), _ptr(cnt))
    return (cl, fl, int(k), cnt) if with_counts else (cl, fl, int(k))


def fit_grid(x, y, eps, min_points, mode=NAIVE, nthreads=None, with_counts=False):
    x, y = _xy(x, y)
    n = x.size
    cl = np.zeros(n, np.int32)
    fl = np.zeros(n, np.uint8)
    cnt = np.zeros(n, np.int64) if with_counts else None
    nt = nthreads or default_threads()
    k = lib().oracle_fit_grid(_ptr(x), _ptr(y), n, float(eps), int(min_points), int(mode), nt,
                              _ptr(cl), _ptr(fl), _ptr(cnt))
    return (cl, fl, int(k), cnt) if with_counts else (cl, fl, int(k))


def ref_partition(x, y, eps, max_points_per_partition, max_parts=1 << 16):
    """EvenSplitPartitioner over the 2*eps cell histogram. Returns (rects[k,4], counts[k])."""
    x, y = _xy(x, y)
    rects = np.zeros((max_parts, 4), np.float64)
    counts = np.zeros(max_parts, np.int64)
    k = lib().ref_partition(_ptr(x), _ptr(y), x.size, float(eps), int(max_points_per_partition),
                            _ptr(rects), _ptr(counts), max_parts)
    if k < 0:
        raise RuntimeError("ref_partition failed")
    if k > max_parts:
        return ref_partition(x, y, eps, max_points_per_partition, int(k))
    return rects[:k].copy(), counts[:k].copy()


def ref_partition_cells(cells, max_points_per_partition, mrs):
    """EvenSplitPartitioner.partition(Set[(rect, count)], max, mrs) for grid-aligned cells
    given as [(x, y, x2, y2, count), ...] (EvenSplitPartitionerSuite.scala:23-60)."""
    cx = np.array([c[0] for c in cells], np.float64)
    cy = np.array([c[1] for c in cells], np.float64)
    cc = np.array([c[4] for c in cells], np.int64)
    mp = 1024
    rects = np.zeros((mp, 4), np.float64)
    counts = np.zeros(mp, np.int64)
    k = lib().ref_partition_cells(_ptr(cx), _ptr(cy), _ptr(cc), len(cells),
                                  int(max_points_per_partition), float(mrs), _ptr(rects),
                                  _ptr(counts), mp)
    if k < 0:
        raise RuntimeError("ref_partition_cells failed")
    return [(tuple(rects[i]), int(counts[i])) for i in range(k)]


def ref_fit_partitions_timed(x, y, eps, min_points, rects, counts, nthreads, budget_s):
    """CPU baseline: restated LocalDBSCANNaive.fit on the reference's partitions (outer =
    main grown by eps, DBSCAN.scala:119,132-137), nthreads workers, until budget_s elapses.
    Returns dict(seconds, parts, outer_points, main_points)."""
    x, y = _xy(x, y)
    rects = np.ascontiguousarray(rects, np.float64)
    counts = np.ascontiguousarray(counts, np.int64)
    pd = np.zeros(1, np.int64)
    po = np.zeros(1, np.int64)
    pm = np.zeros(1, np.int64)
    el = lib().ref_fit_partitions_timed(_ptr(x), _ptr(y), x.size, float(eps), int(min_points),
                                        _ptr(rects), _ptr(counts), len(counts), int(nthreads),
                                        float(budget_s), _ptr(pd), _ptr(po), _ptr(pm))
    return dict(seconds=float(el), parts=int(pd[0]), outer_points=int(po[0]),
                main_points=int(pm[0]))


def ref_train(x, y, eps, min_points, max_points_per_partition, nthreads=None):
    """DBSCAN.train restatement (DBSCAN.scala:72-283). Returns dict with per-point global
    cluster, flag, record count (0 = lost, >1 = duplicated), n_clusters and partitions."""
    x, y = _xy(x, y)
    n = x.size
    cl = np.zeros(n, np.int32)
    fl = np.zeros(n, np.uint8)
    oc = np.zeros(n, np.int32)
    npart = np.zeros(1, np.int64)
    mp = 4096
    rects = np.zeros((mp, 4), np.float64)
    nt = nthreads or default_threads()
    k = lib().ref_train(_ptr(x), _ptr(y), n, float(eps), int(min_points),
                        int(max_points_per_partition), nt, _ptr(cl), _ptr(fl), _ptr(oc),
                        _ptr(npart), _ptr(rects), mp)
    if k < 0:
        raise RuntimeError("ref_train failed")
    npt = int(npart[0])
    return dict(cluster=cl, flag=fl, records=oc, n_clusters=int(k),
                rects=rects[:min(npt, mp)].copy())


def slab_fit(x, y, zone, eps, min_points, nthreads=None):
    """CPU restatement of dbscan_slab_fit_device (node path test double)."""
    x, y = _xy(x, y)
    zone = np.ascontiguousarray(zone, np.uint8)
    n = x.size
    core = np.zeros(n, np.uint8)
    root = np.zeros(n, np.int32)
    nt = nthreads or default_threads()
    lib().oracle_slab_fit(_ptr(x), _ptr(y), _ptr(zone), n, float(eps), int(min_points), nt,
                          _ptr(core), _ptr(root))
    return core, root


def slab_label(x, y, zone, eps, core, root, gid, gs_of_root, label_of_root, mode):
    """CPU restatement of dbscan_slab_label_device (zone-0 entries written)."""
    x, y = _xy(x, y)
    n = x.size
    args = [np.ascontiguousarray(a, t) for a, t in ((zone, np.uint8), (core, np.uint8),
                                                     (root, np.int32), (gid, np.int64),
                                                     (gs_of_root, np.int64),
                                                     (label_of_root, np.int32))]
    cl = np.zeros(n, np.int32)
    fl = np.full(n, NOT_FLAGGED, np.uint8)
    lib().oracle_slab_label(_ptr(x), _ptr(y), _ptr(args[0]), n, float(eps), _ptr(args[1]),
                            _ptr(args[2]), _ptr(args[3]), _ptr(args[4]), _ptr(args[5]),
                            int(mode), _ptr(cl), _ptr(fl))
    return cl, fl


# --------------------------------------------------------------------------------------------
# Pure-Python restatement (small n only), independent of the C code.
# --------------------------------------------------------------------------------------------

def _dist2(p, o):
    """DBSCANPoint.scala:26-30 (Python floats are IEEE doubles; no FMA in CPython)."""
    dx = o[0] - p[0]
    dy = o[1] - p[1]
    return (dx * dx) + (dy * dy)


def py_fit_sequential(points, eps, min_points, mode=NAIVE):
    """LocalDBSCANNaive.fit (mode 0) / LocalDBSCANArchery.fit semantics (mode 1) over
    `points` = list of (x, y) in visit order. Returns (clusters, flags, n_clusters)."""
    eps2 = eps * eps  # LocalDBSCANNaive.scala:33
    n = len(points)
    visited = [False] * n
    cluster = [0] * n
    flag = [NOT_FLAGGED] * n

    def neighbors(p):  # findNeighbors, :72-78 (array order, includes self)
        return [j for j in range(n) if _dist2(points[p], points[j]) <= eps2]

    total = 0
    for i in range(n):
        if visited[i]:
            continue
        visited[i] = True
        nb = neighbors(i)
        if len(nb) < min_points:
            flag[i] = NOISE
            continue
        total += 1
        c = total
        flag[i] = CORE
        cluster[i] = c
        queue = [nb]
        while queue:
            for j in queue.pop(0):
                if not visited[j]:
                    visited[j] = True
                    cluster[j] = c
                    nn = neighbors(j)
                    if len(nn) >= min_points:
                        flag[j] = CORE
                        queue.append(nn)
                    else:
                        flag[j] = BORDER
                if mode != NAIVE and cluster[j] == 0:  # LocalDBSCANArchery re-claim
                    cluster[j] = c
                    flag[j] = BORDER
    return cluster, flag, total


def load_labeled_csv(path):
    """labeled_data.csv rows `x,y,label` (LocalDBSCANArcherySuite.scala:66-77)."""
    data = np.loadtxt(path, delimiter=",", dtype=np.float64)
    return data[:, 0].copy(), data[:, 1].copy(), data[:, 2].copy()
