"""Host-side mirror of the reference's local-fit interface, backed by libdbscan_hip.so.

Mirrors (src/main/scala/org/apache/spark/mllib/clustering/dbscan/):
  DBSCANPoint              DBSCANPoint.scala:21-32   (x = vector(0), y = vector(1), distanceSquared)
  DBSCANLabeledPoint/Flag  DBSCANLabeledPoint.scala:24-47 (Unknown = 0, Flag ordinals, toString)
  LocalDBSCANNaive         LocalDBSCANNaive.scala:31-120  (fit in input order, Naive noise rule)
  LocalDBSCANArchery       LocalDBSCANArchery.scala:32-126 (fit, Noise re-claimed as Border)
Same names, argument meaning and error behaviour: a vector with fewer than two coordinates
raises IndexError (the reference throws IndexOutOfBounds from vector(1)); `fit` never raises on
valid input and returns fresh labeled points in input order with visited = True.
Everything is computed by the gfx950 kernels; there is no CPU path.
"""
from __future__ import annotations

import ctypes
import enum
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib

Unknown = 0  # DBSCANLabeledPoint.scala:26


class Flag(enum.IntEnum):  # DBSCANLabeledPoint.scala:28-31
    Border = 0
    Core = 1
    Noise = 2
    NotFlagged = 3


class DBSCANPoint:
    """case class DBSCANPoint(vector: Vector) -- equality/hash on the whole vector."""

    __slots__ = ("vector",)

    def __init__(self, vector: Sequence[float]):
        self.vector = tuple(float(v) for v in vector)

    @property
    def x(self) -> float:
        return self.vector[0]

    @property
    def y(self) -> float:
        return self.vector[1]

    def distanceSquared(self, other: "DBSCANPoint") -> float:  # DBSCANPoint.scala:26-30
        dx = other.x - self.x
        dy = other.y - self.y
        return (dx * dx) + (dy * dy)

    def __eq__(self, other):
        return isinstance(other, DBSCANPoint) and self.vector == other.vector

    def __hash__(self):
        return hash(self.vector)

    def __repr__(self):
        return f"DBSCANPoint([{','.join(repr(v) for v in self.vector)}])"


class DBSCANLabeledPoint(DBSCANPoint):
    __slots__ = ("flag", "cluster", "visited")

    def __init__(self, vector: Sequence[float]):
        super().__init__(vector.vector if isinstance(vector, DBSCANPoint) else vector)
        self.flag = Flag.NotFlagged
        self.cluster = Unknown
        self.visited = False

    def __str__(self):  # DBSCANLabeledPoint.scala:43-45: s"$vector,$cluster,$flag"
        return f"[{','.join(repr(v) for v in self.vector)}],{self.cluster},{self.flag.name}"


_tls_handles = {}


def default_handle(device: int = 0) -> _lib.Handle:
    h = _tls_handles.get(device)
    if h is None:
        h = _lib.Handle(device)
        _tls_handles[device] = h
    return h


def fit_arrays(x, y, eps: float, min_points: int, mode: int = _lib.MODE_NAIVE,
               handle: Optional[_lib.Handle] = None, cluster_out: Optional[np.ndarray] = None,
               flag_out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray, int]:
    """Fit host arrays (input order = visit order). Returns (cluster int32, flag uint8, k).
    cluster_out / flag_out: caller-owned output arrays to fill (reused across calls, as a JNI
    caller's Java arrays are: no fresh pages to fault in during the copy back)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    if x.shape != y.shape or x.ndim != 1:
        raise ValueError("x and y must be 1-D arrays of equal length")
    n = x.size
    cl = cluster_out if cluster_out is not None else np.zeros(n, np.int32)
    fl = flag_out if flag_out is not None else np.zeros(n, np.uint8)
    if cl.dtype != np.int32 or fl.dtype != np.uint8 or cl.shape != (n,) or fl.shape != (n,) \
            or not (cl.flags.c_contiguous and fl.flags.c_contiguous):
        raise ValueError("cluster_out / flag_out: contiguous int32[n] / uint8[n]")
    k = ctypes.c_int32(0)
    h = handle or default_handle()
    _lib.check(_lib.load().dbscan_fit_h(
        h.ptr, x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p), n,
        float(eps), int(min_points), int(mode), cl.ctypes.data_as(ctypes.c_void_p),
        fl.ctypes.data_as(ctypes.c_void_p), ctypes.byref(k)))
    return cl, fl, int(k.value)


def fit_batch(x, y, offsets, eps: float, min_points: int, mode: int = _lib.MODE_NAIVE,
              handle: Optional[_lib.Handle] = None, cluster_out: Optional[np.ndarray] = None,
              flag_out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Independent local fits of a batch of partitions (dbscan_fit_batch): partition p is
    x[offsets[p]:offsets[p+1]] (visit order = array order), fitted exactly as fit_arrays would
    fit it alone.  Returns (cluster int32[n], flag uint8[n], n_clusters int32[n_parts]) with
    partition-local cluster ids -- DBSCAN.scala:153-154's flatMapValues(fit) over an executor's
    partitions in one call."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    offs = np.ascontiguousarray(offsets, dtype=np.int64)
    if x.shape != y.shape or x.ndim != 1 or offs.ndim != 1 or offs.size < 1:
        raise ValueError("x, y: equal 1-D arrays; offsets: n_parts + 1 values")
    n = x.size
    if offs[0] < 0 or np.any(np.diff(offs) < 0) or offs[-1] > n:
        raise ValueError("offsets: non-decreasing, from >= 0, within the arrays")
    cl = cluster_out if cluster_out is not None else np.zeros(n, np.int32)
    fl = flag_out if flag_out is not None else np.zeros(n, np.uint8)
    if cl.dtype != np.int32 or fl.dtype != np.uint8 or cl.shape != (n,) or fl.shape != (n,) \
            or not (cl.flags.c_contiguous and fl.flags.c_contiguous):
        raise ValueError("cluster_out / flag_out: contiguous int32[n] / uint8[n]")
    nk = np.zeros(max(1, offs.size - 1), np.int32)
    h = handle or default_handle()
    vp = ctypes.c_void_p
    _lib.check(_lib.load().dbscan_fit_batch(
        h.ptr, x.ctypes.data_as(vp), y.ctypes.data_as(vp), offs.ctypes.data_as(vp),
        offs.size - 1, float(eps), int(min_points), int(mode), cl.ctypes.data_as(vp),
        fl.ctypes.data_as(vp), nk.ctypes.data_as(vp)))
    return cl, fl, nk[:offs.size - 1]


def duplicate(x, y, rects, eps: float) -> Tuple[np.ndarray, np.ndarray]:
    """DBSCAN.scala:116-137: the input indices every partition's outer rectangle (rectangle
    grown by eps) holds, each partition in input order.  rects: (k, 4) array of (x, y, x2, y2).
    Returns (offsets int64[k+1], index int64[total])."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    r = np.ascontiguousarray(np.asarray(rects, np.float64).reshape(-1, 4))
    k = r.shape[0]
    offs = np.zeros(k + 1, np.int64)
    L, vp = _lib.load(), ctypes.c_void_p
    tot = L.dbscan_duplicate(x.ctypes.data_as(vp), y.ctypes.data_as(vp), x.size,
                             r.ctypes.data_as(vp), k, float(eps), offs.ctypes.data_as(vp), None,
                             0)
    if tot < 0:
        _lib.check(int(tot))
    idx = np.zeros(max(1, tot), np.int64)
    tot2 = L.dbscan_duplicate(x.ctypes.data_as(vp), y.ctypes.data_as(vp), x.size,
                              r.ctypes.data_as(vp), k, float(eps), offs.ctypes.data_as(vp),
                              idx.ctypes.data_as(vp), idx.size)
    if tot2 != tot:
        _lib.check(int(tot2) if tot2 < 0 else _lib.DBSCAN_EARG)
    return offs, idx[:tot]


def train_node(x, y, eps: float, min_points: int, mode: int = _lib.MODE_NAIVE,
               n_shards: int = 0) -> Tuple[np.ndarray, np.ndarray, int]:
    """Whole-node fit of host arrays in one process (dbscan_train_node): n_shards x-slabs over
    the visible GPUs (0: one per GPU), merged exactly -- the result equals one fit of all
    points.  The DBSCAN.train(...).labeledPoints of DBSCAN.scala:91-283 for one node."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    if x.shape != y.shape or x.ndim != 1:
        raise ValueError("x and y must be 1-D arrays of equal length")
    n = x.size
    cl = np.zeros(n, np.int32)
    fl = np.zeros(n, np.uint8)
    k = ctypes.c_int64(0)
    _lib.check(_lib.load().dbscan_train_node(
        x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p), n, float(eps),
        int(min_points), int(mode), int(n_shards), cl.ctypes.data_as(ctypes.c_void_p),
        fl.ctypes.data_as(ctypes.c_void_p), ctypes.byref(k)))
    return cl, fl, int(k.value)


def train_node_shards() -> List[dict]:
    """What the calling thread's last train_node ran, per shard: the device its worker ran on
    (shard s on device s % device_count), its points with eps halos, its shared points."""
    L = _lib.load()
    k = L.dbscan_train_node_shards(None, None, None, 0)
    _lib.check(int(k) if k < 0 else _lib.DBSCAN_OK)
    dev = (ctypes.c_int32 * max(1, k))()
    pts = (ctypes.c_int64 * max(1, k))()
    sh = (ctypes.c_int64 * max(1, k))()
    L.dbscan_train_node_shards(dev, pts, sh, k)
    return [{"device": int(dev[s]), "points": int(pts[s]), "shared": int(sh[s])} for s in range(k)]


class _LocalDBSCAN:
    _mode = _lib.MODE_NAIVE

    def __init__(self, eps: float, minPoints: int, handle: Optional[_lib.Handle] = None):
        self.eps = float(eps)
        self.minPoints = int(minPoints)
        self.minDistanceSquared = self.eps * self.eps  # LocalDBSCANNaive.scala:33
        self._handle = handle

    def fit(self, points: Iterable[DBSCANPoint]) -> List[DBSCANLabeledPoint]:
        pts = list(points)
        vecs = [p.vector if isinstance(p, DBSCANPoint) else tuple(p) for p in pts]
        x = np.fromiter((v[0] for v in vecs), np.float64, len(vecs))
        y = np.fromiter((v[1] for v in vecs), np.float64, len(vecs))  # IndexError if < 2 dims
        cl, fl, _ = fit_arrays(x, y, self.eps, self.minPoints, self._mode, self._handle)
        out = []
        for v, c, f in zip(vecs, cl.tolist(), fl.tolist()):
            lp = DBSCANLabeledPoint(v)
            lp.cluster = c
            lp.flag = Flag(f)
            lp.visited = True
            out.append(lp)
        return out


class LocalDBSCANNaive(_LocalDBSCAN):
    """LocalDBSCANNaive(eps, minPoints).fit(points) -- the one DBSCAN.train uses."""

    _mode = _lib.MODE_NAIVE


class LocalDBSCANArchery(_LocalDBSCAN):
    """LocalDBSCANArchery(eps, minPoints).fit(points): neighbours are the points whose float32
    coordinates lie in the float32 box (x-eps, y-eps, x+eps, y+eps) AND pass the fp64 predicate
    (LocalDBSCANArchery.scala:38-41,114-124), Noise re-claimed as Border (:103-106).  Visit
    order = input order (archery's R-tree entry order is not reproducible; its labels match up
    to permutation).  f32_box=False: the exact fp64 neighbour set (DBSCAN_MODE_ARCHERY)."""

    _mode = _lib.MODE_ARCHERY_F32BOX

    def __init__(self, eps: float, minPoints: int, handle: Optional[_lib.Handle] = None,
                 f32_box: bool = True):
        super().__init__(eps, minPoints, handle)
        self._mode = _lib.MODE_ARCHERY_F32BOX if f32_box else _lib.MODE_ARCHERY
