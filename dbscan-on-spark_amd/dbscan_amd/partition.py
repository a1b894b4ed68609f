"""Host-side mirror of the reference's spatial partitioner, backed by libdbscan_hip.so.

Mirrors (src/main/scala/org/apache/spark/mllib/clustering/dbscan/):
  DBSCANRectangle        DBSCANRectangle.scala:23-52  (contains, shrink, almostContains)
  EvenSplitPartitioner   EvenSplitPartitioner.scala:26-209
                         partition(toSplit, maxPointsPerPartition, minimumRectangleSize)
  the cell histogram     DBSCAN.scala:91-97, 345-356  (toMinimumBoundingRectangle, corner)
partition_points() is the whole DBSCAN.scala:91-104 step for raw points: the histogram runs on
the GPU (csrc/partition.hip), the splits on the host.  Same names, argument meaning and list
order as the reference; ties between equal-cost splits go to the first candidate (x splits,
then y splits), where the reference iterates a Scala HashSet (not reproducible).
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, NamedTuple, Optional, Tuple

import numpy as np

from . import _lib


class DBSCANRectangle(NamedTuple):  # DBSCANRectangle.scala:23
    x: float
    y: float
    x2: float
    y2: float

    def contains(self, other) -> bool:
        """Rectangle: other inside this box (:28-30); point: inside or on the border (:35-37)."""
        if isinstance(other, DBSCANRectangle):
            return (self.x <= other.x and other.x2 <= self.x2 and self.y <= other.y
                    and other.y2 <= self.y2)
        px, py = other.x, other.y
        return self.x <= px <= self.x2 and self.y <= py <= self.y2

    def shrink(self, amount: float) -> "DBSCANRectangle":  # :42-44
        return DBSCANRectangle(self.x + amount, self.y + amount, self.x2 - amount,
                               self.y2 - amount)

    def almostContains(self, point) -> bool:  # :50-52
        return self.x < point.x < self.x2 and self.y < point.y < self.y2


def _check64(rc: int) -> int:
    if rc < 0:
        _lib.check(int(rc))
    return int(rc)


def _collect(call, max_parts: int = 1 << 12) -> List[Tuple[DBSCANRectangle, int]]:
    while True:
        rects = np.zeros((max_parts, 4), np.float64)
        counts = np.zeros(max_parts, np.int64)
        k = _check64(call(rects.ctypes.data_as(ctypes.c_void_p),
                          counts.ctypes.data_as(ctypes.c_void_p), max_parts))
        if k <= max_parts:
            return [(DBSCANRectangle(*map(float, rects[i])), int(counts[i])) for i in range(k)]
        max_parts = k


def scala_range_count(start: float, end: float, step: float, inclusive: bool = False) -> int:
    """Element count of the Scala 2.10 Double range `start until end by step` (`to` if
    inclusive): NumericRange.count with DoubleAsIfIntegral, as the EvenSplitPartitioner's
    candidate splits use it (EvenSplitPartitioner.scala:150-152; csrc/javanum.hip)."""
    r = _lib.load().dbscan_scala_range_count(float(start), float(end), float(step),
                                             1 if inclusive else 0)
    if r < 0:
        raise ValueError(_lib.load().dbscan_last_error().decode())
    return int(r)


class EvenSplitPartitioner:
    """EvenSplitPartitioner.partition(toSplit, maxPointsPerPartition, minimumRectangleSize)
    (EvenSplitPartitioner.scala:28-35): toSplit is a set of (grid cell, count)."""

    @staticmethod
    def partition(toSplit: Iterable[Tuple[DBSCANRectangle, int]], maxPointsPerPartition: int,
                  minimumRectangleSize: float) -> List[Tuple[DBSCANRectangle, int]]:
        cells = list(toSplit)
        cx = np.array([r.x for r, _ in cells], np.float64)
        cy = np.array([r.y for r, _ in cells], np.float64)
        cc = np.array([c for _, c in cells], np.int64)
        L = _lib.load()
        return _collect(lambda r, c, m: L.dbscan_partition_cells(
            cx.ctypes.data_as(ctypes.c_void_p), cy.ctypes.data_as(ctypes.c_void_p),
            cc.ctypes.data_as(ctypes.c_void_p), len(cells), int(maxPointsPerPartition),
            float(minimumRectangleSize), r, c, m))


def partition_points(x, y, eps: float, maxPointsPerPartition: int,
                     handle: Optional[_lib.Handle] = None) -> List[Tuple[DBSCANRectangle, int]]:
    """DBSCAN.scala:91-104 for raw points: the 2*eps cell histogram (GPU) and
    EvenSplitPartitioner over it.  Returns [(DBSCANRectangle, count), ...] in list order."""
    from .local import default_handle

    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    if x.shape != y.shape or x.ndim != 1:
        raise ValueError("x and y must be 1-D arrays of equal length")
    h = handle or default_handle()
    L = _lib.load()
    return _collect(lambda r, c, m: L.dbscan_partition(
        h.ptr, x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p), x.size,
        float(eps), int(maxPointsPerPartition), r, c, m))
