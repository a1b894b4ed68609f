"""DBSCAN.train(data, eps, minPoints, maxPointsPerPartition) -> DBSCAN (DBSCAN.scala:40-48),
the reference's whole-job API, over libdbscan_hip.so.

  partitions      the reference's [(id, DBSCANRectangle)] list: EvenSplitPartitioner over the
                  2*eps cell histogram (DBSCAN.scala:91-104, 283; cell histogram on the GPU,
                  dbscan_partition), in list order
  labeledPoints   every input point once, in input order (DBSCANLabeledPoint: vector, cluster,
                  flag), from dbscan_train_node: x-slabs over the visible GPUs with eps halos and
                  an exact merge -- equal to ONE LocalDBSCANNaive fit of all points.  The
                  reference's merge (DBSCAN.scala:158-270) can drop or duplicate points and
                  report halo cores as Border; none of that is replicated.
                  Cluster ids are the input-order Naive numbering (the reference's are a
                  permutation of them: DBSCANSuite maps them through `corresponding`).
  cluster, flag   the same labels as numpy arrays (no per-point objects)
  predict(v)      NotImplementedError, as in the reference (DBSCAN.scala:300-302)
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Tuple

import numpy as np

from . import _lib
from .local import DBSCANLabeledPoint, DBSCANPoint, Flag, train_node
from .partition import DBSCANRectangle, partition_points


def _as_xy(data) -> Tuple[np.ndarray, np.ndarray, Optional[list]]:
    if isinstance(data, np.ndarray):
        if data.ndim != 2 or data.shape[1] < 2:
            raise IndexError("DBSCANPoint needs vector(0) and vector(1)")  # DBSCANPoint.scala:23-24
        return (np.ascontiguousarray(data[:, 0], np.float64),
                np.ascontiguousarray(data[:, 1], np.float64), None)
    vecs = [p.vector if isinstance(p, DBSCANPoint) else tuple(p) for p in data]
    x = np.fromiter((v[0] for v in vecs), np.float64, len(vecs))
    y = np.fromiter((v[1] for v in vecs), np.float64, len(vecs))  # IndexError if < 2 dims
    return x, y, vecs


class DBSCAN:
    """The trained model (DBSCAN.scala:59-68)."""

    def __init__(self, eps: float, minPoints: int, maxPointsPerPartition: int,
                 partitions: List[Tuple[int, DBSCANRectangle]], cluster: np.ndarray,
                 flag: np.ndarray, n_clusters: int, data):
        self.eps = float(eps)
        self.minPoints = int(minPoints)
        self.maxPointsPerPartition = int(maxPointsPerPartition)
        self.partitions = partitions
        self.cluster = cluster
        self.flag = flag
        self.n_clusters = n_clusters
        self._data = data
        self._labeled = None

    @staticmethod
    def train(data, eps: float, minPoints: int, maxPointsPerPartition: int,
              n_shards: int = 0, handle: Optional[_lib.Handle] = None) -> "DBSCAN":
        """data: an (n, d >= 2) array or an iterable of vectors / DBSCANPoints (only the first
        two coordinates are used, DBSCAN.scala:33-34).  n_shards = 0: one slab per GPU."""
        x, y, vecs = _as_xy(data)
        cl, fl, k = train_node(x, y, eps, minPoints, _lib.MODE_NAIVE, n_shards)
        parts = partition_points(x, y, eps, maxPointsPerPartition, handle)
        partitions = [(i, r) for i, (r, _) in enumerate(parts)]
        return DBSCAN(eps, minPoints, maxPointsPerPartition, partitions, cl, fl, k,
                      vecs if vecs is not None else data)

    @property
    def minimumRectangleSize(self) -> float:  # DBSCAN.scala:289
        return 2 * self.eps

    @property
    def labeledPoints(self) -> List[DBSCANLabeledPoint]:
        """One DBSCANLabeledPoint per input point, input order (DBSCAN.scala:291-293)."""
        if self._labeled is None:
            out = []
            rows = self._data if not isinstance(self._data, np.ndarray) else self._data.tolist()
            for v, c, f in zip(rows, self.cluster.tolist(), self.flag.tolist()):
                lp = DBSCANLabeledPoint(v)
                lp.cluster = c
                lp.flag = Flag(f)
                lp.visited = True
                out.append(lp)
            self._labeled = out
        return self._labeled

    def predict(self, vector) -> DBSCANLabeledPoint:  # DBSCAN.scala:300-302
        raise NotImplementedError("DBSCAN.predict is not implemented (as in the reference)")
