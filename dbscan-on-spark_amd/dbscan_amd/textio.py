"""The reference's text I/O through libdbscan_hip.so (csrc/csv.hip).

  read_csv(path)                    DBSCANSuite.scala:31-33, DBSCANSample.scala:21:
                                    textFile(path).map(s => Vectors.dense(s.split(',')
                                    .map(_.toDouble))) -> x = field 0, y = field 1
  write_csv(path, x, y, cluster)    DBSCANSample.scala:35: s"${p.x},${p.y},${p.cluster}"
  format_double(v)                  java.lang.Double.toString as JDK 7/8 print it (the reference's
                                    runtime; sun.misc.FloatingDecimal's digits)
"""
from __future__ import annotations

import ctypes
import os
from typing import Tuple

import numpy as np

from . import _lib


def _path(p) -> bytes:
    return os.fsencode(os.fspath(p))


def read_csv(path) -> Tuple[np.ndarray, np.ndarray]:
    """Points of a reference input file as float64 arrays (x, y), in line order."""
    L = _lib.load()
    n = L.dbscan_csv_read(_path(path), None, None, 0)
    if n < 0:
        _lib.check(int(n))
    x = np.zeros(n, np.float64)
    y = np.zeros(n, np.float64)
    k = L.dbscan_csv_read(_path(path), x.ctypes.data_as(ctypes.c_void_p),
                          y.ctypes.data_as(ctypes.c_void_p), n)
    if k < 0:
        _lib.check(int(k))
    return x[:k], y[:k]


def write_csv(path, x, y, cluster) -> None:
    """One "x,y,cluster" line per point, Double.toString for the coordinates."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    c = np.ascontiguousarray(cluster, np.int32)
    if not (x.shape == y.shape == c.shape) or x.ndim != 1:
        raise ValueError("x, y and cluster must be 1-D arrays of equal length")
    _lib.check(_lib.load().dbscan_csv_write(_path(path), x.ctypes.data_as(ctypes.c_void_p),
                                            y.ctypes.data_as(ctypes.c_void_p),
                                            c.ctypes.data_as(ctypes.c_void_p), x.size))


def format_double(v: float) -> str:
    buf = ctypes.create_string_buffer(64)
    k = _lib.load().dbscan_format_double(float(v), buf)
    return buf.raw[:k].decode()
