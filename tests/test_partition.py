"""The product partitioner (csrc/partition.hip, dbscan_amd/partition.py) against the reference's
EvenSplitPartitionerSuite and the oracle's restatement (oracle/reference_pipeline.c).

dbscan_partition_cells is host code (no GPU): EvenSplitPartitionerSuite's two cases and random
cell sets run here on the CPU.  dbscan_partition (GPU cell histogram) is in the gpu tests
below: partitions equal the oracle's exactly, including the split-line/cell-corner defect."""
import numpy as np
import pytest

import oracle as O
from conftest import EPS_03F, gen_blobs

from dbscan_amd.partition import DBSCANRectangle, EvenSplitPartitioner


def _cells(spec):
    return {(DBSCANRectangle(*map(float, c[:4])), c[4]) for c in spec}


def test_should_find_partitions():
    """EvenSplitPartitionerSuite.scala:23-46."""
    sections = _cells([(0, 0, 1, 1, 3), (0, 2, 1, 3, 6), (1, 1, 2, 2, 7), (1, 0, 2, 1, 2),
                       (2, 0, 3, 1, 5), (2, 2, 3, 3, 4)])
    partitions = EvenSplitPartitioner.partition(sections, 9, 1)
    expected = [(DBSCANRectangle(1, 2, 3, 3), 4), (DBSCANRectangle(0, 2, 1, 3), 6),
                (DBSCANRectangle(0, 1, 3, 2), 7), (DBSCANRectangle(2, 0, 3, 1), 5),
                (DBSCANRectangle(0, 0, 2, 1), 5)]
    assert partitions == expected


def test_should_find_two_splits():
    """EvenSplitPartitionerSuite.scala:48-59."""
    sections = _cells([(0, 0, 1, 1, 3), (2, 2, 3, 3, 4), (0, 1, 1, 2, 2)])
    partitions = EvenSplitPartitioner.partition(sections, 4, 1)
    assert partitions[0] == (DBSCANRectangle(1, 0, 3, 3), 4)
    assert partitions[1] == (DBSCANRectangle(0, 1, 1, 3), 2)


@pytest.mark.parametrize("seed", range(6))
def test_random_cell_sets_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    mrs = [1.0, 0.6, 2 * EPS_03F, 0.25, 5.1, 3.0][seed]
    k = int(rng.integers(5, 400))
    ij = {(int(a), int(b)) for a, b in rng.integers(-40, 40, size=(k, 2))}
    spec = [(i * mrs, j * mrs, i * mrs + mrs, j * mrs + mrs, int(rng.integers(1, 50)))
            for i, j in sorted(ij)]
    maxpp = int(rng.integers(20, 400))
    got = EvenSplitPartitioner.partition(_cells(spec), maxpp, mrs)
    ref = O.ref_partition_cells(spec, maxpp, mrs)
    assert [(tuple(r), c) for r, c in got] == [(tuple(map(float, r)), c) for r, c in ref]


def test_rectangle_mirror():
    r = DBSCANRectangle(0.0, 0.0, 2.0, 2.0)
    assert r.contains(DBSCANRectangle(0.0, 1.0, 2.0, 2.0))
    assert not r.contains(DBSCANRectangle(-0.5, 1.0, 2.0, 2.0))
    assert r.shrink(0.5) == DBSCANRectangle(0.5, 0.5, 1.5, 1.5)
    assert r.shrink(-1.0) == DBSCANRectangle(-1.0, -1.0, 3.0, 3.0)


@pytest.mark.gpu
def test_partition_points_labeled_csv(labeled_data):
    """DBSCANSuite (maxPointsPerPartition = 250): 4 partitions of 243/225/142/139 points, equal
    to the oracle's rectangles."""
    from dbscan_amd.partition import partition_points

    x, y, _ = labeled_data
    got = partition_points(x, y, EPS_03F, 250)
    rects, counts = O.ref_partition(x, y, EPS_03F, 250)
    assert [c for _, c in got] == [243, 225, 142, 139] == counts.tolist()
    assert [tuple(r) for r, _ in got] == [tuple(map(float, r)) for r in rects]


@pytest.mark.gpu
@pytest.mark.parametrize("n,maxpp,noise,seed", [(200_000, 8192, 0.2, 1), (1_000_000, 8192, 0.0, 2),
                                               (300_000, 500, 0.1, 3), (50_000, 64, 0.5, 4)])
def test_partition_points_vs_oracle(n, maxpp, noise, seed):
    from dbscan_amd.partition import partition_points

    x, y = gen_blobs(n, noise=noise, seed=seed)
    got = partition_points(x, y, 2.55, maxpp)
    rects, counts = O.ref_partition(x, y, 2.55, maxpp)
    assert len(got) == len(counts)
    np.testing.assert_array_equal(np.array([c for _, c in got]), counts)
    np.testing.assert_array_equal(np.array([tuple(r) for r, _ in got]), rects)


@pytest.mark.parametrize("seed", range(4))
def test_duplicate_into_outer_rectangles(seed):
    """dbscan_duplicate (host code) against a brute-force restatement of DBSCAN.scala:116-137:
    point i goes to partition p iff outer_p = p.shrink(-eps) contains it (inclusive,
    DBSCANRectangle.scala:35-37), each partition's points in input order.  Rectangles from the
    reference's partitioner restated in the oracle; points on the outer borders exactly, NaNs
    and points outside every rectangle included."""
    import dbscan_amd

    rng = np.random.default_rng(seed)
    x, y = gen_blobs(20_000, noise=0.3, seed=seed + 40)
    eps = 2.55 * (0.5 + seed * 0.3)
    rects, _ = O.ref_partition(x, y, eps, 700)
    # points exactly on outer borders, NaNs, and far outside
    k = rng.integers(0, len(rects), 200)
    x[:200] = rects[k, 0] + (-eps)
    y[:200] = rng.uniform(rects[k, 1], rects[k, 3])
    x[200:300] = rects[k[:100], 2] - (-eps)
    x[300:310] = np.nan
    x[310:320] = 1e9
    offs, idx = dbscan_amd.duplicate(x, y, rects, eps)
    ox, oy = rects[:, 0] + (-eps), rects[:, 1] + (-eps)
    ox2, oy2 = rects[:, 2] - (-eps), rects[:, 3] - (-eps)
    assert len(offs) == len(rects) + 1 and offs[0] == 0
    for p in range(len(rects)):
        want = np.flatnonzero((ox[p] <= x) & (x <= ox2[p]) & (oy[p] <= y) & (y <= oy2[p]))
        np.testing.assert_array_equal(idx[offs[p]:offs[p + 1]], want)
