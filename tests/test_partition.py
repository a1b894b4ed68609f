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


def test_murmur3_primitives_known_vectors():
    """The oracle's MurmurHash3 mix / finalization (oracle/jvm.py, restating Scala 2.10's
    scala.util.hashing.MurmurHash3 that DBSCANRectangle.hashCode goes through) against the
    published MurmurHash3_x86_32 verification values (4-byte blocks, byte length mixed in)."""
    import jvm

    def x86_32(blocks, seed):
        h = seed
        for k in blocks:
            h = jvm._mix(h, k)
        return jvm._avalanche(h ^ (4 * len(blocks)))

    assert x86_32([], 0) == 0
    assert x86_32([], 1) == 0x514E28B7
    assert x86_32([0xFFFFFFFF], 0) == 0x76293B50
    assert x86_32([0x87654321], 0) == 0xF55B516B
    assert x86_32([0x87654321], 0x5082EDEE) == 0x2362F9DE
    assert x86_32([0x61616161], 0x9747B28C) == 0x5A97808A
    # BoxesRunTime.hashFromDouble: Int, Long, Float and Double cases
    assert jvm.hash_from_double(3.0) == 3 and jvm.hash_from_double(-1.0) == 0xFFFFFFFF
    assert jvm.hash_from_double(2.0 ** 40) == (2 ** 40 ^ 0) >> 32 ^ (2 ** 40 & 0xFFFFFFFF)
    assert jvm.hash_from_double(0.5) == 0x3F000000
    assert jvm.hash_from_double(0.1) == 0x9999999A ^ 0x3FB99999


def _first_split_candidates(spec, mrs):
    """The first split of the bounding rectangle, restated directly over the cells: every
    candidate (x splits, then y splits) with its cost |count/2 - pointsIn(candidate)|."""
    import jvm

    x0 = min(c[0] for c in spec)
    y0 = min(c[1] for c in spec)
    x2 = max(c[2] for c in spec)
    y2 = max(c[3] for c in spec)
    total = sum(c[4] for c in spec)

    def pin(r):
        return sum(c[4] for c in spec
                   if r[0] <= c[0] and c[2] <= r[2] and r[1] <= c[1] and c[3] <= r[3])

    cands = []
    for axis in (0, 1):
        start = (x0 if axis == 0 else y0) + mrs
        end = x2 if axis == 0 else y2
        v = start
        for _ in range(O.scala_range_count(start, end, mrs)):
            r = (x0, y0, v, y2) if axis == 0 else (x0, y0, x2, v)
            cands.append((r, abs(total // 2 - pin(r)), jvm.split_order_key(*r)))
            v += mrs
    return cands


@pytest.mark.parametrize("shape", ["square", "gaps", "stripes"])
def test_tie_heavy_lattices_vs_oracle(shape):
    """Cell sets built so that equal-cost split candidates are the rule: the product
    (csrc/partition.hip) and the oracle (reference_pipeline.c with oracle/jvm.py's ranks), two
    independent restatements of Scala 2.10's `splits.toSet` order, must pick the same splits.
    The first split is checked to be a tie that the HashTrieSet order decides differently from
    plain candidate order, so the case discriminates."""
    mrs, o = 1.0, 9  # (o: an x offset at which every shape's first tie is decided by rank)
    if shape == "square":  # 16 x 16 unit cells of one point: x = 8 and y = 8 both halve it
        spec = [(i + o, j, i + o + 1, j + 1, 1) for i in range(16) for j in range(16)]
        maxpp = 5
    elif shape == "gaps":  # two blocks with an empty band between them: every x in the band ties
        spec = [(i + o, j, i + o + 1, j + 1, 2) for i in list(range(0, 6)) + list(range(14, 20))
                for j in range(10)]
        maxpp = 7
    else:  # vertical stripes of equal weight with empty columns between them
        spec = [(i + o, j, i + o + 1, j + 1, 3) for i in range(0, 24, 3) for j in range(12)]
        maxpp = 10
    cands = _first_split_candidates(spec, mrs)
    best = min(c[1] for c in cands)
    ties = [c for c in cands if c[1] == best]
    assert len(cands) > 4 and len(ties) > 1
    by_rank = min(ties, key=lambda c: c[2])[0]
    assert by_rank != ties[0][0], "the tie order must matter for this case"
    got = EvenSplitPartitioner.partition(_cells(spec), maxpp, mrs)
    ref = O.ref_partition_cells(spec, maxpp, mrs)
    assert [(tuple(r), c) for r, c in got] == [(tuple(map(float, r)), c) for r, c in ref]
