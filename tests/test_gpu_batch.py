"""Batched fits as ONE tiled fit over per-partition grids (csrc/batch.hip), bit-exact against
the CPU oracle partition by partition.

DBSCAN.scala:150-155 fits every spatial partition on its own (`flatMapValues(new
LocalDBSCANNaive(eps, minPoints).fit(_))`).  dbscan_fit_batch serves an executor's partitions in
one call: batches spanning >= 65536 points (or holding a partition over the one-workgroup
capacity) are fitted as one tiled fit in which each partition has its own eps grid, placed in a
virtual tile grid with empty cells between partitions.  Each partition's labels, flags and
cluster count must equal the oracle's fit of that partition alone (LocalDBSCANNaive.scala:37-118
/ LocalDBSCANArchery.scala:36-112 restated, visit order = the partition's array order, cluster
ids counted from 1 in every partition).  Partitions the virtual grid does not take (absurd
extents, eps below the grid's clique range) are fitted one by one in the same call."""
import numpy as np
import pytest

import oracle as O
from conftest import gen_blobs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dm():
    import dbscan_amd

    if dbscan_amd.load().dbscan_device_count() < 1:
        pytest.fail("no GPU visible to libdbscan_hip.so")
    return dbscan_amd


@pytest.fixture(scope="module")
def handle(dm):
    h = dm.Handle(0)
    yield h
    h.close()


def _check_parts(x, y, offs, eps, mp, mode, got, what=""):
    cl, fl, nk = got
    for p in range(len(offs) - 1):
        a, b = int(offs[p]), int(offs[p + 1])
        rc, rf, rk = O.fit_grid(x[a:b], y[a:b], eps, mp, mode)
        assert int(nk[p]) == rk, f"{what} partition {p} (m={b - a}): {nk[p]} clusters, oracle {rk}"
        bad = np.flatnonzero((cl[a:b] != rc) | (fl[a:b] != rf))
        assert bad.size == 0, f"{what} partition {p} (m={b - a}): {bad.size} mismatches {bad[:8]}"


def _blob_part(rng, m, scale, centre):
    k = int(rng.integers(1, 6))
    c = centre + rng.uniform(-scale, scale, size=(k, 2))
    nb = m - m // 5
    pts = c[rng.integers(0, k, nb)] + rng.normal(0, scale * rng.uniform(0.05, 0.3), size=(nb, 2))
    pts = np.concatenate([pts, centre + rng.uniform(-1.3 * scale, 1.3 * scale, size=(m - nb, 2))])
    pts = pts[rng.permutation(m)]
    return pts[:, 0].copy(), pts[:, 1].copy()


def _mixed_batch(seed, eps):
    """Partitions of many shapes: blobs at varied densities and places (overlapping each other in
    space, like the reference's eps halos), exact duplicates, a lattice at exactly eps, far from
    the origin, non-finite points, an all-NaN partition, empty ones, a far outlier (a sparse
    extent: fitted alone), and one over the one-workgroup capacity."""
    rng = np.random.default_rng(seed)
    xs, ys = [], []

    def add(x, y):
        xs.append(np.asarray(x, np.float64))
        ys.append(np.asarray(y, np.float64))

    for _ in range(12):
        m = int(rng.integers(50, 6000))
        add(*_blob_part(rng, m, eps * rng.uniform(5, 40), rng.uniform(-20 * eps, 20 * eps, 2)))
    add([], [])
    add(np.full(700, 3.25), np.full(700, -1.5))                      # duplicates
    i, j = np.meshgrid(np.arange(40), np.arange(40), indexing="ij")
    add(1e3 + i.ravel() * eps, -7.0 + j.ravel() * eps)               # lattice at exactly eps
    x, y = _blob_part(rng, 3000, eps * 10, np.array([0.0, 0.0]))
    add(1e9 + x, -1e9 + y)                                           # far from the origin
    x, y = _blob_part(rng, 2500, eps * 15, np.array([1.0, 2.0]))
    x[::29] = np.nan
    y[::31] = np.inf
    add(x, y)                                                        # non-finite points
    add(np.full(40, np.nan), np.zeros(40))                           # no finite point
    x, y = _blob_part(rng, 900, eps * 8, np.array([5.0, 5.0]))
    x[17] = 1e7
    add(x, y)                                                        # sparse extent: alone
    add([], [])
    add(*_blob_part(rng, 21000, eps * 60, np.array([-3.0, 4.0])))    # over 8192 points
    add([7.0], [7.0])
    offs = np.concatenate([[0], np.cumsum([a.size for a in xs])]).astype(np.int64)
    return np.concatenate(xs), np.concatenate(ys), offs


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("mp", [0, 1, 4, 10])
def test_mixed_partitions(dm, handle, mode, mp):
    eps = 0.25
    x, y, offs = _mixed_batch(11 + mp, eps)
    assert offs[-1] >= 65536 or np.diff(offs).max() > 8192  # the tiled batch path
    got = dm.fit_batch(x, y, offs, eps, mp, mode, handle=handle)
    _check_parts(x, y, offs, eps, mp, mode, got, f"mode {mode} minPoints {mp}")


def test_batch_equals_single_fits(dm, handle):
    """The batched fit equals the same partitions fitted one call at a time (each through the
    direct fit path), bit for bit; and running the batch twice gives the same labels."""
    x, y, offs = _mixed_batch(5, 0.3)
    got = dm.fit_batch(x, y, offs, 0.3, 6, 0, handle=handle)
    again = dm.fit_batch(x, y, offs, 0.3, 6, 0, handle=handle)
    for u, v in zip(got, again):
        assert np.array_equal(u, v)
    for p in range(len(offs) - 1):
        a, b = int(offs[p]), int(offs[p + 1])
        cl, fl, k = dm.fit_arrays(x[a:b], y[a:b], 0.3, 6, 0, handle=handle)
        assert k == int(got[2][p])
        assert np.array_equal(cl, got[0][a:b]) and np.array_equal(fl, got[1][a:b])


def test_small_cap_zero_routes_every_batch_through_the_tiled_path(dm, handle):
    """dbscan_set_small_max(h, 0): even a small batch (the csv's four reference partitions)
    takes the tiled batch path; labels still equal the sequential oracle per partition."""
    x, y, _ = O.load_labeled_csv(__import__("os").path.join(
        __import__("os").path.dirname(__file__), "golden", "labeled_data.csv"))
    eps = float(np.float32(0.3))
    rects, _ = O.ref_partition(x, y, eps, 250)
    offs, idx = dm.duplicate(x, y, rects, eps)
    px, py = x[idx], y[idx]
    prev = handle.set_small_max(0)
    try:
        for mode in (0, 1):
            cl, fl, nk = dm.fit_batch(px, py, offs, eps, 10, mode, handle=handle)
            for p in range(len(offs) - 1):
                a, b = offs[p], offs[p + 1]
                rc, rf, rk = O.fit_sequential(px[a:b], py[a:b], eps, 10, mode)
                assert int(nk[p]) == rk
                assert np.array_equal(cl[a:b], rc) and np.array_equal(fl[a:b], rf)
    finally:
        handle.set_small_max(prev)


def test_eps_without_clique_grid_fits_alone(dm, handle):
    """eps below 2^-500: the grid side is floored, quarters are no cliques, the virtual grid is
    not used -- every partition is fitted on its own inside the same call."""
    rng = np.random.default_rng(3)
    xs = [rng.uniform(0, 1e-149, 20000) for _ in range(4)]
    ys = [rng.uniform(0, 1e-149, 20000) for _ in range(4)]
    x, y = np.concatenate(xs), np.concatenate(ys)
    offs = np.arange(5, dtype=np.int64) * 20000
    got = dm.fit_batch(x, y, offs, 1e-152, 3, 0, handle=handle)
    _check_parts(x, y, offs, 1e-152, 3, 0, got, "tiny eps")


def test_reference_partitions_of_blobs(dm, handle):
    """G(2*10^6, 20% noise) cut by the reference's EvenSplitPartitioner (maxPointsPerPartition
    8192) and duplicated into eps-grown partitions (DBSCAN.scala:105-137): hundreds of
    partitions in one call, host and device-resident forms equal, every partition equal to its
    own oracle fit."""
    import torch

    from dbscan_amd import device as D

    x, y = gen_blobs(2_000_000, noise=0.2, seed=23)
    parts = dm.partition.partition_points(x, y, 2.55, 8192, handle)
    rects = np.array([r for r, _ in parts])
    offs, idx = dm.duplicate(x, y, rects, 2.55)
    px, py = x[idx], y[idx]
    got = dm.fit_batch(px, py, offs, 2.55, 10, 0, handle=handle)
    tx, ty = torch.from_numpy(px).cuda(), torch.from_numpy(py).cuda()
    dcl = torch.empty(px.size, dtype=torch.int32, device="cuda")
    dfl = torch.empty(px.size, dtype=torch.uint8, device="cuda")
    dnk = torch.empty(len(offs) - 1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    D.fit_batch_tensors_async(tx, ty, offs, 2.55, 10, 0, handle, dcl, dfl, dnk)
    handle.sync()
    assert np.array_equal(dcl.cpu().numpy(), got[0]) and np.array_equal(dfl.cpu().numpy(), got[1])
    assert np.array_equal(dnk.cpu().numpy(), got[2])
    assert len(offs) - 1 > 200
    _check_parts(px, py, offs, 2.55, 10, 0, got, "blobs")


def test_only_sparse_and_empty_partitions(dm, handle):
    """A tiled batch (a partition over the one-workgroup capacity) in which NO partition is
    placed in the virtual grid: every finite partition has a sparse extent (a far outlier), the
    rest are empty or all-NaN.  Every partition must still be fitted (round-3 ADVICE: the empty
    and NaN ones were once left with stale outputs)."""
    rng = np.random.default_rng(8)
    xs, ys = [], []
    for m in (9000, 3000):
        x, y = _blob_part(rng, m, 0.25 * 10, np.array([0.0, 0.0]))
        x[5] = 1e9  # sparse extent: the partition is fitted alone
        xs.append(x)
        ys.append(y)
    xs += [np.array([]), np.full(30, np.nan), np.array([])]
    ys += [np.array([]), np.zeros(30), np.array([])]
    offs = np.concatenate([[0], np.cumsum([a.size for a in xs])]).astype(np.int64)
    x, y = np.concatenate(xs), np.concatenate(ys)
    for mp in (1, 5):
        cl = np.full(x.size, 12345, np.int32)
        fl = np.full(x.size, 7, np.uint8)
        got = dm.fit_batch(x, y, offs, 0.25, mp, 0, handle=handle, cluster_out=cl, flag_out=fl)
        _check_parts(x, y, offs, 0.25, mp, 0, got, f"sparse/empty minPoints {mp}")
        assert not np.any(fl == 7) and not np.any(cl == 12345)
