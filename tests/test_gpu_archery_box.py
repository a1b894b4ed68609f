"""GPU parity for LocalDBSCANArchery with its float32 R-tree search box
(DBSCAN_MODE_ARCHERY_F32BOX; LocalDBSCANArchery.scala:38-41,114-124, Noise re-claim :103-106).

The neighbour relation is directed here (o in N(p) iff d2 <= eps2 and (float)o lies in p's
float32 box), so the oracle is the literal BFS (oracle_fit_sequential for small sets,
oracle_fit_bfs_grid -- the same BFS with grid neighbour queries -- for large ones), with visit
order = input order.  Bit-exact flags and cluster numbers.  The negative-eps sets hold many
one-way core pairs: they exercise the library's one-way-pair resolution."""
import numpy as np
import pytest

import oracle as O
from conftest import EPS_03F, gen_blobs, load_edge_cases, neg_eps_set, one_way_pairs

pytestmark = pytest.mark.gpu

BOX = 2


@pytest.fixture(scope="module")
def dm():
    import dbscan_amd

    if dbscan_amd.load().dbscan_device_count() < 1:
        pytest.fail("no GPU visible to libdbscan_hip.so")
    assert dbscan_amd.MODE_ARCHERY_F32BOX == BOX
    return dbscan_amd


@pytest.fixture(scope="module")
def handle(dm):
    h = dm.Handle(0)
    yield h
    h.close()


def _check(dm, handle, x, y, eps, mp, ref):
    cl, fl, k = dm.fit_arrays(x, y, eps, mp, BOX, handle=handle)
    rc, rf, rk = ref
    bad = np.flatnonzero((cl != rc) | (fl != rf))
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:10]}"
    assert k == rk
    return cl, fl, k


def test_box_labeled_csv(dm, handle, labeled_data, labeled_expected):
    x, y, _ = labeled_data
    cl, fl, k = _check(dm, handle, x, y, EPS_03F, 10, O.fit_sequential(x, y, EPS_03F, 10, BOX))
    np.testing.assert_array_equal(fl, labeled_expected["flag_archery"])
    assert k == 3


def test_box_reference_interface(dm, labeled_data):
    """LocalDBSCANArchery(eps, minPoints).fit(points): the float32 box by default."""
    x, y, lab = labeled_data
    pts = [dm.DBSCANPoint([a, b, c]) for a, b, c in zip(x, y, lab)]
    out = dm.LocalDBSCANArchery(EPS_03F, 10).fit(pts)
    ref = O.fit_sequential(x, y, EPS_03F, 10, BOX)
    assert [p.cluster for p in out] == ref[0].tolist()
    assert [int(p.flag) for p in out] == ref[1].tolist()


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("eps", [-0.02, -0.01])
def test_box_negative_eps_one_way_pairs(dm, handle, seed, eps):
    x, y = neg_eps_set(seed, 800, eps=eps)
    assert one_way_pairs(x, y, eps) > 0
    for mp in (1, 2, 4):
        _check(dm, handle, x, y, eps, mp, O.fit_sequential(x, y, eps, mp, BOX))


@pytest.mark.parametrize("case", load_edge_cases(), ids=lambda c: c["name"])
def test_box_edge_fixtures(dm, handle, case):
    """Every committed edge fixture (NaN/inf, eps 0 / negative / huge, duplicates, lattices at
    exactly eps) in the float32-box mode."""
    x, y, eps, mp = case["x"], case["y"], case["eps"], case["min_points"]
    _check(dm, handle, x, y, eps, mp, O.fit_sequential(x, y, eps, mp, BOX))


@pytest.mark.parametrize("offset", [0.0, 1e4, 1e6])
def test_box_blobs_far_from_origin(dm, handle, offset):
    x, y = gen_blobs(100_000, noise=0.2, seed=21)
    x, y = x + offset, y - offset
    _check(dm, handle, x, y, 2.55, 10, O.fit_bfs_grid(x, y, 2.55, 10, BOX))


def test_box_bench_like_million(dm, handle):
    """G(10^6) at the bench's eps: the float32-box fit equals the oracle and (eps > 0) the
    exact-fp64 archery fit."""
    x, y = gen_blobs(1_000_000, noise=0.1, seed=4)
    cl, fl, k = _check(dm, handle, x, y, 2.55, 10, O.fit_bfs_grid(x, y, 2.55, 10, BOX))
    c1, f1, k1 = dm.fit_arrays(x, y, 2.55, 10, 1, handle=handle)
    assert k1 == k and np.array_equal(c1, cl) and np.array_equal(f1, fl)


def test_box_mode_rejected_by_node_entries(dm):
    from dbscan_amd import _lib

    x, y = gen_blobs(1000, seed=2)
    with pytest.raises(_lib.DBSCANError):
        dm.train_node(x, y, 2.55, 10, BOX, 2)
