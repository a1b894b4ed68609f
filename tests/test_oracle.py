"""CPU tests of the oracle itself: pinned against the reference's golden fixture and
known-answer tests, and the three restatements fuzzed against each other.

Reference tests mirrored (src/test/scala/org/apache/spark/mllib/clustering/dbscan/):
  LocalDBSCANArcherySuite."should cluster"   (:31-53)  -> test_labeled_csv_*
  DBSCANSuite."dbscan"                       (:30-60)  -> test_reference_train_labeled_csv
  EvenSplitPartitionerSuite (two cases)      (:23-60)  -> test_even_split_partitioner_*
"""
import collections

import numpy as np
import pytest

import oracle as O
from conftest import EPS_03F, gen_blobs, load_edge_cases, neg_eps_set, one_way_pairs

# csv column 3 is archery's entry-order numbering; input-order
# Naive ids {1,2,3} correspond to csv labels {1,3,2}; Noise stays 0.
NAIVE_TO_CSV = {0: 0, 1: 1, 2: 3, 3: 2}


@pytest.mark.parametrize("mode", [O.NAIVE, O.ARCHERY])
def test_labeled_csv_sequential_matches_reference_labels(labeled_data, mode):
    x, y, lab = labeled_data
    cl, fl, k = O.fit_sequential(x, y, EPS_03F, 10, mode)
    assert k == 3
    assert np.bincount(fl, minlength=4).tolist() == [54, 677, 18, 0]  # Border, Core, Noise
    mapped = np.array([NAIVE_TO_CSV[c] for c in cl])
    np.testing.assert_array_equal(mapped, lab.astype(np.int64))
    assert sorted(collections.Counter(cl.tolist()).values()) == [18, 243, 243, 245]


def test_labeled_csv_pure_python_matches_c(labeled_data):
    x, y, _ = labeled_data
    pts = list(zip(x.tolist(), y.tolist()))
    for mode in (O.NAIVE, O.ARCHERY):
        pc, pf, pk = O.py_fit_sequential(pts, EPS_03F, 10, mode)
        cl, fl, k = O.fit_sequential(x, y, EPS_03F, 10, mode)
        assert pk == k
        np.testing.assert_array_equal(np.array(pc), cl)
        np.testing.assert_array_equal(np.array(pf), fl)


def test_labeled_expected_fixture(labeled_data, labeled_expected):
    x, y, _ = labeled_data
    for mode, key in ((O.NAIVE, "naive"), (O.ARCHERY, "archery")):
        cl, fl, _ = O.fit_sequential(x, y, EPS_03F, 10, mode)
        np.testing.assert_array_equal(cl, labeled_expected["cluster_" + key])
        np.testing.assert_array_equal(fl, labeled_expected["flag_" + key])


@pytest.mark.parametrize("case", load_edge_cases(), ids=lambda c: c["name"])
def test_edge_case_fixtures(case):
    """Committed edge fixtures: sequential restatement reproduces them, and both closed-form
    restatements agree with it bit-exactly (flags and cluster numbering)."""
    x, y, eps, mp, mode = case["x"], case["y"], case["eps"], case["min_points"], case["mode"]
    cl, fl, k = O.fit_sequential(x, y, eps, mp, mode)
    np.testing.assert_array_equal(cl, case["cluster"])
    np.testing.assert_array_equal(fl, case["flag"])
    assert k == case["n_clusters"]
    for fit in (O.fit_bruteforce, O.fit_grid):
        c2, f2, k2 = fit(x, y, eps, mp, mode)
        np.testing.assert_array_equal(f2, fl)
        np.testing.assert_array_equal(c2, cl)
        assert k2 == k


@pytest.mark.parametrize("seed", range(40))
def test_closed_form_equals_sequential_fuzz(seed):
    """the order-parametrised closed form equals the sequential BFS."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(50, 400))
    k = int(rng.integers(1, 6))
    c = rng.uniform(-2, 2, size=(k, 2))
    pts = c[rng.integers(0, k, n)] + rng.normal(0, rng.uniform(0.05, 0.4), size=(n, 2))
    if seed % 3 == 0:
        pts = np.concatenate([pts, rng.uniform(-3, 3, size=(n // 4, 2))])
    x, y = pts[:, 0].copy(), pts[:, 1].copy()
    eps = float(rng.uniform(0.05, 0.3))
    mp = int(rng.integers(1, 12))
    for mode in (O.NAIVE, O.ARCHERY):
        cs, fs, ks = O.fit_sequential(x, y, eps, mp, mode)
        for fit in (O.fit_bruteforce, O.fit_grid):
            c2, f2, k2 = fit(x, y, eps, mp, mode)
            np.testing.assert_array_equal(f2, fs)
            np.testing.assert_array_equal(c2, cs)
            assert k2 == ks


def test_grid_oracle_counts_equal_bruteforce():
    x, y = gen_blobs(20000, noise=0.2, seed=5)
    _, _, _, cb = O.fit_bruteforce(x[:3000], y[:3000], 60.0, 10, with_counts=True)
    _, _, _, cg = O.fit_grid(x[:3000], y[:3000], 60.0, 10, with_counts=True)
    np.testing.assert_array_equal(cb, cg)


def test_grid_oracle_thread_invariance():
    x, y = gen_blobs(50000, noise=0.1, seed=9)
    eps = 2.55 * np.sqrt(50000 / 1e6) * 4
    a = O.fit_grid(x, y, eps, 10, nthreads=1)
    b = O.fit_grid(x, y, eps, 10, nthreads=8)
    for u, v in zip(a[:2], b[:2]):
        np.testing.assert_array_equal(u, v)
    assert a[2] == b[2]


def test_naive_archery_differ_only_in_noise_reclaim():
    x, y = gen_blobs(3000, noise=0.3, seed=3)
    cn, fn, _ = O.fit_grid(x, y, 60.0 * np.sqrt(3000 / 1e6) * 3, 6, O.NAIVE)
    ca, fa, _ = O.fit_grid(x, y, 60.0 * np.sqrt(3000 / 1e6) * 3, 6, O.ARCHERY)
    diff = fn != fa
    assert np.all(fn[diff] == O.NOISE) and np.all(fa[diff] == O.BORDER)
    same = ~diff
    np.testing.assert_array_equal(cn[same], ca[same])


# ------------------------- archery's float32 search box (mode 2) --------------------------
@pytest.mark.parametrize("seed", range(12))
def test_bfs_grid_equals_sequential(seed):
    """The grid-query BFS (the large-n oracle of every mode) equals the literal O(n^2) BFS,
    modes 0/1/2, on blob fuzz (some far from the origin) and on negative-eps box sets."""
    rng = np.random.default_rng(500 + seed)
    n = int(rng.integers(100, 800))
    c = rng.uniform(-3, 3, size=(4, 2)) + (rng.uniform(1e3, 1e6) if seed % 2 else 0.0)
    pts = c[rng.integers(0, 4, n)] + rng.normal(0, rng.uniform(0.05, 0.4), size=(n, 2))
    x, y = pts[:, 0].copy(), pts[:, 1].copy()
    eps = float(rng.uniform(0.05, 0.3))
    mp = int(rng.integers(1, 10))
    cases = [(x, y, eps, mp), neg_eps_set(seed, 400) + (-0.02, 1 + seed % 4)]
    for cx, cy, e, m in cases:
        for mode in (O.NAIVE, O.ARCHERY, O.ARCHERY_F32BOX):
            a = O.fit_sequential(cx, cy, e, m, mode)
            b = O.fit_bfs_grid(cx, cy, e, m, mode)
            np.testing.assert_array_equal(b[1], a[1])
            np.testing.assert_array_equal(b[0], a[0])
            assert a[2] == b[2]


@pytest.mark.parametrize("offset", [0.0, 1e3, 1e5, 1e7])
def test_f32_box_never_excludes_with_positive_eps(offset):
    """With eps >= 0 archery's float32 box only widens the fp64 neighbourhood (float rounding is
    monotone and the box is inclusive), so mode 2 equals mode 1 bit for bit -- here on blobs at
    growing distances from the origin; SURVEY's 'ulp-scale box edge' difference does not arise.
    A negative eps inverts the box: there the modes differ (next test)."""
    rng = np.random.default_rng(int(offset) % 1000 + 1)
    n = 2000
    c = rng.uniform(-2, 2, size=(6, 2)) + offset
    pts = c[rng.integers(0, 6, n)] + rng.normal(0, 0.2, size=(n, 2))
    x, y = pts[:, 0].copy(), pts[:, 1].copy()
    for eps in (0.05, float(np.float32(0.3)), 0.1 + 2.0 ** -30):
        a = O.fit_bfs_grid(x, y, eps, 5, O.ARCHERY_F32BOX)
        b = O.fit_grid(x, y, eps, 5, O.ARCHERY)
        for u, v in zip(a, b):
            np.testing.assert_array_equal(u, v)
        assert one_way_pairs(x[:1500], y[:1500], eps) == 0


def test_f32_box_negative_eps_is_directed():
    """The negative-eps sets do produce one-way pairs, and mode 2 then differs from mode 1."""
    x, y = neg_eps_set(1)
    assert one_way_pairs(x, y, -0.02) > 0
    a = O.fit_sequential(x, y, -0.02, 3, O.ARCHERY_F32BOX)
    b = O.fit_sequential(x, y, -0.02, 3, O.ARCHERY)
    assert (a[1] != b[1]).any()


def test_f32_box_labeled_csv(labeled_data, labeled_expected):
    """LocalDBSCANArcherySuite 'should cluster' with the float32 box: the same labels as the
    exact fp64 set (677 Core / 54 Border / 18 Noise)."""
    x, y, _ = labeled_data
    cl, fl, k = O.fit_sequential(x, y, EPS_03F, 10, O.ARCHERY_F32BOX)
    np.testing.assert_array_equal(cl, labeled_expected["cluster_archery"])
    np.testing.assert_array_equal(fl, labeled_expected["flag_archery"])
    assert k == 3


# ---------------------------------- reference driver --------------------------------------

def test_even_split_partitioner_should_find_partitions():
    """EvenSplitPartitionerSuite.scala:23-46."""
    cells = [(0, 0, 1, 1, 3), (0, 2, 1, 3, 6), (1, 1, 2, 2, 7), (1, 0, 2, 1, 2), (2, 0, 3, 1, 5),
             (2, 2, 3, 3, 4)]
    got = O.ref_partition_cells(cells, 9, 1)
    expected = [((1, 2, 3, 3), 4), ((0, 2, 1, 3), 6), ((0, 1, 3, 2), 7), ((2, 0, 3, 1), 5),
                ((0, 0, 2, 1), 5)]
    assert [(tuple(float(v) for v in r), c) for r, c in got] == \
        [(tuple(float(v) for v in r), c) for r, c in expected]


def test_even_split_partitioner_should_find_two_splits():
    """EvenSplitPartitionerSuite.scala:48-59."""
    cells = [(0, 0, 1, 1, 3), (2, 2, 3, 3, 4), (0, 1, 1, 2, 2)]
    got = O.ref_partition_cells(cells, 4, 1)
    assert got[0] == ((1.0, 0.0, 3.0, 3.0), 4)
    assert got[1] == ((0.0, 1.0, 1.0, 3.0), 2)


def test_reference_partitions_labeled_csv(labeled_data):
    """4 partitions, 243/225/142/139 main points (maxPPP = 250)."""
    x, y, _ = labeled_data
    rects, counts = O.ref_partition(x, y, EPS_03F, 250)
    assert counts.tolist() == [243, 225, 142, 139]


def test_reference_train_labeled_csv(labeled_data):
    """DBSCANSuite.scala:30-60 -- end-to-end labels equal the csv up to the suite's own
    permutation; every point is reported exactly once on this fixture."""
    x, y, lab = labeled_data
    r = O.ref_train(x, y, EPS_03F, 10, 250)
    assert r["n_clusters"] == 3
    assert np.all(r["records"] == 1)
    pairs = set(zip(r["cluster"].tolist(), lab.astype(int).tolist()))
    assert len(pairs) == 4 and len({a for a, _ in pairs}) == 4  # a bijection
    assert (0, 0) in pairs


def test_band_model_shapes():
    """tests/band_model.py (the host model of the band form's staging capacity that the band
    tests take their exact recall counts from): a dense square overflows whichever axis the
    rows take, a dense strip overflows with its rows along it and not across it, and the
    shipped choice (rows along the axis with fewer cells per row) takes the strip across."""
    import numpy as np

    from band_model import band_overflows, band_recall

    rng = np.random.default_rng(5)
    x, y = rng.uniform(0, 50, 20000), rng.uniform(0, 0.05, 20000)
    assert band_overflows(x, y, 0.2)[0]  # rows along the strip: one row of 20000 points
    assert not band_recall(x, y, 0.2) and not band_recall(y, x, 0.2)
    sx, sy = rng.uniform(0, 0.5, 20000), rng.uniform(0, 0.5, 20000)
    assert band_recall(sx, sy, 0.2) and band_recall(sy, sx, 0.2)
    bx, by = rng.normal(0, 5, 3000), rng.normal(0, 5, 3000)
    assert not band_recall(bx, by, 0.3)
