"""GPU parity on inputs shaped to drive every branch of the tiled fit (fit.hip) -- exact vs the
CPU grid oracle:
  * dense clumps: tiles whose 10x10-cell stage exceeds the LDS capacity (global-memory count
    path), quarter cells with > 32 points and > 8 cores (generic pair tests);
  * minPoints > 12: no neighbour lists, the label pass scans the stencil itself;
  * minPoints 1 and 2: every point core / lists of one neighbour;
  * a grid too fine for 2^23 tiles: the cell side grows, quarter cells stop being cliques and
    the per-point union runs;
  * clusters laid along tile edges and corners (the tile-edge merge);
  * a single tile (extent < 8 eps) and a one-row grid."""
import numpy as np
import pytest

import oracle as O

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
    h.set_band_max(0)  # (this module drives the tiled pipeline; tests/test_gpu_band.py the band)
    yield h
    h.close()


def _check(dm, handle, x, y, eps, mp, modes=(0, 1)):
    for mode in modes:
        cl, fl, k = dm.fit_arrays(x, y, eps, mp, mode, handle=handle)
        rc, rf, rk = O.fit_grid(x, y, eps, mp, mode)
        assert k == rk
        mism = np.flatnonzero((cl != rc) | (fl != rf))
        assert mism.size == 0, f"mode {mode}: {mism.size} mismatches, first {mism[:10]}"


def _clumps(n, seed, sigma, k=6, spread=20.0, noise=0.1):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-spread, spread, size=(k, 2))
    m = n - int(n * noise)
    pts = c[rng.integers(0, k, m)] + rng.normal(0, sigma, size=(m, 2))
    pts = np.concatenate([pts, rng.uniform(-spread * 1.5, spread * 1.5, size=(n - m, 2))])
    pts = pts[rng.permutation(n)]
    return pts[:, 0].copy(), pts[:, 1].copy()


@pytest.mark.parametrize("sigma", [0.05, 0.3, 1.5])
def test_dense_clumps(dm, handle, sigma):
    x, y = _clumps(150_000, seed=int(sigma * 100), sigma=sigma)
    _check(dm, handle, x, y, 0.25, 10)
    assert handle.stats()["clique"] == 1


@pytest.mark.parametrize("mp", [13, 25, 60])
def test_min_points_without_neighbour_lists(dm, handle, mp):
    x, y = _clumps(120_000, seed=mp, sigma=1.0, noise=0.3)
    _check(dm, handle, x, y, 0.3, mp)


@pytest.mark.parametrize("mp", [1, 2, 3, 12])
def test_small_min_points(dm, handle, mp):
    x, y = _clumps(80_000, seed=mp, sigma=0.8, noise=0.4)
    _check(dm, handle, x, y, 0.2, mp)


def test_grid_too_fine_for_tiles(dm, handle):
    """eps so small against the extent that 8x8-cell tiles would exceed 2^23: the host grows
    the cell side and the quarter cells are no longer cliques (per-point union path)."""
    rng = np.random.default_rng(3)
    n = 60_000
    x = rng.uniform(0, 1e4, n)
    y = rng.uniform(0, 1e4, n)
    # pairs and triples at distance < eps so that clusters exist
    x[: n // 3] = x[n // 3: 2 * n // 3] + rng.uniform(-4e-4, 4e-4, n // 3)
    y[: n // 3] = y[n // 3: 2 * n // 3] + rng.uniform(-4e-4, 4e-4, n // 3)
    _check(dm, handle, x, y, 1e-3, 2, modes=(0,))
    st = handle.stats()
    assert st["grid_mode"] == 0 and st["clique"] == 0
    _check(dm, handle, x, y, 1e-3, 2, modes=(1,))


@pytest.mark.parametrize("eps", [0.5, 1.0])
def test_clusters_on_tile_edges_and_corners(dm, handle, eps):
    """Dense lines along multiples of 8*eps (tile edges) and blobs on tile corners."""
    rng = np.random.default_rng(int(eps * 10))
    parts = []
    for k in range(-3, 4):
        t = rng.uniform(-30 * eps, 30 * eps, 4000)
        parts.append(np.stack([np.full_like(t, 8 * eps * k) + rng.normal(0, 0.2 * eps, t.size),
                               t], 1))
        parts.append(np.stack([t, np.full_like(t, 8 * eps * k) +
                               rng.normal(0, 0.2 * eps, t.size)], 1))
    for kx in range(-3, 4):
        for ky in range(-3, 4):
            parts.append(rng.normal(0, 0.6 * eps, (300, 2)) + 8 * eps * np.array([kx, ky]))
    parts.append(rng.uniform(-32 * eps, 32 * eps, (8000, 2)))
    pts = np.concatenate(parts)
    pts = pts[rng.permutation(len(pts))]
    _check(dm, handle, pts[:, 0].copy(), pts[:, 1].copy(), eps, 6)


def test_single_tile_and_single_row(dm, handle):
    rng = np.random.default_rng(11)
    x = rng.normal(0, 0.5, 5000)
    y = rng.normal(0, 0.5, 5000)
    _check(dm, handle, x, y, 0.6, 8)  # extent ~ 6 eps: one tile
    x = rng.uniform(0, 500, 20000)
    y = rng.uniform(0, 0.1, 20000)
    _check(dm, handle, x, y, 0.3, 5)  # one row of cells, many tiles along x


@pytest.mark.parametrize("div,mp", [(1, 5), (1, 3), (3, 29), (3, 10), (5, 40)])
def test_lattice_pairs_at_exactly_eps(dm, handle, div, mp):
    """Lattices of spacing eps/div: every point has lattice neighbours at distance eps exactly
    (up to the fp64 rounding of the coordinates), so the fp32 cell-unit pre-filter of the
    clique-grid count and pair tests (count_wave / count32) finds them ambiguous and the exact
    fp64 predicate decides -- core flags hinge on those pairs when minPoints equals the lattice
    disc count.  div 1: small tiles (one wave each); div 3 / 5: medium and big tiles.  Offsets
    of 1e3 and a few one-ulp nudges make the fp64 differences round both ways."""
    eps = 0.3
    rng = np.random.default_rng(div * 100 + mp)
    side = {1: 120, 3: 150, 5: 160}[div]
    i, j = np.meshgrid(np.arange(side), np.arange(side), indexing="ij")
    x = 1e3 + i.ravel() * (eps / div)
    y = -2e3 + j.ravel() * (eps / div)
    k = rng.choice(x.size, x.size // 10, replace=False)
    x[k] = np.nextafter(x[k], np.where(rng.random(k.size) < 0.5, -np.inf, np.inf))
    k = rng.choice(y.size, y.size // 10, replace=False)
    y[k] = np.nextafter(y[k], np.where(rng.random(k.size) < 0.5, -np.inf, np.inf))
    p = rng.permutation(x.size)
    _check(dm, handle, x[p].copy(), y[p].copy(), eps, mp)
    assert handle.stats()["clique"] == 1
    # the same lattices through the band LDS fit (its own fp32 pre-filter and exact fallback)
    hb = dm.Handle(0)
    try:
        _check(dm, hb, x[p].copy(), y[p].copy(), eps, mp)
        assert hb.stats()["clique"] == 1
    finally:
        hb.close()


@pytest.mark.parametrize("offset,eps", [(1e12, 1e-3), (-3e9, 0.05), (0.0, 1e-150)])
def test_fp32_records_far_from_origin(dm, handle, offset, eps):
    """Tile-relative fp32 records must not lose the fp64 predicate: clumps far from the origin
    (coordinate ulps close to eps), and a tiny eps whose squares sit near the fp64 underflow.
    Exact against the CPU oracle."""
    rng = np.random.default_rng(abs(int(np.log10(abs(offset) + 1))) + 7)
    n = 60_000
    c = rng.uniform(-30 * eps, 30 * eps, size=(12, 2))
    pts = c[rng.integers(0, 12, n)] + rng.normal(0, 0.8 * eps, size=(n, 2))
    x = offset + pts[:, 0]
    y = -offset + pts[:, 1]
    _check(dm, handle, x, y, eps, 8)


@pytest.mark.parametrize("n_tiles", [1, 2, 3, 5])
@pytest.mark.parametrize("per_tile", [9, 10, 31, 32, 33, 64, 65, 192, 193])
def test_small_tile_buckets_and_packing(dm, handle, n_tiles, per_tile):
    """Isolated tiles of chosen stage sizes, around the small-tile bucket edges (32 | 64 | 96 |
    144 | 192) and the two-tiles-per-wave packing: an odd number of packed tiles leaves a wave's
    second segment empty; 9 / 10 points straddle minPoints."""
    rng = np.random.default_rng(n_tiles * 1000 + per_tile)
    eps = 1.0
    xs, ys = [], []
    for t in range(n_tiles):  # tile centres 40 eps apart: every stage holds its own clump only
        cx, cy = 40.0 * t + 4.0, 4.0 + 40.0 * (t % 2)
        xs.append(cx + rng.normal(0, 0.6, per_tile))
        ys.append(cy + rng.normal(0, 0.6, per_tile))
    x, y = np.concatenate(xs), np.concatenate(ys)
    _check(dm, handle, x, y, eps, 10)
