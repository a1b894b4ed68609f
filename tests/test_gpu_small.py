"""The seam's real call pattern on the GPU: partition-sized fits (small.hip, one workgroup per
partition) and batches of them, bit-exact against the CPU oracle.

DBSCAN.scala:150-155 runs `new LocalDBSCANNaive(eps, minPoints).fit(points)` once per spatial
partition (EvenSplitPartitioner.scala:44-209 + the eps halo of DBSCAN.scala:116-137), so the
fits the seam sees hold hundreds to ~10^4 points.  Every case runs through the one-workgroup
kernel (small_fit_kernel), its multi-workgroup form (spread_fit_kernel: ~256 points per
workgroup, two grid barriers; dbscan_set_spread_min) and, where noted, through the tiled pipeline
as well (dbscan_set_small_max(h, 0)), and all must equal the oracle (LocalDBSCANNaive.scala:37-118
/ LocalDBSCANArchery.scala:36-112 restated, visit order = array order)."""
import numpy as np
import pytest

import oracle as O
from conftest import EPS_03F, gen_blobs, load_edge_cases

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


def _eq(got, ref, what=""):
    cl, fl, k = got
    rc, rf, rk = ref
    assert k == rk, f"{what}: {k} clusters, oracle {rk}"
    bad = np.flatnonzero((cl != rc) | (fl != rf))
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first {bad[:10]}"


ONE_WG = 1 << 30  # dbscan_set_spread_min: every LDS fit on one workgroup
NO_BAND = 1 << 30  # dbscan_set_band_min: no LDS-sized fit takes the band form
BAND_MIN = 400  # DBSCAN_BAND_MIN_DEFAULT_POINTS


def _lds_forms(handle):
    """(name, spread_min, band_min) of the three one-launch forms for LDS-sized fits: one
    workgroup, spread from 0 points, the band form from 1 point (where eligible)"""
    return (("small", ONE_WG, NO_BAND), ("spread", 0, NO_BAND), ("band", 0, 0))


def _both_paths(dm, handle, x, y, eps, mp, mode, ref):
    """The one-workgroup fit, the spread fit and the tiled pipeline, each against ref."""
    try:
        for name, spread, band in _lds_forms(handle):
            handle.set_small_max(8192)
            handle.set_spread_min(spread)
            handle.set_band_min(band)
            _eq(dm.fit_arrays(x, y, eps, mp, mode, handle=handle), ref, f"{name} path")
        handle.set_small_max(0)
        _eq(dm.fit_arrays(x, y, eps, mp, mode, handle=handle), ref, "tiled path")
    finally:
        handle.set_small_max(8192)
        handle.set_spread_min(512)
        handle.set_band_min(BAND_MIN)


@pytest.mark.parametrize("mode", [0, 1])
def test_labeled_csv_both_paths(dm, handle, labeled_data, labeled_expected, mode):
    """LocalDBSCANArcherySuite 'should cluster' (749 points) through both fit paths."""
    x, y, _ = labeled_data
    ref = O.fit_sequential(x, y, EPS_03F, 10, mode)
    _both_paths(dm, handle, x, y, EPS_03F, 10, mode, ref)
    handle.set_small_max(8192)
    dm.fit_arrays(x, y, EPS_03F, 10, mode, handle=handle)
    st = handle.stats()
    assert st["core"] == 677 and st["clusters"] == 3 and st["finite"] == 749


def test_labeled_csv_reference_partitions(dm, handle, labeled_data):
    """DBSCANSuite's job (maxPointsPerPartition 250): the reference's 4 partitions, each point
    duplicated into every partition whose eps-grown rectangle holds it (249 / 409 / 235 / 204
    points), then ONE batch call; each partition's labels equal the
    sequential oracle's fit of that partition alone."""
    x, y, _ = labeled_data
    rects, counts = O.ref_partition(x, y, EPS_03F, 250)
    prod = dm.partition.partition_points(x, y, EPS_03F, 250, handle)
    assert np.allclose(rects, np.array([r for r, _ in prod])) and \
        list(counts) == [c for _, c in prod]
    offs, idx = dm.duplicate(x, y, rects, EPS_03F)
    assert list(np.diff(offs)) == [249, 409, 235, 204]
    px, py = x[idx], y[idx]
    for mode in (0, 1):
        cl, fl, nk = dm.fit_batch(px, py, offs, EPS_03F, 10, mode, handle=handle)
        for p in range(len(offs) - 1):
            a, b = offs[p], offs[p + 1]
            _eq((cl[a:b], fl[a:b], int(nk[p])), O.fit_sequential(px[a:b], py[a:b], EPS_03F, 10,
                                                                 mode), f"partition {p}")


@pytest.mark.parametrize("case", load_edge_cases(), ids=lambda c: c["name"])
def test_edge_fixtures_both_paths(dm, handle, case):
    ref = (case["cluster"], case["flag"], case["n_clusters"])
    _both_paths(dm, handle, case["x"], case["y"], case["eps"], case["min_points"], case["mode"],
                ref)


def _fuzz_set(rng, m):
    k = int(rng.integers(1, 8))
    c = rng.uniform(-3, 3, size=(k, 2))
    nb = m - m // 4
    pts = c[rng.integers(0, k, nb)] + rng.normal(0, rng.uniform(0.05, 0.5), size=(nb, 2))
    pts = np.concatenate([pts, rng.uniform(-4, 4, size=(m - nb, 2))])
    pts = pts[rng.permutation(m)]
    return pts[:, 0].copy(), pts[:, 1].copy()


@pytest.mark.parametrize("m", [1, 2, 7, 63, 250, 1000, 2048, 4097, 8191, 8192])
def test_fuzz_sizes(dm, handle, m):
    """Random blobs + noise at every partition size up to the one-workgroup capacity, several
    eps / minPoints, both modes: single fits and the same sets as one batch."""
    rng = np.random.default_rng(7000 + m)
    sets = []
    for trial in range(3):
        x, y = _fuzz_set(rng, m)
        eps = float(rng.uniform(0.03, 0.4))
        mp = int(rng.integers(1, 15))
        sets.append((x, y, eps, mp))
    try:
        for mode in (0, 1):
            for x, y, eps, mp in sets:
                ref = (O.fit_sequential(x, y, eps, mp, mode) if m <= 3000
                       else O.fit_grid(x, y, eps, mp, mode))
                for name, spread, band in _lds_forms(handle):
                    handle.set_spread_min(spread)
                    handle.set_band_min(band)
                    _eq(dm.fit_arrays(x, y, eps, mp, mode, handle=handle), ref, f"{name} m={m}")
    finally:
        handle.set_spread_min(512)
        handle.set_band_min(BAND_MIN)
    # one batch of equal-eps partitions
    x = np.concatenate([s[0] for s in sets])
    y = np.concatenate([s[1] for s in sets])
    offs = np.arange(len(sets) + 1, dtype=np.int64) * m
    eps, mp = sets[0][2], sets[0][3]
    cl, fl, nk = dm.fit_batch(x, y, offs, eps, mp, 0, handle=handle)
    for p in range(len(sets)):
        a, b = offs[p], offs[p + 1]
        _eq((cl[a:b], fl[a:b], int(nk[p])), O.fit_grid(x[a:b], y[a:b], eps, mp, 0), f"batch {p}")


def test_batch_mixed_sizes_and_modes(dm, handle):
    """Empty partitions, partitions over the one-workgroup capacity (tiled pipeline inside the
    same batch) and a non-zero first offset; every partition equals its own oracle fit; the
    float32-box Archery mode runs every partition through the tiled pipeline."""
    rng = np.random.default_rng(5)
    sizes = [0, 1, 300, 0, 8192, 8193, 20000, 5000, 2]
    xs, ys = zip(*[_fuzz_set(rng, s) if s else (np.zeros(0), np.zeros(0)) for s in sizes])
    lead = 17  # offsets need not start at 0: the first 17 entries belong to no partition
    x = np.concatenate([rng.uniform(-1, 1, lead)] + list(xs))
    y = np.concatenate([rng.uniform(-1, 1, lead)] + list(ys))
    offs = lead + np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    for mode in (0, 1, 2):
        cl = np.full(x.size, -7, np.int32)
        fl = np.full(x.size, 9, np.uint8)
        cl, fl, nk = dm.fit_batch(x, y, offs, 0.2, 6, mode, handle=handle, cluster_out=cl,
                                  flag_out=fl)
        assert (cl[:lead] == -7).all() and (fl[:lead] == 9).all()  # untouched
        for p in range(len(sizes)):
            a, b = offs[p], offs[p + 1]
            ref = (O.fit_bfs_grid(x[a:b], y[a:b], 0.2, 6, mode) if mode == 2
                   else O.fit_grid(x[a:b], y[a:b], 0.2, 6, mode))
            _eq((cl[a:b], fl[a:b], int(nk[p])), ref, f"mode {mode} partition {p} (m={sizes[p]})")


def _stress_sets():
    rng = np.random.default_rng(99)
    out = []
    # every point the same: one cell, all pairs within eps (O(m^2) unions)
    out.append(("duplicates", np.full(8192, 1.25), np.full(8192, -3.5), 0.1, 10))
    # lattice at exactly eps (pairs on the threshold: the exact fp64 path decides)
    i, j = np.meshgrid(np.arange(90), np.arange(90), indexing="ij")
    lx, ly = 1e3 + i.ravel() * 0.1, -2e3 + j.ravel() * 0.1
    k = rng.choice(lx.size, lx.size // 10, replace=False)
    lx[k] = np.nextafter(lx[k], np.inf)
    out.append(("lattice_eps", lx, ly, 0.1, 5))
    # far from the origin (coordinate ulps near eps)
    c = rng.uniform(-30e-3, 30e-3, size=(6, 2))
    pts = c[rng.integers(0, 6, 6000)] + rng.normal(0, 0.8e-3, size=(6000, 2))
    out.append(("offset_1e12", 1e12 + pts[:, 0], -1e12 + pts[:, 1], 1e-3, 8))
    # one long row: 8000 cells wide (large fp32 records: a wide pre-filter band)
    t = rng.uniform(0, 800, 8000)
    out.append(("long_row", t, rng.normal(0, 0.02, 8000), 0.1, 4))
    # sparse over a huge extent: the cell side grows until the table fits
    out.append(("sparse_grown", rng.uniform(-1e6, 1e6, 4000), rng.uniform(-1e6, 1e6, 4000),
                1.0, 2))
    pairs = rng.uniform(-1e6, 1e6, (2000, 2))
    pp = np.concatenate([pairs, pairs + rng.uniform(-0.5, 0.5, (2000, 2))])
    out.append(("sparse_pairs", pp[:, 0].copy(), pp[:, 1].copy(), 1.0, 2))
    # non-finite coordinates mixed in, minPoints 0 / 1, eps 0, tiny eps
    x, y = _fuzz_set(rng, 3000)
    x[::37] = np.nan
    y[::53] = np.inf
    out.append(("nonfinite", x, y, 0.2, 5))
    out.append(("minpts0", x, y, 0.2, 0))
    out.append(("minpts1", x, y, 0.2, 1))
    q = np.round(x[:1000] * 4) / 4
    out.append(("eps0", q, np.round(y[:1000] * 4) / 4, 0.0, 2))
    out.append(("eps_tiny", x * 1e-150, y * 1e-150, 1e-151, 3))
    out.append(("eps_negative", x, y, -0.2, 5))
    return out


@pytest.mark.parametrize("name,x,y,eps,mp", _stress_sets(), ids=lambda v: v if isinstance(v, str) else "")
def test_stress_shapes(dm, handle, name, x, y, eps, mp):
    for mode in (0, 1):
        ref = O.fit_grid(x, y, eps, mp, mode)
        _both_paths(dm, handle, x, y, eps, mp, mode, ref)


def test_blob_partitions_batch(dm, handle):
    """G(10^6) cut by the reference's partitioner (maxPointsPerPartition 8192), duplicated into
    eps-grown partitions: the whole batch in one call, and the device-resident async form; each
    partition equals its own oracle fit."""
    import torch

    from dbscan_amd import device as D

    x, y = gen_blobs(1_000_000, noise=0.2, seed=21)
    parts = dm.partition.partition_points(x, y, 2.55, 8192, handle)
    rects = np.array([r for r, _ in parts])
    offs, idx = dm.duplicate(x, y, rects, 2.55)
    assert offs[-1] >= x.size - 100  # (the reference's split-line defect may drop a few)
    px, py = x[idx], y[idx]
    cl, fl, nk = dm.fit_batch(px, py, offs, 2.55, 10, 0, handle=handle)
    tx, ty = torch.from_numpy(px).cuda(), torch.from_numpy(py).cuda()
    dcl = torch.empty(px.size, dtype=torch.int32, device="cuda")
    dfl = torch.empty(px.size, dtype=torch.uint8, device="cuda")
    dnk = torch.empty(len(offs) - 1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    D.fit_batch_tensors_async(tx, ty, offs, 2.55, 10, 0, handle, dcl, dfl, dnk)
    handle.sync()
    assert np.array_equal(dcl.cpu().numpy(), cl) and np.array_equal(dfl.cpu().numpy(), fl)
    assert np.array_equal(dnk.cpu().numpy(), nk)
    big = 0
    for p in range(len(offs) - 1):
        a, b = offs[p], offs[p + 1]
        big += (b - a) > 8192
        _eq((cl[a:b], fl[a:b], int(nk[p])), O.fit_grid(px[a:b], py[a:b], 2.55, 10, 0),
            f"partition {p} (m={b - a})")
    assert len(offs) - 1 > 100


@pytest.mark.parametrize("band_min", [BAND_MIN, NO_BAND])
def test_spread_fits_from_concurrent_handles(dm, band_min):
    """Four executor threads, a handle each, fitting partitions concurrently through the spread
    and band forms (each launch holds its workgroups at grid barriers while the other handles'
    launches share the GPU; NO_BAND: the spread form alone): every fit equals its oracle fit,
    no barrier times out."""
    import threading

    rng = np.random.default_rng(404)
    sets = []
    for m in (600, 1500, 3000, 5000, 8192, 2500, 7000, 4096):
        x, y = _fuzz_set(rng, m)
        sets.append((x, y, float(rng.uniform(0.05, 0.3)), int(rng.integers(2, 12))))
    refs = [O.fit_grid(x, y, e, mp, 0) for x, y, e, mp in sets]
    handles = [dm.Handle(0) for _ in range(4)]
    for hh in handles:
        hh.set_band_min(band_min)
    errors = []

    def worker(t):
        try:
            for rep in range(3):
                for k in range(t, len(sets), 4):
                    x, y, e, mp = sets[k]
                    _eq(dm.fit_arrays(x, y, e, mp, 0, handle=handles[t]), refs[k],
                        f"thread {t} set {k} rep {rep}")
        except Exception as exc:  # (reported below, from the main thread)
            errors.append(exc)

    try:
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    finally:
        for hh in handles:
            hh.close()
    assert not errors, errors[0]


@pytest.mark.parametrize("m", [9000, 65536, 65537])
def test_host_array_fit_around_the_pinned_staging_limit(dm, handle, m):
    """dbscan_fit_h stages partitions of <= 65536 points through one pinned block and one DMA
    each way; above that it copies the caller's arrays directly: both sides of the limit, each
    against the oracle, and the caller's output arrays written in full."""
    rng = np.random.default_rng(65000 + m)
    x, y = _fuzz_set(rng, m)
    x *= 20.0
    y *= 20.0
    cl = np.full(m, -5, np.int32)
    fl = np.full(m, 7, np.uint8)
    got = dm.fit_arrays(x, y, 0.25, 6, 0, handle=handle, cluster_out=cl, flag_out=fl)
    _eq(got, O.fit_grid(x, y, 0.25, 6, 0), f"m={m}")
    assert (cl >= 0).all() and (fl <= 2).all()


def test_spread_fit_barrier_give_up_falls_back(dm):
    """A spread fit whose grid barrier gives up (its workgroups not all resident: forced here by
    the test-only poll bound 0, so every barrier gives up at once) is re-run by the
    one-workgroup kernel in the same call and still equals the oracle -- through dbscan_fit_h
    (host arrays: the labels copied back again), dbscan_fit_device and dbscan_fit_device_async
    + dbscan_sync (the device cluster count rewritten); every re-run is counted.  The
    reference's fit never fails on valid input (DBSCAN.scala:153-154)."""
    import torch

    from dbscan_amd import device as D

    rng = np.random.default_rng(911)
    h = dm.Handle(0)
    try:
        h.set_spread_min(0)
        h.set_band_min(NO_BAND)  # (the band form's own give-up: tests/test_gpu_band.py)
        assert h.set_spread_spin_limit(0) == 1 << 21
        before = h.spread_fallbacks()
        expect = before
        for m in (600, 3000, 8192):
            x, y = _fuzz_set(rng, m)
            ref = O.fit_grid(x, y, 0.2, 5, 0)
            _eq(dm.fit_arrays(x, y, 0.2, 5, 0, handle=h), ref, f"fit_h m={m}")
            expect += 1
            assert h.spread_fallbacks() == expect
            tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
            cl, fl, k = D.fit_tensors(tx, ty, 0.2, 5, 0, h)
            _eq((cl.cpu().numpy(), fl.cpu().numpy(), k), ref, f"device m={m}")
            expect += 1
            cl = torch.full((m,), -9, dtype=torch.int32, device="cuda")
            fl = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
            nk = torch.full((1,), -1, dtype=torch.int32, device="cuda")
            D.fit_tensors_async(tx, ty, 0.2, 5, 0, h, cl, fl, nk)
            h.sync()
            expect += 1
            _eq((cl.cpu().numpy(), fl.cpu().numpy(), int(nk.item())), ref, f"async m={m}")
            assert h.spread_fallbacks() == expect
        # the default bound again: no re-runs
        h.set_spread_spin_limit(1 << 21)
        x, y = _fuzz_set(rng, 5000)
        _eq(dm.fit_arrays(x, y, 0.2, 5, 0, handle=h), O.fit_grid(x, y, 0.2, 5, 0), "default")
        assert h.spread_fallbacks() == expect
    finally:
        h.close()
