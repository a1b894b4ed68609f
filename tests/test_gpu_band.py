"""Partitions in ONE launch of the band form (small.hip band_fit_kernel): 400 <= m <= 65536
points by default (dbscan_set_band_min / _max), ~m/256 workgroups (16..64) each staging its own
cell range's rows plus one row either side, six grid barriers, quarter-level unions (per-core
walks on grown grids), the clusters merged over input indices.  Every result must equal the
oracle (LocalDBSCANNaive.scala:37-118 / LocalDBSCANArchery.scala:36-112 restated, visit order =
array order) and the tiled pipeline (dbscan_set_band_max 0) bit for bit; ranges over the
staging capacity and barriers that give up fall back to the tiled pipeline.  (Sizes up to 8192
run through this form in tests/test_gpu_small.py as well.)"""
import numpy as np
import pytest

import oracle as O
from band_model import band_recall

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dm():
    import dbscan_amd

    if dbscan_amd.load().dbscan_device_count() < 1:
        pytest.fail("no GPU visible to libdbscan_hip.so")
    return dbscan_amd


def _set(rng, m, spread=3.0):
    k = int(rng.integers(2, 10))
    c = rng.uniform(-spread, spread, size=(k, 2))
    nb = m - m // 5
    pts = c[rng.integers(0, k, nb)] + rng.normal(0, rng.uniform(0.05, 0.4), size=(nb, 2))
    pts = np.concatenate([pts, rng.uniform(-spread - 1, spread + 1, size=(m - nb, 2))])
    pts = pts[rng.permutation(m)] * np.sqrt(m / 8192.0)
    return pts[:, 0].copy(), pts[:, 1].copy()


def _eq(got, ref, what):
    cl, fl, k = got
    rc, rf, rk = ref
    assert k == rk, f"{what}: {k} clusters, oracle {rk}"
    bad = np.flatnonzero((cl != rc) | (fl != rf))
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first {bad[:10]}"


@pytest.mark.parametrize("mode", [0, 1])
def test_band_sizes_vs_oracle(dm, mode):
    """Sizes from just above the LDS capacity to the band ceiling, through dbscan_fit_h and
    dbscan_fit_device (the densest of these sets overflow a band and take the fallback; the
    others do not)."""
    import torch

    from dbscan_amd import device as D

    rng = np.random.default_rng(800 + mode)
    h = dm.Handle(0)
    try:
        before = h.spread_fallbacks()
        expect = before
        for m in (8193, 9000, 12345, 16384, 20000, 33333, 50000, 65535, 65536):
            x, y = _set(rng, m)
            eps, mp = (0.12, 6) if m % 2 else (0.2, 10)
            ref = O.fit_grid(x, y, eps, mp, mode)
            _eq(dm.fit_arrays(x, y, eps, mp, mode, handle=h), ref, f"fit_h m={m}")
            tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
            cl, fl, k = D.fit_tensors(tx, ty, eps, mp, mode, h)
            _eq((cl.cpu().numpy(), fl.cpu().numpy(), k), ref, f"device m={m}")
            # the sets the band model says overflow a workgroup's staging (a row band of more
            # than kBandCap points) take the tiled recall, both calls; no other fit does
            expect += 2 * int(band_recall(x, y, eps))
            assert h.spread_fallbacks() == expect, f"m={m}"
        # (mode 1's 50000 / 65535-point sets: 4 recalls; mode 0: none)
        assert expect - before == (0, 4)[mode]
    finally:
        h.close()


def test_band_sparse_partitions_take_no_fallback(dm):
    """Partitions shaped like the seam's halo-grown ones above 8192 points (blobs over tens of
    eps cells per side, rows of a few hundred points): the band form serves them all."""
    rng = np.random.default_rng(42)
    h = dm.Handle(0)
    try:
        before = h.spread_fallbacks()
        for m in (9000, 15000, 19273):
            side = 25 * 2.55
            c = rng.uniform(0, side, size=(6, 2))
            pts = c[rng.integers(0, 6, m)] + rng.normal(0, side / 6, size=(m, 2))
            x, y = pts[:, 0].copy(), pts[:, 1].copy()
            _eq(dm.fit_arrays(x, y, 2.55, 10, 0, handle=h), O.fit_grid(x, y, 2.55, 10, 0),
                f"m={m}")
        assert h.spread_fallbacks() == before
    finally:
        h.close()


def test_band_equals_tiled_and_edge_inputs(dm):
    """Non-finite points, minPoints 1, a large eps (few wide cells), duplicates, visit-order
    permutations; the tiled pipeline (band_max 0) bit for bit."""
    rng = np.random.default_rng(91)
    h = dm.Handle(0)
    try:
        for m, eps, mp in ((15000, 0.12, 1), (30000, 2.0, 25), (40000, 0.05, 3)):
            x, y = _set(rng, m)
            x[::1013] = np.nan
            y[7::2027] = -np.inf
            x[100:200] = x[300:400]  # duplicates
            y[100:200] = y[300:400]
            ref = O.fit_grid(x, y, eps, mp, 0)
            got = dm.fit_arrays(x, y, eps, mp, 0, handle=h)
            _eq(got, ref, f"band m={m}")
            prev = h.set_band_max(0)
            _eq(dm.fit_arrays(x, y, eps, mp, 0, handle=h), ref, f"tiled m={m}")
            h.set_band_max(prev)
            p = rng.permutation(m)
            refp = O.fit_grid(x[p], y[p], eps, mp, 0)
            _eq(dm.fit_arrays(x[p], y[p], eps, mp, 0, handle=h), refp, f"permuted m={m}")
            np.testing.assert_array_equal(refp[1] == 1, ref[1][p] == 1)  # core flags move along
    finally:
        h.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_band_grown_grid_per_core_walks(dm, mode):
    """eps small against the extent: the band grid grows past eps cells, its quarter cells are
    no cliques (stats clique 0) and the unions take the per-core stencil walks; pairs and
    triples within eps make the clusters."""
    rng = np.random.default_rng(77 + mode)
    h = dm.Handle(0)
    try:
        for m in (3000, 20000):
            x = rng.uniform(0, 1e4, m)
            y = rng.uniform(0, 1e4, m)
            k = m // 3
            x[:k] = x[k:2 * k] + rng.uniform(-4e-4, 4e-4, k)
            y[:k] = y[k:2 * k] + rng.uniform(-4e-4, 4e-4, k)
            x[2 * k:2 * k + k // 2] = x[k:k + k // 2] + rng.uniform(-4e-4, 4e-4, k // 2)
            y[2 * k:2 * k + k // 2] = y[k:k + k // 2] + rng.uniform(-4e-4, 4e-4, k // 2)
            ref = O.fit_grid(x, y, 1e-3, 2, mode)
            before = h.spread_fallbacks()
            _eq(dm.fit_arrays(x, y, 1e-3, 2, mode, handle=h), ref, f"m={m}")
            assert h.spread_fallbacks() == before  # (the band form itself ran ...)
            assert h.stats()["clique"] == 0  # (... on a grid without quarter cliques)
    finally:
        h.close()


def _dense_square(rng, m):
    """m points in a 0.5 x 0.5 square: at eps 0.2 every 3-row band holds all of them, whichever
    axis the rows take (over a band's staging capacity)"""
    return rng.uniform(0, 0.5, m), rng.uniform(0, 0.5, m)


def test_band_overflow_and_barrier_fallbacks(dm):
    """Rows denser than a band's staging capacity (20000 points in a square of ~3 x 3 cells)
    and a forced barrier give-up (poll bound 0) both re-run through the tiled pipeline in the
    same call, counted, equal to the oracle.  A thin dense strip (rows along its length would
    hold all of it) takes its rows across instead and needs no recall."""
    rng = np.random.default_rng(5)
    h = dm.Handle(0)
    try:
        m = 20000
        x = rng.uniform(0, 50, m)
        y = rng.uniform(0, 0.05, m)
        before = h.spread_fallbacks()
        _eq(dm.fit_arrays(x, y, 0.2, 10, 0, handle=h), O.fit_grid(x, y, 0.2, 10, 0),
            "dense strip")
        _eq(dm.fit_arrays(y, x, 0.2, 10, 0, handle=h), O.fit_grid(y, x, 0.2, 10, 0),
            "dense strip, transposed")
        assert h.spread_fallbacks() == before
        x, y = _dense_square(rng, m)
        ref = O.fit_grid(x, y, 0.2, 10, 0)
        _eq(dm.fit_arrays(x, y, 0.2, 10, 0, handle=h), ref, "dense square")
        assert h.spread_fallbacks() == before + 1
        x2, y2 = _set(rng, 30000)
        ref2 = O.fit_grid(x2, y2, 0.12, 6, 1)
        h.set_spread_spin_limit(0)
        _eq(dm.fit_arrays(x2, y2, 0.12, 6, 1, handle=h), ref2, "barrier give-up")
        assert h.spread_fallbacks() == before + 2
        h.set_spread_spin_limit(1 << 21)
        _eq(dm.fit_arrays(x2, y2, 0.12, 6, 1, handle=h), ref2, "default bound")
        assert h.spread_fallbacks() == before + 2
    finally:
        h.close()


@pytest.mark.parametrize("nt", [4, 8, 16])
def test_band_from_concurrent_handles(dm, nt):
    """nt executor threads, a handle each, band fits at once (nt x up to 64 workgroups of one
    CU each; the process has 4 hardware queues on the box, so from 8 threads on more fits are
    queued than can run): every fit equals its oracle fit, whether or not a grid barrier gave up
    and the fit was re-run (tools/concurrency_probe.py: no give-ups at 4-16 threads)."""
    import threading

    rng = np.random.default_rng(606)
    sets = []
    for m in (9000, 20000, 40000, 65536, 12000, 30000, 50000, 16000):
        x, y = _set(rng, m)
        sets.append((x, y))
    refs = [O.fit_grid(x, y, 0.12, 6, 0) for x, y in sets]
    handles = [dm.Handle(0) for _ in range(nt)]
    errors = []

    def worker(t):
        try:
            for rep in range(2 * len(sets) // nt + 1):
                k = (t + rep) % len(sets)
                x, y = sets[k]
                _eq(dm.fit_arrays(x, y, 0.12, 6, 0, handle=handles[t]), refs[k],
                    f"thread {t} set {k} rep {rep}")
        except Exception as exc:
            errors.append(exc)

    try:
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(nt)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    finally:
        for hh in handles:
            hh.close()
    assert not errors, errors[0]


def test_band_labels_written_into_pinned_block(dm):
    """dbscan_fit_h up to 16384 points: the LDS kernels write cluster|flag into the handle's
    pinned block themselves (capi.hip kDirectOutMax); above it the labels come back by copy.
    Both sides of the limit, and the recalls that re-run such a fit through the tiled pipeline
    into the same block (a staging overflow, a barrier that gives up), equal the oracle."""
    rng = np.random.default_rng(16384)
    h = dm.Handle(0)
    try:
        for m in (7000, 16384, 16385):
            x, y = _set(rng, m)
            _eq(dm.fit_arrays(x, y, 0.12, 6, 0, handle=h), O.fit_grid(x, y, 0.12, 6, 0),
                f"m={m}")
        before = h.spread_fallbacks()
        x, y = _dense_square(rng, 12000)  # every row band over a band's staging capacity
        _eq(dm.fit_arrays(x, y, 0.2, 10, 1, handle=h), O.fit_grid(x, y, 0.2, 10, 1), "square")
        assert h.spread_fallbacks() == before + 1
        x2, y2 = _set(rng, 9000)
        ref2 = O.fit_grid(x2, y2, 0.12, 6, 0)
        h.set_spread_spin_limit(0)
        _eq(dm.fit_arrays(x2, y2, 0.12, 6, 0, handle=h), ref2, "barrier give-up")
        assert h.spread_fallbacks() == before + 2
        h.set_spread_spin_limit(1 << 21)
        _eq(dm.fit_arrays(x2, y2, 0.12, 6, 0, handle=h), ref2, "default bound")
    finally:
        h.close()


def test_async_queued_fits_all_recalled(dm):
    """Three asynchronous fits of different data queued back to back on one handle (a band fit
    over the one-box limit of 16384 points, a band fit below it in Archery mode, a spread fit),
    every grid barrier giving up at once (spin limit 0), ONE dbscan_sync: each fit has its own
    stats block and recall record, so all three are re-run and each equals the oracle, cluster
    count included (dbscan_fit_device_async must never leave wrong labels, DBSCAN.scala:153-154).
    Then the default bound: the same handle fits again with no re-run (the give-ups left no
    dirty band counters behind)."""
    import torch

    from dbscan_amd import device as D

    rng = np.random.default_rng(606)
    h = dm.Handle(0)
    try:
        assert h.set_spread_spin_limit(0) == 1 << 21
        before = h.spread_fallbacks()
        cases = [(20000, 0.2, 10, 0, None), (9000, 0.12, 6, 1, None), (5000, 0.2, 5, 0, "spread")]
        outs = []
        for m, eps, mp, mode, form in cases:
            x, y = _set(rng, m)
            if form == "spread":
                h.set_band_min(1 << 30)
                h.set_spread_min(0)
            tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
            cl = torch.full((m,), -9, dtype=torch.int32, device="cuda")
            fl = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
            nk = torch.full((1,), -1, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            D.fit_tensors_async(tx, ty, eps, mp, mode, h, cl, fl, nk)
            outs.append((x, y, eps, mp, mode, tx, ty, cl, fl, nk))
        h.sync()
        torch.cuda.synchronize()
        assert h.spread_fallbacks() == before + 3
        for x, y, eps, mp, mode, _, _, cl, fl, nk in outs:
            _eq((cl.cpu().numpy(), fl.cpu().numpy(), int(nk.item())),
                O.fit_grid(x, y, eps, mp, mode), f"queued m={x.size}")
        h.set_spread_spin_limit(1 << 21)
        h.set_band_min(400)
        h.set_spread_min(512)
        for m in (20000, 9000):  # (the seam's halo-grown shape: no staging overflow)
            c = rng.uniform(0, 25 * 2.55, size=(6, 2))
            pts = c[rng.integers(0, 6, m)] + rng.normal(0, 25 * 2.55 / 6, size=(m, 2))
            x, y = pts[:, 0].copy(), pts[:, 1].copy()
            _eq(dm.fit_arrays(x, y, 2.55, 10, 0, handle=h), O.fit_grid(x, y, 2.55, 10, 0),
                f"after m={m}")
        assert h.spread_fallbacks() == before + 3
    finally:
        h.close()


def test_async_overflow_then_another_fit(dm):
    """A queued band fit that overflows its staging (20000 points in a square of ~3 x 3 cells:
    kStError 3) followed by two more queued fits, one dbscan_sync: the square is re-run through
    the tiled pipeline into its own outputs, the fits after it are untouched, all equal the
    oracle."""
    import torch

    from dbscan_amd import device as D

    rng = np.random.default_rng(707)
    h = dm.Handle(0)
    try:
        before = h.spread_fallbacks()
        sets = [_dense_square(rng, 20000) + (0.2, 10, 0)]
        for m in (9000, 3000):
            x, y = _set(rng, m)
            sets.append((x, y, 0.12, 6, m % 2))
        outs = []
        for x, y, eps, mp, mode in sets:
            tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
            cl = torch.full((x.size,), -9, dtype=torch.int32, device="cuda")
            fl = torch.full((x.size,), 9, dtype=torch.uint8, device="cuda")
            nk = torch.full((1,), -1, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            D.fit_tensors_async(tx, ty, eps, mp, mode, h, cl, fl, nk)
            outs.append((tx, ty, cl, fl, nk))
        h.sync()
        torch.cuda.synchronize()
        assert h.spread_fallbacks() == before + 1
        for (x, y, eps, mp, mode), (_, _, cl, fl, nk) in zip(sets, outs):
            _eq((cl.cpu().numpy(), fl.cpu().numpy(), int(nk.item())),
                O.fit_grid(x, y, eps, mp, mode), f"queued m={x.size}")
        st = h.stats()  # the last fit's
        assert st["n"] == 3000
    finally:
        h.close()


def test_async_fits_wrap_the_stats_ring(dm):
    """150 asynchronous LDS fits (one-workgroup, spread and band forms) queued on one handle
    without a sync: more than two turns of the 64-block stats ring, so the ring drains the
    stream and checks the queued fits when it is full; one dbscan_sync; every fit's labels and
    cluster count equal the oracle."""
    import torch

    from dbscan_amd import device as D

    rng = np.random.default_rng(150)
    h = dm.Handle(0)
    try:
        h.set_spread_min(1000)
        h.set_band_min(3000)
        sets, outs = [], []
        for i in range(150):
            m = int(rng.choice([200, 700, 1500, 2500, 5000, 9000]))
            x, y = _set(rng, m)
            mode = i % 2
            tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
            cl = torch.full((m,), -9, dtype=torch.int32, device="cuda")
            fl = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
            nk = torch.full((1,), -1, dtype=torch.int32, device="cuda")
            sets.append((x, y, mode))
            outs.append((tx, ty, cl, fl, nk))
        torch.cuda.synchronize()
        for (x, y, mode), (tx, ty, cl, fl, nk) in zip(sets, outs):
            D.fit_tensors_async(tx, ty, 0.12, 6, mode, h, cl, fl, nk)
        h.sync()
        torch.cuda.synchronize()
        for k, ((x, y, mode), (_, _, cl, fl, nk)) in enumerate(zip(sets, outs)):
            _eq((cl.cpu().numpy(), fl.cpu().numpy(), int(nk.item())),
                O.fit_grid(x, y, 0.12, 6, mode), f"fit {k} m={x.size}")
    finally:
        h.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_band_wide_and_tall_partitions(dm, mode):
    """Partitions much wider than tall (the band grid then takes its rows across, on (y, x))
    and much taller than wide (rows along y), sparse and dense, with non-finite points: each
    equals the oracle, and fitting (y, x) gives the same labels as (x, y) (the predicate
    dx*dx + dy*dy is symmetric, so every form must be too)."""
    rng = np.random.default_rng(4242 + mode)
    h = dm.Handle(0)
    try:
        before = h.spread_fallbacks()
        for m, w, hgt, eps, mp in ((3000, 40.0, 2.0, 0.2, 5), (12000, 60.0, 1.0, 0.12, 6),
                                   (20000, 200.0, 6.0, 0.3, 10), (50000, 300.0, 3.0, 0.15, 8)):
            k = int(rng.integers(3, 12))
            c = np.column_stack([rng.uniform(0, w, k), rng.uniform(0, hgt, k)])
            pts = c[rng.integers(0, k, m)] + rng.normal(0, eps * 3, size=(m, 2))
            x, y = pts[:, 0].copy(), pts[:, 1].copy()
            x[::997] = np.nan
            ref = O.fit_grid(x, y, eps, mp, mode)
            _eq(dm.fit_arrays(x, y, eps, mp, mode, handle=h), ref, f"wide m={m}")
            _eq(dm.fit_arrays(y, x, eps, mp, mode, handle=h), ref, f"tall m={m}")
            expect = int(band_recall(x, y, eps)) + int(band_recall(y, x, eps))
            assert h.spread_fallbacks() - before == expect, f"m={m}"
            before += expect
    finally:
        h.close()


def test_async_queue_fuzz(dm):
    """A seeded mix of queued work on one handle -- single fits of every form (one-workgroup,
    spread, band, tiled), batches of partitions, forced barrier give-ups switched on and off
    between enqueues, syncs at random points -- and one final dbscan_sync: every queued fit's
    labels and cluster counts equal the oracle, and the handle's re-run count equals the
    number of queued spread / band fits that ran with the give-up forced or overflowed
    (DBSCAN.scala:150-155: an executor's fits never come back wrong)."""
    import torch

    from dbscan_amd import device as D

    rng = np.random.default_rng(2026)
    h = dm.Handle(0)
    try:
        h.set_spread_min(1000)
        h.set_band_min(2500)
        before = h.spread_fallbacks()
        expect = 0
        jobs = []
        for step in range(40):
            give_up = bool(rng.random() < 0.5)
            h.set_spread_spin_limit(0 if give_up else 1 << 21)
            kind = rng.choice(["single", "single", "single", "batch", "sync"])
            if kind == "sync":
                h.sync()
                continue
            mode = int(rng.integers(0, 2))
            eps, mp = (0.2, 10) if rng.random() < 0.5 else (0.12, 6)
            if kind == "single":
                m = int(rng.choice([300, 1500, 4000, 9000, 20000, 70000]))
                if m <= 9000 and rng.random() < 0.3:  # (the oracle's cost grows as m^2 here)
                    x, y = _dense_square(rng, m)
                else:
                    x, y = _set(rng, m)
                tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
                cl = torch.full((m,), -9, dtype=torch.int32, device="cuda")
                fl = torch.full((m,), 9, dtype=torch.uint8, device="cuda")
                nk = torch.full((1,), -1, dtype=torch.int32, device="cuda")
                torch.cuda.synchronize()
                D.fit_tensors_async(tx, ty, eps, mp, mode, h, cl, fl, nk)
                jobs.append(("single", [(x, y)], eps, mp, mode, (tx, ty, cl, fl, nk)))
                lds = m <= 65536 and m >= 1000  # (spread from 1000, band from 2500 points)
                if lds and (give_up or (m >= 2500 and band_recall(x, y, eps))):
                    expect += 1
            else:
                sizes = rng.integers(50, 3000, size=int(rng.integers(3, 12)))
                parts = [_set(rng, int(s)) for s in sizes]
                x = np.concatenate([p[0] for p in parts])
                y = np.concatenate([p[1] for p in parts])
                offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
                tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
                cl = torch.full((x.size,), -9, dtype=torch.int32, device="cuda")
                fl = torch.full((x.size,), 9, dtype=torch.uint8, device="cuda")
                nk = torch.full((len(sizes),), -1, dtype=torch.int32, device="cuda")
                torch.cuda.synchronize()
                D.fit_batch_tensors_async(tx, ty, offs, eps, mp, mode, h, cl, fl, nk)
                jobs.append(("batch", parts, eps, mp, mode, (tx, ty, cl, fl, nk)))
        h.sync()
        torch.cuda.synchronize()
        h.set_spread_spin_limit(1 << 21)
        for k, (kind, parts, eps, mp, mode, (_, _, cl, fl, nk)) in enumerate(jobs):
            cl, fl, nk = cl.cpu().numpy(), fl.cpu().numpy(), nk.cpu().numpy()
            o = 0
            for p, (x, y) in enumerate(parts):
                m = x.size
                _eq((cl[o:o + m], fl[o:o + m], int(nk[p])), O.fit_grid(x, y, eps, mp, mode),
                    f"job {k} ({kind}) part {p} m={m}")
                o += m
        assert h.spread_fallbacks() - before == expect
    finally:
        h.close()
