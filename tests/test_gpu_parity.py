"""GPU parity tests: the gfx950 fit through the C-ABI vs the CPU oracle, bit-exact.

Flags and cluster numbers are integer outputs of an integer/predicate pipeline, so the bar
is exact equality (flags bit-exact; cluster ids bit-exact for Naive mode with
visit order = input order).  Mirrors the reference's LocalDBSCANArcherySuite ("should
cluster", :31-53) on the golden csv, plus the edge fixtures and random fuzz."""
import ctypes
import threading

import numpy as np
import pytest

import oracle as O
from conftest import EPS_03F, gen_blobs, load_edge_cases

pytestmark = pytest.mark.gpu

NAIVE_TO_CSV = {0: 0, 1: 1, 2: 3, 3: 2}


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


def _check(dm, handle, x, y, eps, mp, mode, ref=None):
    cl, fl, k = dm.fit_arrays(x, y, eps, mp, mode, handle=handle)
    if ref is None:
        ref = O.fit_grid(x, y, eps, mp, mode)
    rc, rf, rk = ref
    assert k == rk
    mism = np.flatnonzero((cl != rc) | (fl != rf))
    assert mism.size == 0, f"{mism.size} mismatches, first {mism[:10]}"
    return cl, fl, k


@pytest.mark.parametrize("mode", [0, 1])
def test_should_cluster_labeled_csv(dm, handle, labeled_data, labeled_expected, mode):
    """LocalDBSCANArcherySuite 'should cluster' on the GPU: exact vs the oracle and the
    committed fixture, and equal to the reference's csv labels up to SURVEY's permutation."""
    x, y, lab = labeled_data
    cl, fl, k = _check(dm, handle, x, y, EPS_03F, 10, mode, O.fit_sequential(x, y, EPS_03F, 10,
                                                                              mode))
    key = "naive" if mode == 0 else "archery"
    np.testing.assert_array_equal(cl, labeled_expected["cluster_" + key])
    np.testing.assert_array_equal(fl, labeled_expected["flag_" + key])
    np.testing.assert_array_equal(np.array([NAIVE_TO_CSV[c] for c in cl]), lab.astype(int))
    st = handle.stats()
    assert st["core"] == 677 and st["clusters"] == 3


def test_reference_interface_on_gpu(dm, labeled_data):
    x, y, lab = labeled_data
    pts = [dm.DBSCANPoint([a, b, c]) for a, b, c in zip(x, y, lab)]
    out = dm.LocalDBSCANNaive(EPS_03F, 10).fit(pts)
    assert len(out) == len(pts) and all(p.visited for p in out)
    assert [p.vector for p in out] == [p.vector for p in pts]  # input order, fresh objects
    assert sum(p.flag == dm.Flag.Core for p in out) == 677
    with pytest.raises(IndexError):
        dm.LocalDBSCANNaive(0.3, 1).fit([dm.DBSCANPoint([1.0])])


@pytest.mark.parametrize("case", load_edge_cases(), ids=lambda c: c["name"])
def test_edge_fixtures(dm, handle, case):
    ref = (case["cluster"], case["flag"], case["n_clusters"])
    _check(dm, handle, case["x"], case["y"], case["eps"], case["min_points"], case["mode"], ref)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_vs_sequential(dm, handle, seed):
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(200, 3000))
    k = int(rng.integers(1, 8))
    c = rng.uniform(-3, 3, size=(k, 2))
    pts = c[rng.integers(0, k, n)] + rng.normal(0, rng.uniform(0.05, 0.5), size=(n, 2))
    pts = np.concatenate([pts, rng.uniform(-4, 4, size=(n // 3, 2))])
    x, y = pts[:, 0].copy(), pts[:, 1].copy()
    eps = float(rng.uniform(0.03, 0.3))
    mp = int(rng.integers(1, 15))
    for mode in (0, 1):
        _check(dm, handle, x, y, eps, mp, mode, O.fit_sequential(x, y, eps, mp, mode))


@pytest.mark.parametrize("n,noise,dense", [(100_000, 0.2, 1.0), (300_000, 0.0, 8.0),
                                           (1_000_000, 0.2, 1.0)])
def test_blobs_vs_grid_oracle(dm, handle, n, noise, dense):
    x, y = gen_blobs(n, noise=noise, dense=dense, seed=n)
    for mode in (0, 1):
        _check(dm, handle, x, y, 2.55, 10, mode)


def test_full_size_config2(dm, handle):
    """BASELINE config 2 size (10^7 points, eps 2.55, minPoints 10): exact vs the closed-form
    grid oracle (C, pthreads), plus size-independent properties: idempotence and core flags
    invariant under a permutation of the visit order."""
    n = 10_000_000
    x, y = gen_blobs(n, noise=0.0, seed=1)
    cl, fl, k = _check(dm, handle, x, y, 2.55, 10, 0)
    cl2, fl2, k2 = dm.fit_arrays(x, y, 2.55, 10, 0, handle=handle)
    assert k2 == k and np.array_equal(cl, cl2) and np.array_equal(fl, fl2)
    perm = np.random.default_rng(7).permutation(n)
    clp, flp, kp = dm.fit_arrays(x[perm], y[perm], 2.55, 10, 0, handle=handle)
    assert kp == k
    np.testing.assert_array_equal(flp == 1, (fl == 1)[perm])


def test_device_entry_equals_host_entry(dm, handle):
    import torch

    from dbscan_amd import device as D

    x, y = gen_blobs(200_000, noise=0.1, seed=11)
    cl, fl, k = dm.fit_arrays(x, y, 2.55, 10, 0, handle=handle)
    tx = torch.from_numpy(x).cuda()
    ty = torch.from_numpy(y).cuda()
    dcl, dfl, dk = D.fit_tensors(tx, ty, 2.55, 10, 0, handle)
    assert dk == k
    np.testing.assert_array_equal(dcl.cpu().numpy(), cl)
    np.testing.assert_array_equal(dfl.cpu().numpy(), fl)


def test_device_generator_statistics(dm, handle):
    """G(n) on the device: k_bar ~ 49 at eps 2.55 (SURVEY §8d calibration), checked with the
    GPU fit's own stats on 10^6 points and against the oracle on the same data."""
    from dbscan_amd import device as D

    x, y = D.generate_blobs(1_000_000, 0.0, 1.0, 1, handle)
    hx, hy = x.cpu().numpy(), y.cpu().numpy()
    cl, fl, k = _check(dm, handle, hx, hy, 2.55, 10, 0)
    core_frac = float((fl == 1).mean())
    assert 0.75 < core_frac < 0.97, core_frac


def test_two_threads_two_handles(dm):
    x, y = gen_blobs(200_000, noise=0.2, seed=3)
    ref = O.fit_grid(x, y, 2.55, 10, 0)
    results = [None, None]

    def run(i):
        h = dm.Handle(0)
        results[i] = dm.fit_arrays(x, y, 2.55, 10, 0, handle=h)
        h.close()

    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for r in results:
        assert r[2] == ref[2]
        np.testing.assert_array_equal(r[0], ref[0])
        np.testing.assert_array_equal(r[1], ref[1])


def test_argument_errors(dm, handle):
    from dbscan_amd import _lib

    L = _lib.load()
    k = ctypes.c_int32(0)
    assert L.dbscan_fit_h(handle.ptr, None, None, -1, 0.3, 1, 0, None, None, ctypes.byref(k)) \
        == _lib.DBSCAN_EARG
    assert L.dbscan_fit_h(handle.ptr, None, None, 5, 0.3, 1, 0, None, None, ctypes.byref(k)) \
        == _lib.DBSCAN_EARG
    a = np.zeros(4)
    c = np.zeros(4, np.int32)
    f = np.zeros(4, np.uint8)
    p = lambda v: v.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert L.dbscan_fit_h(handle.ptr, p(a), p(a), 4, 0.3, 1, 7, p(c), p(f), ctypes.byref(k)) \
        == _lib.DBSCAN_EARG
    assert L.dbscan_fit_h(handle.ptr, p(a), p(a), 0, 0.3, 1, 0, p(c), p(f), ctypes.byref(k)) \
        == _lib.DBSCAN_OK and k.value == 0


@pytest.mark.parametrize("n", [100_000, 9_000_000])
def test_async_cluster_count_from_the_output_kernel(dm, handle, n):
    """dbscan_fit_device_async on the tiled pipeline: the cluster count lands in the caller's
    device word, written by the output kernel itself (FitArgs::n_clusters_dev; 100k points:
    the plain sort's permute_out_kernel, 9M: the bucketed sort's permute_out_bucket_kernel), and
    equals the synchronous fit's count and labels (the oracle digest of the full-size configs
    pins those)."""
    import torch
    from dbscan_amd import device as D

    x, y = D.generate_blobs(n, 0.1, 1.0, 11, handle)
    cl = torch.empty(n, dtype=torch.int32, device="cuda")
    fl = torch.empty(n, dtype=torch.uint8, device="cuda")
    nk = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    D.fit_tensors_async(x, y, 2.55, 10, 0, handle, cl, fl, nk)
    handle.sync()
    cl2 = torch.empty_like(cl)
    fl2 = torch.empty_like(fl)
    _, _, k2 = D.fit_tensors(x, y, 2.55, 10, 0, handle, cl2, fl2)
    torch.cuda.synchronize()
    assert int(nk.item()) == int(k2) > 0
    assert torch.equal(cl, cl2) and torch.equal(fl, fl2)
    assert int(cl.max().item()) == int(k2)


def test_async_fits_back_to_back(dm, handle):
    """dbscan_fit_device_async: several fits of different inputs (grid, all-pairs, no-finite)
    enqueued without any host synchronization, each output buffer equal to the oracle after
    one dbscan_sync; the cluster count lands in device memory."""
    import torch
    from dbscan_amd import device as D

    cases = []
    x, y = gen_blobs(20000, noise=0.2, seed=5)
    cases.append((x, y, 2.55 * 0.9, 10, 0))
    xs, ys = gen_blobs(3000, seed=6)
    cases.append((xs, ys, 1e200, 4, 1))  # eps*eps = +inf: all pairs
    cases.append((np.full(500, np.nan), np.zeros(500), 1.0, 1, 0))  # nothing in the grid
    cases.append((x, y, 2.55, 10, 1))
    outs = []
    for cx, cy, eps, mp, mode in cases:
        tx = torch.tensor(cx, dtype=torch.float64, device="cuda")
        ty = torch.tensor(cy, dtype=torch.float64, device="cuda")
        cl = torch.empty(cx.size, dtype=torch.int32, device="cuda")
        fl = torch.empty(cx.size, dtype=torch.uint8, device="cuda")
        nk = torch.full((1,), -1, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        D.fit_tensors_async(tx, ty, eps, mp, mode, handle, cl, fl, nk)
        outs.append((tx, ty, cl, fl, nk))
    handle.sync()
    torch.cuda.synchronize()
    for (cx, cy, eps, mp, mode), (_, _, cl, fl, nk) in zip(cases, outs):
        rc, rf, rk = O.fit_grid(cx, cy, eps, mp, mode)
        assert int(nk.item()) == rk
        np.testing.assert_array_equal(cl.cpu().numpy(), rc)
        np.testing.assert_array_equal(fl.cpu().numpy(), rf)
    st = handle.stats()  # the last fit's
    assert st["n"] == 20000 and st["finite"] == 20000
