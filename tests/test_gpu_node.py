"""Node path with the real HIP slab kernels: 2, 3 and 8 ranks on the one GPU of the test box, gloo
for the exchange (RCCL needs one GPU per rank; the collectives are the same calls).  The
union of the ranks' owned labels must equal one fit of the whole data set, bit for bit."""
import ctypes

import numpy as np
import pytest

import oracle as O
from conftest import gen_blobs
from test_node import run_ranks

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,mode,n", [(2, 0, 400_000), (3, 1, 200_000), (2, 0, 2_000_000)])
def test_gpu_node_equals_single_fit(tmp_path, world, mode, n):
    x, y = gen_blobs(n, noise=0.2, seed=n + world)
    eps = 2.55 * np.sqrt(n / 1e6) / np.sqrt(n / 1e6)  # bench calibration (k_bar ~ 49 at any n)
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, world, eps, 10, mode, use_gpu=True,
                                        timeout=600)
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, eps, 10, mode)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("chunks", [False, True], ids=["global", "chunks"])
def test_gpu_node_world8_config3_shape(tmp_path, chunks):
    """The N = 8 rehearsal of the bench's node path with the HIP slab kernels: 8 ranks (gloo)
    sharing the one test GPU, 7 cuts, 2*10^6 points of config 3's shape (20% noise), both the
    global-input and the host-chunk form; bit-exact against one oracle fit."""
    n = 2_000_000
    x, y = gen_blobs(n, noise=0.2, seed=2)
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, 8, 2.55, 10, 0, use_gpu=True,
                                        timeout=800, chunks=chunks)
    assert np.all(seen == 1)
    assert len(parts[0]["cuts"]) == 7
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, 0)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("chunks", [False, True], ids=["global", "chunks"])
def test_gpu_node_bucketed_slabs(tmp_path, chunks):
    """Slabs of >= 2^23 points take the bucketed sort (zones and the shared points' slots ride
    in the place records, labels at the places): 2 ranks over 1.8*10^7 points of config 3's
    shape, the global-input and host-chunk forms, bit-exact against one oracle fit."""
    n = 18_000_000
    x, y = gen_blobs(n, noise=0.2, seed=3)
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, 2, 2.55, 10, 0, use_gpu=True,
                                        timeout=800, chunks=chunks)
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, 0)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}


@pytest.mark.parametrize("world,mode", [(2, 0), (3, 1)])
def test_gpu_node_chunks_equals_single_fit(tmp_path, world, mode):
    """Host-to-slab path with the HIP slab kernels: each rank starts from its chunk of the input,
    all_to_all routes points to slabs and labels back (gloo between ranks on the one GPU)."""
    n = 500_000
    x, y = gen_blobs(n, noise=0.2, seed=n + world + 5)
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, world, 2.55, 10, mode, use_gpu=True,
                                        timeout=600, chunks=True)
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, mode)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}


@pytest.mark.parametrize("env", [{"DBSCAN_NODE_COMM_STREAM": "1"},
                                 {"NODE_WORKER_SHARE_STREAM": "0"}],
                         ids=["comm_stream", "own_stream"])
def test_gpu_node_stream_variants(tmp_path, env):
    """The node step's optional stream arrangements: the roots' gather and sort on a stream of
    their own (DBSCAN_NODE_COMM_STREAM=1), and the handle on its own stream ordered by events
    (share_stream=False): both bit-exact against one fit."""
    n = 300_000
    x, y = gen_blobs(n, noise=0.2, seed=17)
    cl, fl, seen, ks, _ = run_ranks(tmp_path, x, y, 2, 2.55, 10, 0, use_gpu=True, timeout=600,
                                    env_extra=env)
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, 0)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}


def test_set_stream_bind_and_restore():
    """dbscan_set_stream: a fit on a caller's torch stream, back on the handle's own stream
    (own = 1), both equal to the oracle; destroying a handle bound to the null stream."""
    import torch

    import dbscan_amd
    from dbscan_amd import _lib
    from dbscan_amd import device as D

    L = _lib.load()
    x, y = gen_blobs(200_000, noise=0.1, seed=23)
    ref = O.fit_grid(x, y, 2.55, 10, 0)
    tx, ty = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    h = dbscan_amd.Handle(0)
    s = torch.cuda.Stream()
    _lib.check(L.dbscan_set_stream(h.ptr, ctypes.c_void_p(s.cuda_stream), 0))
    assert h.stream == s.cuda_stream
    with torch.cuda.stream(s):
        cl, fl, k = D.fit_tensors(tx, ty, 2.55, 10, 0, h)
    s.synchronize()
    assert k == ref[2]
    np.testing.assert_array_equal(cl.cpu().numpy(), ref[0])
    _lib.check(L.dbscan_set_stream(h.ptr, None, 1))  # back to the handle's own stream
    assert h.stream not in (0, s.cuda_stream)
    cl2, fl2, k2 = D.fit_tensors(tx, ty, 2.55, 10, 0, h)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(cl2.cpu().numpy(), ref[0])
    np.testing.assert_array_equal(fl2.cpu().numpy(), ref[1])
    h2 = dbscan_amd.Handle(0)
    _lib.check(L.dbscan_set_stream(h2.ptr, None, 0))  # the null stream
    D.fit_tensors_async(tx, ty, 2.55, 10, 0, h2, torch.empty_like(cl), torch.empty_like(fl),
                        None)
    h2.close()  # waits for the fit on the null stream before freeing its buffers
    h.close()


@pytest.mark.parametrize("chunks", [False, True], ids=["global", "chunks"])
def test_gpu_node_rccl_world1(tmp_path, chunks):
    """The node step over RCCL: one rank on the test GPU with the collectives forced (all_gather,
    all_to_all_single on device tensors, the dtypes the exchange uses), so the nccl calls the
    driver's multi-GPU runs make are exercised here; bit-exact against one fit."""
    n = 300_000
    x, y = gen_blobs(n, noise=0.2, seed=19)
    env = {"NODE_WORKER_BACKEND": "nccl", "NODE_WORKER_FORCE_COLLECTIVES": "1"}
    cl, fl, seen, ks, _ = run_ranks(tmp_path, x, y, 1, 2.55, 10, 0, use_gpu=True, timeout=300,
                                    chunks=chunks, env_extra=env)
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, 0)
    np.testing.assert_array_equal(cl, rc)
    np.testing.assert_array_equal(fl, rf)
    assert ks == {rk}


@pytest.mark.parametrize("chunks", [False, True], ids=["global", "chunks"])
def test_gpu_node_single_rank(tmp_path, chunks):
    """One rank, no forced collectives: the one-rank shortcuts (from_chunk's local form,
    chunk_labels returning the slab's labels, run() as the direct fit) over two steps: the
    labels of both steps and both cluster counts equal one oracle fit."""
    x, y = gen_blobs(300_000, noise=0.1, seed=77)
    cl, fl, seen, ks, _ = run_ranks(tmp_path, x, y, 1, 2.55, 10, 0, use_gpu=True, chunks=chunks)
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, 0)
    np.testing.assert_array_equal(cl, rc)
    np.testing.assert_array_equal(fl, rf)
    assert ks == {rk}


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_slab_select_kernel_equals_torch_zones(world):
    """dbscan_slab_select_device (HipSlabOps.select, from_global's slab on the GPU) against the
    torch restatement of node.py zones() + the ordered selection: the same x, y, zone, gid and
    shared slab indices for every rank, NaN / inf points, points on the cuts and within ulps of
    the halo margins, coinciding cuts (an empty slab)."""
    import torch

    import dbscan_amd
    from dbscan_amd import node

    rng = np.random.default_rng(world + 40)
    n, eps = 300_000, 2.55
    x, y = gen_blobs(n, noise=0.2, seed=world + 40)
    xs = np.sort(x[np.isfinite(x)])
    cuts = [float(np.floor(xs[k * xs.size // world] / (2 * eps)) * 2 * eps) for k in range(1, world)]
    if world == 8:
        cuts[3] = cuts[2]
    R = node.reach(eps)
    special = []
    for c in cuts:
        m1, m2 = node.margin1(c, R), node.margin2(c, R)
        for v in (c, c - m1, c + m1, c - m2, c + m2):
            special += [v, np.nextafter(v, -np.inf), np.nextafter(v, np.inf)]
    k = len(special)
    x[:k] = special
    x[k:k + 5] = [np.nan, np.inf, -np.inf, np.nan, 0.0]
    y[k + 5] = np.nan
    p = rng.permutation(n)
    x, y = x[p], y[p]
    h = dbscan_amd.Handle(0)
    ops = node.HipSlabOps(h)
    try:
        tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        for rank in range(world):
            sx, sy, sz, sg, sh = ops.select(tx, ty, cuts, rank, eps)
            if cuts:
                z, shm = node.zones(tx, rank, cuts, eps)
            else:
                z = torch.zeros(n, dtype=torch.uint8, device="cuda")
                shm = torch.zeros(n, dtype=torch.bool, device="cuda")
            idx = torch.nonzero(z != node.OUT).flatten()
            assert torch.equal(sg, idx)
            assert torch.equal(sz, z[idx])
            assert torch.equal(sx.view(torch.int64), tx[idx].view(torch.int64))
            assert torch.equal(sy.view(torch.int64), ty[idx].view(torch.int64))
            assert torch.equal(sh, torch.nonzero(shm[idx]).flatten())
    finally:
        ops.close()
        h.close()


def test_gpu_merge_kernels_vs_double():
    """dbscan_merge_union_device / dbscan_slab_merge_roots_device / dbscan_merge_reset_device
    against the numpy restatement (tests/node_worker.py) on random record graphs with long
    chains, repeated nodes and skipped records."""
    import torch

    import dbscan_amd
    from dbscan_amd import node
    from node_worker import OracleSlabOps

    dbscan_amd.load()
    h = dbscan_amd.Handle(0)
    ops = node.HipSlabOps(h)
    ref = OracleSlabOps()
    rng = np.random.default_rng(3)
    n_total = 200_000
    par = torch.full((n_total,), -1, dtype=torch.int32, device="cuda")
    for trial in range(3):
        m = 50_000
        a = rng.integers(0, n_total, m)
        b = np.minimum(a, rng.integers(0, n_total, m))  # b <= a, like a local root
        b[rng.random(m) < 0.1] = -1
        ta, tb = torch.tensor(a, device="cuda"), torch.tensor(b, device="cuda")
        ops.merge(ta, tb, par)
        rpar = torch.full((n_total,), -1, dtype=torch.int32)
        ref.merge(torch.tensor(a), torch.tensor(b), rpar)
        np.testing.assert_array_equal(par.cpu().numpy(), rpar.numpy())
        # local roots of a synthetic slab: every 7th point (if core) roots its 7-run
        n = 30_000
        gid = torch.arange(n, dtype=torch.int64, device="cuda") * 5
        core = torch.tensor((rng.random(n) < 0.7).astype(np.uint8), device="cuda")
        ar = torch.arange(n, device="cuda")
        root = torch.where(core != 0, torch.where(ar % 7 == 0, ar, ar // 7 * 7),
                           torch.full_like(ar, -1)).to(torch.int32)
        zone = torch.tensor(rng.integers(0, 2, n).astype(np.uint8), device="cuda")
        gs = torch.zeros(n, dtype=torch.int64, device="cuda")
        own = ops.merge_roots(zone, gid, root, par, gs)
        rgs = torch.zeros(n, dtype=torch.int64)
        rown = ref.merge_roots(zone.cpu(), gid.cpu(), root.cpu(), rpar, rgs)
        rlr = ref.lroots.numpy()
        assert own.cpu().tolist() == rown.tolist()  # increasing gid order
        np.testing.assert_array_equal(gs.cpu().numpy()[rlr], rgs.numpy()[rlr])
        ops.merge_reset(ta, tb, par)
        assert bool((par == -1).all())
    h.close()


@pytest.mark.parametrize("shards,mode,noise,bad", [(2, 0, 0.2, 0), (3, 1, 0.1, 40), (4, 0, 0.0, 0),
                                                    (7, 0, 0.3, 10)])
def test_train_node_single_process(shards, mode, noise, bad):
    """dbscan_train_node (one process, n_shards slabs on the visible GPUs -- here all on one):
    the global labels equal one fit of the whole set, bit for bit, NaN/inf points included."""
    import dbscan_amd

    n = 300_000
    x, y = gen_blobs(n, noise=noise, seed=shards * 7 + mode)
    if bad:
        rng = np.random.default_rng(bad)
        idx = rng.choice(n, bad, replace=False)
        x[idx[: bad // 2]] = np.nan
        y[idx[bad // 2:]] = -np.inf
    cl, fl, k = dbscan_amd.train_node(x, y, 2.55, 10, mode, shards)
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, mode)
    assert k == rk
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)


def test_train_node_unshardable_and_labeled_csv(labeled_data):
    """eps*eps = +inf (all pairs) falls back to one fit; the reference's csv through the node
    entry equals the local fit (DBSCANSuite, maxPointsPerPartition small -> several slabs)."""
    import dbscan_amd
    from conftest import EPS_03F

    x, y, _ = labeled_data
    cl, fl, k = dbscan_amd.train_node(x, y, EPS_03F, 10, 0, 4)
    rc, rf, rk = O.fit_sequential(x, y, EPS_03F, 10, 0)
    assert k == rk == 3
    np.testing.assert_array_equal(cl, rc)
    np.testing.assert_array_equal(fl, rf)
    xs, ys = gen_blobs(2000, seed=9)
    cl, fl, k = dbscan_amd.train_node(xs, ys, 1e200, 5, 1, 3)
    rc, rf, rk = O.fit_grid(xs, ys, 1e200, 5, 1)
    assert k == rk
    np.testing.assert_array_equal(cl, rc)
    np.testing.assert_array_equal(fl, rf)


def test_lean_slab_fit_matches_full():
    """dbscan_slab_fit_shared_device_async (the node step's form) against the full slab fit on
    the same slab: identical core/root at the shared points, root[r] == r at exactly the local
    roots and -1 elsewhere."""
    import torch

    import dbscan_amd
    from dbscan_amd import node

    dbscan_amd.load()
    x, y = gen_blobs(600_000, noise=0.2, seed=5)
    tx, ty = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    cuts = node.make_cuts(tx, 3, 2.55)
    h = dbscan_amd.Handle(0)
    ops = node.HipSlabOps(h)
    for rank in range(3):
        z, sh = node.zones(tx, rank, cuts, 2.55)
        idx = torch.nonzero(z != node.OUT).flatten()
        sx, sy, sz = tx[idx].contiguous(), ty[idx].contiguous(), z[idx].contiguous()
        shared = torch.nonzero(sh[idx]).flatten()
        core_f, root_f = [t.clone() for t in ops.fit(sx, sy, sz, 2.55, 10)]
        core_l, root_l = [t.clone() for t in ops.fit(sx, sy, sz, 2.55, 10, shared=shared)]
        torch.cuda.synchronize()
        assert shared.numel() > 0
        assert torch.equal(core_l[shared], core_f[shared])
        assert torch.equal(root_l[shared], root_f[shared])
        ar = torch.arange(root_f.numel(), device="cuda", dtype=torch.int32)
        is_root = root_f == ar
        assert torch.equal(root_l == ar, is_root)
        rest = torch.ones_like(is_root)
        rest[shared] = False
        rest &= ~is_root
        assert bool((root_l[rest] == -1).all())
    h.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_two_part_slab_label_matches_one_part(mode):
    """dbscan_slab_roots_prepare_device + dbscan_slab_label_finish_device_async (the node step's
    form) against dbscan_slab_merge_roots_device + dbscan_slab_label_device_async on the same
    slab fits (zones 0/1/2 of a 3-way cut): identical owned roots, labels and flags; zone 1/2
    entries untouched.  A fit in between invalidates the prepared state."""
    import torch

    import dbscan_amd
    from dbscan_amd import _lib, node

    dbscan_amd.load()
    x, y = gen_blobs(500_000, noise=0.2, seed=11)
    tx, ty = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    cuts = node.make_cuts(tx, 3, 2.55)
    h = dbscan_amd.Handle(0)
    ops = node.HipSlabOps(h)
    for rank in range(3):
        z, sh = node.zones(tx, rank, cuts, 2.55)
        idx = torch.nonzero(z != node.OUT).flatten()
        sx, sy, sz = tx[idx].contiguous(), ty[idx].contiguous(), z[idx].contiguous()
        gid = idx.to(torch.int64).contiguous()
        shared = torch.nonzero(sh[idx]).flatten()
        par = torch.full((x.size,), -1, dtype=torch.int32, device="cuda")
        out = []
        for two_part in (False, True):
            _, root = ops.fit(sx, sy, sz, 2.55, 10, shared=shared)
            gs = torch.zeros(sx.numel(), dtype=torch.int64, device="cuda")
            own = ops.merge_roots(sz, gid, root, par, gs, mode=mode if two_part else None)
            own = own.clone()
            cl, fl = ops.label(sz, gid, gs, torch.sort(own)[0], mode)
            torch.cuda.synchronize()
            out.append((own.cpu(), cl.cpu(), fl.cpu()))
        assert torch.equal(out[0][0], out[1][0])
        assert torch.equal(out[0][1], out[1][1])
        assert torch.equal(out[0][2], out[1][2])
        outside = (sz != 0).cpu()
        assert bool((out[1][2][outside] == 3).all()) and bool((out[1][1][outside] == 0).all())
        assert bool((out[1][2][~outside] <= 2).all())
    # finish without a prepare since the last fit: an argument error, not stale labels
    ops.fit(sx, sy, sz, 2.55, 10, shared=shared)
    cl = torch.zeros(sx.numel(), dtype=torch.int32, device="cuda")
    fl = torch.zeros(sx.numel(), dtype=torch.uint8, device="cuda")
    roots = torch.zeros(1, dtype=torch.int64, device="cuda")
    rc = _lib.load().dbscan_slab_label_finish_device_async(
        h.ptr, node._p(sz), node._p(gs), node._p(roots), 1, node._p(cl), node._p(fl))
    assert rc == _lib.DBSCAN_EARG
    h.close()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_route_kernel_equals_torch_zones(world):
    """dbscan_route_slabs_device (HipSlabOps.route, the HIP routing of NodeJob.from_chunk) against
    the torch restatement of node.py zones() (_route_torch): the same rows (x bits, y bits,
    gid * 8 + zone * 2 + shared) in the same order and the same per-rank counts, on a chunk with
    NaN / inf coordinates, points exactly on the cuts and within ulps of the halo margins, and
    cuts that coincide (empty slabs)."""
    import torch

    import dbscan_amd
    from dbscan_amd import node

    rng = np.random.default_rng(world)
    n, start, eps = 300_000, 12_345, 2.55
    x, y = gen_blobs(n, noise=0.2, seed=world)
    xs = np.sort(x[np.isfinite(x)])
    cuts = [float(np.floor(xs[k * xs.size // world] / (2 * eps)) * 2 * eps) for k in range(1, world)]
    if world == 8:
        cuts[3] = cuts[2]  # an empty slab
    R = node.reach(eps)
    special = []
    for c in cuts:
        m1, m2 = node.margin1(c, R), node.margin2(c, R)
        for v in (c, c - m1, c + m1, c - m2, c + m2):
            special += [v, np.nextafter(v, -np.inf), np.nextafter(v, np.inf)]
    k = len(special)
    x[:k] = special
    x[k:k + 5] = [np.nan, np.inf, -np.inf, np.nan, 0.0]
    y[k + 5] = np.nan
    x = x[rng.permutation(n)]
    h = dbscan_amd.Handle(0)
    ops = node.HipSlabOps(h)
    try:
        tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        rows, counts = ops.route(tx, ty, start, cuts, eps)
        trows, tcounts = node.NodeJob._route_torch(tx, ty, start, cuts, eps, world)
        assert counts == tcounts
        assert torch.equal(rows, trows)
    finally:
        ops.close()
        h.close()
