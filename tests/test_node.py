"""Multi-rank node path (slab sharding + exact merge) on CPU with gloo.

The slabs are fitted by the oracle's CPU restatement of the slab semantics (test double for
the HIP slab fit); everything else -- zones, records, collectives, global min-label merge,
cluster numbering -- is the product code in dbscan_amd/node.py.  The bar: the union of the
ranks' owned labels equals ONE fit of the whole data set (oracle), bit for bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import oracle as O
from conftest import ROOT, gen_blobs

WORKER = os.path.join(ROOT, "tests", "node_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(tmp_path, x, y, world, eps, min_points, mode, use_gpu=False, timeout=300,
              chunks=False, env_extra=None):
    data = tmp_path / "data.npz"
    np.savez(data, x=x, y=y)
    port = _free_port()
    env = dict(os.environ)
    env["NODE_WORKER_CHUNKS"] = "1" if chunks else "0"
    env.update(env_extra or {})
    env.setdefault("OMP_NUM_THREADS", "2")
    procs = [subprocess.Popen([sys.executable, WORKER, str(r), str(world), str(port), str(data),
                               str(tmp_path), repr(float(eps)), str(min_points), str(mode),
                               "1" if use_gpu else "0"], env=env)
             for r in range(world)]
    for p in procs:
        assert p.wait(timeout=timeout) == 0
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    n = x.size
    cl = np.full(n, -7, np.int64)
    fl = np.full(n, 9, np.int64)
    seen = np.zeros(n, np.int64)
    for pt in parts:
        cl[pt["gid"]] = pt["cluster"]
        fl[pt["gid"]] = pt["flag"]
        np.add.at(seen, pt["gid"], 1)
    ks = {int(v) for pt in parts for v in pt["k"]}
    return cl, fl, seen, ks, parts


def _data(n, seed, noise=0.15, bad=0):
    x, y = gen_blobs(n, noise=noise, seed=seed)
    if bad:
        rng = np.random.default_rng(seed)
        idx = rng.choice(n, bad, replace=False)
        x[idx[: bad // 2]] = np.nan
        y[idx[bad // 2:]] = np.inf
    return x, y


@pytest.mark.parametrize("world,mode", [(2, 0), (3, 0), (2, 1), (4, 0)])
def test_node_merge_equals_single_fit(tmp_path, world, mode):
    n = 40_000
    x, y = _data(n, seed=world * 10 + mode, bad=20)
    eps = 60.0 * np.sqrt(n / 1e6)  # ~ the bench's k_bar at this scale
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, world, eps, 10, mode)
    assert np.all(seen == 1), "every point owned by exactly one rank"
    rc, rf, rk = O.fit_grid(x, y, eps, 10, mode)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}
    # the slabs really are shards: each holds well under the whole set
    assert max(int(pt["n_slab"][0]) for pt in parts) < 0.8 * n


def test_node_single_rank_equals_single_fit(tmp_path):
    x, y = _data(20_000, seed=5)
    cl, fl, seen, ks, _ = run_ranks(tmp_path, x, y, 1, 25.0, 8, 0)
    rc, rf, rk = O.fit_grid(x, y, 25.0, 8, 0)
    np.testing.assert_array_equal(cl, rc)
    np.testing.assert_array_equal(fl, rf)


@pytest.mark.parametrize("chunks", [False, True], ids=["global", "chunks"])
def test_node_forced_collectives_one_rank(tmp_path, chunks):
    """Comm.force: the collectives run at one rank too (the GPU suite's RCCL check uses it)."""
    n = 20_000
    x, y = _data(n, seed=5)
    eps = 60.0 * np.sqrt(n / 1e6)
    cl, fl, seen, ks, _ = run_ranks(tmp_path, x, y, 1, eps, 10, 0, chunks=chunks,
                                    env_extra={"NODE_WORKER_FORCE_COLLECTIVES": "1"})
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, eps, 10, 0)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}


def test_node_cluster_spanning_every_slab(tmp_path):
    """A long horizontal band crosses every cut: the merge must chain local components across
    all ranks (diameter > 2 in the record graph)."""
    rng = np.random.default_rng(3)
    t = rng.uniform(0, 1000, 30_000)
    x = t.copy()
    y = rng.normal(0, 0.4, t.size)
    x = np.concatenate([x, rng.uniform(0, 1000, 3000)])
    y = np.concatenate([y, rng.uniform(-50, 50, 3000)])
    perm = rng.permutation(x.size)
    x, y = x[perm], y[perm]
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, 4, 0.5, 5, 0)
    rc, rf, rk = O.fit_grid(x, y, 0.5, 5, 0)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert len(parts[0]["cuts"]) == 3


def test_zone_margins_cover_the_predicate():
    """zones(): zone-0 points' neighbours lie in zones 0/1, zone-1 points' neighbours in 0/1/2;
    shared masks of adjacent ranks agree point for point."""
    import dbscan_amd.node as node

    rng = np.random.default_rng(0)
    eps = 0.3
    cut = 1.0
    # points straddling the cut at distances eps +- a few ulps
    base = np.array([cut, cut - eps, cut + eps, np.nextafter(cut - eps, -9),
                     np.nextafter(cut + eps, 9), cut - 2 * eps, cut + 2 * eps])
    x = torch.from_numpy(np.concatenate([base, rng.uniform(0, 2, 5000)]))
    z0, s0 = node.zones(x, 0, [cut], eps)
    z1, s1 = node.zones(x, 1, [cut], eps)
    own0, own1 = z0 == 0, z1 == 0
    assert torch.all(own0 ^ own1)
    xs = x.numpy()
    for r, z, own in ((0, z0, own0), (1, z1, own1)):
        zz = z.numpy()
        for i in np.flatnonzero(own.numpy())[:400]:
            nb = np.abs(xs - xs[i]) <= eps
            assert np.all(zz[nb] <= 1)
        for i in np.flatnonzero(zz == 1)[:400]:
            nb = np.abs(xs - xs[i]) <= eps
            assert np.all(zz[nb] <= 2)
    # a point is shared iff it is in zone 0/1 of both ranks
    both = ((z0 <= 1) & (z1 <= 1))
    assert torch.equal(s0 & (z0 <= 1), both & (z0 <= 1))
    assert torch.equal(s1 & (z1 <= 1), both & (z1 <= 1))


def test_merge_double_components():
    """The numpy restatement of the merge kernels (test double) on a known record graph:
    roots are the smallest gid of each component; untouched entries stay -1; reset restores."""
    from node_worker import OracleSlabOps

    ops = OracleSlabOps()
    a = torch.tensor([10, 11, 12, 30, 31, 40], dtype=torch.int64)
    b = torch.tensor([11, 12, 13, 31, 5, -1], dtype=torch.int64)
    par = torch.full((64,), -1, dtype=torch.int32)
    ops.merge(a, b, par)
    assert par[[10, 11, 12, 13]].tolist() == [10] * 4
    assert par[[30, 31, 5]].tolist() == [5] * 3
    assert par[40] == -1 and par[0] == -1
    ops.merge_reset(a, b, par)
    assert bool((par == -1).all())


@pytest.mark.parametrize("world,mode,bad", [(2, 0, 0), (3, 1, 12), (4, 0, 0)])
def test_node_chunks_all_to_all_equals_single_fit(tmp_path, world, mode, bad):
    """Host-to-slab path (NodeJob.from_chunk + chunk_labels): each rank starts from its chunk of
    the input only; one all_to_all routes points to their slabs, one routes the labels back to
    the chunk owners.  The chunks' labels, concatenated, equal one fit of the whole set."""
    n = 30_000
    x, y = _data(n, seed=world * 3 + mode, bad=bad)
    eps = 60.0 * np.sqrt(n / 1e6)
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, world, eps, 10, mode, chunks=True)
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, eps, 10, mode)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}
    assert max(int(pt["n_slab"][0]) for pt in parts) < 0.8 * n


@pytest.mark.parametrize("chunks", [False, True], ids=["global", "chunks"])
def test_node_world8_rehearsal(tmp_path, chunks):
    """The N = 8 shape of the bench's node path on CPU (gloo, 8 ranks, 7 cuts): blobs + noise
    plus a horizontal band that crosses every slab, so the merge chains local components through
    all 8 ranks; both the global-input and the host-chunk (two all_to_all) forms.  The union of
    the ranks' owned labels equals one oracle fit of the whole set."""
    rng = np.random.default_rng(88)
    n = 48_000
    x, y = _data(n, seed=88, bad=16)
    s = np.sqrt(n / 1e6)
    t = rng.uniform(-1100 * s, 1100 * s, 12_000)
    x = np.concatenate([x, t])
    y = np.concatenate([y, rng.normal(0, 0.3, t.size)])
    p = rng.permutation(x.size)
    x, y = x[p], y[p]
    eps = 60.0 * s
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, 8, eps, 10, 0, chunks=chunks,
                                        timeout=600)
    assert np.all(seen == 1)
    rc, rf, rk = O.fit_grid(x, y, eps, 10, 0)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}
    assert len(parts[0]["cuts"]) == 7
    band = np.abs(y) < 1.0
    assert len(np.unique(rc[band & (rf == 1)])) == 1  # the band is one cluster across the slabs
