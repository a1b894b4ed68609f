"""bench.py's workload selection (CPU): N = 1 times BASELINE config 2, N > 1 config 3
weak-scaled (exactly config 3, G(10^8, 20% noise, seed 2), at N = 8), and the N > 1 node job
on config-3-shaped data shards into slabs under gloo."""
import numpy as np

import bench
import oracle as O
from conftest import gen_blobs
from test_node import run_ranks


def test_config2_at_one_gpu():
    a = bench.workload_defaults(bench.parse([]), 1)
    assert (a.points_per_gpu, a.noise, a.seed, a.dense, a.eps, a.min_points) == \
        (10_000_000, 0.0, 1, 1.0, 2.55, 10)


def test_config3_at_eight_gpus():
    a = bench.workload_defaults(bench.parse(["--gpus", "8"]), 8)
    assert a.points_per_gpu * 8 == 100_000_000
    assert (a.noise, a.seed, a.dense, a.eps, a.min_points) == (0.2, 2, 1.0, 2.55, 10)
    a = bench.workload_defaults(bench.parse(["--gpus", "2"]), 2)
    assert (a.points_per_gpu, a.noise, a.seed) == (12_500_000, 0.2, 2)


def test_explicit_flags_win():
    a = bench.workload_defaults(bench.parse(["--noise", "0.1", "--seed", "7"]), 4)
    assert (a.noise, a.seed, a.points_per_gpu) == (0.1, 7, 12_500_000)


def test_config3_shaped_job_shards_into_slabs(tmp_path):
    """The N > 1 step on G(n, 20% noise, seed 2) (config 3's shape, scaled down) over two gloo
    ranks: every point owned once, each slab well under the whole set, labels equal one fit."""
    n = 60_000
    x, y = gen_blobs(n, noise=0.2, seed=2)
    cl, fl, seen, ks, parts = run_ranks(tmp_path, x, y, 2, 2.55, 10, 0)
    assert np.all(seen == 1)
    assert max(int(pt["n_slab"][0]) for pt in parts) < 0.7 * n
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, 0)
    np.testing.assert_array_equal(fl, rf)
    np.testing.assert_array_equal(cl, rc)
    assert ks == {rk}
