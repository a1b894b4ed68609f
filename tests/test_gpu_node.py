"""Node path with the real HIP slab kernels: 2-3 ranks on the one GPU of the test box, gloo
for the exchange (RCCL needs one GPU per rank; the collectives are the same calls).  The
union of the ranks' owned labels must equal one fit of the whole data set, bit for bit."""
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


def test_gpu_node_single_rank(tmp_path):
    x, y = gen_blobs(300_000, noise=0.1, seed=77)
    cl, fl, seen, ks, _ = run_ranks(tmp_path, x, y, 1, 2.55, 10, 0, use_gpu=True)
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, 0)
    np.testing.assert_array_equal(cl, rc)
    np.testing.assert_array_equal(fl, rf)
