"""Large fits through the bucketed sort (csrc/primitives.hip bucket_sort: an MSD pass on the top
8 key bits into padded per-band segments, then LSD passes inside the segments), bit-exact
against the CPU oracle.

Fits of >= 2^23 points take this path (kBucketMinPoints); the BASELINE configs 2-5 (per-GPU
shares) run through it in tests/test_gpu_configs.py.  Here: sizes just over the threshold
with non-finite points (sentinel keys, which share the last band with real keys), both
LocalDBSCANNaive and LocalDBSCANArchery rules, archery's float32 box (its own output kernels),
an input with no finite point (no key bits: the MSD pass alone sorts), and idempotence."""
import numpy as np
import pytest

import oracle as O
from conftest import gen_blobs

pytestmark = pytest.mark.gpu

N = (1 << 23) + 4099


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


@pytest.fixture(scope="module")
def data():
    x, y = gen_blobs(N, noise=0.2, seed=31)
    x[::1009] = np.nan
    y[5::2003] = np.inf
    x[7::4001] = -np.inf
    return x, y


def _eq(got, ref, what):
    cl, fl, k = got
    rc, rf, rk = ref
    assert k == rk, f"{what}: {k} clusters, oracle {rk}"
    bad = np.flatnonzero((cl != rc) | (fl != rf))
    assert bad.size == 0, f"{what}: {bad.size} mismatches, first {bad[:10]}"


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", [0, 1])
def test_over_threshold_vs_oracle(dm, handle, data, mode):
    x, y = data
    got = dm.fit_arrays(x, y, 2.55, 10, mode, handle=handle)
    st = handle.stats()
    assert st["n"] == N and st["finite"] == N - int((~np.isfinite(x) | ~np.isfinite(y)).sum())
    _eq(got, O.fit_grid(x, y, 2.55, 10, mode), f"mode {mode}")
    again = dm.fit_arrays(x, y, 2.55, 10, mode, handle=handle)
    assert again[2] == got[2] and np.array_equal(again[0], got[0]) and \
        np.array_equal(again[1], got[1])


@pytest.mark.timeout(600)
def test_float32_box_equals_exact_archery(dm, handle, data):
    """Archery's float32 search box only widens the fp64 neighbourhood for eps >= 0 (DESIGN.md
    §1), so on these coordinates mode 2 equals mode 1 bit for bit; mode 2 labels through its
    own kernels (box_label) and the bucketed output gather."""
    x, y = data
    a = dm.fit_arrays(x, y, 2.55, 10, 1, handle=handle)
    b = dm.fit_arrays(x, y, 2.55, 10, 2, handle=handle)
    assert a[2] == b[2] and np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("mp", [0, 3])
def test_no_finite_point(dm, handle, mp):
    """No finite coordinate: nothing is binned (key width 0); every point is Noise, or its own
    one-point cluster when minPoints <= 0 (a NaN point has no neighbour, not even itself)."""
    x = np.full(N, np.nan)
    y = np.zeros(N)
    cl, fl, k = dm.fit_arrays(x, y, 2.55, mp, 0, handle=handle)
    if mp <= 0:
        assert k == N and (fl == 1).all() and np.array_equal(cl, np.arange(1, N + 1, dtype=np.int32))
    else:
        assert k == 0 and (fl == 2).all() and (cl == 0).all()


@pytest.mark.timeout(600)
def test_dense_band(dm, handle):
    """90% of the points in a narrow horizontal band: a few band segments hold most keys (the
    per-segment offsets over segments of thousands of tiles), the other segments few."""
    rng = np.random.default_rng(8)
    m = N
    x = rng.uniform(-4000, 4000, m)
    y = np.where(rng.random(m) < 0.9, rng.normal(0, 30.0, m), rng.uniform(-4000, 4000, m))
    _eq(dm.fit_arrays(x, y, 2.55, 10, 0, handle=handle), O.fit_grid(x, y, 2.55, 10, 0),
        "dense band")
