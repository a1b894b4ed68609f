"""Shared pytest setup: the `gpu` marker and import paths.

`-m "not gpu"` tests run here on CPU (oracle vs golden vectors, host logic, C-ABI exports,
multi-rank gloo paths); `-m gpu` tests are the parity tests proper and need a MI355X.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dbscan-on-spark_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

EPS_03F = float(np.float32(0.3))  # Scala `eps = 0.3F` widened to Double (SURVEY key fact 4b)


if os.environ.get("DBSCAN_SEGV_TRACE") == "1":  # debug runs: native backtraces after finalize
    import atexit
    import ctypes

    _segv = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools",
                                     "segv_trace.so"))
    atexit.register(_segv.segv_trace_install)  # (re-installed last: after torch's handlers)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def labeled_data():
    import oracle as O

    return O.load_labeled_csv(os.path.join(GOLDEN, "labeled_data.csv"))


@pytest.fixture(scope="session")
def labeled_expected():
    a = np.loadtxt(os.path.join(GOLDEN, "labeled_expected.csv"), delimiter=",", dtype=np.int64)
    return dict(flag_naive=a[:, 1], cluster_naive=a[:, 2], flag_archery=a[:, 3],
                cluster_archery=a[:, 4])


def load_edge_cases():
    with open(os.path.join(GOLDEN, "edge_cases.json")) as f:
        recs = json.load(f)
    for r in recs:
        r["x"] = np.array([float.fromhex(v) for v in r["x"]], np.float64)
        r["y"] = np.array([float.fromhex(v) for v in r["y"]], np.float64)
        r["eps"] = float.fromhex(r["eps"])
        r["cluster"] = np.array(r["cluster"], np.int32)
        r["flag"] = np.array(r["flag"], np.uint8)
    return recs


def gen_blobs(n, noise=0.0, dense=1.0, seed=1, k=32):
    """Host copy of the SURVEY §8d generator G(n, noise, dense, seed) (numpy RNG; used for
    parity inputs -- the bench uses the device generator, whose values differ bitwise)."""
    rng = np.random.default_rng(seed)
    s = np.sqrt(n / 1e6)
    n_noise = int(round(n * noise))
    n_blob = n - n_noise
    centres = rng.uniform(-1000 * s, 1000 * s, size=(k, 2))
    sig = rng.uniform(20 * s, 60 * s, size=k)
    sig[:4] /= dense
    lab = rng.integers(0, k, size=n_blob)
    pts = centres[lab] + rng.normal(size=(n_blob, 2)) * sig[lab, None]
    nz = rng.uniform(-1100 * s, 1100 * s, size=(n_noise, 2))
    allp = np.concatenate([pts, nz])
    perm = rng.permutation(n)
    allp = allp[perm]
    return allp[:, 0].copy(), allp[:, 1].copy()


def neg_eps_set(seed, n=600, scale=1e6, eps=-0.02):
    """Archery float32-box stress set: points near float32 rounding midpoints far from the
    origin with a NEGATIVE eps.  The fp64 predicate treats eps like |eps|, but archery's float32
    box (x-eps .. x+eps, LocalDBSCANArchery.scala:118-124) is inverted: empty, or one float
    wide where both edges round to the same float.  So the neighbour relation is directed and
    many pairs hold one way only (the case the one-way-pair resolution exists for)."""
    rng = np.random.default_rng(seed)
    u = float(np.spacing(np.float32(scale)))
    k = int(rng.integers(3, 9))
    cx = scale + (rng.integers(0, 50, k) + 0.5) * u
    cy = -scale + (rng.integers(0, 50, k) + 0.5) * u
    lab = rng.integers(0, k, n)
    x = cx[lab] + rng.normal(0, abs(eps) * 0.7, n)
    y = cy[lab] + rng.normal(0, abs(eps) * 0.7, n)
    return x, y


def one_way_pairs(x, y, eps):
    """Number of ordered pairs (p, o) with o in N(p) but p not in N(o) under archery's float32
    box + fp64 predicate (numpy, O(n^2): small sets only)."""
    f = np.float32
    dx = x[None, :] - x[:, None]
    dy = y[None, :] - y[:, None]
    w = dx * dx + dy * dy <= eps * eps
    x1, x2 = (x - eps).astype(f)[:, None], (x + eps).astype(f)[:, None]
    y1, y2 = (y - eps).astype(f)[:, None], (y + eps).astype(f)[:, None]
    fx, fy = x.astype(f)[None, :], y.astype(f)[None, :]
    fwd = w & (x1 <= fx) & (fx <= x2) & (y1 <= fy) & (fy <= y2)
    return int((fwd != fwd.T).sum())
