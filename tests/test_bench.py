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


def test_gpus_n_without_launcher_starts_n_ranks(monkeypatch, capfd):
    """`python bench.py --gpus N` with no WORLD_SIZE (the driver's BENCH form) must not time one
    GPU: it starts N ranks through torch.distributed.run as a child.  The probe ranks (gloo, no
    GPU) report the process group they joined; device count mocked to N."""
    import json

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "visible_devices", lambda: 3)
    argv = ["--gpus", "3", "--backend", "gloo", "--launch-probe"]
    rc = bench.launch_ranks(bench.parse(argv), argv)
    assert rc == 0
    lines = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and [r["rank"] for r in d["devices"]] == [0, 1, 2]


def test_gpus_n_refused_without_n_devices(monkeypatch, capfd):
    """Fewer visible GPUs than --gpus: exit 2 before anything runs, never an n_gpus=1 line."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "visible_devices", lambda: 1)
    rc = bench.launch_ranks(bench.parse(["--gpus", "8"]), ["--gpus", "8"])
    assert rc == 2
    out = capfd.readouterr()
    assert "n_gpus" not in out.out and "refusing" in out.err


def test_gpus_n_cli_exits_nonzero_without_gpus():
    """The CLI form end to end in this GPU-less container: non-zero, no JSON line."""
    import os
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")}
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "{" not in r.stdout


def test_launcher_not_used_under_torchrun(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.launch_ranks(bench.parse(["--gpus", "2"]), ["--gpus", "2"]) is None
    monkeypatch.delenv("WORLD_SIZE")
    assert bench.launch_ranks(bench.parse([]), []) is None
