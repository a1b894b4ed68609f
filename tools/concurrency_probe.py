"""Many executor threads, a handle each, fitting partition-sized inputs at once through the
LDS forms (band fits of 9000-65536 points: up to 64 workgroups of one CU each, grid barriers
in one plain launch): wall time per fit, how many fits were recalled (a barrier that gave up, or
a staging overflow, re-run through the tiled pipeline), and every label checked against the
oracle.  Spark local[N] with N > 4 (the process has 4 hardware queues on the box):
    python3 tools/concurrency_probe.py [threads ...]      (default 4 8 12 16)"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "dbscan-on-spark_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import dbscan_amd  # noqa: E402
import oracle as O  # noqa: E402  (the checker)


def make_sets(rng, sizes):
    out = []
    for m in sizes:
        k = int(rng.integers(2, 10))
        c = rng.uniform(-3, 3, size=(k, 2))
        nb = m - m // 5
        pts = c[rng.integers(0, k, nb)] + rng.normal(0, rng.uniform(0.05, 0.4), size=(nb, 2))
        pts = np.concatenate([pts, rng.uniform(-4, 4, size=(m - nb, 2))])
        pts = pts[rng.permutation(m)] * np.sqrt(m / 8192.0)
        out.append((pts[:, 0].copy(), pts[:, 1].copy()))
    return out


def main():
    nts = [int(a) for a in sys.argv[1:]] or [4, 8, 12, 16]
    rng = np.random.default_rng(4242)
    sets = make_sets(rng, [9000, 20000, 40000, 65536, 12000, 30000, 50000, 65536])
    refs = [O.fit_grid(x, y, 0.12, 6, 0) for x, y in sets]
    per = 6  # fits per thread
    for nt in nts:
        hs = [dbscan_amd.Handle(0) for _ in range(nt)]
        for hh in hs:  # workspaces allocated before the clock
            dbscan_amd.fit_arrays(sets[0][0], sets[0][1], 0.12, 6, 0, handle=hh)
        rec0 = sum(hh.spread_fallbacks() for hh in hs)
        bad = []
        lat = []
        lock = threading.Lock()

        def worker(t):
            for r in range(per):
                k = (t + r) % len(sets)
                x, y = sets[k]
                t0 = time.perf_counter()
                cl, fl, nk = dbscan_amd.fit_arrays(x, y, 0.12, 6, 0, handle=hs[t])
                dt = time.perf_counter() - t0
                rc, rf, rk = refs[k]
                ok = nk == rk and np.array_equal(cl, rc) and np.array_equal(fl, rf)
                with lock:
                    lat.append(dt)
                    if not ok:
                        bad.append((t, r, k))

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(nt)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        wall = time.perf_counter() - t0
        recalls = sum(hh.spread_fallbacks() for hh in hs) - rec0
        for hh in hs:
            hh.close()
        lat = np.array(lat) * 1e6
        print(f"threads {nt:2d}: {nt * per} fits in {wall * 1e3:8.1f} ms ({wall / (nt * per) * 1e6:7.1f}"
              f" us per fit), per-call latency p50 {np.median(lat):8.1f} max {lat.max():10.1f} us, "
              f"recalled {recalls}, label mismatches {len(bad)}", flush=True)
        if bad:
            print("  mismatches (thread, rep, set):", bad[:10], flush=True)


if __name__ == "__main__":
    main()
