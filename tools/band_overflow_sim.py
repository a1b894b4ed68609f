"""Host simulation of the band form's staging capacity (small.hip band_fit_kernel: band_make_grid,
the row-cost ranges, the staged row span of every workgroup) over the seam's partitions of G(10^7):
which partitions overflow a workgroup's staging (kStError 3 -> the tiled recall), and how many
would with the grid's rows taken along the other axis.  CPU only (numpy restatement of the
device generator, the oracle's EvenSplitPartitioner, the library's host-side duplication).
    python tools/band_overflow_sim.py [n]"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "dbscan-on-spark_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from band_model import band_overflows  # noqa: E402


def _mix(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def gen_blobs_device(n, noise, dense, seed):
    """capi.hip gen_blobs_kernel restated (values within an ulp of the device's)."""
    with np.errstate(over="ignore"):
        def sm(st):  # splitmix64 on scalars (python ints)
            st = (st + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
            z = st
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
            return st, z ^ (z >> 31)

        def u01(v):
            return ((v >> 11) + 1.0) * 2.0 ** -53

        s = np.sqrt(n / 1e6)
        st = (seed * 0x2545F4914F6CDD1D + 0x1234567) & 0xFFFFFFFFFFFFFFFF
        cx, cy, sg = [], [], []
        for b in range(32):
            st, v = sm(st)
            cx.append((2.0 * u01(v) - 1.0) * 1000.0 * s)
            st, v = sm(st)
            cy.append((2.0 * u01(v) - 1.0) * 1000.0 * s)
            st, v = sm(st)
            sig = (20.0 + 40.0 * u01(v)) * s
            if b < 4 and dense > 0:
                sig /= dense
            sg.append(sig)
        cx, cy, sg = np.array(cx), np.array(cy), np.array(sg)
        i = np.arange(n, dtype=np.uint64)
        state = np.uint64(seed) ^ (i * np.uint64(0xD1B54A32D192ED03))
        g = np.uint64(0x9E3779B97F4A7C15)
        outs = []
        for _ in range(5):
            state = state + g
            outs.append(_mix(state))
        ud = lambda v: ((v >> np.uint64(11)).astype(np.float64) + 1.0) * 2.0 ** -53  # noqa: E731
        u0, r1, u2, u3 = ud(outs[1]), outs[2], ud(outs[3]), ud(outs[4])
        b = (r1 % np.uint64(32)).astype(np.int64)
        rad = np.sqrt(-2.0 * np.log(u2))
        th = 6.283185307179586 * u3
        x = cx[b] + sg[b] * rad * np.cos(th)
        y = cy[b] + sg[b] * rad * np.sin(th)
        nz = u0 <= noise
        half = 1100.0 * s
        x[nz] = (2.0 * u2[nz] - 1.0) * half
        y[nz] = (2.0 * u3[nz] - 1.0) * half
        return x, y


def main():
    import dbscan_amd
    import oracle as O

    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
    eps, maxp = 2.55, 8192
    x, y = gen_blobs_device(n, 0.0, 1.0, 1)
    rects, _ = O.ref_partition(x, y, eps, maxp)
    offs, idx = dbscan_amd.duplicate(x, y, rects, eps)
    px, py = x[idx], y[idx]
    sizes = np.diff(offs)
    res = {k: [] for k in ("shipped", "gscale", "transposed+gscale")}
    for p in range(len(sizes)):
        a, b = offs[p], offs[p + 1]
        if b - a < 400 or b - a > 65536:
            continue
        X, Y = px[a:b], py[a:b]
        o, nx, ny = band_overflows(X, Y, eps, False)
        og, nxg, nyg = band_overflows(X, Y, eps, True)
        # rows along the axis that gives the shorter rows (fewer cells per row)
        ot = band_overflows(Y, X, eps, True)[0] if nxg > nyg else og
        for k, v in (("shipped", o), ("gscale", og), ("transposed+gscale", ot)):
            if v:
                res[k].append((p, int(b - a), nx, ny))
    print(f"{len(sizes)} partitions, {int(sizes.sum())} points with halos")
    for k, v in res.items():
        print(f"band overflows, {k}: {len(v)}: {v}")


if __name__ == "__main__":
    main()
