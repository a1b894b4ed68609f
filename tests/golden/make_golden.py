"""Generate the committed golden fixtures under tests/golden/ (run from the repo root):

    python tests/golden/make_golden.py

* labeled_data.csv -- copied verbatim from the reference's
  src/test/resources/labeled_data.csv (Apache-2.0 test data: x,y,label).
* labeled_expected.csv -- per-point (flag, cluster) of the oracle's literal sequential
  restatement in Naive and Archery-rule modes for eps = (double)0.3F, minPoints = 10 (the
  reference's LocalDBSCANArcherySuite / DBSCANSuite parameters).  tests/test_oracle.py pins
  these against the reference's own label column (up to the permutation SURVEY.md §4 found).
* edge_cases.json -- small synthetic inputs stressing the predicate boundary
  (d2 = eps2 +- ulps), duplicates, NaN/inf, eps <= 0, tiny/huge scales, minPoints <= 1,
  and visit-order effects, with the sequential oracle's outputs.  Floats are stored as
  float.hex() strings so they round-trip bit-exactly.
* jvm_printed_doubles.txt -- every decimal number printed in the reference's source comments
  (debug output of the author's JVM run, e.g. DBSCAN.scala:73-101's vectors and
  DBSCANRectangle corners, EvenSplitPartitioner.scala:186-197), one per line with its file:line:
  java.lang.Double.toString outputs of the reference's runtime, so format_double must print
  each parsed value back as the same string.  Needs /root/reference (generation only).
* config5_oracle_digest.json -- NOT made here: needs an MI355X (the device generator's 10^9
  points) and ~3 minutes of the oracle on the box's cores.  Written by
  `DBSCAN_TEST_FULL_SCALE=1 pytest tests/test_gpu_configs.py -k config5_full_size_vs_oracle`
  (gpurun_out/config5_oracle_digest.json: sha256 of oracle_fit_grid's cluster and flag arrays,
  cluster and core counts) and copied here.
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

EPS_03F = float(np.float32(0.3))  # Scala `eps = 0.3F` widened to Double


def _hex(a):
    return [float(v).hex() for v in a]


def boundary_ulp(rng, n_pairs, eps):
    """Pairs at distance eps along random directions, perturbed by -3..3 ulps per coord, so
    d2 lands within a few ulps of eps2 on both sides of the predicate."""
    xs, ys = [], []
    for _ in range(n_pairs):
        bx, by = rng.uniform(-5, 5), rng.uniform(-5, 5)
        th = rng.uniform(0, 2 * math.pi)
        ox, oy = bx + eps * math.cos(th), by + eps * math.sin(th)
        for _ in range(int(rng.integers(-3, 4))):
            ox = math.nextafter(ox, math.inf)
        for _ in range(int(rng.integers(-3, 4))):
            oy = math.nextafter(oy, -math.inf)
        xs += [bx, ox]
        ys += [by, oy]
    # axis-aligned exact-eps pairs: dx = eps exactly representable offsets
    for k in range(n_pairs // 4):
        bx = float(k) * 0.75
        xs += [bx, bx + eps, math.nextafter(bx + eps, math.inf), math.nextafter(bx + eps, -math.inf)]
        ys += [3.0, 3.0, 3.0, 3.0]
    return np.array(xs), np.array(ys)


def blobs(rng, n, k, spread, sigma):
    c = rng.uniform(-spread, spread, size=(k, 2))
    lab = rng.integers(0, k, size=n)
    p = c[lab] + rng.normal(0, sigma, size=(n, 2))
    return p[:, 0].copy(), p[:, 1].copy()


def cases():
    rng = np.random.default_rng(20240611)
    out = []

    def add(name, x, y, eps, mps, modes=(0, 1)):
        for m in modes:
            out.append(dict(name=f"{name}/mode{m}", x=np.asarray(x, np.float64),
                            y=np.asarray(y, np.float64), eps=float(eps), min_points=int(mps),
                            mode=m))

    x, y = boundary_ulp(rng, 300, EPS_03F)
    add("boundary_ulp_mp2", x, y, EPS_03F, 2)
    add("boundary_ulp_mp3", x, y, EPS_03F, 3)
    x, y = boundary_ulp(rng, 200, 1.0)
    add("boundary_ulp_eps1", x, y, 1.0, 2)
    # duplicates
    base = rng.uniform(-1, 1, size=(60, 2))
    rep = base[rng.integers(0, 60, size=600)]
    add("duplicates", rep[:, 0], rep[:, 1], 0.05, 12)
    add("duplicates_eps0", rep[:, 0], rep[:, 1], 0.0, 10)
    add("duplicates_epsneg", rep[:, 0], rep[:, 1], -0.05, 12)
    # non-finite coordinates mixed into blobs
    x, y = blobs(rng, 800, 4, 3.0, 0.3)
    bad = rng.choice(800, size=40, replace=False)
    specials = [math.nan, math.inf, -math.inf]
    for t, i in enumerate(bad):
        if t % 2:
            x[i] = specials[t % 3]
        else:
            y[i] = specials[(t + 1) % 3]
    add("nonfinite_mp5", x, y, 0.25, 5)
    add("nonfinite_mp1", x, y, 0.25, 1)
    add("nonfinite_mp0", x, y, 0.25, 0)
    add("nonfinite_mpneg", x, y, 0.25, -3)
    # eps = +inf (eps2 = inf: every finite pair is a neighbour) and NaN
    add("eps_inf", x[:200], y[:200], math.inf, 150)
    add("eps_huge", x[:200], y[:200], 1e200, 150)
    add("eps_nan", x[:200], y[:200], math.nan, 1)
    # underflow: eps = 0 with sub-1e-162 offsets (squares underflow to 0 -> neighbours)
    ux = np.concatenate([np.full(20, 1e-300), 1e-300 + np.arange(20) * 1e-170, [0.0, 1e-150]])
    uy = np.zeros_like(ux)
    add("eps0_underflow", ux, uy, 0.0, 5)
    # huge coordinates and a far outlier (grid capping path)
    hx, hy = blobs(rng, 400, 3, 1e6, 2.0)
    hx = np.concatenate([hx, [1e300, -1e300, 5e307]])
    hy = np.concatenate([hy, [0.0, 1e300, -5e307]])
    add("far_outliers", hx, hy, 3.0, 6)
    add("tiny_scale", hx[:400] * 1e-290, hy[:400] * 1e-290, 3e-290, 6)
    # visit-order effects: random blobs with noise, random permutations
    for s in range(4):
        x, y = blobs(rng, 1200, 6, 4.0, 0.35)
        nx = rng.uniform(-5, 5, 300)
        ny = rng.uniform(-5, 5, 300)
        x = np.concatenate([x, nx])
        y = np.concatenate([y, ny])
        perm = rng.permutation(x.size)
        add(f"blobs_noise_{s}", x[perm], y[perm], 0.22, 8)
    # one long chain (union depth) and a dense clump
    t = np.arange(1500) * 0.099
    add("chain", t, np.sin(t) * 0.01, 0.1, 2)
    cx, cy = blobs(rng, 1500, 1, 0.0, 0.02)
    add("dense_clump", cx, cy, 0.01, 40)
    add("empty", [], [], 0.3, 10)
    add("single", [0.5], [0.5], 0.3, 1)
    add("single_noise", [0.5], [0.5], 0.3, 2)
    return out


def jvm_printed_doubles():
    import re

    src = "/root/reference/src/main/scala/org/apache/spark/mllib/clustering/dbscan"
    seen, out = set(), []
    for name in sorted(os.listdir(src)):
        with open(os.path.join(src, name)) as f:
            for ln, line in enumerate(f, 1):
                if "//" not in line or "licen" in line.lower():
                    continue
                for m in re.finditer(r"(?<![\w.])-?\d+\.\d+(?:E-?\d+)?", line.split("//", 1)[1]):
                    v = m.group(0)
                    if v not in seen:
                        seen.add(v)
                        out.append(f"{v} {name}:{ln}")
    with open(os.path.join(HERE, "jvm_printed_doubles.txt"), "w") as f:
        f.write("# Double.toString outputs printed in the reference's comments (value file:line)\n")
        f.write("\n".join(out) + "\n")
    print(f"wrote {len(out)} JVM-printed doubles")


def main():
    O.build()
    if os.path.isdir("/root/reference"):
        jvm_printed_doubles()
    # labeled_data expected outputs
    x, y, lab = O.load_labeled_csv(os.path.join(HERE, "labeled_data.csv"))
    cn, fn, _ = O.fit_sequential(x, y, EPS_03F, 10, O.NAIVE)
    ca, fa, _ = O.fit_sequential(x, y, EPS_03F, 10, O.ARCHERY)
    with open(os.path.join(HERE, "labeled_expected.csv"), "w") as f:
        f.write("# index,flag_naive,cluster_naive,flag_archery,cluster_archery "
                "(eps=(double)0.3F, minPoints=10; Flag: Border=0 Core=1 Noise=2)\n")
        for i in range(x.size):
            f.write(f"{i},{fn[i]},{cn[i]},{fa[i]},{ca[i]}\n")
    recs = []
    for c in cases():
        cl, fl, k = O.fit_sequential(c["x"], c["y"], c["eps"], c["min_points"], c["mode"])
        recs.append(dict(name=c["name"], eps=float(c["eps"]).hex(), min_points=c["min_points"],
                         mode=c["mode"], x=_hex(c["x"]), y=_hex(c["y"]),
                         cluster=cl.tolist(), flag=fl.tolist(), n_clusters=k))
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump(recs, f, separators=(",", ":"))
    print(f"wrote {len(recs)} edge cases")


if __name__ == "__main__":
    main()
