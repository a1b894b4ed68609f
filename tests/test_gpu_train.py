"""DBSCAN.train(data, eps, minPoints, maxPointsPerPartition) -- the reference's whole-job API
(DBSCAN.scala:40-48) -- in its Python and C++ mirrors, on the GPU.  Mirrors DBSCANSuite."dbscan"
(DBSCANSuite.scala:30-60): the csv with eps = 0.3F, minPoints = 10, maxPointsPerPartition = 250;
labels equal the csv's up to permutation (the suite itself maps ids through `corresponding`),
and the partitions equal the reference's EvenSplitPartitioner list."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from conftest import EPS_03F, ROOT, gen_blobs

pytestmark = pytest.mark.gpu


def test_dbscan_suite_labeled_csv(labeled_data):
    import dbscan_amd

    x, y, lab = labeled_data
    vectors = [[a, b, c] for a, b, c in zip(x, y, lab)]  # Vectors.dense(line.split(','))
    model = dbscan_amd.DBSCAN.train(vectors, eps=EPS_03F, minPoints=10, maxPointsPerPartition=250)
    pts = model.labeledPoints
    assert len(pts) == len(vectors) and [p.vector for p in pts] == [tuple(v) for v in vectors]
    pairs = {(p.cluster, int(v[2])) for p, v in zip(pts, vectors)}
    assert len(pairs) == 4 and len({a for a, _ in pairs}) == 4 and (0, 0) in pairs  # bijection
    assert sum(p.flag == dbscan_amd.Flag.Core for p in pts) == 677
    assert sum(p.flag == dbscan_amd.Flag.Noise for p in pts) == 18
    rects, counts = O.ref_partition(x, y, EPS_03F, 250)
    assert [i for i, _ in model.partitions] == [0, 1, 2, 3]
    assert [tuple(r) for _, r in model.partitions] == [tuple(map(float, r)) for r in rects]
    assert model.minimumRectangleSize == 2 * EPS_03F
    with pytest.raises(NotImplementedError):
        model.predict([0.0, 0.0])


@pytest.mark.parametrize("shards", [0, 3])
def test_train_numpy_blobs_equals_one_fit(shards):
    import dbscan_amd

    x, y = gen_blobs(300_000, noise=0.2, seed=31)
    model = dbscan_amd.DBSCAN.train(np.stack([x, y], 1), 2.55, 10, 8192, n_shards=shards)
    rc, rf, rk = O.fit_grid(x, y, 2.55, 10, 0)
    assert model.n_clusters == rk
    np.testing.assert_array_equal(model.cluster, rc)
    np.testing.assert_array_equal(model.flag, rf)
    rects, _ = O.ref_partition(x, y, 2.55, 8192)
    np.testing.assert_array_equal(np.array([tuple(r) for _, r in model.partitions]), rects)
    with pytest.raises(IndexError):
        dbscan_amd.DBSCAN.train(np.zeros((5, 1)), 1.0, 2, 10)


def test_cpp_train_mirror(tmp_path, labeled_data):
    """include/dbscan_local.hpp's dbscan::DBSCAN::train (g++ only, linked to libdbscan_hip.so)
    on the csv: labels equal the Python mirror's, partitions the reference's."""
    from dbscan_amd import _lib

    x, y, lab = labeled_data
    data = tmp_path / "pts.txt"
    np.savetxt(data, np.stack([x, y], 1), fmt="%.17g")
    src = tmp_path / "train.cpp"
    src.write_text(r'''
#include <cstdio>
#include <fstream>
#include "dbscan_local.hpp"
int main(int argc, char** argv) {
    std::ifstream in(argv[1]);
    std::vector<dbscan::DBSCANPoint> pts;
    double a, b;
    while (in >> a >> b) pts.emplace_back(std::vector<double>{a, b});
    auto m = dbscan::DBSCAN::train(pts, (double)0.3f, 10, 250);
    for (const auto& p : m.labeledPoints()) std::printf("%d %d\n", p.cluster, (int)p.flag);
    for (const auto& pr : m.partitions())
        std::printf("P %d %.17g %.17g %.17g %.17g\n", pr.first, pr.second.x, pr.second.y,
                    pr.second.x2, pr.second.y2);
    // the seam's own pattern: duplicate into eps-grown partitions, one batch of local fits
    auto parts = dbscan::duplicate(pts, m.partitions(), (double)0.3f);
    auto res = dbscan::LocalDBSCANNaive((double)0.3f, 10).fitAll(parts);
    for (size_t g = 0; g < res.size(); ++g)
        for (const auto& p : res[g]) std::printf("Q %zu %d %d\n", g, p.cluster, (int)p.flag);
    return 0;
}
''')
    exe = tmp_path / "train"
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(exe), "-L", libdir, "-ldbscan_hip", f"-Wl,-rpath,{libdir}"],
                   check=True)
    out = subprocess.run([str(exe), str(data)], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    lab_lines = [l.split() for l in out if l and not l[0] in "PQ"]
    cl = np.array([int(a) for a, _ in lab_lines])
    fl = np.array([int(b) for _, b in lab_lines])
    rc, rf, _ = O.fit_sequential(x, y, EPS_03F, 10, 0)
    np.testing.assert_array_equal(cl, rc)
    np.testing.assert_array_equal(fl, rf)
    parts = [tuple(map(float, l.split()[2:])) for l in out if l.startswith("P")]
    rects, _ = O.ref_partition(x, y, EPS_03F, 250)
    assert parts == [tuple(map(float, r)) for r in rects]
    import dbscan_amd

    offs, idx = dbscan_amd.duplicate(x, y, rects, EPS_03F)
    q = np.array([[int(v) for v in l.split()[1:]] for l in out if l.startswith("Q")])
    assert q.shape[0] == offs[-1] == 1097
    for g in range(len(rects)):
        a, b = offs[g], offs[g + 1]
        rc, rf, _ = O.fit_sequential(x[idx[a:b]], y[idx[a:b]], EPS_03F, 10, 0)
        assert (q[a:b, 0] == g).all()
        np.testing.assert_array_equal(q[a:b, 1], rc)
        np.testing.assert_array_equal(q[a:b, 2], rf)


def test_dbscan_sample_file_flow(tmp_path):
    """DBSCANSample.scala:17-35 end to end from files: sc.textFile(labeled_data.csv) parsed by
    dbscan_csv_read -> DBSCAN.train(eps = 0.1, minPoints = 3, maxPointsPerPartition = 400) on the
    GPU -> model.labeledPoints written as "${p.x},${p.y},${p.cluster}" by dbscan_csv_write.
    Expected text: the csv's own coordinate fields (they are exactly what JDK 7/8's
    Double.toString prints for those doubles) and the oracle's restated DBSCAN.train
    (ref_train: the reference's partitioner, halos, per-partition LocalDBSCANNaive and merge)
    cluster ids, mapped through the one bijection between the two numberings (the reference
    numbers global clusters in its collect order).  saveAsTextFile's line order follows the
    Spark partitions, so the lines are compared as a multiset.  Every point appears once in
    both (the reference's known defects drop no point and split no cluster on this input)."""
    import dbscan_amd
    from dbscan_amd import textio

    src = os.path.join(ROOT, "tests", "golden", "labeled_data.csv")
    x, y = textio.read_csv(src)
    fields = [l.split(",") for l in open(src).read().splitlines() if l]
    np.testing.assert_array_equal(x, np.array([float(f[0]) for f in fields]))
    np.testing.assert_array_equal(y, np.array([float(f[1]) for f in fields]))
    model = dbscan_amd.DBSCAN.train(np.stack([x, y], 1), eps=0.1, minPoints=3,
                                    maxPointsPerPartition=400)
    out = tmp_path / "labeled_data_result.txt"
    textio.write_csv(out, x, y, model.cluster)
    got = out.read_text().splitlines()
    ref = O.ref_train(x, y, 0.1, 3, 400)
    assert (ref["records"] == 1).all() and len(ref["rects"]) == 2
    pairs = set(zip(ref["cluster"].tolist(), model.cluster.tolist()))
    assert len(pairs) == len(set(ref["cluster"].tolist())) == len(set(model.cluster.tolist()))
    to_ours = dict(pairs)
    assert to_ours.get(0, 0) == 0  # Noise stays 0
    want = [f"{f[0]},{f[1]},{to_ours[c]}" for f, c in zip(fields, ref["cluster"].tolist())]
    assert sorted(got) == sorted(want)
    assert model.n_clusters == ref["n_clusters"] == 26
