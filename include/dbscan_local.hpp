// dbscan_local.hpp -- C++ host-side mirror of the reference's local-fit interface over the
// C-ABI of libdbscan_hip.so (dbscan_hip.h).  Header-only; callers need only g++ and
// -ldbscan_hip (no HIP headers).  Same names, argument meaning and error behaviour as
// (src/main/scala/org/apache/spark/mllib/clustering/dbscan/):
//   DBSCANPoint          DBSCANPoint.scala:21-32        x = vector(0), y = vector(1)
//   DBSCANLabeledPoint   DBSCANLabeledPoint.scala:24-47 flag, cluster (Unknown = 0), visited
//   LocalDBSCANNaive     LocalDBSCANNaive.scala:31-120  fit(points) in input order
//   LocalDBSCANArchery   LocalDBSCANArchery.scala:32-126 (float32 search box: mode 2)
//   DBSCANRectangle      DBSCANRectangle.scala:23-53
//   DBSCAN::train        DBSCAN.scala:40-48,72-283: labeledPoints (input order) + partitions
// A vector with fewer than two coordinates throws std::out_of_range (the reference's
// IndexOutOfBounds from vector(1)); HIP failures throw std::runtime_error with
// dbscan_last_error().  There is no CPU fallback.
#pragma once

#include <algorithm>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "dbscan_hip.h"

namespace dbscan {

constexpr int Unknown = 0;  // DBSCANLabeledPoint.scala:26

enum class Flag : unsigned char { Border = 0, Core = 1, Noise = 2, NotFlagged = 3 };

struct DBSCANPoint {
    std::vector<double> vector;
    explicit DBSCANPoint(std::vector<double> v) : vector(std::move(v)) {}
    double x() const { return vector.at(0); }
    double y() const { return vector.at(1); }
    double distanceSquared(const DBSCANPoint& other) const {  // DBSCANPoint.scala:26-30
        const double dx = other.x() - x();
        const double dy = other.y() - y();
        return (dx * dx) + (dy * dy);
    }
    bool operator==(const DBSCANPoint& o) const { return vector == o.vector; }
};

struct DBSCANLabeledPoint : DBSCANPoint {
    Flag flag = Flag::NotFlagged;
    int cluster = Unknown;
    bool visited = false;
    explicit DBSCANLabeledPoint(const DBSCANPoint& p) : DBSCANPoint(p.vector) {}
};

// Owns one dbscan_handle (one HIP stream, grow-only device buffers).
class Handle {
   public:
    explicit Handle(int device = 0) : h_(dbscan_create(device)) {
        if (!h_) throw std::runtime_error(std::string("dbscan_create: ") + dbscan_last_error());
    }
    ~Handle() { dbscan_destroy(h_); }
    Handle(const Handle&) = delete;
    Handle& operator=(const Handle&) = delete;
    dbscan_handle* get() const { return h_; }

   private:
    dbscan_handle* h_;
};

namespace detail {
inline std::vector<DBSCANLabeledPoint> fit(Handle* h, double eps, int minPoints, int mode,
                                           const std::vector<DBSCANPoint>& points) {
    const int64_t n = (int64_t)points.size();
    std::vector<double> xs((size_t)n), ys((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        xs[(size_t)i] = points[(size_t)i].x();
        ys[(size_t)i] = points[(size_t)i].y();
    }
    std::vector<int32_t> cl((size_t)n);
    std::vector<uint8_t> fl((size_t)n);
    int32_t k = 0;
    const int rc = h ? dbscan_fit_h(h->get(), xs.data(), ys.data(), n, eps, minPoints, mode,
                                    cl.data(), fl.data(), &k)
                     : dbscan_fit(xs.data(), ys.data(), n, eps, minPoints, mode, cl.data(),
                                  fl.data(), &k);
    if (rc != DBSCAN_OK) throw std::runtime_error(std::string("dbscan_fit: ") + dbscan_last_error());
    std::vector<DBSCANLabeledPoint> out;
    out.reserve((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        DBSCANLabeledPoint lp(points[(size_t)i]);
        lp.cluster = cl[(size_t)i];
        lp.flag = static_cast<Flag>(fl[(size_t)i]);
        lp.visited = true;
        out.push_back(std::move(lp));
    }
    return out;
}
// One fit per partition in one call (dbscan_fit_batch): result p equals fit(parts[p]).
inline std::vector<std::vector<DBSCANLabeledPoint>> fit_all(
    Handle* h, double eps, int minPoints, int mode,
    const std::vector<std::vector<DBSCANPoint>>& parts) {
    std::vector<int64_t> offs(1, 0);
    std::vector<double> xs, ys;
    for (const auto& pt : parts) {
        for (const auto& p : pt) {
            xs.push_back(p.x());
            ys.push_back(p.y());
        }
        offs.push_back((int64_t)xs.size());
    }
    const size_t n = xs.size();
    std::vector<int32_t> cl(n), k(parts.size());
    std::vector<uint8_t> fl(n);
    std::unique_ptr<Handle> own;
    if (!h) own.reset(h = new Handle(0));
    const int rc = dbscan_fit_batch(h->get(), xs.data(), ys.data(), offs.data(),
                                    (int32_t)parts.size(), eps, minPoints, mode, cl.data(),
                                    fl.data(), k.data());
    if (rc != DBSCAN_OK)
        throw std::runtime_error(std::string("dbscan_fit_batch: ") + dbscan_last_error());
    std::vector<std::vector<DBSCANLabeledPoint>> out(parts.size());
    for (size_t g = 0; g < parts.size(); ++g) {
        out[g].reserve(parts[g].size());
        for (size_t i = 0; i < parts[g].size(); ++i) {
            const size_t j = (size_t)offs[g] + i;
            DBSCANLabeledPoint lp(parts[g][i]);
            lp.cluster = cl[j];
            lp.flag = static_cast<Flag>(fl[j]);
            lp.visited = true;
            out[g].push_back(std::move(lp));
        }
    }
    return out;
}
}  // namespace detail

// new LocalDBSCANNaive(eps, minPoints).fit(points)   (LocalDBSCANNaive.scala:31,37)
class LocalDBSCANNaive {
   public:
    LocalDBSCANNaive(double eps, int minPoints, Handle* h = nullptr)
        : eps_(eps), minPoints_(minPoints), minDistanceSquared(eps * eps), h_(h) {}
    std::vector<DBSCANLabeledPoint> fit(const std::vector<DBSCANPoint>& points) const {
        return detail::fit(h_, eps_, minPoints_, DBSCAN_MODE_NAIVE, points);
    }
    // flatMapValues(fit) over many partitions at once (DBSCAN.scala:153-154, dbscan_fit_batch)
    std::vector<std::vector<DBSCANLabeledPoint>> fitAll(
        const std::vector<std::vector<DBSCANPoint>>& partitions) const {
        return detail::fit_all(h_, eps_, minPoints_, DBSCAN_MODE_NAIVE, partitions);
    }

   private:
    double eps_;
    int minPoints_;

   public:
    const double minDistanceSquared;  // LocalDBSCANNaive.scala:33

   private:
    Handle* h_;
};

// new LocalDBSCANArchery(eps, minPoints).fit(points)  (LocalDBSCANArchery.scala:32,36): the
// float32 R-tree search box + fp64 filter (:38-41,114-124); f32Box = false takes the exact fp64
// neighbour set.  Visit order = input order (archery's R-tree entry order is not reproducible).
class LocalDBSCANArchery {
   public:
    LocalDBSCANArchery(double eps, int minPoints, Handle* h = nullptr, bool f32Box = true)
        : eps_(eps), minPoints_(minPoints), h_(h), f32Box_(f32Box) {}
    std::vector<DBSCANLabeledPoint> fit(const std::vector<DBSCANPoint>& points) const {
        return detail::fit(h_, eps_, minPoints_,
                           f32Box_ ? DBSCAN_MODE_ARCHERY_F32BOX : DBSCAN_MODE_ARCHERY, points);
    }

   private:
    double eps_;
    int minPoints_;
    Handle* h_;
    bool f32Box_;
};

// DBSCANRectangle.scala:23 -- (x, y) lower-left, (x2, y2) upper-right
struct DBSCANRectangle {
    double x, y, x2, y2;
    bool operator==(const DBSCANRectangle& o) const {
        return x == o.x && y == o.y && x2 == o.x2 && y2 == o.y2;
    }
};

// DBSCAN.scala:116-137: every point into every partition whose eps-grown rectangle
// (shrink(-eps), borders included) contains it, each partition in input order -- the input of
// flatMapValues(fit) / LocalDBSCANNaive::fitAll (dbscan_duplicate).
inline std::vector<std::vector<DBSCANPoint>> duplicate(
    const std::vector<DBSCANPoint>& data,
    const std::vector<std::pair<int, DBSCANRectangle>>& partitions, double eps) {
    const int64_t n = (int64_t)data.size(), k = (int64_t)partitions.size();
    std::vector<double> xs((size_t)n), ys((size_t)n), rects((size_t)(4 * k));
    for (int64_t i = 0; i < n; ++i) {
        xs[(size_t)i] = data[(size_t)i].x();
        ys[(size_t)i] = data[(size_t)i].y();
    }
    for (int64_t p = 0; p < k; ++p) {
        const DBSCANRectangle& r = partitions[(size_t)p].second;
        rects[(size_t)(4 * p)] = r.x;
        rects[(size_t)(4 * p + 1)] = r.y;
        rects[(size_t)(4 * p + 2)] = r.x2;
        rects[(size_t)(4 * p + 3)] = r.y2;
    }
    std::vector<int64_t> offs((size_t)k + 1);
    const int64_t tot = dbscan_duplicate(xs.data(), ys.data(), n, rects.data(), k, eps,
                                         offs.data(), nullptr, 0);
    if (tot < 0) throw std::runtime_error(std::string("dbscan_duplicate: ") + dbscan_last_error());
    std::vector<int64_t> idx((size_t)std::max<int64_t>(tot, 1));
    if (dbscan_duplicate(xs.data(), ys.data(), n, rects.data(), k, eps, offs.data(), idx.data(),
                         (int64_t)idx.size()) != tot)
        throw std::runtime_error(std::string("dbscan_duplicate: ") + dbscan_last_error());
    std::vector<std::vector<DBSCANPoint>> out((size_t)k);
    for (int64_t p = 0; p < k; ++p)
        for (int64_t j = offs[(size_t)p]; j < offs[(size_t)p + 1]; ++j)
            out[(size_t)p].push_back(data[(size_t)idx[(size_t)j]]);
    return out;
}

// DBSCAN.train(data, eps, minPoints, maxPointsPerPartition) (DBSCAN.scala:40-48).
//   partitions()    the reference's (id, rectangle) list: EvenSplitPartitioner over the 2*eps
//                   cell histogram, in list order (DBSCAN.scala:91-104, 283)
//   labeledPoints() every input point once, in input order, from dbscan_train_node: x-slabs
//                   over the visible GPUs with eps halos and an exact merge, equal to ONE
//                   LocalDBSCANNaive fit of all points.  (The reference's own merge can drop or
//                   duplicate points and report halo cores as Border; cluster
//                   ids here are the input-order Naive numbering, equal to the reference's up
//                   to permutation.)
//   nShards = 0: one slab per visible GPU.
class DBSCAN {
   public:
    static DBSCAN train(const std::vector<DBSCANPoint>& data, double eps, int minPoints,
                        int maxPointsPerPartition, int nShards = 0, Handle* h = nullptr) {
        DBSCAN m(eps, minPoints, maxPointsPerPartition);
        const int64_t n = (int64_t)data.size();
        std::vector<double> xs((size_t)n), ys((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            xs[(size_t)i] = data[(size_t)i].x();
            ys[(size_t)i] = data[(size_t)i].y();
        }
        std::vector<int32_t> cl((size_t)n);
        std::vector<uint8_t> fl((size_t)n);
        int64_t k = 0;
        if (dbscan_train_node(xs.data(), ys.data(), n, eps, minPoints, DBSCAN_MODE_NAIVE, nShards,
                              cl.data(), fl.data(), &k) != DBSCAN_OK)
            throw std::runtime_error(std::string("dbscan_train_node: ") + dbscan_last_error());
        m.labeled_.reserve((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            DBSCANLabeledPoint lp(data[(size_t)i]);
            lp.cluster = cl[(size_t)i];
            lp.flag = static_cast<Flag>(fl[(size_t)i]);
            lp.visited = true;
            m.labeled_.push_back(std::move(lp));
        }
        m.nClusters_ = k;
        std::unique_ptr<Handle> own;
        if (!h) {
            own.reset(new Handle(0));
            h = own.get();
        }
        std::vector<double> rects;
        std::vector<int64_t> counts;
        int64_t cap = 0, np = 0;
        do {  // the return value is the full partition count: grow and call again if needed
            cap = np > cap ? np : (cap ? cap : 256);
            rects.assign((size_t)cap * 4, 0.0);
            counts.assign((size_t)cap, 0);
            np = dbscan_partition(h->get(), xs.data(), ys.data(), n, eps, maxPointsPerPartition,
                                  rects.data(), counts.data(), cap);
            if (np < 0)
                throw std::runtime_error(std::string("dbscan_partition: ") + dbscan_last_error());
        } while (np > cap);
        for (int64_t i = 0; i < np; ++i)
            m.partitions_.push_back({(int)i, DBSCANRectangle{rects[(size_t)(4 * i)],
                                                             rects[(size_t)(4 * i + 1)],
                                                             rects[(size_t)(4 * i + 2)],
                                                             rects[(size_t)(4 * i + 3)]}});
        return m;
    }
    const std::vector<DBSCANLabeledPoint>& labeledPoints() const { return labeled_; }
    const std::vector<std::pair<int, DBSCANRectangle>>& partitions() const { return partitions_; }
    int64_t numClusters() const { return nClusters_; }
    double minimumRectangleSize() const { return 2 * eps; }  // DBSCAN.scala:289
    DBSCANLabeledPoint predict(const std::vector<double>&) const {  // DBSCAN.scala:300-302
        throw std::logic_error("DBSCAN.predict is not implemented (as in the reference)");
    }
    const double eps;
    const int minPoints;
    const int maxPointsPerPartition;

   private:
    DBSCAN(double e, int mp, int mpp) : eps(e), minPoints(mp), maxPointsPerPartition(mpp) {}
    std::vector<DBSCANLabeledPoint> labeled_;
    std::vector<std::pair<int, DBSCANRectangle>> partitions_;
    int64_t nClusters_ = 0;
};

}  // namespace dbscan
