// dbscan_local.hpp -- C++ host-side mirror of the reference's local-fit interface over the
// C-ABI of libdbscan_hip.so (dbscan_hip.h).  Header-only; callers need only g++ and
// -ldbscan_hip (no HIP headers).  Same names, argument meaning and error behaviour as
// (src/main/scala/org/apache/spark/mllib/clustering/dbscan/):
//   DBSCANPoint          DBSCANPoint.scala:21-32        x = vector(0), y = vector(1)
//   DBSCANLabeledPoint   DBSCANLabeledPoint.scala:24-47 flag, cluster (Unknown = 0), visited
//   LocalDBSCANNaive     LocalDBSCANNaive.scala:31-120  fit(points) in input order
//   LocalDBSCANArchery   LocalDBSCANArchery.scala:32-126
// A vector with fewer than two coordinates throws std::out_of_range (the reference's
// IndexOutOfBounds from vector(1)); HIP failures throw std::runtime_error with
// dbscan_last_error().  There is no CPU fallback.
#pragma once

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
}  // namespace detail

// new LocalDBSCANNaive(eps, minPoints).fit(points)   (LocalDBSCANNaive.scala:31,37)
class LocalDBSCANNaive {
   public:
    LocalDBSCANNaive(double eps, int minPoints, Handle* h = nullptr)
        : eps_(eps), minPoints_(minPoints), minDistanceSquared(eps * eps), h_(h) {}
    std::vector<DBSCANLabeledPoint> fit(const std::vector<DBSCANPoint>& points) const {
        return detail::fit(h_, eps_, minPoints_, DBSCAN_MODE_NAIVE, points);
    }

   private:
    double eps_;
    int minPoints_;

   public:
    const double minDistanceSquared;  // LocalDBSCANNaive.scala:33

   private:
    Handle* h_;
};

// new LocalDBSCANArchery(eps, minPoints).fit(points)  (LocalDBSCANArchery.scala:32,36);
// visit order = input order (archery's R-tree entry order is not reproducible).
class LocalDBSCANArchery {
   public:
    LocalDBSCANArchery(double eps, int minPoints, Handle* h = nullptr)
        : eps_(eps), minPoints_(minPoints), h_(h) {}
    std::vector<DBSCANLabeledPoint> fit(const std::vector<DBSCANPoint>& points) const {
        return detail::fit(h_, eps_, minPoints_, DBSCAN_MODE_ARCHERY, points);
    }

   private:
    double eps_;
    int minPoints_;
    Handle* h_;
};

}  // namespace dbscan
