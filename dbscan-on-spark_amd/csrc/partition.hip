// partition.hip -- the reference's spatial partitioner with its data-parallel
// part on the GPU:
//   DBSCAN.scala:91-97      every point -> its minimum bounding rectangle (a 2*eps cell with
//                           lower corner corner(p) = (shiftIfNegative(p) / mrs).intValue * mrs,
//                           DBSCAN.scala:345-356), counted per cell     -> cell_range + cell_hist
//                           kernels: a dense histogram over the occupied cell-index window
//   EvenSplitPartitioner.scala:44-209  findPartitions over (cell, count): recursive best split
//                           (cost |count/2 - pointsIn(candidate)|, candidates every mrs from the
//                           box corner by repeated fp addition, Scala 2.10 NumericRange), until
//                           every partition holds <= maxPointsPerPartition or cannot be split
//                                                                    -> host, over a summed-area
//                           table, O(box width + height) per split with a two-pointer walk
// pointsInRectangle counts the cells CONTAINED in a rectangle (DBSCANRectangle.scala:28-30) with
// the reference's exact fp comparisons, so the split-line/cell-corner defect (a
// split line an ulp off a cell corner drops that cell's points) is reproduced, not repaired.
// Ties between equal-cost splits (split's reduceLeft over `splits.toSet`, :111-119, :161): the
// first minimum in the iteration order of a Scala 2.10 immutable Set -- candidate order (x
// splits, then y splits) for at most four candidates (Set1..Set4), else a HashTrieSet, which
// iterates by the improved hash of each DBSCANRectangle (split_rank below).  Two candidates
// whose 32-bit hashes collide would iterate in ListSet order: not modelled (never observed).
#include "../../include/dbscan_hip.h"
#include "internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace dbscan {
namespace {

// Scala Double.intValue: truncation toward zero, NaN -> 0, saturating to Int.
__host__ __device__ inline int64_t scala_int(double v) {
    if (v != v) return 0;
    if (v >= 2147483647.0) return 2147483647;
    if (v <= -2147483648.0) return -2147483648LL;
    return (int64_t)v;
}

// DBSCAN.scala:352-356 corner(p) as a cell index: corner = index * mrs.
__host__ __device__ inline int64_t corner_index(double p, double mrs) {
    const double s = p < 0 ? p - mrs : p;
    return scala_int(s / mrs);
}

__global__ __launch_bounds__(kBlock) void cell_range_kernel(const double* __restrict__ x,
                                                            const double* __restrict__ y,
                                                            int64_t n, double mrs,
                                                            int64_t* __restrict__ part) {
    __shared__ int64_t sm[kBlock / 64][4];
    int64_t a = INT64_MAX, b = INT64_MIN, c = INT64_MAX, d = INT64_MIN;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        const int64_t ci = corner_index(x[i], mrs), cj = corner_index(y[i], mrs);
        a = ci < a ? ci : a;
        b = ci > b ? ci : b;
        c = cj < c ? cj : c;
        d = cj > d ? cj : d;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t a2 = __shfl_xor(a, o, 64), b2 = __shfl_xor(b, o, 64);
        const int64_t c2 = __shfl_xor(c, o, 64), d2 = __shfl_xor(d, o, 64);
        a = a2 < a ? a2 : a;
        b = b2 > b ? b2 : b;
        c = c2 < c ? c2 : c;
        d = d2 > d ? d2 : d;
    }
    const int w = threadIdx.x >> 6;
    if (__lane_id() == 0) {
        sm[w][0] = a;
        sm[w][1] = b;
        sm[w][2] = c;
        sm[w][3] = d;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kBlock / 64; ++k) {
            a = sm[k][0] < a ? sm[k][0] : a;
            b = sm[k][1] > b ? sm[k][1] : b;
            c = sm[k][2] < c ? sm[k][2] : c;
            d = sm[k][3] > d ? sm[k][3] : d;
        }
        part[4 * blockIdx.x + 0] = a;
        part[4 * blockIdx.x + 1] = b;
        part[4 * blockIdx.x + 2] = c;
        part[4 * blockIdx.x + 3] = d;
    }
}

__global__ __launch_bounds__(kBlock) void cell_hist_kernel(const double* __restrict__ x,
                                                           const double* __restrict__ y,
                                                           int64_t n, double mrs, int64_t imin,
                                                           int64_t jmin, int64_t w,
                                                           uint32_t* __restrict__ hist) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int64_t ci = corner_index(x[i], mrs) - imin, cj = corner_index(y[i], mrs) - jmin;
    atomicAdd(&hist[cj * w + ci], 1u);
}

struct Rect {
    double x, y, x2, y2;
};

// Dense cell window [imin, imin+W) x [jmin, jmin+H) with a summed-area table.
class CellGrid {
public:
    CellGrid(double mrs, int64_t imin, int64_t jmin, int64_t W, int64_t H,
             const std::vector<uint32_t>& hist)
        : mrs_(mrs), imin_(imin), jmin_(jmin), W_(W), H_(H), sat_((W + 1) * (H + 1), 0) {
        for (int64_t j = 0; j < H; ++j) {
            int64_t row = 0;
            for (int64_t i = 0; i < W; ++i) {
                row += hist[j * W + i];
                sat_[(j + 1) * (W + 1) + i + 1] = sat_[j * (W + 1) + i + 1] + row;
            }
        }
    }
    double lo(int64_t i) const { return (double)i * mrs_; }  // cell corners, DBSCAN.scala:352
    double hi(int64_t i) const { return (double)i * mrs_ + mrs_; }
    // first window column whose cell starts at or after v (cells contained from the left)
    int64_t first_col(double v) const { return first_ge(v, imin_, W_); }
    int64_t first_row(double v) const { return first_ge(v, jmin_, H_); }
    int64_t last_col(double v) const { return last_le(v, imin_, W_); }
    int64_t last_row(double v) const { return last_le(v, jmin_, H_); }
    // points in the cells of columns [i0, i1] x rows [j0, j1] (absolute indices, inclusive)
    int64_t count(int64_t i0, int64_t i1, int64_t j0, int64_t j1) const {
        if (i0 > i1 || j0 > j1) return 0;
        const int64_t a0 = i0 - imin_, a1 = i1 - imin_ + 1, b0 = j0 - jmin_, b1 = j1 - jmin_ + 1;
        const int64_t w = W_ + 1;
        return sat_[b1 * w + a1] - sat_[b0 * w + a1] - sat_[b1 * w + a0] + sat_[b0 * w + a0];
    }
    // EvenSplitPartitioner.pointsInRectangle (:175-181): cells with r.x <= c.x, c.x2 <= r.x2,
    // r.y <= c.y, c.y2 <= r.y2
    int64_t points_in(const Rect& r) const {
        return count(first_col(r.x), last_col(r.x2), first_row(r.y), last_row(r.y2));
    }
    int64_t imin() const { return imin_; }
    int64_t jmin() const { return jmin_; }
    int64_t W() const { return W_; }
    int64_t H() const { return H_; }

private:
    int64_t first_ge(double v, int64_t base, int64_t len) const {
        int64_t a = base, b = base + len;
        while (a < b) {
            const int64_t m = a + ((b - a) >> 1);
            if (v <= lo(m)) b = m; else a = m + 1;
        }
        return a;
    }
    int64_t last_le(double v, int64_t base, int64_t len) const {
        int64_t a = base, b = base + len;
        while (a < b) {
            const int64_t m = a + ((b - a) >> 1);
            if (hi(m) <= v) a = m + 1; else b = m;
        }
        return a - 1;
    }
    double mrs_;
    int64_t imin_, jmin_, W_, H_;
    std::vector<int64_t> sat_;
};

// ---- Scala 2.10.4 hashing of a DBSCANRectangle (a case class of four Doubles) -------------
// scala.runtime.BoxesRunTime.hashFromDouble: a boxed Double's ## -- the Int value when exact,
// else the Long's hashCode when exact, else the Float's (floatToIntBits), else the Double's.
uint32_t boxed_double_hash(double d) {
    if (d == d && d > -2147483649.0 && d < 2147483648.0) {
        const int32_t i = (int32_t)d;  // (truncation: in range)
        if ((double)i == d) return (uint32_t)i;
    }
    if (d == d && d >= -9223372036854775808.0 && d < 9223372036854775808.0) {
        const int64_t l = (int64_t)d;
        if ((double)l == d) {
            const uint64_t u = (uint64_t)l;
            return (uint32_t)(u ^ (u >> 32));
        }
    }
    // Java's (long) saturates: 2^63 becomes Long.MaxValue, which compares equal to 2^63 as a
    // double (NaN: Java's (int) / (long) give 0, which is not == NaN: falls through too)
    if (d == 9223372036854775808.0) return 0x80000000u;  // Long.MaxValue.hashCode
    const float f = (float)d;
    if ((double)f == d) {
        uint32_t b;
        memcpy(&b, &f, 4);
        return b;
    }
    uint64_t u;
    memcpy(&u, &d, 8);
    if (d != d) u = 0x7FF8000000000000ull;  // Double.doubleToLongBits: canonical NaN
    return (uint32_t)(u ^ (u >> 32));
}
// scala.util.hashing.MurmurHash3.productHash(rect, 0xcafebabe): mix per field, finalize
uint32_t rect_case_hash(const Rect& r) {
    const auto rotl = [](uint32_t v, int k) { return (v << k) | (v >> (32 - k)); };
    uint32_t h = 0xCAFEBABEu;
    const double f[4] = {r.x, r.y, r.x2, r.y2};
    for (double v : f) {
        uint32_t k = boxed_double_hash(v) * 0xCC9E2D51u;
        k = rotl(k, 15) * 0x1B873593u;
        h = rotl(h ^ k, 13) * 5u + 0xE6546B64u;
    }
    h ^= 4u;  // finalizeHash(h, productArity)
    h = (h ^ (h >> 16)) * 0x85EBCA6Bu;
    h = (h ^ (h >> 13)) * 0xC2B2AE35u;
    return h ^ (h >> 16);
}
// Iteration rank of a rectangle in a Scala 2.10 immutable.HashSet (HashTrieSet): the element's
// hash goes through HashSet.improve, then the trie indexes 5-bit groups from the low bits up and
// iterates children in index order -- i.e. ascending order of the groups read low group first.
uint32_t split_rank(const Rect& r) {
    uint32_t h = rect_case_hash(r);
    h += ~(h << 9);
    h ^= h >> 14;
    h += h << 4;
    h ^= h >> 10;
    uint32_t key = 0;
    for (int lvl = 0; lvl < 6; ++lvl) key = (key << 5) | ((h >> (5 * lvl)) & 31u);
    return (key << 2) | (h >> 30);
}

// Number of elements of the Scala 2.10 Double range `start until end by step`
// (EvenSplitPartitioner.scala:150-152): NumericRange.count, restated exactly in javanum.hip;
// the elements themselves come by repeated addition from start (NumericRange.foreach).
int64_t range_len(double start, double end, double step) {
    return scala_range_count(start, end, step, false);
}

// EvenSplitPartitioner.split (:105-123) + complement (:128-143).  Candidates along one axis:
// the box grows to v = start, start + mrs, ... (repeated addition); the contained columns (or
// rows) only grow with v, so a two-pointer walk finds each candidate's count in O(1).
bool best_split(const CellGrid& g, const Rect& box, double mrs, Rect* s1, Rect* s2) {
    const int64_t half = g.points_in(box) / 2;  // Int division, :81
    const int64_t c0 = g.first_col(box.x), c1 = g.last_col(box.x2);
    const int64_t r0 = g.first_row(box.y), r1 = g.last_row(box.y2);
    bool have = false;
    int64_t best_cost = 0;
    Rect best = box;
    int64_t lens[2];
    for (int axis = 0; axis < 2; ++axis)
        lens[axis] = range_len((axis == 0 ? box.x : box.y) + mrs, axis == 0 ? box.x2 : box.y2, mrs);
    // the candidate Set (findPossibleSplits' toSet) is a HashTrieSet above 4 DISTINCT
    // rectangles: a step below ulp(v) repeats a value (the x and y candidates never coincide)
    const auto distinct = [&](int axis, int64_t cap) {
        int64_t d = 0;
        double v = (axis == 0 ? box.x : box.y) + mrs, prev = 0.0;
        for (int64_t k = 0; k < lens[axis] && d < cap; ++k, v += mrs) {
            if (k == 0 || v != prev) ++d;
            prev = v;
        }
        return d;
    };
    const bool trie = lens[0] + lens[1] > 4 && distinct(0, 5) + distinct(1, 5) > 4;
    uint32_t best_rank = 0;
    for (int axis = 0; axis < 2; ++axis) {
        const double start = (axis == 0 ? box.x : box.y) + mrs;
        const int64_t len = lens[axis];
        const int64_t base = axis == 0 ? g.imin() : g.jmin();
        const int64_t lim = base + (axis == 0 ? g.W() : g.H());
        int64_t last = (axis == 0 ? c0 : r0) - 1;  // last contained column/row so far
        double v = start;
        for (int64_t k = 0; k < len; ++k, v += mrs) {
            while (last + 1 < lim && g.hi(last + 1) <= v) ++last;
            const int64_t cnt = axis == 0 ? g.count(c0, last, r0, r1) : g.count(c0, c1, r0, last);
            const int64_t cost = std::llabs(half - cnt);
            const Rect cand = axis == 0 ? Rect{box.x, box.y, v, box.y2} : Rect{box.x, box.y, box.x2, v};
            if (!have || cost < best_cost) {
                best_cost = cost;
                best = cand;
                have = true;
                if (trie) best_rank = split_rank(cand);
            } else if (trie && cost == best_cost) {
                const uint32_t rk = split_rank(cand);
                if (rk < best_rank) {
                    best = cand;
                    best_rank = rk;
                }
            }
        }
    }
    if (!have) return false;
    *s1 = best;
    if (best.y2 == box.y2) *s2 = Rect{best.x2, best.y, box.x2, box.y2};
    else if (best.x2 == box.x2) *s2 = Rect{best.x, best.y2, box.x2, box.y2};
    else return false;  // "rectangle is not a proper sub-rectangle"
    return true;
}

}  // namespace

// EvenSplitPartitioner.findPartitions (:44-64) + partition (:66-103) over the histogram.
int64_t split_partitions(double mrs, int64_t imin, int64_t jmin, int64_t W, int64_t H,
                         const std::vector<uint32_t>& hist, int64_t max_points,
                         std::vector<Partition>* out) {
    out->clear();
    const CellGrid g(mrs, imin, jmin, W, H, hist);
    // findBoundingRectangle (:183-209) over the occupied cells
    Rect bound{INFINITY, INFINITY, -INFINITY, -INFINITY};
    for (int64_t j = 0; j < H; ++j)
        for (int64_t i = 0; i < W; ++i) {
            if (!hist[j * W + i]) continue;
            bound.x = std::min(bound.x, g.lo(imin + i));
            bound.y = std::min(bound.y, g.lo(jmin + j));
            bound.x2 = std::max(bound.x2, g.hi(imin + i));
            bound.y2 = std::max(bound.y2, g.hi(jmin + j));
        }
    if (!(bound.x <= bound.x2)) return 0;  // no cells
    struct RC {
        Rect r;
        int64_t c;
    };
    std::vector<RC> stack{{bound, g.points_in(bound)}}, done;
    while (!stack.empty()) {  // the tail recursion: head of `remaining` first
        const RC cur = stack.back();
        stack.pop_back();
        const Rect& b = cur.r;
        if (cur.c > max_points && (b.x2 - b.x > mrs * 2 || b.y2 - b.y > mrs * 2)) {  // :168-171
            Rect s1, s2;
            if (!best_split(g, b, mrs, &s1, &s2)) return -1;
            stack.push_back({s2, g.points_in(s2)});
            stack.push_back({s1, g.points_in(s1)});  // s1 :: s2 :: rest
        } else {
            done.push_back(cur);  // also "Can't split" (:89-91)
        }
    }
    // `partitioned` is built by prepending (:91,:96): reverse; drop empty partitions (:63)
    for (auto it = done.rbegin(); it != done.rend(); ++it)
        if (it->c > 0) out->push_back({it->r.x, it->r.y, it->r.x2, it->r.y2, it->c});
    return (int64_t)out->size();
}

int64_t run_partition(hipStream_t s, Workspace& ws, const double* d_x, const double* d_y,
                      int64_t n, double eps, int64_t max_points, std::vector<Partition>* out) {
    out->clear();
    if (n == 0) return 0;
    const double mrs = 2 * eps;  // DBSCAN.scala:289 minimumRectangleSize
    const int nb = (int)std::min<int64_t>(1024, (n + kBlock - 1) / kBlock);
    int64_t* part = static_cast<int64_t*>(ws.scan_tmp.ensure((size_t)nb * 4 * sizeof(int64_t)));
    hipLaunchKernelGGL(cell_range_kernel, dim3(nb), dim3(kBlock), 0, s, d_x, d_y, n, mrs, part);
    DBSCAN_HIP_CHECK(hipGetLastError());
    std::vector<int64_t> hp((size_t)nb * 4);
    DBSCAN_HIP_CHECK(hipMemcpyAsync(hp.data(), part, hp.size() * sizeof(int64_t),
                                    hipMemcpyDeviceToHost, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    int64_t imin = INT64_MAX, imax = INT64_MIN, jmin = INT64_MAX, jmax = INT64_MIN;
    for (int b = 0; b < nb; ++b) {
        imin = std::min(imin, hp[4 * b]);
        imax = std::max(imax, hp[4 * b + 1]);
        jmin = std::min(jmin, hp[4 * b + 2]);
        jmax = std::max(jmax, hp[4 * b + 3]);
    }
    const int64_t W = imax - imin + 1, H = jmax - jmin + 1;
    if ((double)(W + 1) * (double)(H + 1) > kMaxPartitionCells)
        throw ArgError{"dbscan_partition: the 2*eps cell window is too large for a dense "
                       "histogram (spread or non-finite coordinates)"};
    uint32_t* hist = static_cast<uint32_t*>(ws.key2.ensure((size_t)(W * H) * sizeof(uint32_t)));
    DBSCAN_HIP_CHECK(hipMemsetAsync(hist, 0, (size_t)(W * H) * sizeof(uint32_t), s));
    hipLaunchKernelGGL(cell_hist_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, s, d_x, d_y, n, mrs, imin, jmin, W, hist);
    DBSCAN_HIP_CHECK(hipGetLastError());
    std::vector<uint32_t> h((size_t)(W * H));
    DBSCAN_HIP_CHECK(hipMemcpyAsync(h.data(), hist, h.size() * sizeof(uint32_t),
                                    hipMemcpyDeviceToHost, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    const int64_t k = split_partitions(mrs, imin, jmin, W, H, h, max_points, out);
    if (k < 0) throw ArgError{"dbscan_partition: rectangle is not a proper sub-rectangle"};
    return k;
}

int64_t partition_cells(const double* cell_x, const double* cell_y, const int64_t* counts,
                        int64_t ncells, int64_t max_points, double mrs,
                        std::vector<Partition>* out) {
    out->clear();
    if (ncells == 0) return 0;
    std::vector<int64_t> ci(ncells), cj(ncells);
    int64_t imin = INT64_MAX, imax = INT64_MIN, jmin = INT64_MAX, jmax = INT64_MIN;
    for (int64_t k = 0; k < ncells; ++k) {
        ci[k] = (int64_t)std::llround(cell_x[k] / mrs);
        cj[k] = (int64_t)std::llround(cell_y[k] / mrs);
        if ((double)ci[k] * mrs != cell_x[k] || (double)cj[k] * mrs != cell_y[k])
            throw ArgError{"dbscan_partition_cells: a cell is not on the mrs grid"};
        imin = std::min(imin, ci[k]);
        imax = std::max(imax, ci[k]);
        jmin = std::min(jmin, cj[k]);
        jmax = std::max(jmax, cj[k]);
    }
    const int64_t W = imax - imin + 1, H = jmax - jmin + 1;
    if ((double)(W + 1) * (double)(H + 1) > kMaxPartitionCells)
        throw ArgError{"dbscan_partition_cells: cell window too large"};
    std::vector<uint32_t> h((size_t)(W * H), 0);
    for (int64_t k = 0; k < ncells; ++k) h[(cj[k] - jmin) * W + (ci[k] - imin)] += (uint32_t)counts[k];
    const int64_t r = split_partitions(mrs, imin, jmin, W, H, h, max_points, out);
    if (r < 0) throw ArgError{"dbscan_partition_cells: rectangle is not a proper sub-rectangle"};
    return r;
}

// DBSCAN.scala:116-137: localMargins = (p.shrink(eps), p, p.shrink(-eps)) and
//   duplicated = for (point, ((inner, main, outer), id)) if outer.contains(point) yield (id, point)
// i.e. every point goes to every partition whose outer rectangle (main grown by eps, the
// reference's own fp arithmetic: x + (-eps), x2 - (-eps)) contains it, borders included
// (DBSCANRectangle.scala:35-37).  Each partition's points come out in input order (the order
// groupByKey hands a partition to LocalDBSCANNaive.fit).  Host threads over chunks of the input;
// a bucket grid over the outer rectangles replaces the reference's scan of every partition per
// point (the same decisions).  Returns the total; fills offsets_out[n_parts + 1] and, when
// index_out is given and capacity >= total, index_out.
int64_t duplicate_points(const double* x, const double* y, int64_t n, const double* rects,
                         int64_t n_parts, double eps, int64_t* offsets_out, int64_t* index_out,
                         int64_t capacity) {
    struct Box {
        double x, y, x2, y2;
    };
    std::vector<Box> outer((size_t)n_parts);
    bool finite = true;
    double bx0 = INFINITY, bx1 = -INFINITY, by0 = INFINITY, by1 = -INFINITY;
    for (int64_t p = 0; p < n_parts; ++p) {
        const double* r = rects + 4 * p;
        Box b{r[0] + (-eps), r[1] + (-eps), r[2] - (-eps), r[3] - (-eps)};  // shrink(-eps)
        outer[(size_t)p] = b;
        finite = finite && std::isfinite(b.x) && std::isfinite(b.y) && std::isfinite(b.x2) &&
                 std::isfinite(b.y2);
        bx0 = std::min(bx0, b.x);
        bx1 = std::max(bx1, b.x2);
        by0 = std::min(by0, b.y);
        by1 = std::max(by1, b.y2);
    }
    // bucket grid: bucket(v) = floor((v - b0) * ib), clamped; monotone in v, so a point inside
    // a box lies in one of the buckets the box registered in
    int G = 1;
    if (finite && n_parts > 0) {
        G = (int)std::min<double>(4096.0, 2.0 * std::ceil(std::sqrt((double)n_parts)) + 1.0);
        if (!(bx1 > bx0) || !(by1 > by0) || !std::isfinite(bx1 - bx0) || !std::isfinite(by1 - by0))
            G = 1;
    }
    const double ibx = G > 1 ? G / (bx1 - bx0) : 0.0, iby = G > 1 ? G / (by1 - by0) : 0.0;
    auto bucket = [&](double v, double b0, double ib) -> int {
        if (G == 1) return 0;
        const double t = std::floor((v - b0) * ib);
        if (!(t > 0)) return 0;  // (NaN too)
        return t >= G - 1 ? G - 1 : (int)t;
    };
    std::vector<int32_t> head((size_t)G * G + 1, 0), lst;
    for (int pass = 0; pass < 2; ++pass) {
        std::vector<int32_t> fill;
        if (pass == 1) {
            for (size_t k = 1; k < head.size(); ++k) head[k] += head[k - 1];
            lst.resize((size_t)head.back());
            fill.assign(head.begin(), head.end() - 1);
        }
        for (int64_t p = 0; p < n_parts; ++p) {
            const Box& b = outer[(size_t)p];
            const int i0 = bucket(b.x, bx0, ibx), i1 = bucket(b.x2, bx0, ibx);
            const int j0 = bucket(b.y, by0, iby), j1 = bucket(b.y2, by0, iby);
            for (int j = j0; j <= j1; ++j)
                for (int i = i0; i <= i1; ++i) {
                    const size_t c = (size_t)j * G + i;
                    if (pass == 0) ++head[c + 1];
                    else lst[(size_t)fill[c]++] = (int32_t)p;
                }
        }
    }
    int T = (int)std::min<int64_t>(16, std::max<int64_t>(1, n / 65536));
    const unsigned hc = std::thread::hardware_concurrency();
    if (hc > 0) T = std::min<int>(T, (int)hc);
    const int64_t chunk = (n + T - 1) / std::max(T, 1);
    std::vector<std::vector<int64_t>> cnt((size_t)T, std::vector<int64_t>((size_t)n_parts, 0));
    auto visit = [&](int t, bool write, std::vector<int64_t>* pos) {
        const int64_t a = t * chunk, e = std::min<int64_t>(n, a + chunk);
        for (int64_t i = a; i < e; ++i) {
            const double px = x[i], py = y[i];
            const size_t c = (size_t)bucket(py, by0, iby) * G + bucket(px, bx0, ibx);
            for (int32_t k = head[c]; k < head[c + 1]; ++k) {
                const int32_t p = lst[(size_t)k];
                const Box& b = outer[(size_t)p];
                if (b.x <= px && px <= b.x2 && b.y <= py && py <= b.y2) {  // contains
                    if (write) index_out[(*pos)[(size_t)p]++] = i;
                    else ++cnt[(size_t)t][(size_t)p];
                }
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(visit, t, false, nullptr);
        for (auto& h : th) h.join();
    }
    int64_t total = 0;
    std::vector<std::vector<int64_t>> pos((size_t)T, std::vector<int64_t>((size_t)n_parts, 0));
    for (int64_t p = 0; p < n_parts; ++p) {
        offsets_out[p] = total;
        for (int t = 0; t < T; ++t) {
            pos[(size_t)t][(size_t)p] = total;
            total += cnt[(size_t)t][(size_t)p];
        }
    }
    offsets_out[n_parts] = total;
    if (index_out && capacity >= total) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(visit, t, true, &pos[(size_t)t]);
        for (auto& h : th) h.join();
    }
    return total;
}

}  // namespace dbscan
