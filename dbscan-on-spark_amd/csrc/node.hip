// node.hip -- dbscan_train_node: the whole-node entry of SURVEY.md §8b, one process driving
// every GPU of the node.  The C++ twin of dbscan_amd/node.py (which runs one process per GPU
// over RCCL); the same slab plan, the same exact merge:
//   DBSCAN.scala:91-137    partition the plane, grow partitions by eps, duplicate points
//                          -> n_shards x-slabs at count quantiles snapped to the 2*eps grid,
//                             each with its 2-zone halo (node.py: make_cuts, zones)
//   DBSCAN.scala:150-155   LocalDBSCANNaive.fit per partition
//                          -> the lean slab fit per shard, shard s on device s % device_count,
//                             one host thread and one handle (HIP stream) per device; shards
//                             sharing a device run one after another on its handle and are
//                             re-fitted before their label (one workspace per device, so 8
//                             shards of 10^9 points fit one GPU's HBM)
//   DBSCAN.scala:158-222   band points, findAdjacencies, DBSCANGraph, global ids
//                          -> records (gid of a shared core, gid of its local root) merged by
//                             merge.hip's lock-free union-find on every device (the records are
//                             a thin band: O(1e5) at 1e8 pts), global s(K) per local root,
//                             cluster id = rank of s(K)
//   DBSCAN.scala:232-270   relabel                  -> dbscan_slab_label_device per shard
// The result equals ONE fit of all points, bit for bit.
#include "../../include/dbscan_hip.h"
#include "internal.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <memory>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <vector>

namespace dbscan {
namespace {

constexpr uint8_t kOut = 255;

double reach(double eps) { return std::max(std::fabs(eps) * (1.0 + 0x1p-40), 0x1p-500); }
double ulp(double c) {
    c = std::fabs(c);
    return std::nextafter(c, INFINITY) - c;
}
double margin1(double c, double R) { return R * (1.0 + 0x1p-10) + 16.0 * ulp(c); }
double margin2(double c, double R) { return 2.0 * margin1(c, R) + 16.0 * ulp(c); }

// Host threads for the slab plan: OMP_NUM_THREADS when set (the GPU box's per-GPU CPU share),
// else the hardware's, at most 64.
int64_t host_threads() {
    int64_t n = (int64_t)std::thread::hardware_concurrency();
    if (const char* e = std::getenv("OMP_NUM_THREADS")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v > 0) n = std::min<int64_t>(n > 0 ? n : v, v);
    }
    return std::max<int64_t>(1, std::min<int64_t>(n, 64));
}

// DBSCAN_NODE_TRACE=1: phase wall times on stderr (observability only; nothing computed changes)
struct PhaseTrace {
    bool on = false;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    PhaseTrace() {
        const char* e = std::getenv("DBSCAN_NODE_TRACE");
        on = e && e[0] == '1';
    }
    void mark(const char* what) {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[train_node] %-22s %9.3f s\n", what,
                     std::chrono::duration<double>(t - t0).count());
        t0 = t;
    }
};

template <class F>
void parallel_for(int nth, F&& f) {
    if (nth <= 1) {
        f(0);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nth; ++t) th.emplace_back([&, t]() { f(t); });
    for (auto& t : th) t.join();
}

// Host arrays of the slab plan: resize() leaves the elements uninitialized (every element is
// written before it is read), so the 10^9-point plan's ~40 GB are first touched by the parallel
// fill instead of being zeroed by one thread.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
template <class T>
using HostVec = std::vector<T, NoInitAlloc<T>>;

// node.py make_cuts: world-1 cuts at count quantiles of a strided sample of the finite x,
// snapped down to the 2*eps grid, non-decreasing.  The finite count and the sample (every
// step-th finite x in input order) by host threads over contiguous chunks.
std::vector<double> make_cuts(const double* x, int64_t n, int world, double eps) {
    std::vector<double> cuts;
    if (world <= 1 || !std::isfinite(eps * eps)) return cuts;
    const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), n / 65536 + 1));
    const auto chunk = [&](int t) { return std::make_pair(n * t / nth, n * (t + 1) / nth); };
    std::vector<int64_t> fin(nth + 1, 0);
    parallel_for(nth, [&](int t) {
        const auto [i0, i1] = chunk(t);
        int64_t c = 0;
        for (int64_t i = i0; i < i1; ++i) c += std::isfinite(x[i]) ? 1 : 0;
        fin[t + 1] = c;
    });
    for (int t = 0; t < nth; ++t) fin[t + 1] += fin[t];
    const int64_t nfin = fin[nth];
    if (nfin == 0) return cuts;
    const int64_t step = std::max<int64_t>(1, nfin / (1 << 20));
    // finite index k is sampled when k % step == 0; chunk t starts at finite index fin[t]
    std::vector<int64_t> soff(nth + 1, 0);
    for (int t = 0; t < nth; ++t) soff[t + 1] = (fin[t + 1] + step - 1) / step;
    std::vector<double> xf((size_t)soff[nth]);
    parallel_for(nth, [&](int t) {
        const auto [i0, i1] = chunk(t);
        int64_t k = fin[t], o = soff[t];
        for (int64_t i = i0; i < i1; ++i)
            if (std::isfinite(x[i])) {
                if (k % step == 0) xf[(size_t)o++] = x[i];
                ++k;
            }
    });
    std::sort(xf.begin(), xf.end());
    const double grid = 2.0 * std::fabs(eps);
    const int64_t m = (int64_t)xf.size();
    for (int r = 1; r < world; ++r) {
        const double q = xf[std::min<int64_t>(m - 1, r * m / world)];
        double c = (grid > 0 && std::isfinite(q / grid)) ? std::floor(q / grid) * grid : q;
        if (!cuts.empty() && c < cuts.back()) c = cuts.back();
        cuts.push_back(c);
    }
    return cuts;
}

// node.py zones(): zone of x for shard r (0 owned, 1 inner halo, 2 outer halo, kOut) and
// whether the point is shared (in zone 0/1 of an adjacent shard as well).  The margins depend on
// the cut values alone, so they are computed once per shard (ZoneCut), not per point.
struct ZoneCut {
    bool has_lo = false, has_hi = false;
    double lo = 0, hi = 0, m1lo = 0, m2lo = 0, m1hi = 0, m2hi = 0;
};

std::vector<ZoneCut> zone_cuts(int world, const std::vector<double>& cuts, double R) {
    std::vector<ZoneCut> zc(world);
    for (int r = 0; r < world; ++r) {
        ZoneCut& z = zc[r];
        z.has_lo = r > 0;
        z.has_hi = r < world - 1;
        if (z.has_lo) {
            z.lo = cuts[r - 1];
            z.m1lo = margin1(z.lo, R);
            z.m2lo = margin2(z.lo, R);
        }
        if (z.has_hi) {
            z.hi = cuts[r];
            z.m1hi = margin1(z.hi, R);
            z.m2hi = margin2(z.hi, R);
        }
    }
    return zc;
}

__host__ __device__ inline uint8_t zone_of(double x, int r, int world, const ZoneCut& c,
                                           bool* shared) {
    bool own = (!c.has_lo || x >= c.lo) && (!c.has_hi || x < c.hi);
    if (r == 0 && world > 1 && x != x) own = true;
    bool in1 = false, in2 = false, sh = false;
    if (c.has_lo) {
        in1 = in1 || (x >= c.lo - c.m1lo && x < c.lo);
        in2 = in2 || (x >= c.lo - c.m2lo && x < c.lo - c.m1lo);
        sh = sh || (own && x <= c.lo + c.m1lo);
    }
    if (c.has_hi) {
        in1 = in1 || (x >= c.hi && x <= c.hi + c.m1hi);
        in2 = in2 || (x > c.hi + c.m1hi && x <= c.hi + c.m2hi);
        sh = sh || (own && x >= c.hi - c.m1hi);
    }
    const uint8_t z = own ? 0 : (in1 ? 1 : (in2 ? 2 : kOut));
    *shared = sh || z == 1;
    return z;
}

// ---- the slab plan on the device -------------------------------------------------------
// Shard r's points (zone != kOut for r) in increasing global visit order, by an ordered
// three-kernel compaction over all n points: per-block counts of the shard's points and of its
// shared points, an exclusive scan of each, a ballot-ranked write.  kPlanTile points per block.
constexpr int kPlanTile = 8192;  // 32 rounds of 256

__global__ __launch_bounds__(kBlock) void plan_count_kernel(const double* __restrict__ x,
                                                            int64_t n, int r, int world,
                                                            ZoneCut zc,
                                                            int32_t* __restrict__ cnt_sel,
                                                            int32_t* __restrict__ cnt_sh) {
    __shared__ int ws[2][kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kPlanTile;
    int c = 0, h = 0;
    for (int k = 0; k < kPlanTile / kBlock; ++k) {
        const int64_t i = base + k * kBlock + threadIdx.x;
        if (i >= n) break;
        bool sh = false;
        const uint8_t z = zone_of(x[i], r, world, zc, &sh);
        c += z != kOut ? 1 : 0;
        h += (z != kOut && sh) ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o, 64);
        h += __shfl_xor(h, o, 64);
    }
    if (__lane_id() == 0) {
        ws[0][threadIdx.x >> 6] = c;
        ws[1][threadIdx.x >> 6] = h;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        int t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += ws[threadIdx.x][w];
        (threadIdx.x ? cnt_sh : cnt_sel)[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kBlock) void plan_write_kernel(
    const double* __restrict__ x, const double* __restrict__ y, int64_t n, int r, int world,
    ZoneCut zc, const int32_t* __restrict__ off_sel, const int32_t* __restrict__ off_sh,
    double* __restrict__ sx, double* __restrict__ sy, uint8_t* __restrict__ sz,
    int64_t* __restrict__ sgid, int64_t* __restrict__ sshared) {
    __shared__ int wc[2][2][kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kPlanTile;
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int o = off_sel[blockIdx.x], oh = off_sh[blockIdx.x];
    for (int k = 0; k < kPlanTile / kBlock; ++k) {
        if (base + k * kBlock >= n) break;  // (block-uniform)
        const int64_t i = base + k * kBlock + threadIdx.x;
        bool sh = false;
        uint8_t z = kOut;
        double xi = 0;
        if (i < n) {
            xi = x[i];
            z = zone_of(xi, r, world, zc, &sh);
        }
        const bool in = z != kOut;
        sh = sh && in;
        const uint64_t b = __ballot(in), bh = __ballot(sh);
        if (lane == 0) {
            wc[k & 1][0][w] = __popcll(b);
            wc[k & 1][1][w] = __popcll(bh);
        }
        __syncthreads();
        int before = 0, total = 0, beforeh = 0, totalh = 0;
#pragma unroll
        for (int v = 0; v < kBlock / 64; ++v) {
            const int c = wc[k & 1][0][v], ch = wc[k & 1][1][v];
            before += v < w ? c : 0;
            total += c;
            beforeh += v < w ? ch : 0;
            totalh += ch;
        }
        if (in) {
            const int64_t q = (int64_t)o + before + __popcll(b & lt);
            sx[q] = xi;
            sy[q] = y[i];
            sz[q] = z;
            sgid[q] = i;
            if (sh) sshared[oh + beforeh + __popcll(bh & lt)] = q;
        }
        o += total;
        oh += totalh;
    }
}

// The merge records of a shard: (gid of a shared point, gid of its local root, or -1 when the
// point is not core here) -- node.py NodeJob.run's records.
__global__ __launch_bounds__(kBlock) void plan_records_kernel(
    const int64_t* __restrict__ sshared, int64_t ns, const int64_t* __restrict__ sgid,
    const uint8_t* __restrict__ score, const int32_t* __restrict__ sroot, int64_t* __restrict__ a,
    int64_t* __restrict__ b) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= ns) return;
    const int64_t p = sshared[k];
    const int32_t r = sroot[p];
    a[k] = sgid[p];
    b[k] = (score[p] != 0 && r >= 0) ? sgid[r] : -1;
}

// The zone-0 labels of a shard (slab order) into the whole job's output arrays (input order).
__global__ __launch_bounds__(kBlock) void plan_scatter_kernel(
    int64_t m, const uint8_t* __restrict__ sz, const int64_t* __restrict__ sgid,
    const int32_t* __restrict__ cl, const uint8_t* __restrict__ fl, int32_t* __restrict__ out_cl,
    uint8_t* __restrict__ out_fl) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= m || sz[p] != 0) return;
    const int64_t g = sgid[p];
    out_cl[g] = cl[p];
    out_fl[g] = fl[p];
}

unsigned nblocks(int64_t m) { return (unsigned)std::max<int64_t>(1, (m + kBlock - 1) / kBlock); }

// chunk_labels' rows (node.py): the zone-0 points of a slab, in slab order (ascending gid), as
// (gid, cluster << 8 | flag) int64 pairs -- the same ordered compaction as the plan kernels.
__global__ __launch_bounds__(kBlock) void owned_count_kernel(const uint8_t* __restrict__ zone,
                                                             int64_t m,
                                                             int32_t* __restrict__ cnt) {
    __shared__ int ws[kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kPlanTile;
    int c = 0;
    for (int k = 0; k < kPlanTile / kBlock; ++k) {
        const int64_t i = base + k * kBlock + threadIdx.x;
        if (i >= m) break;
        c += zone[i] == 0 ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (__lane_id() == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += ws[w];
        cnt[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kBlock) void owned_write_kernel(
    const uint8_t* __restrict__ zone, const int64_t* __restrict__ gid,
    const int32_t* __restrict__ cl, const uint8_t* __restrict__ fl, int64_t m,
    const int32_t* __restrict__ off, int64_t* __restrict__ rows) {
    __shared__ int wc[2][kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kPlanTile;
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int o = off[blockIdx.x];
    for (int k = 0; k < kPlanTile / kBlock; ++k) {
        if (base + k * kBlock >= m) break;  // (block-uniform)
        const int64_t i = base + k * kBlock + threadIdx.x;
        const bool in = i < m && zone[i] == 0;
        const uint64_t b = __ballot(in);
        if (lane == 0) wc[k & 1][w] = __popcll(b);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int v = 0; v < kBlock / 64; ++v) {
            before += v < w ? wc[k & 1][v] : 0;
            total += wc[k & 1][v];
        }
        if (in) {
            const int64_t q = (int64_t)o + before + __popcll(b & lt);
            rows[2 * q] = gid[i];
            rows[2 * q + 1] = ((int64_t)cl[i] << 8) | (int64_t)fl[i];
        }
        o += total;
    }
}

// from_chunk's received rows (x bits, y bits, gid * 8 + zone * 2 + shared) into the slab's
// columns, and the slab indices of its shared points (an ordered compaction: count, scan, write).
__global__ __launch_bounds__(kBlock) void unpack_count_kernel(const int64_t* __restrict__ rows,
                                                              int64_t k,
                                                              int32_t* __restrict__ cnt) {
    __shared__ int ws[kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kPlanTile;
    int c = 0;
    for (int j = 0; j < kPlanTile / kBlock; ++j) {
        const int64_t i = base + j * kBlock + threadIdx.x;
        if (i >= k) break;
        c += (int)(rows[3 * i + 2] & 1);
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (__lane_id() == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += ws[w];
        cnt[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kBlock) void unpack_write_kernel(
    const int64_t* __restrict__ rows, int64_t k, const int32_t* __restrict__ off,
    double* __restrict__ sx, double* __restrict__ sy, uint8_t* __restrict__ sz,
    int64_t* __restrict__ sgid, int64_t* __restrict__ sshared) {
    __shared__ int wc[2][kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kPlanTile;
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int o = off[blockIdx.x];
    for (int j = 0; j < kPlanTile / kBlock; ++j) {
        if (base + j * kBlock >= k) break;  // (block-uniform)
        const int64_t i = base + j * kBlock + threadIdx.x;
        bool sh = false;
        if (i < k) {
            const int64_t a = rows[3 * i], b = rows[3 * i + 1], code = rows[3 * i + 2];
            sx[i] = __longlong_as_double(a);
            sy[i] = __longlong_as_double(b);
            sz[i] = (uint8_t)((code >> 1) & 3);
            sgid[i] = code >> 3;
            sh = (code & 1) != 0;
        }
        const uint64_t bb = __ballot(sh);
        if (lane == 0) wc[j & 1][w] = __popcll(bb);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int v = 0; v < kBlock / 64; ++v) {
            before += v < w ? wc[j & 1][v] : 0;
            total += wc[j & 1][v];
        }
        if (sh) sshared[o + before + __popcll(bb & lt)] = i;
        o += total;
    }
}

// chunk_labels' scatter: rows (gid, cluster << 8 | flag) received by the chunk's owner.
__global__ __launch_bounds__(kBlock) void label_scatter_kernel(const int64_t* __restrict__ rows,
                                                               int64_t k, int64_t start, int64_t m,
                                                               int32_t* __restrict__ cl,
                                                               uint8_t* __restrict__ fl) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= k) return;
    const int64_t g = rows[2 * j] - start;
    const int64_t v = rows[2 * j + 1];
    if (g < 0 || g >= m) return;  // (never: every row was routed to its chunk's owner)
    cl[g] = (int32_t)(v >> 8);
    fl[g] = (uint8_t)(v & 255);
}

// ---- the node path's host-to-slab routing (node.py NodeJob.from_chunk) ------------------
// Every point of a rank's input chunk goes to each slab whose zones 0/1/2 hold it, as a 24-B row
// (x bits, y bits, gid * 8 + zone * 2 + shared), rows grouped by destination rank, ascending gid
// within each.  One count pass (per block and destination), one scan over the [dest][block]
// counts, one ballot-ranked write pass: every destination's rows in one kernel pass each.
constexpr int kRouteTile = 4096;  // points per block (16 rounds of 256)
constexpr int kRouteMaxWorld = 64;

__global__ __launch_bounds__(kBlock) void route_count_kernel(const double* __restrict__ x,
                                                             int64_t m, int world,
                                                             const ZoneCut* __restrict__ zc,
                                                             int32_t* __restrict__ cnt) {
    __shared__ int c[kRouteMaxWorld];
    for (int d = threadIdx.x; d < world; d += kBlock) c[d] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kRouteTile;
    for (int k = 0; k < kRouteTile / kBlock; ++k) {
        const int64_t i = base + k * kBlock + threadIdx.x;
        if (i >= m) break;
        const double xi = x[i];
        for (int d = 0; d < world; ++d) {
            bool sh = false;
            if (zone_of(xi, d, world, zc[d], &sh) != kOut) atomicAdd(&c[d], 1);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < world; d += kBlock) cnt[(int64_t)d * gridDim.x + blockIdx.x] = c[d];
}

__global__ __launch_bounds__(kBlock) void route_write_kernel(
    const double* __restrict__ x, const double* __restrict__ y, int64_t m, int64_t start,
    int world, const ZoneCut* __restrict__ zc, const int32_t* __restrict__ off,
    int64_t* __restrict__ rows) {
    __shared__ int wc[2][kRouteMaxWorld][kBlock / 64];
    __shared__ int base_d[kRouteMaxWorld];
    const int nb = gridDim.x;
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int d = threadIdx.x; d < world; d += kBlock) base_d[d] = off[(int64_t)d * nb + blockIdx.x];
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kRouteTile;
    for (int k = 0; k < kRouteTile / kBlock; ++k) {
        if (base + k * kBlock >= m) break;  // (block-uniform)
        const int64_t i = base + k * kBlock + threadIdx.x;
        double xi = 0, yi = 0;
        if (i < m) {
            xi = x[i];
            yi = y[i];
        }
        for (int d = 0; d < world; ++d) {
            bool sh = false;
            const uint8_t z = i < m ? zone_of(xi, d, world, zc[d], &sh) : kOut;
            const uint64_t b = __ballot(z != kOut);
            if (lane == 0) wc[k & 1][d][w] = __popcll(b);
        }
        __syncthreads();
        for (int d = 0; d < world; ++d) {
            bool sh = false;
            const uint8_t z = i < m ? zone_of(xi, d, world, zc[d], &sh) : kOut;
            const uint64_t b = __ballot(z != kOut);
            int before = 0, total = 0;
#pragma unroll
            for (int v = 0; v < kBlock / 64; ++v) {
                const int c = wc[k & 1][d][v];
                before += v < w ? c : 0;
                total += c;
            }
            if (z != kOut) {
                const int64_t q = (int64_t)base_d[d] + before + __popcll(b & lt);
                rows[3 * q] = (int64_t)__double_as_longlong(xi);
                rows[3 * q + 1] = (int64_t)__double_as_longlong(yi);
                rows[3 * q + 2] = (start + i) * 8 + (int64_t)z * 2 + (sh ? 1 : 0);
            }
            __syncthreads();  // (every thread has read base_d[d] before it advances)
            if (threadIdx.x == 0) base_d[d] += total;
        }
        __syncthreads();
    }
}

// A shard on its device: the slab (x, y, zone, gid in increasing gid), its shared points, the
// slab fit's outputs and each local root's global s(K).
struct DevShard {
    int64_t m = 0, ns = 0;
    double *x = nullptr, *y = nullptr;
    uint8_t *zone = nullptr, *core = nullptr;
    int64_t *gid = nullptr, *shared = nullptr, *gs = nullptr;
    int32_t* root = nullptr;
    std::vector<int64_t> a, b, own;  // host: merge records, owned global roots
    int32_t rc = DBSCAN_OK;
    std::string err;
    void release() {
        for (void* p : {(void*)x, (void*)y, (void*)zone, (void*)core, (void*)gid, (void*)shared,
                        (void*)gs, (void*)root})
            (void)hipFree(p);
        x = y = nullptr;
        zone = core = nullptr;
        gid = shared = gs = nullptr;
        root = nullptr;
    }
};

// HIP failures inside a device worker: thrown, caught per worker
struct HipFail {
    hipError_t e;
    const char* what;
};
inline void hcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw HipFail{e, what};
}
inline void ccheck(int32_t rc) {
    if (rc != DBSCAN_OK) throw rc;
}

// One device worker's outcome.  Every exception a worker body can throw (HipFail, an rc from
// the C-ABI, dbscan::HipError from DBSCAN_HIP_CHECK / DevBuf, dbscan::ArgError, std::bad_alloc
// from the host vectors, anything else) is mapped here: an exception escaping a std::thread
// would std::terminate the whole process -- the executor JVM included.
struct WorkerStatus {
    int32_t rc = DBSCAN_OK;
    std::string err;
};

inline void worker_status_from_current(WorkerStatus& ws) {
    try {
        throw;
    } catch (const HipFail& e) {
        ws.rc = (e.e == hipErrorOutOfMemory || e.e == hipErrorMemoryAllocation) ? DBSCAN_EOOM
                                                                                : DBSCAN_EHIP;
        ws.err = std::string(e.what) + ": " + hipGetErrorString(e.e);
    } catch (int32_t rc) {
        ws.rc = rc;
        ws.err = dbscan_last_error();
    } catch (const HipError& e) {
        ws.rc = (e.err == hipErrorOutOfMemory || e.err == hipErrorMemoryAllocation) ? DBSCAN_EOOM
                                                                                    : DBSCAN_EHIP;
        ws.err = e.what;
    } catch (const ArgError& e) {
        ws.rc = DBSCAN_EARG;
        ws.err = e.what;
    } catch (const std::bad_alloc&) {
        ws.rc = DBSCAN_EOOM;
        ws.err = "host allocation failed";
    } catch (const std::exception& e) {
        ws.rc = DBSCAN_EHIP;
        ws.err = e.what();
    } catch (...) {
        ws.rc = DBSCAN_EHIP;
        ws.err = "unknown error in a device worker";
    }
    if (ws.rc == DBSCAN_OK) ws.rc = DBSCAN_EHIP;  // (a thrown DBSCAN_OK is still a failure)
}

// f(w) for w < nworkers on one host thread each; false when any worker failed (its status set)
template <class F>
bool run_workers(int nworkers, std::vector<WorkerStatus>& st, F&& f) {
    std::vector<std::thread> th;
    for (int w = 0; w < nworkers; ++w)
        th.emplace_back([&, w]() {
            try {
                f(w);
            } catch (...) {
                worker_status_from_current(st[(size_t)w]);
            }
        });
    for (auto& t : th) t.join();
    for (auto& s : st)
        if (s.rc != DBSCAN_OK) return false;
    return true;
}

// dbscan_train_node's shard -> device plan: shard s runs on device s % ndev; one host worker per
// device in use (nworkers = min(world, ndev)) runs its shards s = w, w + nworkers, ... in order.
struct NodePlan {
    int world = 0, nworkers = 0;
    std::vector<std::vector<int>> shards_of;  // per worker (= device index)
};
NodePlan node_plan(int world, int ndev) {
    NodePlan p;
    p.world = std::max(0, world);
    p.nworkers = std::max(0, std::min(p.world, ndev));
    p.shards_of.resize((size_t)p.nworkers);
    for (int s = 0; s < p.world && p.nworkers > 0; ++s) p.shards_of[(size_t)(s % p.nworkers)].push_back(s);
    return p;
}

// The call's status from its workers': the first failed worker's (in device order), else OK.
int32_t first_failure(const std::vector<WorkerStatus>& wst, std::string* err) {
    for (const auto& d : wst)
        if (d.rc != DBSCAN_OK) {
            if (err) *err = d.err;
            return d.rc;
        }
    return DBSCAN_OK;
}

// What the calling thread's last dbscan_train_node ran: per shard, the device its worker ran on
// (read back from the worker's hipGetDevice), its points with halos and its shared points.
struct NodeRecord {
    std::vector<int32_t> device;
    std::vector<int64_t> points, shared;
};
thread_local NodeRecord g_node_record;

}  // namespace

int32_t node_record(int32_t* device_out, int64_t* points_out, int64_t* shared_out, int32_t max) {
    const NodeRecord& r = g_node_record;
    const int32_t k = (int32_t)r.device.size();
    for (int32_t s = 0; s < k && s < max; ++s) {
        if (device_out) device_out[s] = r.device[(size_t)s];
        if (points_out) points_out[s] = r.points[(size_t)s];
        if (shared_out) shared_out[s] = r.shared[(size_t)s];
    }
    return k;
}

// The plan and the worker error path of dbscan_train_node on the host alone: ndev mocked
// devices, the same node_plan and run_workers; worker w records the device it runs as for each
// of its shards (ran_on[s]) and throws a HIP failure when w == fail_device; rc_of_device[w] is
// each worker's status; returns the call's status as dbscan_train_node would.
int32_t node_plan_selftest(int32_t n_shards, int32_t ndev, int32_t fail_device, int32_t* ran_on,
                           int32_t* rc_of_device) {
    const NodePlan plan = node_plan(n_shards, ndev);
    std::vector<WorkerStatus> wst((size_t)plan.nworkers);
    for (int s = 0; s < plan.world; ++s) ran_on[s] = -1;
    run_workers(plan.nworkers, wst, [&](int w) {
        for (int s : plan.shards_of[(size_t)w]) {
            ran_on[s] = w;  // (train_node: the worker's hipSetDevice(w), read back per shard)
            if (w == fail_device) throw HipFail{hipErrorInvalidValue, "selftest shard"};
        }
    });
    for (int w = 0; w < plan.nworkers; ++w) rc_of_device[w] = wst[(size_t)w].rc;
    std::string err;
    return first_failure(wst, &err);
}

// The worker error mapping on the host alone (no device): worker w throws kind w (0 none,
// 1 HipFail OOM, 2 HipFail other, 3 rc EARG, 4 HipError, 5 ArgError, 6 bad_alloc,
// 7 std::runtime_error, 8 an int64); its rc goes to rcs[w].  The C-ABI selftest behind it.
int32_t worker_selftest(int32_t* rcs, int32_t n) {
    std::vector<WorkerStatus> st((size_t)std::max(0, n));
    run_workers(n, st, [](int w) {
        switch (w % 9) {
            case 1: throw HipFail{hipErrorOutOfMemory, "selftest"};
            case 2: throw HipFail{hipErrorInvalidValue, "selftest"};
            case 3: throw (int32_t)DBSCAN_EARG;
            case 4: throw HipError(hipErrorInvalidValue, "selftest", __FILE__, __LINE__);
            case 5: throw ArgError{"selftest"};
            case 6: throw std::bad_alloc();
            case 7: throw std::runtime_error("selftest");
            case 8: throw (int64_t)7;
            default: return;
        }
    });
    for (int w = 0; w < n; ++w) rcs[w] = st[(size_t)w].rc;
    return DBSCAN_OK;
}

// NodeJob.from_global's slab selection on the device (the plan kernels of dbscan_train_node):
// slab `rank`'s points (zones 0/1/2) in input order and the slab indices of its shared points.
// Returns the slab's point count (ns_out: its shared points); writes when sx != nullptr and
// capacity >= that count.  Synchronizes the stream.
int64_t select_slab(hipStream_t s, DevBuf& scratch, ScanState& scan, const double* x,
                    const double* y, int64_t n, const double* cuts, int32_t n_cuts, int32_t rank,
                    double eps, double* sx, double* sy, uint8_t* sz, int64_t* sgid,
                    int64_t* sshared, int64_t capacity, int64_t* ns_out) {
    const int world = n_cuts + 1;
    if (rank < 0 || rank >= world) throw ArgError{"slab select: rank out of range"};
    if (n >= (int64_t)INT32_MAX) throw ArgError{"slab select: more than 2^31 - 1 points"};
    *ns_out = 0;
    if (n == 0) return 0;
    const std::vector<double> cv(cuts, cuts + n_cuts);
    const std::vector<ZoneCut> zc = zone_cuts(world, cv, reach(eps));
    const int64_t nb = (n + kPlanTile - 1) / kPlanTile;
    int32_t* cnt = static_cast<int32_t*>(scratch.ensure((4 * nb + 4) * sizeof(int32_t)));
    int32_t *cs = cnt, *ch = cnt + nb, *os = cnt + 2 * nb, *oh = cnt + 3 * nb, *tot = cnt + 4 * nb;
    hipLaunchKernelGGL(plan_count_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, x, n, rank,
                       world, zc[rank], cs, ch);
    DBSCAN_HIP_CHECK(hipGetLastError());
    exclusive_scan(s, 0, cs, os, nb, tot, scan);
    exclusive_scan(s, 0, ch, oh, nb, tot + 1, scan);
    int32_t t2[2];
    DBSCAN_HIP_CHECK(hipMemcpyAsync(t2, tot, sizeof(t2), hipMemcpyDeviceToHost, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    *ns_out = t2[1];
    if (!sx || capacity < t2[0]) return t2[0];
    hipLaunchKernelGGL(plan_write_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, x, y, n, rank,
                       world, zc[rank], os, oh, sx, sy, sz, sgid, sshared);
    DBSCAN_HIP_CHECK(hipGetLastError());
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    return t2[0];
}

// chunk_labels' rows: the zone-0 points of a slab as (gid, cluster << 8 | flag), slab order.
// Returns the row count; writes when rows != nullptr and capacity suffices.
int64_t owned_rows(hipStream_t s, DevBuf& scratch, ScanState& scan, const uint8_t* zone,
                   const int64_t* gid, const int32_t* cl, const uint8_t* fl, int64_t m,
                   int64_t* rows, int64_t capacity) {
    if (m == 0) return 0;
    if (m >= (int64_t)INT32_MAX) throw ArgError{"owned rows: more than 2^31 - 1 points"};
    const int64_t nb = (m + kPlanTile - 1) / kPlanTile;
    int32_t* cnt = static_cast<int32_t*>(scratch.ensure((2 * nb + 2) * sizeof(int32_t)));
    int32_t *cs = cnt, *os = cnt + nb, *tot = cnt + 2 * nb;
    hipLaunchKernelGGL(owned_count_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, zone, m, cs);
    DBSCAN_HIP_CHECK(hipGetLastError());
    exclusive_scan(s, 0, cs, os, nb, tot, scan);
    int32_t t = 0;
    DBSCAN_HIP_CHECK(hipMemcpyAsync(&t, tot, sizeof(t), hipMemcpyDeviceToHost, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    if (!rows || capacity < t) return t;
    hipLaunchKernelGGL(owned_write_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, zone, gid, cl,
                       fl, m, os, rows);
    DBSCAN_HIP_CHECK(hipGetLastError());
    return t;
}

int64_t unpack_rows(hipStream_t s, DevBuf& scratch, ScanState& scan, const int64_t* rows,
                    int64_t k, double* sx, double* sy, uint8_t* sz, int64_t* sgid,
                    int64_t* sshared) {
    if (k == 0) return 0;
    if (k >= (int64_t)INT32_MAX) throw ArgError{"unpack rows: more than 2^31 - 1 rows"};
    const int64_t nb = (k + kPlanTile - 1) / kPlanTile;
    int32_t* cnt = static_cast<int32_t*>(scratch.ensure((2 * nb + 2) * sizeof(int32_t)));
    int32_t *cs = cnt, *os = cnt + nb, *tot = cnt + 2 * nb;
    hipLaunchKernelGGL(unpack_count_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, rows, k, cs);
    DBSCAN_HIP_CHECK(hipGetLastError());
    exclusive_scan(s, 0, cs, os, nb, tot, scan);
    hipLaunchKernelGGL(unpack_write_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, rows, k, os,
                       sx, sy, sz, sgid, sshared);
    DBSCAN_HIP_CHECK(hipGetLastError());
    int32_t t = 0;
    DBSCAN_HIP_CHECK(hipMemcpyAsync(&t, tot, sizeof(t), hipMemcpyDeviceToHost, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    return t;
}

void label_scatter(hipStream_t s, const int64_t* rows, int64_t k, int64_t start, int64_t m,
                   int32_t* cl, uint8_t* fl) {
    if (k <= 0) return;
    hipLaunchKernelGGL(label_scatter_kernel, dim3(nblocks(k)), dim3(kBlock), 0, s, rows, k, start,
                       m, cl, fl);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

// Routing of one chunk (see route_write_kernel): counts_out[d] = rows for rank d; rows written
// when rows != nullptr and capacity (rows) suffices.  Returns the total row count.
int64_t route_slabs(hipStream_t s, DevBuf& scratch, DevBuf& tabbuf, const double* x,
                    const double* y, int64_t m, int64_t start, const double* cuts, int32_t n_cuts,
                    double eps, int64_t* rows, int64_t capacity, int64_t* counts_out) {
    const int world = n_cuts + 1;
    if (world > kRouteMaxWorld) throw ArgError{"route: more than 64 slabs"};
    for (int d = 0; d < world; ++d) counts_out[d] = 0;
    if (m == 0) return 0;
    const std::vector<double> cv(cuts, cuts + n_cuts);
    const std::vector<ZoneCut> zc = zone_cuts(world, cv, reach(eps));
    ZoneCut* dzc = static_cast<ZoneCut*>(tabbuf.ensure(world * sizeof(ZoneCut)));
    DBSCAN_HIP_CHECK(hipMemcpyAsync(dzc, zc.data(), world * sizeof(ZoneCut), hipMemcpyHostToDevice, s));
    const int64_t nb = (m + kRouteTile - 1) / kRouteTile;
    int32_t* cnt = static_cast<int32_t*>(scratch.ensure((2 * nb * world + 8) * sizeof(int32_t)));
    int32_t* off = cnt + nb * world;
    hipLaunchKernelGGL(route_count_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, x, m, world,
                       dzc, cnt);
    DBSCAN_HIP_CHECK(hipGetLastError());
    // per destination: the sum of its blocks (host), then one scan for the offsets
    std::vector<int32_t> hc((size_t)(nb * world));
    DBSCAN_HIP_CHECK(hipMemcpyAsync(hc.data(), cnt, hc.size() * sizeof(int32_t),
                                    hipMemcpyDeviceToHost, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    int64_t total = 0;
    for (int d = 0; d < world; ++d) {
        int64_t c = 0;
        for (int64_t b = 0; b < nb; ++b) c += hc[(size_t)(d * nb + b)];
        counts_out[d] = c;
        total += c;
    }
    if (!rows || capacity < total) return total;
    if (total >= (int64_t)INT32_MAX) throw ArgError{"route: more than 2^31 rows"};
    std::vector<int32_t> ho((size_t)(nb * world));
    int64_t run = 0;
    for (size_t k = 0; k < ho.size(); ++k) {
        ho[k] = (int32_t)run;
        run += hc[k];
    }
    DBSCAN_HIP_CHECK(hipMemcpyAsync(off, ho.data(), ho.size() * sizeof(int32_t),
                                    hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(route_write_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, x, y, m, start,
                       world, dzc, off, rows);
    DBSCAN_HIP_CHECK(hipGetLastError());
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));  // (the host vectors go out of scope)
    return total;
}

// dbscan_train_node: the slab plan, the slab fits, the merge and the labels all on the
// devices (round 4; rounds 1-3 built the plan and merged on the host: 16.9 s for 10^9 points on
// one GPU, 7.3 s of it the host plan).  Per device (one host thread and one handle each; shard
// s on device s % device_count):
//   A  upload x, y; for each of its shards: zone + ordered compaction (plan_*_kernel), the lean
//      slab fit (dbscan_slab_fit_shared_device_async: roots at the shared points only), the
//      merge records (gid, root gid) -> host
//   B  (host) every shard's records, concatenated
//   C  union of all records on each device (dbscan_merge_union_device: the same lock-free
//      union as node.py's ranks), each shard's local roots -> global s(K) and its owned global
//      roots (dbscan_slab_merge_roots_device) -> host
//   D  (host) the owned roots of all shards, sorted: cluster id = 1 + rank of s(K)
//   E  per shard: re-fit when its device held other shards since (one workspace per device),
//      label (dbscan_slab_label_device), scatter the zone-0 labels into the output by gid;
//      one device: the whole output on the device, one copy back; several: each device's
//      labels copied back and scattered by host threads.
int32_t train_node(const double* x, const double* y, int64_t n, double eps, int32_t min_points,
                   int32_t mode, int32_t n_shards, int32_t* cluster_out, uint8_t* flag_out,
                   int64_t* n_clusters_out, std::string* err) {
    const int ndev = dbscan_device_count();
    if (ndev <= 0) {
        *err = "no HIP device visible";
        return DBSCAN_EHIP;
    }
    if (n_shards <= 0) n_shards = ndev;
    PhaseTrace tr;
    const std::vector<double> cuts = make_cuts(x, n, n_shards, eps);
    tr.mark("cuts");
    if (cuts.empty()) {  // one slab (or eps*eps not finite: all-pairs / no-pairs do not shard)
        g_node_record.device.assign(1, 0);
        g_node_record.points.assign(1, n);
        g_node_record.shared.assign(1, 0);
        dbscan_handle* h = dbscan_create(0);
        if (!h) {
            *err = dbscan_last_error();
            return DBSCAN_EHIP;
        }
        int32_t k = 0;
        const int32_t rc = dbscan_fit_h(h, x, y, n, eps, min_points, mode, cluster_out, flag_out, &k);
        if (rc != DBSCAN_OK) *err = dbscan_last_error();
        dbscan_destroy(h);
        *n_clusters_out = k;
        return rc;
    }
    if (n >= (int64_t)INT32_MAX) {
        *err = "dbscan_train_node: more than 2^31 - 1 points";
        return DBSCAN_EARG;
    }
    const int world = (int)cuts.size() + 1;
    const std::vector<ZoneCut> zc = zone_cuts(world, cuts, reach(eps));
    const NodePlan plan = node_plan(world, ndev);
    const int nworkers = plan.nworkers;
    const bool shared_dev = world > nworkers;
    NodeRecord& rec = g_node_record;
    rec.device.assign((size_t)world, -1);
    rec.points.assign((size_t)world, 0);
    rec.shared.assign((size_t)world, 0);
    std::vector<DevShard> sh(world);
    std::vector<dbscan_handle*> hs(nworkers, nullptr);
    for (int w = 0; w < nworkers; ++w) {
        hs[w] = dbscan_create(w);
        if (!hs[w]) {
            *err = dbscan_last_error();
            for (auto* h : hs)
                if (h) dbscan_destroy(h);
            return DBSCAN_EHIP;
        }
    }
    struct Dev {  // per device: the union's parent array and records, output arrays
        int32_t* parent = nullptr;
        int64_t *ra = nullptr, *rb = nullptr, *roots = nullptr;
        int32_t* out_cl = nullptr;
        uint8_t* out_fl = nullptr;
    };
    std::vector<Dev> dv(nworkers);
    std::vector<WorkerStatus> wst(nworkers);
    // runs f(w) on one host thread per device; a failure of any kind is recorded per device
    auto each_device = [&](auto&& f) {
        return run_workers(nworkers, wst, [&](int w) {
            hcheck(hipSetDevice(w), "hipSetDevice");
            f(w);
        });
    };
    auto lean_fit = [&](int r, int w) {
        DevShard& s = sh[r];
        ccheck(dbscan_slab_fit_shared_device_async(hs[w], s.x, s.y, s.zone, s.m, eps, min_points,
                                                   s.shared, s.ns, s.core, s.root));
    };
    int32_t rc = DBSCAN_OK;
    int64_t nroots = 0;
    std::vector<int64_t> all_roots;
    const bool ok = [&]() {
        // ---- A: plan + lean slab fits + records ----
        if (!each_device([&](int w) {
                hipStream_t st = static_cast<hipStream_t>(dbscan_stream(hs[w]));
                double *dx = nullptr, *dy = nullptr;
                int32_t* cnt = nullptr;
                const int64_t nb = (n + kPlanTile - 1) / kPlanTile;
                try {
                    hcheck(hipMalloc(&dx, n * sizeof(double)), "upload");
                    hcheck(hipMalloc(&dy, n * sizeof(double)), "upload");
                    hcheck(hipMalloc(&cnt, (4 * nb + 4) * sizeof(int32_t)), "plan");
                    hcheck(hipMemcpyAsync(dx, x, n * sizeof(double), hipMemcpyHostToDevice, st),
                           "upload");
                    hcheck(hipMemcpyAsync(dy, y, n * sizeof(double), hipMemcpyHostToDevice, st),
                           "upload");
                    int32_t* cs = cnt;
                    int32_t* ch = cnt + nb;
                    int32_t* os = cnt + 2 * nb;
                    int32_t* oh = cnt + 3 * nb;
                    int32_t* tot = cnt + 4 * nb;
                    dbscan::Workspace scratch;  // (the scans' look-back state)
                    for (int r : plan.shards_of[(size_t)w]) {
                        DevShard& s = sh[r];
                        int dev = -1;
                        hcheck(hipGetDevice(&dev), "hipGetDevice");
                        rec.device[(size_t)r] = dev;
                        hipLaunchKernelGGL(plan_count_kernel, dim3((unsigned)nb), dim3(kBlock), 0,
                                           st, dx, n, r, world, zc[r], cs, ch);
                        hcheck(hipGetLastError(), "plan count");
                        exclusive_scan(st, 0, cs, os, nb, tot, scratch.scan);
                        exclusive_scan(st, 0, ch, oh, nb, tot + 1, scratch.scan);
                        int32_t t2[2];
                        hcheck(hipMemcpyAsync(t2, tot, sizeof(t2), hipMemcpyDeviceToHost, st),
                               "plan");
                        hcheck(hipStreamSynchronize(st), "plan");
                        s.m = t2[0];
                        s.ns = t2[1];
                        rec.points[(size_t)r] = s.m;
                        rec.shared[(size_t)r] = s.ns;
                        const int64_t m = std::max<int64_t>(1, s.m);
                        hcheck(hipMalloc(&s.x, m * sizeof(double)), "shard");
                        hcheck(hipMalloc(&s.y, m * sizeof(double)), "shard");
                        hcheck(hipMalloc(&s.zone, m), "shard");
                        hcheck(hipMalloc(&s.core, m), "shard");
                        hcheck(hipMalloc(&s.gid, m * sizeof(int64_t)), "shard");
                        hcheck(hipMalloc(&s.gs, m * sizeof(int64_t)), "shard");
                        hcheck(hipMalloc(&s.root, m * sizeof(int32_t)), "shard");
                        hcheck(hipMalloc(&s.shared, std::max<int64_t>(1, s.ns) * sizeof(int64_t)),
                               "shard");
                        hipLaunchKernelGGL(plan_write_kernel, dim3((unsigned)nb), dim3(kBlock), 0,
                                           st, dx, dy, n, r, world, zc[r], os, oh, s.x, s.y,
                                           s.zone, s.gid, s.shared);
                        hcheck(hipGetLastError(), "plan write");
                        if (s.m == 0) continue;
                        lean_fit(r, w);
                        s.a.resize((size_t)s.ns);
                        s.b.resize((size_t)s.ns);
                        if (s.ns > 0) {
                            int64_t* rec = nullptr;
                            hcheck(hipMalloc(&rec, 2 * s.ns * sizeof(int64_t)), "records");
                            hipLaunchKernelGGL(plan_records_kernel, dim3(nblocks(s.ns)),
                                               dim3(kBlock), 0, st, s.shared, s.ns, s.gid, s.core,
                                               s.root, rec, rec + s.ns);
                            hcheck(hipMemcpyAsync(s.a.data(), rec, s.ns * sizeof(int64_t),
                                                  hipMemcpyDeviceToHost, st), "records");
                            hcheck(hipMemcpyAsync(s.b.data(), rec + s.ns, s.ns * sizeof(int64_t),
                                                  hipMemcpyDeviceToHost, st), "records");
                            hcheck(hipStreamSynchronize(st), "records");
                            (void)hipFree(rec);
                        }
                        ccheck(dbscan_sync(hs[w]));
                    }
                } catch (...) {
                    (void)hipFree(dx);
                    (void)hipFree(dy);
                    (void)hipFree(cnt);
                    throw;
                }
                (void)hipFree(dx);
                (void)hipFree(dy);
                (void)hipFree(cnt);
            }))
            return false;
        tr.mark("plan + slab fits");
        // ---- B: all records ----
        std::vector<int64_t> A, B;
        for (auto& s : sh) {
            A.insert(A.end(), s.a.begin(), s.a.end());
            B.insert(B.end(), s.b.begin(), s.b.end());
            std::vector<int64_t>().swap(s.a);
            std::vector<int64_t>().swap(s.b);
        }
        const int64_t nrec = (int64_t)A.size();
        // ---- C: the union on every device, global s(K) per local root, owned roots ----
        if (!each_device([&](int w) {
                hipStream_t st = static_cast<hipStream_t>(dbscan_stream(hs[w]));
                Dev& d = dv[w];
                hcheck(hipMalloc(&d.parent, n * sizeof(int32_t)), "merge");
                hcheck(hipMemsetAsync(d.parent, 0xFF, n * sizeof(int32_t), st), "merge");
                hcheck(hipMalloc(&d.ra, std::max<int64_t>(1, nrec) * sizeof(int64_t)), "merge");
                hcheck(hipMalloc(&d.rb, std::max<int64_t>(1, nrec) * sizeof(int64_t)), "merge");
                if (nrec > 0) {
                    hcheck(hipMemcpyAsync(d.ra, A.data(), nrec * sizeof(int64_t),
                                          hipMemcpyHostToDevice, st), "merge");
                    hcheck(hipMemcpyAsync(d.rb, B.data(), nrec * sizeof(int64_t),
                                          hipMemcpyHostToDevice, st), "merge");
                    ccheck(dbscan_merge_union_device(d.ra, d.rb, nrec, d.parent, st));
                }
                for (int r : plan.shards_of[(size_t)w]) {
                    DevShard& s = sh[r];
                    if (s.m == 0) continue;
                    int64_t* own = nullptr;
                    hcheck(hipMalloc(&own, s.m * sizeof(int64_t)), "roots");
                    int64_t k = 0;
                    const int32_t rc2 = dbscan_slab_merge_roots_device(
                        hs[w], s.m, s.zone, s.gid, s.root, d.parent, s.gs, own, &k);
                    if (rc2 == DBSCAN_OK) {
                        s.own.resize((size_t)k);
                        const hipError_t e = k > 0 ? hipMemcpyAsync(s.own.data(), own,
                                                                    k * sizeof(int64_t),
                                                                    hipMemcpyDeviceToHost, st)
                                                   : hipSuccess;
                        const hipError_t e2 = hipStreamSynchronize(st);
                        (void)hipFree(own);
                        hcheck(e, "roots");
                        hcheck(e2, "roots");
                    } else {
                        (void)hipFree(own);
                        throw rc2;
                    }
                }
                (void)hipFree(d.ra);
                (void)hipFree(d.rb);
                (void)hipFree(d.parent);
                d.ra = d.rb = nullptr;
                d.parent = nullptr;
            }))
            return false;
        // ---- D: numbering ----
        for (auto& s : sh) all_roots.insert(all_roots.end(), s.own.begin(), s.own.end());
        std::sort(all_roots.begin(), all_roots.end());
        nroots = (int64_t)all_roots.size();
        tr.mark("merge + numbering");
        // ---- E: labels ----
        const bool one = nworkers == 1;
        std::vector<std::vector<int32_t>> hcl(world);
        std::vector<std::vector<uint8_t>> hfl(world);
        std::vector<std::vector<int64_t>> hgid(world);
        if (!each_device([&](int w) {
                hipStream_t st = static_cast<hipStream_t>(dbscan_stream(hs[w]));
                Dev& d = dv[w];
                hcheck(hipMalloc(&d.roots, std::max<int64_t>(1, nroots) * sizeof(int64_t)), "label");
                if (nroots > 0)
                    hcheck(hipMemcpyAsync(d.roots, all_roots.data(), nroots * sizeof(int64_t),
                                          hipMemcpyHostToDevice, st), "label");
                if (one) {
                    hcheck(hipMalloc(&d.out_cl, n * sizeof(int32_t)), "output");
                    hcheck(hipMalloc(&d.out_fl, n), "output");
                }
                for (int r : plan.shards_of[(size_t)w]) {
                    DevShard& s = sh[r];
                    if (s.m == 0) continue;
                    if (shared_dev) lean_fit(r, w);  // (the handle's last fit was another shard's)
                    int32_t* cl = nullptr;
                    uint8_t* fl = nullptr;
                    hcheck(hipMalloc(&cl, s.m * sizeof(int32_t)), "label");
                    hcheck(hipMalloc(&fl, s.m), "label");
                    const int32_t rc2 = dbscan_slab_label_device(hs[w], s.zone, s.gid, s.gs,
                                                                 d.roots, nroots, mode, cl, fl);
                    if (rc2 != DBSCAN_OK) {
                        (void)hipFree(cl);
                        (void)hipFree(fl);
                        throw rc2;
                    }
                    if (one) {
                        hipLaunchKernelGGL(plan_scatter_kernel, dim3(nblocks(s.m)), dim3(kBlock),
                                           0, st, s.m, s.zone, s.gid, cl, fl, d.out_cl, d.out_fl);
                        hcheck(hipGetLastError(), "label scatter");
                    } else {  // several devices: the slab-order labels and gids back to the host
                        hcl[r].resize((size_t)s.m);
                        hfl[r].resize((size_t)s.m);
                        hgid[r].resize((size_t)s.m);
                        hcheck(hipMemcpyAsync(hcl[r].data(), cl, s.m * sizeof(int32_t),
                                              hipMemcpyDeviceToHost, st), "label");
                        hcheck(hipMemcpyAsync(hfl[r].data(), fl, s.m, hipMemcpyDeviceToHost, st),
                               "label");
                        hcheck(hipMemcpyAsync(hgid[r].data(), s.gid, s.m * sizeof(int64_t),
                                              hipMemcpyDeviceToHost, st), "label");
                    }
                    hcheck(hipStreamSynchronize(st), "label");
                    (void)hipFree(cl);
                    (void)hipFree(fl);
                    if (!one) {  // zone-0 flags of the slab for the host scatter
                        std::vector<uint8_t> z((size_t)s.m);
                        hcheck(hipMemcpy(z.data(), s.zone, s.m, hipMemcpyDeviceToHost), "label");
                        for (int64_t p = 0; p < s.m; ++p)
                            if (z[(size_t)p] != 0) hgid[r][(size_t)p] = -1;
                    }
                    s.release();
                }
                if (one) {
                    hcheck(hipMemcpyAsync(cluster_out, d.out_cl, n * sizeof(int32_t),
                                          hipMemcpyDeviceToHost, st), "output");
                    hcheck(hipMemcpyAsync(flag_out, d.out_fl, n, hipMemcpyDeviceToHost, st),
                           "output");
                    hcheck(hipStreamSynchronize(st), "output");
                }
                (void)hipFree(d.roots);
                (void)hipFree(d.out_cl);
                (void)hipFree(d.out_fl);
                d.roots = nullptr;
                d.out_cl = nullptr;
                d.out_fl = nullptr;
            }))
            return false;
        tr.mark("slab labels + output");
        if (!one) {  // host scatter of every shard's zone-0 labels (disjoint writes)
            const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), n / 65536 + 1));
            parallel_for(nth, [&](int t) {
                for (int r = 0; r < world; ++r) {
                    const int64_t m = (int64_t)hgid[r].size(), p0 = m * t / nth,
                                  p1 = m * (t + 1) / nth;
                    for (int64_t p = p0; p < p1; ++p) {
                        const int64_t g = hgid[r][(size_t)p];
                        if (g < 0) continue;
                        cluster_out[g] = hcl[r][(size_t)p];
                        flag_out[g] = hfl[r][(size_t)p];
                    }
                }
            });
            tr.mark("output scatter");
        }
        return true;
    }();
    if (!ok) {
        rc = first_failure(wst, err);
        if (rc == DBSCAN_OK) rc = DBSCAN_EHIP;
    }
    for (int w = 0; w < nworkers; ++w) {
        (void)hipSetDevice(w);
        Dev& d = dv[w];
        for (void* p : {(void*)d.parent, (void*)d.ra, (void*)d.rb, (void*)d.roots,
                        (void*)d.out_cl, (void*)d.out_fl})
            (void)hipFree(p);
        for (int r : plan.shards_of[(size_t)w]) sh[r].release();
    }
    for (auto* h : hs) dbscan_destroy(h);
    if (rc == DBSCAN_OK) *n_clusters_out = nroots;
    tr.mark("teardown");
    return rc;
}

}  // namespace dbscan
