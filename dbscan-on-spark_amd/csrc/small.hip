// small.hip -- the local fit of one partition held entirely in LDS, in one launch, for the
// partition sizes DBSCAN.train hands the seam, and its batched form.
//
// DBSCAN.scala:150-155 calls `new LocalDBSCANNaive(eps, minPoints).fit(points)` once per spatial
// partition: at most maxPointsPerPartition points (EvenSplitPartitioner.scala:44-209) plus the
// eps halo (DBSCAN.scala:116-137) -- hundreds to ~10^4 points.  The tiled pipeline of fit.hip is
// ~45 launches whose fixed cost dominates at that size; here a partition of <= kSmallMaxPoints
// points is fitted in one launch: by one workgroup of 1024 threads (small_fit_kernel; a batch of
// an executor's partitions is one launch with one workgroup per partition, dbscan_fit_batch), or
// by ~n/256 workgroups that each stage the whole partition and meet at two grid barriers
// (spread_fit_kernel, below).
//
// Same closed form as fit.hip (LocalDBSCANNaive.scala:37-118,
// LocalDBSCANArchery.scala:103-106), same fp64 predicate (DBSCANPoint.scala:26-30), same results
// bit for bit, partition-local cluster ids 1..k in the order the reference opens them:
//   load    x, y of the partition (fp64, coalesced) into registers; bbox of the finite points
//   grid    cells of side >= eps (the 3x3 stencil holds every accepted pair, DESIGN.md "grid
//           soundness"), the side doubled along the longer axis until the dense cell table fits
//           kSmCells entries
//   sort    counting sort by cell in LDS (histogram with LDS atomics, scan, scatter); each slot
//           keeps an fp32 record of its coordinates (units of the base cell side, origin at the
//           bbox centre) and (visit index << 16 | cell)
//   count   each slot scans the 3 row ranges of its stencil, early exit at minPoints; the fp32
//           pre-filter decides far from the threshold (band sized from the records' magnitude,
//           below), the exact fp64 predicate on the global coordinates inside the band
//   union   union-find in LDS over core-core pairs, each unordered pair once; the root with the
//           larger visit index is hooked under the smaller, so a root IS s(K)
//   number  roots flagged by visit index, popcount scan: cluster id = 1 + roots before s(K)
//   label   cores: their root's id; non-cores: min s(K) over core neighbours + the Naive /
//           Archery rule; written in input order
// The order of the slots inside a cell depends on LDS atomics; nothing above depends on it.
//
// fp32 pre-filter bound.  u = fl64((v*0.5 - c*0.5) * (2/h0)) is the coordinate in units of the
// base side h0 (= eps-ish), |u| <= Rr; r = fl32(u), |r - u| <= 2^-24 Rr; the fp64 steps add a
// common scale error (relative ~2^-51) that only matters far below the band.  For a pair near
// the threshold (|du| <= ~1 per axis) dx_f = fl32(r_q - r_p) is within E = 2^-23 (Rr + 1) of
// the exact scaled difference, so F = fl32(dx_f^2 + dy_f^2) (one fused step or two roundings)
// is within 4E + 2E^2 + 2^-22 e2 of d^2/h0^2, e2 = eps2/h0^2.  With M = 2^-20 (Rr + 4) +
// 2^-20 e2 (> twice that): F <= rd(e2 - M) => the reference's fp64 d2 <= eps2 holds;
// F > ru(e2 + M) => it does not; otherwise the fp64 predicate runs on the two points' global
// coordinates.  Rr > 2^20 (absurd extents against eps) turns the pre-filter off: every
// candidate takes the exact path.
#include "../../include/dbscan_hip.h"
#include "internal.h"

#include <algorithm>
#include <cmath>
#include <vector>

namespace dbscan {
namespace {

constexpr int kSmT = 1024;                  // threads per workgroup
constexpr int kSmW = kSmT / 64;             // waves per workgroup
constexpr int kSmN = (int)kSmallMaxPoints;  // points a workgroup holds
constexpr int kSmPer = kSmN / kSmT;         // points per thread in the load phase
constexpr int kSmCells = 8192;              // dense cell table entries
constexpr int kSmCellPer = kSmCells / kSmT;
constexpr uint32_t kNoCell = 0xFFFFu;
constexpr uint32_t kCellMask = 0x1FFFu;  // info: visit << 16 | quadrant << 13 | cell
static_assert(kSmN % kSmT == 0 && kSmCells % kSmT == 0, "whole rounds per thread");

// DBSCAN_AB_STAMPS (timing builds only, never the shipped library): thread 0 of workgroup 0
// records the 100 MHz clock at the phase boundaries (dbscan_ab_small_stamps).
#if DBSCAN_AB_STAMPS
__device__ long long g_sm_stamps[24];
#define SM_STAMP(k)                                                               \
    do {                                                                          \
        if (threadIdx.x == 0 && blockIdx.x == 0) g_sm_stamps[(k)] = wall_clock64(); \
    } while (0)
// band_fit_kernel, every workgroup: [g][0..7] = clock at the stage's end, the count's end,
// after barrier 1, at barrier 2's arrival; own points, staged points; clock before and after
// the union walks
__device__ long long g_band_wg[64 * 12];
#define BAND_WG(k, v)                                           \
    do {                                                        \
        if (threadIdx.x == 0) g_band_wg[blockIdx.x * 12 + (k)] = (v); \
    } while (0)
#else
#define BAND_WG(k, v) \
    do {              \
    } while (0)
#define SM_STAMP(k) \
    do {            \
    } while (0)
#endif
static_assert(kSmN <= 65536 && kSmCells < 65535, "16-bit visit indices, cells and cell starts");

// DBSCANPoint.scala:26-30 as used at LocalDBSCANNaive.scala:77 (no FMA: -ffp-contract=off and
// the pragma)
__device__ __forceinline__ bool sm_within(double px, double py, double ox, double oy,
                                          double eps2) {
#pragma clang fp contract(off)
    const double dx = ox - px;
    const double dy = oy - py;
    const double a = dx * dx;
    const double b = dy * dy;
    return (a + b) <= eps2;
}

__device__ __forceinline__ float sm_d2(float2 a, float2 b) {
    const float dx = b.x - a.x, dy = b.y - a.y;
    return __builtin_fmaf(dx, dx, dy * dy);
}

struct SmGrid {
    double xmin2, ymin2, invx, invy;  // cell = floor((v*0.5 - vmin*0.5) * inv), as make_grid
    double cx2, cy2, invs;            // record = fl32((v*0.5 - c*0.5) * invs)
    float lo, hi;                     // F <= lo: neighbour; F > hi: not; else exact fp64
    int nx, ny, ncells, nf, exact_only, bad;
    int clique;  // the side was not grown and <= |eps|*(1+2^-14): quarter cells are cliques
    int swap;    // band grids: x and y exchanged (rows along the input's x axis)
};

// Workgroup exclusive scan of one int per thread; *total = the sum.  ws: kSmW + 1 ints.
__device__ int sm_excl_scan(int v, int* ws, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    if (w == 0) {
        const int s = lane < kSmW ? ws[lane] : 0;
        int si = s;
#pragma unroll
        for (int o = 1; o < kSmW; o <<= 1) {
            const int u = __shfl_up(si, o, 64);
            if (lane >= o) si += u;
        }
        if (lane < kSmW) ws[lane] = si - s;
        if (lane == kSmW - 1) ws[kSmW] = si;
    }
    __syncthreads();
    const int r = ws[w] + incl - v;
    *total = ws[kSmW];
    __syncthreads();
    return r;
}

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

// Union-find over slots in LDS.  Parents always have a strictly smaller visit index than their
// children (roots are hooked larger-under-smaller), so there are no cycles and path halving
// only ever shortcuts to an ancestor.
__device__ __forceinline__ int sm_ld(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int sm_find(int* par, int x) {
    while (true) {
        const int p = sm_ld(par + x);
        if (p == x) return x;
        const int g = sm_ld(par + p);
        if (g != p) __hip_atomic_store(par + x, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        x = g;
    }
}
// Unites a's and b's sets from ra, a (possibly stale) root of a's set, hooking the root with the
// larger visit index under the other; returns a root of the merged set at the
// time of the hook (an ancestor of every member of both sets since), so the caller's next walk
// starts from it instead of finding a's root again from a.
__device__ int sm_unite_from(int* par, const uint32_t* info, int ra, int b) {
    while (true) {
        ra = sm_find(par, ra);
        b = sm_find(par, b);
        if (ra == b) return ra;
        int hi = ra, lo = b;  // hi: the root with the larger visit index, hooked under lo
        if ((info[ra] >> 16) < (info[b] >> 16)) {
            hi = b;
            lo = ra;
        }
        if (atomicCAS(par + hi, hi, lo) == hi) return lo;
    }
}

// The grid of one partition (one thread).  Sides as make_grid (fit.hip): >= R*(1+2^-16) with
// R = max(|eps|*(1+2^-40), 2^-500); doubled along the axis with more cells until nx*ny fits.
__device__ void sm_make_grid(double xmin, double xmax, double ymin, double ymax, int nf,
                             double eps, double eps2, SmGrid* g) {
    g->nf = nf;
    g->bad = 0;
    g->exact_only = 0;
    g->nx = g->ny = g->ncells = 1;
    g->clique = 0;
    if (nf == 0) return;
    double R = fabs(eps) * (1.0 + 0x1p-40);
    if (R < 0x1p-500) R = 0x1p-500;
    const double h0 = R * (1.0 + 0x1p-16);
    double hx = h0, hy = h0;
    auto cells = [](double vmax, double vmin, double h) {
        return floor((vmax * 0.5 - vmin * 0.5) * (2.0 / h)) + 1.0;
    };
    bool ok = false;
    double cx = 1, cy = 1;
    for (int it = 0; it < 4096; ++it) {
        cx = cells(xmax, xmin, hx);
        cy = cells(ymax, ymin, hy);
        if (cx * cy <= (double)kSmCells) {
            ok = true;
            break;
        }
        if (cx >= cy) hx *= 2.0; else hy *= 2.0;
    }
    if (!ok) {
        g->bad = 1;
        return;
    }
    g->nx = (int)cx;
    g->ny = (int)cy;
    g->clique = (hx == h0 && hy == h0 && h0 <= fabs(eps) * (1.0 + 0x1p-14)) ? 1 : 0;
    g->ncells = g->nx * g->ny;
    g->xmin2 = xmin * 0.5;
    g->ymin2 = ymin * 0.5;
    g->invx = 2.0 / hx;
    g->invy = 2.0 / hy;
    // fp32 records around the bbox centre, in units of h0
    g->cx2 = xmin * 0.5 + (xmax * 0.5 - xmin * 0.5) * 0.5;
    g->cy2 = ymin * 0.5 + (ymax * 0.5 - ymin * 0.5) * 0.5;
    g->invs = 2.0 / h0;
    const double rr = fmax((xmax * 0.5 - xmin * 0.5), (ymax * 0.5 - ymin * 0.5)) * g->invs * 0.5 +
                      1.0;
    const double e2 = eps2 * (0.5 * g->invs) * (0.5 * g->invs);
    if (!(rr <= 0x1p20) || !(e2 <= 0x1p20)) {
        g->exact_only = 1;
        g->lo = 0.f;
        g->hi = 0.f;
        return;
    }
    const double M = (rr + 4.0) * 0x1p-20 + e2 * 0x1p-20;
    g->lo = __double2float_rd(e2 - M);
    g->hi = __double2float_ru(e2 + M);
}

// A partition staged in one workgroup's LDS (small_fit_kernel, spread_fit_kernel).
struct SmLds {
    float2 rec[kSmN];           // fp32 records by slot
    uint32_t info[kSmN];        // visit index << 16 | quadrant << 13 | cell (kNoCell: no cell)
    int par[kSmN];              // sort cursors, then union-find parents
    uint16_t cst[kSmCells + 2];  // first slot of every cell; cst[ncells] = nf
    uint8_t core[kSmN];         // by slot
    uint32_t rbits[kSmN / 32];  // roots by visit index
    int wrank[kSmN / 32];       // roots before each word
    double red[5][kSmW];
    int wsc[kSmW + 1];
    int nonfin;
    int band[8];  // spread fits: the union's slots [band[0], band[1]), the published pair count
                  // band[2], the count's and labels' slots [band[4], band[5])
    SmGrid G;
    uint32_t sbest[kSmT / 3 + 1];  // row-split phases: per-point counters / min roots
};

// What the stencil walks read in registers (from L.G, once per kernel)
struct SmCtx {
    const double* px;
    const double* py;
    double eps2;
    float lo, hi;
    int nx, ny;
    bool exact_only;
};

// ---- load + bbox + grid + counting sort by cell (points [0, m) of px, py) ----
// false: the grid could not be sized.  occupied: this thread's share of the occupied cells.
// The order of the slots inside a cell depends on LDS atomics; nothing computed from the stage
// depends on it (spread_fit_kernel's workgroups each stage the partition, in their own order).
__device__ __forceinline__ bool sm_stage(SmLds& L, const double* __restrict__ px,
                                         const double* __restrict__ py, int m, double eps,
                                         double eps2, int& occupied) {
    const int tid = threadIdx.x;
    double vx[kSmPer], vy[kSmPer];
    double mnx = INFINITY, mxx = -INFINITY, mny = INFINITY, mxy = -INFINITY, nfin = 0;
#pragma unroll
    for (int k = 0; k < kSmPer; ++k) {
        const int i = tid + k * kSmT;
        vx[k] = 0;
        vy[k] = 0;
        if (i < m) {
            vx[k] = px[i];
            vy[k] = py[i];
            if (isfinite(vx[k]) && isfinite(vy[k])) {
                mnx = fmin(mnx, vx[k]);
                mxx = fmax(mxx, vx[k]);
                mny = fmin(mny, vy[k]);
                mxy = fmax(mxy, vy[k]);
                nfin += 1;
            }
        }
    }
    if (tid < kSmN / 32) L.rbits[tid] = 0;
    if (tid == 0) L.nonfin = 0;
    {
        const int lane = tid & 63, w = tid >> 6;
        mnx = wave_min(mnx);
        mxx = wave_max(mxx);
        mny = wave_min(mny);
        mxy = wave_max(mxy);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nfin += __shfl_xor(nfin, o, 64);
        if (lane == 0) {
            L.red[0][w] = mnx;
            L.red[1][w] = mxx;
            L.red[2][w] = mny;
            L.red[3][w] = mxy;
            L.red[4][w] = nfin;
        }
        __syncthreads();
        if (tid == 0) {
            for (int k = 1; k < kSmW; ++k) {
                L.red[0][0] = fmin(L.red[0][0], L.red[0][k]);
                L.red[1][0] = fmax(L.red[1][0], L.red[1][k]);
                L.red[2][0] = fmin(L.red[2][0], L.red[2][k]);
                L.red[3][0] = fmax(L.red[3][0], L.red[3][k]);
                L.red[4][0] += L.red[4][k];
            }
            sm_make_grid(L.red[0][0], L.red[1][0], L.red[2][0], L.red[3][0], (int)L.red[4][0], eps,
                         eps2, &L.G);
        }
        __syncthreads();
    }
    SM_STAMP(1);
    if (L.G.bad) return false;  // (unreachable for finite bboxes: 4096 doublings span any extent)
    const int nf = L.G.nf, nx = L.G.nx, ny = L.G.ny, ncells = L.G.ncells;

    for (int c = tid; c < ncells; c += kSmT) L.par[c] = 0;
    __syncthreads();
    int mycell[kSmPer];
#pragma unroll
    for (int k = 0; k < kSmPer; ++k) {
        const int i = tid + k * kSmT;
        mycell[k] = -1;
        if (i < m && isfinite(vx[k]) && isfinite(vy[k])) {
            // quarter-grid coordinates: floor(2t) >> 1 == floor(t) exactly (2t is exact)
            int qx = (int)floor(2.0 * ((vx[k] * 0.5 - L.G.xmin2) * L.G.invx));
            int qy = (int)floor(2.0 * ((vy[k] * 0.5 - L.G.ymin2) * L.G.invy));
            qx = min(max(qx, 0), 2 * nx - 1);
            qy = min(max(qy, 0), 2 * ny - 1);
            const int c = (qy >> 1) * nx + (qx >> 1);
            mycell[k] = c | (((qy & 1) << 1 | (qx & 1)) << 13);
            atomicAdd(&L.par[c], 1);
        }
    }
    __syncthreads();
    occupied = 0;
    {
        int cnt[kSmCellPer], sum = 0;
#pragma unroll
        for (int k = 0; k < kSmCellPer; ++k) {
            const int c = tid * kSmCellPer + k;
            cnt[k] = c < ncells ? L.par[c] : 0;
            sum += cnt[k];
            occupied += cnt[k] > 0 ? 1 : 0;
        }
        int tot = 0;
        int run = sm_excl_scan(sum, L.wsc, &tot);
#pragma unroll
        for (int k = 0; k < kSmCellPer; ++k) {
            const int c = tid * kSmCellPer + k;
            if (c < ncells) {
                L.par[c] = run;
                L.cst[c] = (uint16_t)run;
            }
            run += cnt[k];
        }
        if (tid == 0) L.cst[ncells] = (uint16_t)nf;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmPer; ++k) {
        const int i = tid + k * kSmT;
        if (i >= m) continue;
        if (mycell[k] >= 0) {
            const int s = atomicAdd(&L.par[mycell[k] & kCellMask], 1);
            L.rec[s] = make_float2((float)((vx[k] * 0.5 - L.G.cx2) * L.G.invs),
                                   (float)((vy[k] * 0.5 - L.G.cy2) * L.G.invs));
            L.info[s] = ((uint32_t)i << 16) | (uint32_t)mycell[k];
        } else {
            const int s = nf + atomicAdd(&L.nonfin, 1);
            L.info[s] = ((uint32_t)i << 16) | kNoCell;
        }
    }
    __syncthreads();
    return true;
}

__device__ __forceinline__ SmCtx sm_ctx(const SmLds& L, const double* px, const double* py,
                                        double eps2) {
    return {px, py, eps2, L.G.lo, L.G.hi, L.G.nx, L.G.ny, L.G.exact_only != 0};
}

// neighbour test of slots p (record me) and q (record rq).  (The stencil helpers take the LDS
// layout as a template: SmLds, the whole partition; BandLds, one band of it.)
template <class LT>
__device__ __forceinline__ bool sm_pair(const LT& L, const SmCtx& c, int p, float2 me, int q,
                                        float2 rq) {
    if (!c.exact_only) {
        const float F = sm_d2(me, rq);
        if (F <= c.lo) return true;
        if (F > c.hi) return false;
    }
    const int vp = (int)(L.info[p] >> 16), vq = (int)(L.info[q] >> 16);
    return sm_within(c.px[vp], c.py[vp], c.px[vq], c.py[vq], c.eps2);
}

// f(q, rec[q], w) for every slot q >= qmin of slot p's 3x3 stencil (three row ranges, own row
// first), w = the 6x6 quarter-window position of q's cell: (row 0..2) * 3 + col 0..2 (rows cy-1,
// cy, cy+1 -> 0, 1, 2); f returns false to stop.  The candidates' records are loaded kSmBatch at
// a time (their LDS reads in flight together: the walks are bound by the latency of dependent
// LDS reads, not by their count).  only = 0..2: that row alone (row-split phases), -1: all three.
constexpr int kSmBatch = 4;
template <class LT, class F>
__device__ __forceinline__ void sm_for_stencil(const LT& L, const SmCtx& cx_, int p, int qmin,
                                               F&& f, int only) {
    const int nx = cx_.nx, ny = cx_.ny;
    const int c = (int)(L.info[p] & kCellMask);
    const int cy = c / nx, cx = c - cy * nx;
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, nx - 1);
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        if (only >= 0 && d != only) continue;
        const int r = d == 0 ? cy : (d == 1 ? cy - 1 : cy + 1);
        if (r < 0 || r >= ny) continue;
        const int rb = r * nx;
        const int e = L.cst[rb + x1 + 1];
        // boundaries of the row's second and third cell (q's column = x0 + crossings)
        const int b1 = x0 + 1 <= x1 ? (int)L.cst[rb + x0 + 1] : 0x7FFFFFFF;
        const int b2 = x0 + 2 <= x1 ? (int)L.cst[rb + x0 + 2] : 0x7FFFFFFF;
        const int wr = (r - cy + 1) * 3 + (x0 - cx + 1);
        for (int q = max((int)L.cst[rb + x0], qmin); q < e; q += kSmBatch) {
            float2 rq[kSmBatch];
#pragma unroll
            for (int u = 0; u < kSmBatch; ++u) rq[u] = L.rec[min(q + u, e - 1)];
#pragma unroll
            for (int u = 0; u < kSmBatch; ++u) {
                const int qq = q + u;
                if (qq < e && !f(qq, rq[u], wr + (qq >= b1 ? 1 : 0) + (qq >= b2 ? 1 : 0)))
                    return;
            }
        }
    }
}

// |N(p)| capped at minPoints over stencil row `only` (-1: all rows; LocalDBSCANNaive.scala:52-56)
template <class LT>
__device__ __forceinline__ int sm_count(const LT& L, const SmCtx& c, int p, int min_points,
                                        int only) {
    const float2 me = L.rec[p];
    int cnt = 0;
    sm_for_stencil(L, c, p, 0, [&](int q, float2 rq, int) {
        cnt += sm_pair(L, c, p, me, q, rq) ? 1 : 0;
        return cnt < min_points;
    }, only);
    return cnt;
}

// Core p's unions over core-core pairs (each unordered pair from its smaller slot: q > p) in
// stencil row `only` (-1: all rows), union-find over slots in L.par.
// Clique grids: p unites with the FIRST core q > p of each quarter cell (side ~eps/2, a clique)
// of its stencil within eps, and no other of that quarter.  Enough: the cores of one quarter
// are chained (each to the next core of its quarter), and a pair p < q within eps makes p unite
// with some core of q's quarter.  So a dense cell costs a few unions per point instead of one
// per neighbour.  reach_k: record -> cell-local coordinate offsets (clique grids).
template <class LT>
__device__ __forceinline__ void sm_union_walk(LT& L, const SmCtx& cx_, int p, int only,
                                              bool quarters, double reach_kx, double reach_ky) {
    const int nx = cx_.nx, ny = cx_.ny;
    const float2 me = L.rec[p];
    uint64_t done = 0;  // quarters of the 6x6 window around p's cell already joined
    // a root of p's set (possibly stale: it stays an ancestor of p, so a q whose parent it is
    // belongs to p's set already and needs neither a pair test nor a union)
    int rp = sm_find(L.par, p);
    // the stencil walk of sm_for_stencil with each batch's records, infos, core flags and
    // parents loaded together (the walk is bound by dependent LDS reads: one round trip per
    // batch instead of three per candidate).  A parent read before a union of this batch is
    // still an ancestor of that candidate, so `parent == rp` still proves p's set.
    const int c = (int)(L.info[p] & kCellMask);
    const int cy = c / nx, cx = c - cy * nx;
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, nx - 1);
    if (quarters && !cx_.exact_only) {
        // quarters of the 6x6 window wholly beyond eps of p (their nearest point farther than
        // the F threshold plus a margin over the fp32 records' error) count as done
        const float tx = (float)((double)me.x + reach_kx - (double)cx);
        const float ty = (float)((double)me.y + reach_ky - (double)cy);
        const float mg = (fabsf(me.x) + fabsf(me.y) + 4.0f) * 0x1p-18f + 0x1p-12f;
        const float rr = (sqrtf(cx_.hi) + mg) * (sqrtf(cx_.hi) + mg);
        // (one stencil row: only its two quarter rows of the window)
        const int wa = only < 0 ? -1 : (only == 0 ? 1 : (only == 1 ? 0 : 2));
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            if (wa >= 0 && (a >> 1) != wa) continue;
            const float y0 = 0.5f * (float)a - 1.0f,
                        dy = fmaxf(0.0f, fmaxf(y0 - ty, ty - (y0 + 0.5f)));
#pragma unroll
            for (int b = 0; b < 6; ++b) {
                const float xb = 0.5f * (float)b - 1.0f;
                const float dx = fmaxf(0.0f, fmaxf(xb - tx, tx - (xb + 0.5f)));
                if (dx * dx + dy * dy > rr) done |= 1ull << (a * 6 + b);
            }
        }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        if (only >= 0 && d != only) continue;
        const int r = d == 0 ? cy : (d == 1 ? cy - 1 : cy + 1);
        if (r < 0 || r >= ny) continue;
        const int rb = r * nx;
        const int e = L.cst[rb + x1 + 1];
        const int b1 = x0 + 1 <= x1 ? (int)L.cst[rb + x0 + 1] : 0x7FFFFFFF;
        const int b2 = x0 + 2 <= x1 ? (int)L.cst[rb + x0 + 2] : 0x7FFFFFFF;
        const int wr = (r - cy + 1) * 3 + (x0 - cx + 1);
        for (int q = max((int)L.cst[rb + x0], p + 1); q < e; q += kSmBatch) {
            if (quarters) {
                // every quarter of q's cell done: the rest of the cell needs no visit
                const int w = wr + (q >= b1 ? 1 : 0) + (q >= b2 ? 1 : 0);
                const int sh = 2 * (w / 3) * 6 + 2 * (w % 3);
                const uint64_t m4 = (3ull << sh) | (3ull << (sh + 6));
                if ((done & m4) == m4) {
                    q = min(q < b1 ? b1 : (q < b2 ? b2 : e), e) - kSmBatch;
                    continue;
                }
            }
            float2 rq[kSmBatch];
            uint32_t iq[kSmBatch];
            int pq[kSmBatch];
            bool cq[kSmBatch];
#pragma unroll
            for (int u = 0; u < kSmBatch; ++u) {
                const int qq = min(q + u, e - 1);
                rq[u] = L.rec[qq];
                iq[u] = L.info[qq];
                cq[u] = L.core[qq] != 0;
                pq[u] = sm_ld(L.par + qq);
            }
#pragma unroll
            for (int u = 0; u < kSmBatch; ++u) {
                const int qq = q + u;
                if (qq >= e || !cq[u]) continue;
                int bit = 0;
                if (quarters) {
                    const int w = wr + (qq >= b1 ? 1 : 0) + (qq >= b2 ? 1 : 0);
                    const int qd = (int)((iq[u] >> 13) & 3u);
                    bit = (2 * (w / 3) + (qd >> 1)) * 6 + 2 * (w % 3) + (qd & 1);
                    if ((done >> bit) & 1ull) continue;
                }
                if (pq[u] == rp) {
                    if (quarters) done |= 1ull << bit;
                    continue;
                }
                if (sm_pair(L, cx_, p, me, qq, rq[u])) {
                    // unite from the root p's walk holds (finding p's root again measured
                    // slower: 370 -> 348 us at 8192 points)
                    rp = sm_unite_from(L.par, L.info, rp, qq);
                    if (quarters) done |= 1ull << bit;
                }
            }
        }
    }
}

// The smallest root visit index among non-core p's core neighbours in stencil row `only`
// (root_of(q): the root visit index of core slot q)
template <class RootF>
__device__ __forceinline__ uint32_t sm_best_root(const SmLds& L, const SmCtx& c, int p, int only,
                                                 RootF root_of) {
    const float2 me = L.rec[p];
    uint32_t best = 0xFFFFFFFFu;
    sm_for_stencil(L, c, p, 0, [&](int q, float2 rq, int) {
        if (L.core[q]) {
            const uint32_t s = root_of(q);
            if (s < best && sm_pair(L, c, p, me, q, rq)) best = s;
        }
        return true;
    }, only);
    return best;
}

// 1 + roots with a smaller visit index (the reference's cluster id of the cluster s(K) opens)
__device__ __forceinline__ int sm_cluster_of(const SmLds& L, uint32_t s) {
    return L.wrank[s >> 5] + __popc(L.rbits[s >> 5] & ((1u << (s & 31u)) - 1u)) + 1;
}

// Slot p's label (LocalDBSCANNaive.scala:89-106; Archery re-claim LocalDBSCANArchery.scala:
// 103-106): cores their root's cluster (root_v: the root's visit index), non-cores the cluster
// of best (min s(K) over core neighbours) under the Naive / Archery rule; written in input order.
__device__ __forceinline__ void sm_write_label(const SmLds& L, int p, uint32_t root_v,
                                               uint32_t best, int mode, int32_t* cl_out,
                                               uint8_t* fl_out) {
    const uint32_t v = L.info[p] >> 16;
    int cid = 0;
    uint8_t f = DBSCAN_FLAG_NOISE;
    if (L.core[p]) {
        cid = sm_cluster_of(L, root_v);
        f = DBSCAN_FLAG_CORE;
    } else if (best != 0xFFFFFFFFu && (mode != DBSCAN_MODE_NAIVE || best < v)) {
        cid = sm_cluster_of(L, best);
        f = DBSCAN_FLAG_BORDER;
    }
    cl_out[v] = cid;
    fl_out[v] = f;
}

// The fit statistics of an LDS fit: the handle's device state (st, gp) and, when given, the
// same words in the handle's pinned host block (mirror: read back without a copy).
__device__ __forceinline__ void sm_zero_stats(int32_t* st, double* mirror, int tid) {
    if (tid < kStCount) {
        if (st) st[tid] = 0;
        if (mirror) reinterpret_cast<int32_t*>(mirror + kMiscState)[tid] = 0;
    }
}
__device__ __forceinline__ void sm_set_stat(int32_t* st, double* mirror, int k, int32_t v) {
    if (st) st[k] = v;
    if (mirror) reinterpret_cast<int32_t*>(mirror + kMiscState)[k] = v;
}

// One partition per workgroup.  offs == nullptr: one partition [0, single_n) (blockIdx 0);
// else partition list[blockIdx.x] = points [offs[p], offs[p+1]).  nclusters[p] (or st) gets its
// cluster count.  st/gp (single fits only): the handle's fit statistics.
__global__ __launch_bounds__(kSmT, 1) void small_fit_kernel(
    const double* __restrict__ x, const double* __restrict__ y, const int64_t* __restrict__ offs,
    const int32_t* __restrict__ list, int64_t single_n, double eps, double eps2, int min_points,
    int mode, int32_t* __restrict__ cluster, uint8_t* __restrict__ flag,
    int32_t* __restrict__ nclusters, GridParams* __restrict__ gp, int32_t* __restrict__ st,
    double* __restrict__ mirror) {
    __shared__ SmLds L;

    const int tid = threadIdx.x;
    int64_t off = 0, m64 = single_n;
    int part = 0;
    if (offs) {
        part = list[blockIdx.x];
        off = offs[part];
        m64 = offs[part + 1] - off;
    }
    const int m = (int)m64;  // the host routes only m <= kSmN here
    const double* px = x + off;
    const double* py = y + off;
    SM_STAMP(0);
    sm_zero_stats(st, mirror, tid);  // (the fit state: no memset ahead of the launch)
    int occupied = 0;
    if (!sm_stage(L, px, py, m, eps, eps2, occupied)) {
        if (tid == 0) sm_set_stat(st, mirror, kStError, 1);
        return;
    }
    SM_STAMP(2);
    const int nf = L.G.nf, nx = L.G.nx, ny = L.G.ny;
    const SmCtx c = sm_ctx(L, px, py, eps2);

    // Row split (partitions of <= kSmT / 3 points, where most threads would idle): each point's
    // three stencil rows are walked by three threads, counts summed and label minima taken in
    // LDS -- a third of the dependent chain per thread.
    const bool split = 3 * m <= kSmT;

    // ---- count: core <=> |N(p)| >= minPoints (LocalDBSCANNaive.scala:52-56,99-101) ----
    int ncore_local = 0;
    if (split) {
        if (tid < m) L.par[tid] = 0;  // (per-point counters until the union needs par)
        __syncthreads();
        if (tid < 3 * m && min_points > 0) {
            const int p = tid / 3, d = tid - 3 * (tid / 3);
            if (p < nf) {  // a row alone reaching minPoints decides the point
                const int cnt = sm_count(L, c, p, min_points, d);
                if (cnt) atomicAdd(&L.par[p], cnt);
            }
        }
        __syncthreads();
        if (tid < m) {
            const bool cc = min_points <= 0 || (tid < nf && L.par[tid] >= min_points);
            L.core[tid] = cc ? 1 : 0;
            L.par[tid] = tid;
            ncore_local = cc ? 1 : 0;
        }
    } else {
        for (int p = tid; p < m; p += kSmT) {
            bool cc = min_points <= 0;
            if (!cc && p < nf) cc = sm_count(L, c, p, min_points, -1) >= min_points;
            L.core[p] = cc ? 1 : 0;
            L.par[p] = p;
            ncore_local += cc ? 1 : 0;
        }
    }
    __syncthreads();
    SM_STAMP(3);

    // ---- union over core-core pairs ----
    const bool quarters = L.G.clique != 0;
    // record -> cell-local coordinate: (v*0.5 - xmin2)*invx - cx = rec + (cx2 - xmin2)*invx - cx
    // (clique grids: invx = invy = invs)
    const double reach_kx = (L.G.cx2 - L.G.xmin2) * L.G.invx;
    const double reach_ky = (L.G.cy2 - L.G.ymin2) * L.G.invy;
    const int R = split ? 3 : 1;  // stencil rows per work item
    for (int it = tid; it < nf * R; it += kSmT) {
        // (row-major items, as band_fit_kernel: 250 / 2000 points 56.5 / 99.7 -> 51.7 / 89.8
        // us per call)
        const int p = split ? it % nf : it, only = split ? it / nf : -1;
        if (L.core[p]) sm_union_walk(L, c, p, only, quarters, reach_kx, reach_ky);
    }
    __syncthreads();
    SM_STAMP(4);

    // ---- roots: s(K) flagged by visit index; then every core points at its root ----
    // (read-only walks first, writes after a barrier: a path-halving find racing with the
    // compression could leave a pointer one ancestor short of the root)
    int myroot[kSmPer];
#pragma unroll
    for (int k = 0; k < kSmPer; ++k) {
        const int p = tid + k * kSmT;
        myroot[k] = -1;
        if (p < m && L.core[p]) {
            int r = p;
            for (int u = L.par[r]; u != r; u = L.par[r]) r = u;
            myroot[k] = r;
            if (r == p) {
                const uint32_t v = L.info[p] >> 16;
                atomicOr(&L.rbits[v >> 5], 1u << (v & 31u));
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmPer; ++k)
        if (myroot[k] >= 0) L.par[tid + k * kSmT] = myroot[k];
    int nclust = 0;
    {
        const int v = tid < kSmN / 32 ? __popc(L.rbits[tid]) : 0;
        const int r = sm_excl_scan(v, L.wsc, &nclust);  // (its barriers also order the compression)
        if (tid < kSmN / 32) L.wrank[tid] = r;
    }
    __syncthreads();
    SM_STAMP(5);

    // ---- labels ----
    int32_t* cl_out = cluster + off;
    uint8_t* fl_out = flag + off;
    const auto root_of = [&](int q) { return L.info[L.par[q]] >> 16; };
    if (split) {
        if (tid < m) L.sbest[tid] = 0xFFFFFFFFu;
        __syncthreads();
        if (tid < 3 * m) {
            const int p = tid / 3;
            if (!L.core[p] && p < nf) {
                const uint32_t b = sm_best_root(L, c, p, tid - 3 * p, root_of);
                if (b != 0xFFFFFFFFu) atomicMin(&L.sbest[p], b);
            }
        }
        __syncthreads();
        if (tid < m)
            sm_write_label(L, tid, L.core[tid] ? root_of(tid) : 0u, L.sbest[tid], mode, cl_out,
                           fl_out);
    } else {
        for (int p = tid; p < m; p += kSmT) {
            const bool cc = L.core[p] != 0;
            sm_write_label(L, p, cc ? root_of(p) : 0u,
                           (!cc && p < nf) ? sm_best_root(L, c, p, -1, root_of) : 0xFFFFFFFFu,
                           mode, cl_out, fl_out);
        }
    }

    SM_STAMP(6);
    // ---- counts and statistics ----
    {
        int tot = 0;
        (void)sm_excl_scan(ncore_local, L.wsc, &tot);
        int occ = 0;
        (void)sm_excl_scan(occupied, L.wsc, &occ);
        if (tid == 0) {
            if (nclusters) nclusters[part] = nclust;
            sm_set_stat(st, mirror, kStNf, nf);
            sm_set_stat(st, mirror, kStCore, tot);
            sm_set_stat(st, mirror, kStClusters, nclust);
            sm_set_stat(st, mirror, kStCells, nf > 0 ? occ : 0);
            GridParams g{L.G.xmin2, L.G.ymin2, L.G.invx, L.G.invy, (uint32_t)nx, (uint32_t)ny,
                         1u, 1u, 0};
            if (gp) *gp = g;
            if (mirror) *reinterpret_cast<GridParams*>(mirror + kMiscGrid) = g;
        }
    }
}

// ---------------------------------------------------------------------------------------
// The same fit spread over G workgroups of one launch (spread_fit_kernel): a partition of a
// few thousand points keeps one CU busy for hundreds of microseconds in small_fit_kernel (the
// count and union walks are chains of dependent LDS reads, eight points per thread), while a
// launch chain of the tiled pipeline costs ~45 kernel boundaries.  Here every workgroup stages
// the WHOLE partition in its LDS (the same stage as small_fit_kernel, in its own slot order),
// owns the slots of a contiguous cell range holding ~1/G of the points, and
//   count   counts its own points; core flags by input index to global memory
//   -- grid barrier 1 --
//   union   reads every core flag; walks its own cores' stencils (the union rule above) into a
//           union-find over its staged slots; publishes every non-root core of that forest as
//           (input index, its root's input index)
//   -- grid barrier 2 --
//   merge   unites every workgroup's published pairs in a union-find over input indices: the
//           union of all forests, so each root is the smallest input index of its cluster's
//           cores, s(K), in every workgroup alike; numbering as small_fit_kernel
//   label   its own points (and the non-finite points, last workgroup) in input order
// Every edge of the closed form is found by the workgroup owning the smaller cell (cells are
// ordered alike in every stage; a cell's quarters, and so its chains, have one owner), so the
// merged forest has the components small_fit_kernel finds, and the results are the same bit
// for bit.  Two grid barriers (every workgroup resident: the host caps the grid far below one
// workgroup per CU); the arrival counter is reset by the last workgroup to leave.
// ---------------------------------------------------------------------------------------
constexpr int kSpreadMaxWG = 32;  // (64 measured no faster: the workgroups' chains do not shorten)

static_assert(kSpreadMaxWG <= 64 && 2 * 64 + 1 <= kSmN / 32, "merge tables in SmLds::wrank");

struct SpreadArgs {
    uint8_t* core;     // [n] core flags by input index (count -> union)
    uint32_t* pairs;   // [G][n] published (input index << 16 | root input index)
    int32_t* npairs;   // [G]
    uint32_t* bar;     // [2] arrivals, departures (zero between launches)
};

__device__ __forceinline__ uint32_t sp_load(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Grid-wide barrier: every wave drains its stores, the workgroup meets, one lane releases
// (agent fence, then its own drain) and adds its arrival, polls the count relaxed with a sleep
// until `target` arrivals, and acquires (agent fence: this CU's stale lines dropped) before the
// workgroup meets again and reads what the others published.  The poll gives up after ~2^21
// rounds (seconds) and flags st[kStError] = 2: the fit then fails loudly instead of hanging.
// A workgroup that gives up also raises the launch's abort word bar[2], which every poll reads
// beside the count: once one barrier of a launch has failed, every later wait of every
// workgroup ends at once (the result is discarded and re-run by the host) instead of spinning
// to the bound again.  bar[2] is cleared by the last workgroup to leave.
__device__ void sp_grid_sync(uint32_t* bar, uint32_t target, int32_t* st, double* mirror,
                             uint32_t spin_limit) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // (spin_limit 0: give up at once, the test of the fallback; the host re-runs the fit)
        for (uint32_t spins = 0; spin_limit == 0 || sp_load(bar) < target;) {
            if (sp_load(bar + 2) != 0u) break;  // (another workgroup gave up: flagged already)
            __builtin_amdgcn_s_sleep(2);
            if (++spins > spin_limit) {
                __hip_atomic_store(bar + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(st + kStError, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (mirror)
                    __hip_atomic_store(reinterpret_cast<int32_t*>(mirror + kMiscState) + kStError,
                                       2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// Union-find over input indices (merge phase): the larger root hooked under the smaller.
__device__ __forceinline__ void sm_unite_v(int* par, int a, int b) {
    while (true) {
        a = sm_find(par, a);
        b = sm_find(par, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(par + a, a, b) == a) return;
    }
}

// The wave-cooperative walks of the spread form: p is the same in every lane of the wave.
// |N(p)| capped at minPoints: 64 candidates of a stencil row per step, hits by ballot.
template <class LT>
__device__ __forceinline__ int sp_count_wave(const LT& L, const SmCtx& c, int p,
                                             int min_points) {
    const int lane = (int)(threadIdx.x & 63);
    const float2 me = L.rec[p];
    const int cc = (int)(L.info[p] & kCellMask);
    const int cy = cc / c.nx, cx = cc - cy * c.nx;
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, c.nx - 1);
    int cnt = 0;
    for (int d = 0; d < 3 && cnt < min_points; ++d) {
        const int r = d == 0 ? cy : (d == 1 ? cy - 1 : cy + 1);
        if (r < 0 || r >= c.ny) continue;
        const int e = L.cst[r * c.nx + x1 + 1];
        for (int q0 = L.cst[r * c.nx + x0]; q0 < e && cnt < min_points; q0 += 64) {
            const int q = q0 + lane;
            const bool hit = q < e && sm_pair(L, c, p, me, q, L.rec[q]);
            cnt += __popcll(__ballot(hit));
        }
    }
    return cnt;
}

// The smallest root visit index among non-core p's core neighbours (sm_best_root), 64
// candidates per step, the minimum taken across the wave.
__device__ __forceinline__ uint32_t sp_best_root_wave(const SmLds& L, const SmCtx& c, int p) {
    const int lane = (int)(threadIdx.x & 63);
    const float2 me = L.rec[p];
    const int cc = (int)(L.info[p] & kCellMask);
    const int cy = cc / c.nx, cx = cc - cy * c.nx;
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, c.nx - 1);
    uint32_t best = 0xFFFFFFFFu;
    for (int d = 0; d < 3; ++d) {
        const int r = d == 0 ? cy : (d == 1 ? cy - 1 : cy + 1);
        if (r < 0 || r >= c.ny) continue;
        const int e = L.cst[r * c.nx + x1 + 1];
        for (int q = L.cst[r * c.nx + x0] + lane; q < e; q += 64) {
            if (!L.core[q]) continue;
            const uint32_t s = (uint32_t)L.par[L.info[q] >> 16];
            if (s < best && sm_pair(L, c, p, me, q, L.rec[q])) best = s;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, 64));
    return best;
}

__global__ __launch_bounds__(kSmT, 1) void spread_fit_kernel(
    const double* __restrict__ x, const double* __restrict__ y, int m, double eps, double eps2,
    int min_points, int mode, int32_t* __restrict__ cluster, uint8_t* __restrict__ flag,
    GridParams* __restrict__ gp, int32_t* st, double* mirror, SpreadArgs sa,
    uint32_t spin_limit) {
    __shared__ SmLds L;
    const int tid = threadIdx.x;
    const int g = blockIdx.x, G = gridDim.x;
    SM_STAMP(0);
    // (the fit state: no memset ahead of launch) -- except kStError, which the host clears
    // before the launch: a late workgroup 0 must not erase a barrier failure another workgroup
    // has already flagged
    if (g == 0 && tid != kStError) sm_zero_stats(st, mirror, tid);
    int occupied = 0;
    // (every workgroup computes the same grid: a grid that cannot be sized returns them all
    // here, before any barrier)
    if (!sm_stage(L, x, y, m, eps, eps2, occupied)) {
        if (tid == 0 && g == 0) sm_set_stat(st, mirror, kStError, 1);
        return;
    }
    SM_STAMP(2);
    const int nf = L.G.nf, nx = L.G.nx, ny = L.G.ny, ncells = L.G.ncells;
    const SmCtx c = sm_ctx(L, x, y, eps2);
    // the owned cells: a contiguous cell range holding ~1/G of the walks' work, estimated per
    // cell as its points x its stencil's points (cell counts are alike in every stage); the
    // prefix of the estimate before each cell in par (free until the union)
    {
        int w[kSmCellPer], sum = 0;
#pragma unroll
        for (int k = 0; k < kSmCellPer; ++k) {
            const int cc = tid * kSmCellPer + k;
            w[k] = 0;
            if (cc < ncells) {
                const int npt = (int)L.cst[cc + 1] - (int)L.cst[cc];
                if (npt > 0) {
                    const int cy = cc / nx, cx = cc - cy * nx;
                    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, nx - 1);
                    int cand = 0;
                    for (int r = max(cy - 1, 0); r <= min(cy + 1, ny - 1); ++r)
                        cand += (int)L.cst[r * nx + x1 + 1] - (int)L.cst[r * nx + x0];
                    w[k] = npt * cand;
                }
            }
            sum += w[k];
        }
        int tot = 0;
        int run = sm_excl_scan(sum, L.wsc, &tot);
#pragma unroll
        for (int k = 0; k < kSmCellPer; ++k) {
            const int cc = tid * kSmCellPer + k;
            if (cc < ncells) L.par[cc] = run;
            run += w[k];
        }
        __syncthreads();
        if (tid < 2) {
            const int64_t want = (int64_t)(g + tid) * tot / G;
            int lo = 0, hi = ncells;  // smallest cell k whose prefix is >= want (ncells: tot)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if ((int64_t)L.par[mid] >= want) hi = mid; else lo = mid + 1;
            }
            L.band[tid] = g + tid == G ? nf : (int)L.cst[lo];
            if (tid == 0) L.band[2] = 0;
        } else if (tid < 4) {
            // the count and the labels: ~nf/G points each (cell starts are alike in every stage;
            // the walks' work estimate would give the sparse bands far more points to count)
            const int want = (int)((int64_t)(g + tid - 2) * nf / G);
            int lo = 0, hi = ncells;  // smallest cell k with cst[k] >= want (cst[ncells] = nf)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if ((int)L.cst[mid] >= want) hi = mid; else lo = mid + 1;
            }
            L.band[tid + 2] = g + tid - 2 == G ? nf : (int)L.cst[lo];
        }
        __syncthreads();
    }
    const int s0 = L.band[0], s1 = L.band[1], nb = s1 - s0;
    const int c0 = L.band[4], c1 = L.band[5];

    // ---- count (own slots): one wave per own point, its 64 lanes over 64 candidates of a
    // stencil row at a time, hits counted by a ballot (one thread per row measured slower from
    // 2000 points: 19.8 -> 18.1 us at 2000, 26.9 -> 24.6 at 8192) ----
    for (int p = c0 + (tid >> 6); p < c1; p += kSmW) {
        const bool cc = min_points <= 0 || sp_count_wave(L, c, p, min_points) >= min_points;
        if ((tid & 63) == 0) sa.core[L.info[p] >> 16] = cc ? 1 : 0;
    }
    SM_STAMP(7);
    sp_grid_sync(sa.bar, (uint32_t)G, st, mirror, spin_limit);
    SM_STAMP(8);

    // ---- union of the own cores' walks (union-find over this stage's slots) ----
    for (int p = tid; p < m; p += kSmT) {
        L.core[p] = p < nf ? sa.core[L.info[p] >> 16] : (min_points <= 0 ? 1 : 0);
        L.par[p] = p;
    }
    __syncthreads();
    const bool quarters = L.G.clique != 0;
    const double reach_kx = (L.G.cx2 - L.G.xmin2) * L.G.invx;
    const double reach_ky = (L.G.cy2 - L.G.ymin2) * L.G.invy;
    // (one thread per stencil row: the wave-cooperative form, a serial unite per joined quarter,
    // measured 48 -> 92 us at 8192 points)
    for (int it = tid; it < nb * 3; it += kSmT) {
        // (row-major items, as band_fit_kernel: 8192 points 155 -> 137 us per call)
        const int d = it / nb, i = it - d * nb;
        if (L.core[s0 + i]) sm_union_walk(L, c, s0 + i, d, quarters, reach_kx, reach_ky);
    }
    __syncthreads();
    SM_STAMP(9);
    // publish the forest: every core slot that is not a root, with its root (read-only walks)
    uint32_t* mine = sa.pairs + (int64_t)g * m;
    for (int p = tid; p < nf; p += kSmT) {
        if (!L.core[p] || L.par[p] == p) continue;
        int r = p;
        for (int u = L.par[r]; u != r; u = L.par[r]) r = u;
        const int k = atomicAdd(&L.band[2], 1);
        mine[k] = (L.info[p] & 0xFFFF0000u) | (L.info[r] >> 16);
    }
    __syncthreads();
    if (tid == 0) sa.npairs[g] = L.band[2];
    SM_STAMP(10);
    sp_grid_sync(sa.bar, 2u * (uint32_t)G, st, mirror, spin_limit);
    SM_STAMP(11);

    // ---- merge: every workgroup's pairs into a union-find over input indices ----
    for (int v = tid; v < m; v += kSmT) L.par[v] = v;
    if (tid < G) L.wrank[tid] = (int)sp_load(reinterpret_cast<uint32_t*>(sa.npairs + tid));
    __syncthreads();
    if (tid == 0) {  // list starts (wrank[64 + h]) and the total (wrank[128])
        int acc = 0;
        for (int h = 0; h < G; ++h) {
            L.wrank[64 + h] = acc;
            acc += L.wrank[h];
        }
        L.wrank[128] = acc;
    }
    __syncthreads();
    {
        // eight pairs per thread and round, their loads in flight together
        constexpr int kMergeBatch = 8;
        const int total = L.wrank[128];
        for (int k0 = tid; k0 < total; k0 += kSmT * kMergeBatch) {
            uint32_t w[kMergeBatch];
#pragma unroll
            for (int u = 0; u < kMergeBatch; ++u) {
                const int k = k0 + u * kSmT;
                w[u] = 0xFFFFFFFFu;
                if (k < total) {
                    int lo = 0;  // the list holding flat index k
#pragma unroll
                    for (int sh = 32; sh > 0; sh >>= 1)
                        if (lo + sh < G && L.wrank[64 + lo + sh] <= k) lo += sh;
                    w[u] = sa.pairs[(int64_t)lo * m + (k - L.wrank[64 + lo])];
                }
            }
#pragma unroll
            for (int u = 0; u < kMergeBatch; ++u)
                if (w[u] != 0xFFFFFFFFu) sm_unite_v(L.par, (int)(w[u] >> 16), (int)(w[u] & 0xFFFFu));
        }
    }
    __syncthreads();
    SM_STAMP(12);
    // roots: s(K) flagged by visit index, then every core's parent is its root
    int myroot[kSmPer];
#pragma unroll
    for (int k = 0; k < kSmPer; ++k) {
        const int p = tid + k * kSmT;
        myroot[k] = -1;
        if (p < m && L.core[p]) {
            const int v = (int)(L.info[p] >> 16);
            int r = v;
            for (int u = L.par[r]; u != r; u = L.par[r]) r = u;
            myroot[k] = r;
            if (r == v) atomicOr(&L.rbits[v >> 5], 1u << (v & 31));
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmPer; ++k)
        if (myroot[k] >= 0) L.par[L.info[tid + k * kSmT] >> 16] = myroot[k];
    int nclust = 0;
    {
        const int v = tid < kSmN / 32 ? __popc(L.rbits[tid]) : 0;
        const int r = sm_excl_scan(v, L.wsc, &nclust);
        if (tid < kSmN / 32) L.wrank[tid] = r;
    }
    __syncthreads();
    SM_STAMP(13);

    // ---- labels of the own slots (+ the non-finite points: the last workgroup) ----
    const auto root_of = [&](int q) { return (uint32_t)L.par[L.info[q] >> 16]; };
    for (int p = c0 + tid; p < c1; p += kSmT)  // cores: one thread each
        if (L.core[p]) sm_write_label(L, p, root_of(p), 0xFFFFFFFFu, mode, cluster, flag);
    for (int p = c0 + (tid >> 6); p < c1; p += kSmW) {  // non-cores: a wave each
        if (L.core[p]) continue;
        const uint32_t b = sp_best_root_wave(L, c, p);
        if ((tid & 63) == 0) sm_write_label(L, p, 0u, b, mode, cluster, flag);
    }
    if (g == G - 1)
        for (int p = nf + tid; p < m; p += kSmT)
            sm_write_label(L, p, L.core[p] ? root_of(p) : 0u, 0xFFFFFFFFu, mode, cluster, flag);

    SM_STAMP(14);
    // ---- statistics (workgroup 0) and the barrier reset (the last workgroup to leave) ----
    if (g == 0) {
        int ncore = 0;
        for (int p = tid; p < m; p += kSmT) ncore += L.core[p];
        int tot = 0, occ = 0;
        (void)sm_excl_scan(ncore, L.wsc, &tot);
        (void)sm_excl_scan(occupied, L.wsc, &occ);
        if (tid == 0) {
            sm_set_stat(st, mirror, kStNf, nf);
            sm_set_stat(st, mirror, kStCore, tot);
            sm_set_stat(st, mirror, kStClusters, nclust);
            sm_set_stat(st, mirror, kStCells, nf > 0 ? occ : 0);
            GridParams gg{L.G.xmin2, L.G.ymin2, L.G.invx, L.G.invy, (uint32_t)nx, (uint32_t)ny,
                          1u, 1u, L.G.clique};
            *gp = gg;
            if (mirror) *reinterpret_cast<GridParams*>(mirror + kMiscGrid) = gg;
        }
    }
    if (tid == 0 &&
        __hip_atomic_fetch_add(sa.bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (uint32_t)G - 1) {
        __hip_atomic_store(sa.bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sa.bar + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sa.bar + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------------------
// Partitions above the one-workgroup capacity (kSmallMaxPoints < m <= kBandMaxPoints: a dense
// region's rectangle plus its eps halo, DBSCAN.scala:116-137) in ONE launch (band_fit_kernel):
// the tiled pipeline's ~45 kernel boundaries cost ~5 us each on the GPU whatever enqueues them.
// G = 64 workgroups (one per CU by their LDS), each owning a range of cells of ~1/G of the
// partition's cost (below) and staging only the rows of those cells plus one cell row on
// either side (the 3x3 stencil of an owned point never leaves the staged rows):
//   slice   each workgroup reads ~m/G points, one per thread: the non-finite ones labelled
//           noise, the slice's bbox published
//   -- grid barrier A --
//   grid    the G boxes reduced in one order (the same grid everywhere; cells of side >= eps,
//           grown only while the grid is too large for the band tables); the slice's points
//           per cell row added to global row counts
//   -- grid barrier B --
//   bands   the row counts -> cost prefix -> this workgroup's cell range (alike everywhere);
//           the slice's points scattered to a global row-sorted array (each row's piece
//           claimed once per workgroup)
//   -- grid barrier C --
//   stage   the staged rows' records (one contiguous piece of the row-sorted array) counting-
//           sorted by cell in LDS (fp32 records as small.hip)
//   count   its own points (a thread or a wave each); core flags by input index
//   -- grid barrier 1 --
//   union   the staged slots' core flags; its own cores' stencil walks (sm_union_walk) into an
//           LDS forest over the staged slots; every non-root staged core published as
//           (input index, its root's input index).  An edge between two ranges is walked by the
//           owner of the smaller cell, as in spread_fit_kernel
//   -- grid barrier 2 --
//   merge   the published pairs united in a union-find over input indices in global memory
//           (larger index hooked under the smaller: a root IS s(K))
//   -- grid barrier 3 --
//   label   each staged core's root (its s(K)) into LDS; the root flags of all points read
//           from the global forest (a core is a root iff it is its own parent) -> popcount ranks
//           (cluster id = 1 + roots before s(K)); own cores their root's id, own non-cores the
//           min s(K) over their staged core neighbours + the Naive / Archery rule
// Same results bit for bit as every other form (the GPU tests compare them with the oracle).
// A range over the staging capacity (rows too dense, or too many sparse rows), or a barrier
// that gives up, flags st[kStError] (3 / 2): the host then re-runs the fit through the tiled
// pipeline in the same call.
constexpr int kBandT = 1024;
constexpr int kBandCap = 7168;    // staged points per workgroup (and staged cells)
constexpr int kBandCells = kBandCap;
constexpr int kBandMaxWG = 64;
constexpr int kBandFullBox = 16384;  // up to here every workgroup reduces the whole bbox
// a point's count + walk work without neighbours, in cell densities (0, 1 and 4 measured within
// 2% of 2 at 12k-65k points)
constexpr int kBandC0 = 2;
constexpr int kBandWords = (int)(kBandMaxPoints / 32);
static_assert(kBandMaxPoints <= 65536, "16-bit visit indices");
static_assert(kBandCells <= 8191, "13-bit cells in info");

struct BandLds {
    float2 rec[kBandCap];
    uint32_t info[kBandCap];  // visit << 16 | quadrant << 13 | staged cell; first: cell counts
    int par[kBandCap];        // row counts, then sort cursors, then the LDS union-find
    uint8_t core[kBandCap];
    uint16_t cst[kBandCells + 2];
    uint32_t rbits[kBandWords];
    int wrank[kBandWords];
    double red[5][kBandT / 64];
    int wsc[kBandT / 64 + 1];
    int meta[16];
    SmGrid G;
};

struct BandArgs {
    uint8_t* core;    // [m] core flags by input index
    int32_t* par;     // [m] union-find over input indices
    uint32_t* pairs;  // [G][kBandCap] published (input index << 16 | root input index)
    int32_t* npairs;  // [G]
    int32_t* cnt;     // [2] cores, occupied cells
    uint32_t* bar;    // [2] arrivals, departures (zero between launches)
    double* box;      // [G][5] the slices' min x, max x, min y, max y, finite count
    uint32_t* rowcnt; // [kBandCap] points per grid row (zero between launches)
    uint32_t* rowcur; // [kBandCap] claimed per grid row (zero between launches)
    double2* rxy;     // [m] the finite points' coordinates sorted by grid row
    int32_t* ridx;    // [m] their input indices
};

// The band grid (one thread): sides as sm_make_grid, doubled along the axis over its share of
// the limits until nx <= kBandCells / 3 and ny < kBandCap (row counts live in par) and the
// whole grid holds <= 24 * kBandCells * G / kBandMaxWG cells: with G ranges of ~1/G of the cost
// below (at most twice the points + cells) each range fits its tables with room for its halo
// rows (the bound scaled by G: sparse partitions of a few thousand points over hundreds of cells
// per side, fitted by G = 16..20 workgroups, overflowed a fixed 24 * kBandCells)
__device__ void band_make_grid(double xmin, double xmax, double ymin, double ymax, int nf,
                               double eps, double eps2, int G, SmGrid* g) {
    g->nf = nf;
    g->bad = 0;
    g->exact_only = 0;
    g->nx = g->ny = g->ncells = 1;
    g->clique = 0;
    if (nf == 0) return;
    double R = fabs(eps) * (1.0 + 0x1p-40);
    if (R < 0x1p-500) R = 0x1p-500;
    const double h0 = R * (1.0 + 0x1p-16);
    double hx = h0, hy = h0;
    auto cells = [](double vmax, double vmin, double h) {
        return floor((vmax * 0.5 - vmin * 0.5) * (2.0 / h)) + 1.0;
    };
    // (ny + 1 row counts live in par[kBandCap])
    constexpr double kNx = kBandCells / 3, kNy = kBandCap - 1;
    const double kAll = 24.0 * kBandCells * (double)G / (double)kBandMaxWG;
    bool ok = false;
    double cx = 1, cy = 1;
    for (int it = 0; it < 4096; ++it) {
        cx = cells(xmax, xmin, hx);
        cy = cells(ymax, ymin, hy);
        if (cx <= kNx && cy <= kNy && cx * cy <= kAll) {
            ok = true;
            break;
        }
        if (cx / kNx >= cy / kNy) hx *= 2.0; else hy *= 2.0;
    }
    if (!ok) {
        g->bad = 1;
        return;
    }
    g->nx = (int)cx;
    g->ny = (int)cy;
    g->clique = (hx == h0 && hy == h0 && h0 <= fabs(eps) * (1.0 + 0x1p-14)) ? 1 : 0;
    g->ncells = g->nx * g->ny;
    g->xmin2 = xmin * 0.5;
    g->ymin2 = ymin * 0.5;
    g->invx = 2.0 / hx;
    g->invy = 2.0 / hy;
    g->cx2 = xmin * 0.5 + (xmax * 0.5 - xmin * 0.5) * 0.5;
    g->cy2 = ymin * 0.5 + (ymax * 0.5 - ymin * 0.5) * 0.5;
    g->invs = 2.0 / h0;
    const double rr = fmax((xmax * 0.5 - xmin * 0.5), (ymax * 0.5 - ymin * 0.5)) * g->invs * 0.5 +
                      1.0;
    const double e2 = eps2 * (0.5 * g->invs) * (0.5 * g->invs);
    if (!(rr <= 0x1p20) || !(e2 <= 0x1p20)) {
        g->exact_only = 1;
        g->lo = 0.f;
        g->hi = 0.f;
        return;
    }
    const double M = (rr + 4.0) * 0x1p-20 + e2 * 0x1p-20;
    g->lo = __double2float_rd(e2 - M);
    g->hi = __double2float_ru(e2 + M);
}

// Exclusive prefix of an int64 over the workgroup (kBandT threads); ws: kBandT / 64 + 1 slots
__device__ int64_t bd_scan64(int64_t v, int64_t* ws, int64_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t run = 0;
        for (int k = 0; k < kBandT / 64; ++k) {
            const int64_t t = ws[k];
            ws[k] = run;
            run += t;
        }
        ws[kBandT / 64] = run;
    }
    __syncthreads();
    const int64_t r = ws[w] + incl - v;
    *total = ws[kBandT / 64];
    __syncthreads();
    return r;
}

// Global union-find over input indices (the merge): agent-scope loads, CAS hooks of the larger
// root under the smaller
// (parents only decrease along a path; the bound keeps a forest of a run whose barrier gave
// up, and whose result is discarded, from looping)
__device__ __forceinline__ int bd_find(int32_t* par, int x) {
    for (int k = 0; k < kBandMaxPoints; ++k) {
        const int p = __hip_atomic_load(par + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == x || (unsigned)p >= (unsigned)kBandMaxPoints) return x;
        x = p;
    }
    return x;
}
__device__ __forceinline__ double bd_load(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(
        reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
        __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void bd_unite(int32_t* par, int a, int b) {
    for (int k = 0; k < kBandMaxPoints; ++k) {
        a = bd_find(par, a);
        b = bd_find(par, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        int expected = a;
        if (__hip_atomic_compare_exchange_strong(par + a, &expected, b, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
    }
}

static_assert(kBandMaxPoints <= (int64_t)kBandMaxWG * kBandT, "one slice point per thread");

__global__ __launch_bounds__(kBandT, 1) void band_fit_kernel(
    const double* __restrict__ x, const double* __restrict__ y, int m, double eps, double eps2,
    int min_points, int mode, int32_t* __restrict__ cluster, uint8_t* __restrict__ flag,
    GridParams* __restrict__ gp, int32_t* st, double* mirror, BandArgs ba, uint32_t spin_limit) {
    __shared__ BandLds L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int g = blockIdx.x, G = gridDim.x;
    constexpr int kW = kBandT / 64;
    SM_STAMP(0);
    // (the fit state: kStError is cleared by the host before the launch, see spread_fit_kernel)
    if (g == 0 && tid != kStError) sm_zero_stats(st, mirror, tid);
    if (g == 0 && tid < 2) ba.cnt[tid] = 0;  // (added to after barrier 1 only)

    // ---- this workgroup's slice of the input, one point per thread: the non-finite points'
    // labels, the slice's bbox published ----
    const int chunk = (m + G - 1) / G;  // (<= kBandT: m <= kBandMaxPoints = kBandMaxWG * kBandT)
    const int pi = g * chunk + tid;
    const bool have = tid < chunk && pi < m;
    double px = 0.0, py = 0.0;
    bool fin = false;
    if (have) {
        px = x[pi];
        py = y[pi];
        fin = isfinite(px) && isfinite(py);
        if (!fin) {  // nobody's neighbour: noise (minPoints >= 1)
            cluster[pi] = 0;
            flag[pi] = DBSCAN_FLAG_NOISE;
            ba.core[pi] = 0;  // (the numbering reads every point's core flag)
        }
    }
    // (up to kBandFullBox points every workgroup reduces the whole bbox itself, from L2, instead
    // of publishing its slice's and meeting at a barrier)
    const bool fullbox = m <= kBandFullBox;
    uint32_t nbar = 0;  // grid barriers met so far
    {
        double mnx = fin ? px : INFINITY, mxx = fin ? px : -INFINITY;
        double mny = fin ? py : INFINITY, mxy = fin ? py : -INFINITY, nfin = fin ? 1.0 : 0.0;
        if (fullbox) {
            mnx = mny = INFINITY;
            mxx = mxy = -INFINITY;
            nfin = 0.0;
            for (int i0 = tid; i0 < m; i0 += 4 * kBandT) {
                double a[4], b[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = i0 + u * kBandT;
                    a[u] = i < m ? x[i] : NAN;
                    b[u] = i < m ? y[i] : NAN;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (isfinite(a[u]) && isfinite(b[u])) {
                        mnx = fmin(mnx, a[u]);
                        mxx = fmax(mxx, a[u]);
                        mny = fmin(mny, b[u]);
                        mxy = fmax(mxy, b[u]);
                        nfin += 1.0;
                    }
            }
        }
        const int w = tid >> 6;
        mnx = wave_min(mnx);
        mxx = wave_max(mxx);
        mny = wave_min(mny);
        mxy = wave_max(mxy);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nfin += __shfl_xor(nfin, o, 64);
        if (lane == 0) {
            L.red[0][w] = mnx;
            L.red[1][w] = mxx;
            L.red[2][w] = mny;
            L.red[3][w] = mxy;
            L.red[4][w] = nfin;
        }
        __syncthreads();
        if (tid < 5) {
            double v = L.red[tid][0];
            for (int k = 1; k < kW; ++k) {
                const double u = L.red[tid][k];
                v = tid == 4 ? v + u : ((tid & 1) ? fmax(v, u) : fmin(v, u));
            }
            if (fullbox) L.red[tid][0] = v; else ba.box[g * 5 + tid] = v;
        }
    }
    SM_STAMP(1);
    if (!fullbox) sp_grid_sync(ba.bar, (++nbar) * (uint32_t)G, st, mirror, spin_limit);
    SM_STAMP(2);

    // ---- the grid from the G partial boxes (one reduction tree: the same grid everywhere) ----
    if (!fullbox && tid < 5 * 64) {  // wave j reduces quantity j over the G <= 64 boxes
        const int j = tid >> 6;
        double v = lane < G ? bd_load(ba.box + lane * 5 + j)
                            : (j == 4 ? 0.0 : ((j & 1) ? -INFINITY : INFINITY));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double u = __shfl_xor(v, o, 64);
            v = j == 4 ? v + u : ((j & 1) ? fmax(v, u) : fmin(v, u));
        }
        if (lane == 0) L.red[j][0] = v;
    }
    __syncthreads();
    if (tid == 0) {
        band_make_grid(L.red[0][0], L.red[1][0], L.red[2][0], L.red[3][0], (int)L.red[4][0], eps,
                       eps2, G, &L.G);
        // rows along the axis that makes them shorter: a dense partition wider than tall (the
        // strips EvenSplitPartitioner cuts out of a cluster's core) would stage rows of
        // thousands of points and overflow (tools/band_overflow_sim.py: 6 of the 1597 G(10^7)
        // partitions with rows along y alone, none this way).  Every geometric step below runs
        // on (y, x); the exact predicate reads the input's own x, y by index, and
        // fl(dx*dx) + fl(dy*dy) is the same sum either way round.
        L.G.swap = 0;
        if (!L.G.bad && L.G.nf > 0 && L.G.nx > L.G.ny) {
            band_make_grid(L.red[2][0], L.red[3][0], L.red[0][0], L.red[1][0], (int)L.red[4][0],
                           eps, eps2, G, &L.G);
            L.G.swap = 1;
        }
    }
    __syncthreads();
    const int nf = L.G.nf, nx = L.G.nx, ny = L.G.ny;
    const bool swp = L.G.swap != 0;
    const double* X = swp ? y : x;  // (the geometry's coordinates)
    const double* Y = swp ? x : y;
    if (swp) {
        const double t = px;
        px = py;
        py = t;
    }
    // the cell of a finite point (quarter bits << 13 above the cell is the caller's)
    const auto cell_of = [&](double a, double b, int& row, int& col, int& quad) {
        int qx = (int)floor(2.0 * ((a * 0.5 - L.G.xmin2) * L.G.invx));
        int qy = (int)floor(2.0 * ((b * 0.5 - L.G.ymin2) * L.G.invy));
        qx = min(max(qx, 0), 2 * nx - 1);
        qy = min(max(qy, 0), 2 * ny - 1);
        row = qy >> 1;
        col = qx >> 1;
        quad = ((qy & 1) << 1) | (qx & 1);
    };
    const bool gbad = L.G.bad != 0 || nf == 0;  // (bad: unreachable for finite bboxes)
    int prow = -1, pcol = 0, pquad = 0;
    if (fin && !gbad) cell_of(px, py, prow, pcol, pquad);
    // the row histogram: of the whole partition in LDS (up to kBandFullBox points: no global
    // row counts, no barrier), else of the slice, added to the global row counts
    if (!gbad) {
        for (int r = tid; r < ny; r += kBandT) L.info[r] = 0u;
        __syncthreads();
        if (fullbox) {
            for (int i = tid; i < m; i += kBandT) {
                const double a = X[i], b = Y[i];
                if (isfinite(a) && isfinite(b)) {
                    int row, col, quad;
                    cell_of(a, b, row, col, quad);
                    atomicAdd(&L.info[row], 1u);
                }
            }
        } else {
            if (prow >= 0) atomicAdd(&L.info[prow], 1u);
            __syncthreads();
            for (int r = tid; r < ny; r += kBandT)
                if (L.info[r]) atomicAdd(ba.rowcnt + r, L.info[r]);
        }
    }
    SM_STAMP(3);
    if (!fullbox) sp_grid_sync(ba.bar, (++nbar) * (uint32_t)G, st, mirror, spin_limit);
    __syncthreads();
    SM_STAMP(4);

    // ---- the bands: cell ranges of equal cost ----
    // A cell of row r holding n points costs n a(r) + b.  The work: a point's count and walks,
    // ~ kBandC0 + the row's points per cell (its stencil's density), so a(r) >= kBandC0 nx +
    // pts(r) (in units of 1 / nx), and a cell's table entry, b >= nx.  The floors a(r) >= fp
    // and b >= fr / nx, with fp = 3 Tw / (G Pmax) and fr = 3 Tw / (G Rmax) (Tw: the total work
    // alone), keep each range within Pmax = kBandCap / 2 own points and Rmax = kBandCells / nx
    // - 2 own rows (the halo rows take the rest).  Workgroup g owns the cells whose cost offset
    // (row-major) lies in [g T / G, (g + 1) T / G); it stages the rows of those cells and one
    // halo row either side.  Dense rows shared by several workgroups are staged by each of
    // them, with the cells split between them.
    int ra = 0, rb = 0, sa = 0, sb = 0, p_ra = 0, p_rb = 0;
    int64_t lo_g = 0, hi_g = 0, c_ra = 0, c_rb = 0, fpt = 0, bcell = 1;
    bool bad = gbad;
    if (!gbad) {
        int64_t* C = reinterpret_cast<int64_t*>(L.rec);  // [ny + 1] cost prefix (until staging)
        int64_t* ws64 = reinterpret_cast<int64_t*>(&L.red[0][0]);
        {  // exclusive prefixes over the rows: par[r] = points in rows < r, C[r] = their cost
            constexpr int kRowsPer = (kBandCap + kBandT - 1) / kBandT;
            int v[kRowsPer], sum = 0;
            int64_t q = 0;
#pragma unroll
            for (int k = 0; k < kRowsPer; ++k) {
                const int r = tid * kRowsPer + k;
                v[k] = r >= ny ? 0
                       : fullbox ? (int)L.info[r]
                                 : (int)__hip_atomic_load(ba.rowcnt + r, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                v[k] = min(max(v[k], 0), kBandMaxPoints);  // (a gave-up barrier: stay in bounds)
                sum += v[k];
                q += (int64_t)v[k] * ((int64_t)kBandC0 * nx + v[k]);
            }
            int64_t qtot = 0;
            (void)bd_scan64(q, ws64, &qtot);
            const int64_t tw = qtot + (int64_t)nx * nx * ny;
            const int64_t rmax = max(1, kBandCells / nx - 2), pmax = kBandCap / 2;
            fpt = (3 * tw + G * pmax - 1) / (G * pmax);
            const int64_t fr = (3 * tw + G * rmax - 1) / (G * rmax);
            bcell = max((int64_t)nx, (fr + nx - 1) / nx);
            const auto a_of = [&](int pts) {
                return max((int64_t)kBandC0 * nx + pts, fpt);
            };
            int64_t cs = 0;
#pragma unroll
            for (int k = 0; k < kRowsPer; ++k)
                if (tid * kRowsPer + k < ny) cs += (int64_t)v[k] * a_of(v[k]) + nx * bcell;
            int64_t T = 0;
            int64_t crun = bd_scan64(cs, ws64, &T);
            int tot = 0;
            int run = sm_excl_scan(sum, L.wsc, &tot);
#pragma unroll
            for (int k = 0; k < kRowsPer; ++k) {
                const int r = tid * kRowsPer + k;
                if (r < ny) {
                    L.par[r] = run;
                    C[r] = crun;
                    crun += (int64_t)v[k] * a_of(v[k]) + nx * bcell;
                }
                run += v[k];
            }
            if (tid == 0) {
                L.par[ny] = tot;
                C[ny] = T;
            }
            __syncthreads();
            // (the row counts of every slice add up to nf unless a barrier gave up)
            if (tot != nf) bad = true;
        }
        const int64_t T = C[ny];
        lo_g = (int64_t)g * T / G;
        hi_g = g + 1 == G ? T : (int64_t)(g + 1) * T / G;
        if (tid < 2) {
            // the last row r with C[r] <= the offset (costs are > 0: C increases strictly)
            const int64_t want = tid ? hi_g : lo_g;
            int lo = 0, hi = ny;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (C[mid] <= want) lo = mid; else hi = mid - 1;
            }
            L.meta[tid] = lo;
        }
        // each of the slice's rows: its piece of the row-sorted records claimed (info: cursor)
        if (!fullbox)
            for (int r = tid; r < ny; r += kBandT) {
                const uint32_t k = L.info[r];
                if (k) L.info[r] = (uint32_t)L.par[r] + atomicAdd(ba.rowcur + r, k);
            }
        __syncthreads();
        ra = L.meta[0];
        rb = L.meta[1];  // (ny: the range runs to the end)
        if (lo_g < hi_g) {
            sa = ra > 0 ? ra - 1 : 0;
            sb = rb + 2 < ny ? rb + 2 : ny;
        } else {
            sa = sb = ra;  // (an empty range stages nothing)
        }
        c_ra = C[ra];
        p_ra = L.par[ra + 1] - L.par[ra];
        c_rb = rb < ny ? C[rb] : T;
        p_rb = rb < ny ? L.par[rb + 1] - L.par[rb] : 0;
        // the slice's records to their rows' pieces
        if (!fullbox && prow >= 0) {
            const uint32_t k = atomicAdd(&L.info[prow], 1u);
            if (k < (uint32_t)L.par[prow + 1] && k < (uint32_t)m) {
                ba.rxy[k] = make_double2(px, py);
                ba.ridx[k] = pi;
            }
        }
    }
    const int row0 = bad ? 0 : L.par[sa];
    int S = bad ? 0 : L.par[sb] - L.par[sa];
    if (S > kBandCap || (sb - sa) * nx > kBandCells) {  // over the staging capacity
        bad = true;
        S = 0;
    }
    if (bad && !gbad && tid == 0) {
        __hip_atomic_store(st + kStError, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mirror)
            __hip_atomic_store(reinterpret_cast<int32_t*>(mirror + kMiscState) + kStError, 3,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    SM_STAMP(5);
    uint16_t* slist = reinterpret_cast<uint16_t*>(L.rbits);  // (fullbox: the staged points)
    static_assert(sizeof(L.rbits) + sizeof(L.wrank) >= kBandCap * sizeof(uint16_t),
                  "the staged list fits rbits + wrank");
    if (!fullbox) {
        sp_grid_sync(ba.bar, (++nbar) * (uint32_t)G, st, mirror, spin_limit);
        // (every workgroup has read the row counts and claimed its pieces: this workgroup's
        // share of them zeroed for the next launch)
        for (int r = g * kBandT + tid; r < kBandCap; r += G * kBandT) {
            ba.rowcnt[r] = 0u;
            ba.rowcur[r] = 0u;
        }
    } else if (S > 0) {
        // the staged rows' points listed by input index (one append per wave)
        if (tid == 0) L.meta[8] = 0;
        __syncthreads();
        for (int i0 = 0; i0 < m; i0 += kBandT) {
            const int i = i0 + tid;
            bool in = false;
            if (i < m) {
                const double a = X[i], b = Y[i];
                if (isfinite(a) && isfinite(b)) {
                    int row, col, quad;
                    cell_of(a, b, row, col, quad);
                    in = row >= sa && row < sb;
                }
            }
            const uint64_t bl = __ballot(in);
            int base = 0;
            if (lane == 0 && bl) base = atomicAdd(&L.meta[8], __popcll(bl));
            base = __shfl(base, 0, 64);
            const int k = base + __popcll(bl & (lane ? (~0ull >> (64 - lane)) : 0ull));
            if (in && k < kBandCap) slist[k] = (uint16_t)i;
        }
        __syncthreads();
        S = min(S, min(L.meta[8], kBandCap));
    }
    SM_STAMP(6);

    // ---- stage the rows [sa, sb): their records, a counting sort by staged cell ----
    const int srows = sb - sa, scells = srows * nx;
    constexpr int kStPer = kBandCap / kBandT;
    // each thread's staged points in registers: the fp32 record and the info word (input index
    // << 16 | quadrant << 13 | staged cell; ~0u: none)
    float2 srec[kStPer];
    uint32_t sinf[kStPer];
    if (S > 0) {
        for (int cc = tid; cc < scells; cc += kBandT) L.info[cc] = 0u;
#pragma unroll
        for (int k = 0; k < kStPer; ++k) {
            const int j = tid + k * kBandT;
            sinf[k] = ~0u;
            srec[k] = make_float2(0.f, 0.f);
            if (j < S) {
                const int i = fullbox ? (int)slist[j] : ba.ridx[row0 + j];
                const double2 r = fullbox ? make_double2(X[i], Y[i]) : ba.rxy[row0 + j];
                if (i >= 0 && i < m && isfinite(r.x) && isfinite(r.y)) {
                    int row, col, quad;
                    cell_of(r.x, r.y, row, col, quad);
                    if (row >= sa && row < sb) {  // (always, unless a barrier gave up)
                        sinf[k] = ((uint32_t)i << 16) | ((uint32_t)quad << 13) |
                                  (uint32_t)((row - sa) * nx + col);
                        srec[k] = make_float2((float)((r.x * 0.5 - L.G.cx2) * L.G.invs),
                                              (float)((r.y * 0.5 - L.G.cy2) * L.G.invs));
                    }
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kStPer; ++k)
            if (sinf[k] != ~0u) atomicAdd(&L.info[sinf[k] & kCellMask], 1u);
        __syncthreads();
        {
            constexpr int kCellPer = (kBandCells + kBandT - 1) / kBandT;
            int cnt[kCellPer], sum = 0;
#pragma unroll
            for (int k = 0; k < kCellPer; ++k) {
                const int cc = tid * kCellPer + k;
                cnt[k] = cc < scells ? (int)L.info[cc] : 0;
                sum += cnt[k];
            }
            int tot = 0;
            int run = sm_excl_scan(sum, L.wsc, &tot);
#pragma unroll
            for (int k = 0; k < kCellPer; ++k) {
                const int cc = tid * kCellPer + k;
                if (cc < scells) {
                    L.par[cc] = run;
                    L.cst[cc] = (uint16_t)run;
                }
                run += cnt[k];
            }
            if (tid == 0) L.cst[scells] = (uint16_t)tot;
            S = tot;  // (the records placed: S unless a barrier gave up)
        }
        __syncthreads();
        // placed one quadrant after the other: each cell's slots grouped by quarter, in order
        for (uint32_t qq = 0; qq < 3u; ++qq) {
#pragma unroll
            for (int k = 0; k < kStPer; ++k) {
                if (sinf[k] != ~0u && ((sinf[k] >> 13) & 3u) == qq) {
                    const int s = atomicAdd(&L.par[sinf[k] & kCellMask], 1);
                    L.rec[s] = srec[k];
                    L.info[s] = sinf[k];
                    sinf[k] = ~0u;
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < kStPer; ++k) {
            if (sinf[k] != ~0u) {
                const int s = atomicAdd(&L.par[sinf[k] & kCellMask], 1);
                L.rec[s] = srec[k];
                L.info[s] = sinf[k];
            }
        }
        // own cells [ca, cb) (staged numbering): the first cells of rows ra / rb whose cost
        // offset reaches lo_g / hi_g, one wave each
        if (tid < 128) {
            const int w = tid >> 6, lane = tid & 63;
            const int row = w ? rb : ra;
            int res = scells;  // (rb == ny: to the end)
            if (row < ny) {
                const int64_t target = w ? hi_g : lo_g;
                const int pr = w ? p_rb : p_ra;
                const int64_t ar = max((int64_t)kBandC0 * nx + pr, fpt);
                int64_t base = w ? c_rb : c_ra;
                const int c0 = (row - sa) * nx;
                res = c0 + nx;  // (none in the row: the next row's first cell)
                for (int j0 = 0; j0 < nx; j0 += 64) {
                    const int j = j0 + lane;
                    int64_t cost = 0;
                    if (j < nx) {
                        const int n = (int)L.cst[c0 + j + 1] - (int)L.cst[c0 + j];
                        cost = (int64_t)n * ar + bcell;
                    }
                    int64_t incl = cost;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const int64_t t = __shfl_up(incl, d, 64);
                        if (lane >= d) incl += t;
                    }
                    const uint64_t hit = __ballot(j < nx && base + incl - cost >= target);
                    if (hit) {
                        res = c0 + j0 + __ffsll((unsigned long long)hit) - 1;
                        break;
                    }
                    base += __shfl(incl, 63, 64);
                }
            }
            if (lane == 0) L.meta[4 + w] = res;
        }
        __syncthreads();
    }
    SM_STAMP(7);
    BAND_WG(0, wall_clock64());
    // the staged stencil context: rows [sa, sb) as rows 0 .. srows - 1
    const SmCtx c{x, y, eps2, L.G.lo, L.G.hi, nx, srows, L.G.exact_only != 0};
    // own slots: the cells [ca, cb)
    const int ca = S > 0 ? L.meta[4] : 0, cb = S > 0 ? L.meta[5] : 0;
    const int s0 = S > 0 ? (int)L.cst[ca] : 0;
    const int s1 = S > 0 ? (int)L.cst[cb] : 0;
    int occupied = 0;
    for (int cc = ca + tid; cc < cb; cc += kBandT) occupied += L.cst[cc + 1] > L.cst[cc] ? 1 : 0;

    // ---- count (own points): a thread each when they fill a quarter of the workgroup, else
    // a wave each (64 candidates per step, ballot counts) ----
    int ncore = 0;
    // the staged slots' LDS forest, and their core flags: the own ones from the count, the
    // halo's after barrier 1
    for (int p = tid; p < S; p += kBandT) {
        L.par[p] = p;
        L.core[p] = 0;
    }
    __syncthreads();
    // (a thread per point from 256 own points: 128, 64 and always measured within 1-4%)
    if (s1 - s0 >= kBandT / 4) {
        for (int p = s0 + tid; p < s1; p += kBandT) {
            const bool cc = sm_count(L, c, p, min_points, -1) >= min_points;
            const int v = (int)(L.info[p] >> 16);
            ba.core[v] = cc ? 1 : 0;
            ba.par[v] = v;
            L.core[p] = cc ? 1 : 0;
            ncore += cc ? 1 : 0;
        }
    } else {
        for (int p = s0 + (tid >> 6); p < s1; p += kW) {
            const bool cc = sp_count_wave(L, c, p, min_points) >= min_points;
            if (lane == 0) {
                const int v = (int)(L.info[p] >> 16);
                ba.core[v] = cc ? 1 : 0;
                ba.par[v] = v;
                L.core[p] = cc ? 1 : 0;
                ncore += cc ? 1 : 0;
            }
        }
    }
    // own quarters' chains and list, ahead of barrier 1 (they need only the own core flags)
    __syncthreads();
    const bool quarters = L.G.clique != 0;
    uint32_t* qlist = L.rbits;  // (rbits and wrank are free until the numbering)
    constexpr int kQMax = 2 * kBandWords;
    static_assert(sizeof(L.rbits) + sizeof(L.wrank) == kQMax * sizeof(uint32_t) &&
                      offsetof(BandLds, wrank) == offsetof(BandLds, rbits) + sizeof(L.rbits),
                  "qlist spans rbits and wrank");
    if (quarters) {
        if (tid == 0) L.meta[6] = 0;
        __syncthreads();
        // each own core chained to the previous core of its quarter (one union per thread), own
        // quarter runs holding a core listed.  (Chaining the halo quarters too made the
        // distance-2 pass shorter but published ~2x the pairs: 65536 points 222 -> 241 us.)
        for (int sl = s0 + tid; sl < s1; sl += kBandT) {
            const uint32_t inf = L.info[sl];
            const int cell = (int)(inf & kCellMask);
            const uint32_t qd = (inf >> 13) & 3u;
            const int cb0 = L.cst[cell];
            const bool start = sl == cb0 || ((L.info[sl - 1] >> 13) & 3u) != qd;
            if (L.core[sl]) {
                for (int t = sl - 1; t >= cb0 && ((L.info[t] >> 13) & 3u) == qd; --t)
                    if (L.core[t]) {
                        (void)sm_unite_from(L.par, L.info, t, sl);
                        break;
                    }
            }
            if (!start) continue;
            const int ce = L.cst[cell + 1];
            int e = sl + 1;
            bool any = L.core[sl] != 0;
            while (e < ce && ((L.info[e] >> 13) & 3u) == qd) {
                any = any || L.core[e] != 0;
                ++e;
            }
            if (any) {
                const int k = atomicAdd(&L.meta[6], 1);
                if (k < kQMax) qlist[k] = (uint32_t)sl | ((uint32_t)e << 16);
            }
        }
        __syncthreads();
    }
    SM_STAMP(8);
    BAND_WG(1, wall_clock64());
    sp_grid_sync(ba.bar, (++nbar) * (uint32_t)G, st, mirror, spin_limit);
    SM_STAMP(9);
    BAND_WG(2, wall_clock64());

    // ---- union: the staged core flags, own cores' walks, the forest published ----
    {
        int tot = 0, occ = 0;
        (void)sm_excl_scan(ncore, L.wsc, &tot);
        (void)sm_excl_scan(occupied, L.wsc, &occ);
        if (tid == 0) {
            if (tot) atomicAdd(&ba.cnt[0], tot);
            if (occ) atomicAdd(&ba.cnt[1], occ);
        }
    }
    for (int p = tid; p < S; p += kBandT)
        if (p < s0 || p >= s1) L.core[p] = ba.core[L.info[p] >> 16];
    if (tid == 0) L.meta[2] = 0;
    __syncthreads();
    BAND_WG(6, wall_clock64());
    const double reach_kx = (L.G.cx2 - L.G.xmin2) * L.G.invx;
    const double reach_ky = (L.G.cy2 - L.G.ymin2) * L.G.invy - (double)sa;  // (staged rows)
    // Quarter-level unions (clique grids: a quarter cell's cores are one clique; the staged
    // slots of a cell are grouped by quarter): each own core chained to the previous core of
    // its quarter; then for each own quarter holding a core and each of the 12 quarters after
    // it (quarter-grid offsets within 2, row-major order) a core pair within eps searched and
    // united -- adjacent quarters first, then (after a barrier) the distance-2 ones, skipped
    // when already in one set, their far cores pruned by the other quarter's box.  Every
    // quarter pair is tested by the owner of its smaller quarter, which stages both.  Against
    // the per-core stencil walks: 133 / 147 / 171 / 191 -> 112 / 138 / 155 / 178 us per kernel
    // at 12k / 20k / 40k / 65k points (the walks repeat each quarter's work for every core).
    bool walked = false;
    if (quarters) {
        const int nq = L.meta[6];
        BAND_WG(8, wall_clock64());
        BAND_WG(10, nq);
        if (nq <= kQMax) {
            walked = true;
            const auto run_of = [&](int cell, uint32_t qd, int& b, int& e) {
                int lo = L.cst[cell], hi = L.cst[cell + 1];
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (((L.info[mid] >> 13) & 3u) < qd) lo = mid + 1; else hi = mid;
                }
                b = lo;
                hi = L.cst[cell + 1];
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (((L.info[mid] >> 13) & 3u) <= qd) lo = mid + 1; else hi = mid;
                }
                e = lo;
            };
            for (int pass = 0; pass < 2; ++pass) {
                const int K = pass ? 8 : 4;
                for (int it = tid; it < nq * K; it += kBandT) {
                    const int k = it / nq, qi = it - k * nq;
                    const uint32_t rq = qlist[qi];
                    const int qs = (int)(rq & 0xFFFFu), qe = (int)(rq >> 16);
                    const uint32_t inf = L.info[qs];
                    const int cell = (int)(inf & kCellMask);
                    const int qd = (int)((inf >> 13) & 3u);
                    const int cy = cell / nx, cx = cell - cy * nx;
                    // forward offsets (dx, dy): adjacent (1,0) (-1,1) (0,1) (1,1); distance 2
                    // (2,0) (-2,1) (2,1) (-2,2) (-1,2) (0,2) (1,2) (2,2)
                    const int dx = pass ? (k == 0 ? 2 : (k == 1 ? -2 : (k == 2 ? 2 : k - 5)))
                                        : (k == 0 ? 1 : k - 2);
                    const int dy = pass ? (k == 0 ? 0 : (k < 3 ? 1 : 2)) : (k == 0 ? 0 : 1);
                    const int hx = 2 * cx + (qd & 1) + dx, hy = 2 * cy + (qd >> 1) + dy;
                    if (hx < 0 || hx >= 2 * nx || hy < 0 || hy >= 2 * srows) continue;
                    int b2, e2;
                    run_of((hy >> 1) * nx + (hx >> 1), (uint32_t)(((hy & 1) << 1) | (hx & 1)), b2,
                           e2);
                    int fb = -1;
                    for (int t = b2; t < e2; ++t)
                        if (L.core[t]) {
                            fb = t;
                            break;
                        }
                    if (fb < 0) continue;
                    int fa = qs;
                    while (!L.core[fa]) ++fa;
                    if (sm_find(L.par, fa) == sm_find(L.par, fb)) continue;
                    // the other quarter's box in the records' cell units, and a squared reach
                    // over the fp32 threshold with the records' error margin
                    const double bx0 = 0.5 * (double)hx - reach_kx;
                    const double by0 = 0.5 * (double)hy - reach_ky;
                    bool found = false;
                    // (far pairs: the other quarter's cores near this quarter's box, as a mask;
                    // 16384 / 20000 / 65536 points 135 / 149 / 216 -> 127 / 138 / 192 us)
                    uint64_t bm = ~0ull;
                    const bool masked = pass && !c.exact_only && e2 - fb <= 64;
                    if (masked) {
                        const double ax0 = 0.5 * (double)(2 * cx + (qd & 1)) - reach_kx;
                        const double ay0 = 0.5 * (double)(2 * cy + (qd >> 1)) - reach_ky;
                        bm = 0ull;
                        for (int b = fb; b < e2; ++b) {
                            if (!L.core[b]) continue;
                            const float2 rb = L.rec[b];
                            const float ddx = (float)fmax(0.0, fmax(ax0 - (double)rb.x,
                                                                    (double)rb.x - (ax0 + 0.5)));
                            const float ddy = (float)fmax(0.0, fmax(ay0 - (double)rb.y,
                                                                    (double)rb.y - (ay0 + 0.5)));
                            const float mg = (fabsf(rb.x) + fabsf(rb.y) + 4.0f) * 0x1p-18f + 0x1p-12f;
                            const float rr = (sqrtf(c.hi) + mg) * (sqrtf(c.hi) + mg);
                            if (ddx * ddx + ddy * ddy <= rr) bm |= 1ull << (b - fb);
                        }
                        if (!bm) continue;
                    }
                    for (int a = fa; a < qe && !found; ++a) {
                        if (!L.core[a]) continue;
                        const float2 ra = L.rec[a];
                        if (pass && !c.exact_only) {
                            const float ddx = (float)fmax(0.0, fmax(bx0 - (double)ra.x,
                                                                    (double)ra.x - (bx0 + 0.5)));
                            const float ddy = (float)fmax(0.0, fmax(by0 - (double)ra.y,
                                                                    (double)ra.y - (by0 + 0.5)));
                            const float mg = (fabsf(ra.x) + fabsf(ra.y) + 4.0f) * 0x1p-18f + 0x1p-12f;
                            const float rr = (sqrtf(c.hi) + mg) * (sqrtf(c.hi) + mg);
                            if (ddx * ddx + ddy * ddy > rr) continue;
                        }
                        if (masked) {
                            for (uint64_t mm = bm; mm; mm &= mm - 1) {
                                const int b = fb + __ffsll((unsigned long long)mm) - 1;
                                if (sm_pair(L, c, a, ra, b, L.rec[b])) {
                                    (void)sm_unite_from(L.par, L.info, a, b);
                                    found = true;
                                    break;
                                }
                            }
                            continue;
                        }
                        for (int b = fb; b < e2; ++b) {
                            if (!L.core[b]) continue;
                            if (sm_pair(L, c, a, ra, b, L.rec[b])) {
                                (void)sm_unite_from(L.par, L.info, a, b);
                                found = true;
                                break;
                            }
                        }
                    }
                }
                __syncthreads();
                BAND_WG(9 + 2 * pass, wall_clock64());
            }
        }
    }
    // (other grids, or more own quarters than the list holds: per-core stencil walks; row-
    // major items: the lanes of a wave walk one stencil row of consecutive points, mostly of
    // one cell, so their LDS reads coincide: 107 -> 58 us per workgroup at 65536 points)
    for (int it = walked ? 0x7FFFFFFF : tid; it < (s1 - s0) * 3; it += kBandT) {
        const int d = it / (s1 - s0), i = it - d * (s1 - s0);
        if (L.core[s0 + i]) sm_union_walk(L, c, s0 + i, d, quarters, reach_kx, reach_ky);
    }
    __syncthreads();
    SM_STAMP(10);
    BAND_WG(7, wall_clock64());
    uint32_t* mine = ba.pairs + (int64_t)g * kBandCap;
    for (int p = tid; p < S; p += kBandT) {
        if (!L.core[p] || L.par[p] == p) continue;
        int r = p;
        for (int u = L.par[r]; u != r; u = L.par[r]) r = u;
        const int k = atomicAdd(&L.meta[2], 1);
        mine[k] = (L.info[p] & 0xFFFF0000u) | (L.info[r] >> 16);
    }
    __syncthreads();
    const int npairs = L.meta[2];
    SM_STAMP(11);
    BAND_WG(3, wall_clock64());
    BAND_WG(4, s1 - s0);
    BAND_WG(5, S);
    sp_grid_sync(ba.bar, (++nbar) * (uint32_t)G, st, mirror, spin_limit);
    SM_STAMP(12);

    // ---- merge: this workgroup's pairs into the global union-find over input indices ----
    // (v's local root r is the smallest index of its LDS set, r < v: while v is still a
    // global root, one CAS hooks it under r; otherwise the full union)
    for (int k = tid; k < npairs; k += kBandT) {
        const uint32_t w = mine[k];
        const int v = (int)(w >> 16), r = (int)(w & 0xFFFFu);
        int expected = v;
        if (!__hip_atomic_compare_exchange_strong(ba.par + v, &expected, r, __ATOMIC_RELAXED,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            bd_unite(ba.par, v, r);
    }
    SM_STAMP(13);
    sp_grid_sync(ba.bar, (++nbar) * (uint32_t)G, st, mirror, spin_limit);
    SM_STAMP(14);

    // ---- roots of every staged core (read-only walks: every union is done) into L.par (the
    // LDS forest is published); root bits of all points straight from the global forest (a
    // core is a root iff it is its own parent), so no barrier between roots and numbering ----
    // (plain loads: the forest is final after the barrier, which invalidated the L1)
    for (int p = tid; p < S; p += kBandT) {
        if (!L.core[p]) continue;
        int r = (int)(L.info[p] >> 16);
        for (int k = 0; k < kBandMaxPoints; ++k) {
            const int u = ba.par[r];
            if (u == r || (unsigned)u >= (unsigned)kBandMaxPoints) break;
            r = u;
        }
        L.par[p] = r;
    }
    SM_STAMP(15);
    SM_STAMP(16);
    const int nw = (m + 31) / 32;
    int nclust = 0;
    {
        // (four points per thread by one 4-byte and one 16-byte load, two steps' loads in
        // flight together; a root word from 8 lanes' nibbles)
        constexpr int kChunk = 4 * kBandT;
        for (int u0 = 0; u0 < nw * 32; u0 += 2 * kChunk) {
            uint32_t cw[2];
            int4 pv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ub = u0 + h * kChunk + 4 * tid;
                cw[h] = ub < m ? *reinterpret_cast<const uint32_t*>(ba.core + ub) : 0u;
                pv[h] = ub < m ? *reinterpret_cast<const int4*>(ba.par + ub) : make_int4(-1, -1, -1, -1);
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ub = u0 + h * kChunk + 4 * tid;
                uint32_t nib = 0;
                nib |= ((cw[h] & 0xFFu) && pv[h].x == ub && ub < m) ? 1u : 0u;
                nib |= ((cw[h] & 0xFF00u) && pv[h].y == ub + 1 && ub + 1 < m) ? 2u : 0u;
                nib |= ((cw[h] & 0xFF0000u) && pv[h].z == ub + 2 && ub + 2 < m) ? 4u : 0u;
                nib |= ((cw[h] & 0xFF000000u) && pv[h].w == ub + 3 && ub + 3 < m) ? 8u : 0u;
                uint32_t wv = nib << (4 * (lane & 7));
                wv |= (uint32_t)__shfl_xor((int)wv, 1, 64);
                wv |= (uint32_t)__shfl_xor((int)wv, 2, 64);
                wv |= (uint32_t)__shfl_xor((int)wv, 4, 64);
                if ((lane & 7) == 0 && ub < nw * 32) L.rbits[ub >> 5] = wv;
            }
        }
        __syncthreads();
        constexpr int kWPer = kBandWords / kBandT;
        int v[kWPer], sum = 0;
#pragma unroll
        for (int k = 0; k < kWPer; ++k) {
            const int wd = tid * kWPer + k;
            const uint32_t bits = wd < nw ? L.rbits[wd] : 0u;
            if (wd >= nw && wd < kBandWords) L.rbits[wd] = 0u;
            v[k] = __popc(bits);
            sum += v[k];
        }
        int run = sm_excl_scan(sum, L.wsc, &nclust);
#pragma unroll
        for (int k = 0; k < kWPer; ++k) {
            const int wd = tid * kWPer + k;
            if (wd < kBandWords) L.wrank[wd] = run;
            run += v[k];
        }
        __syncthreads();
    }
    SM_STAMP(17);
    const auto cluster_of = [&](uint32_t s) {
        return L.wrank[s >> 5] + __popc(L.rbits[s >> 5] & ((1u << (s & 31u)) - 1u)) + 1;
    };
    for (int p = s0 + tid; p < s1; p += kBandT) {  // cores: one thread each
        if (!L.core[p]) continue;
        const uint32_t v = L.info[p] >> 16;
        cluster[v] = cluster_of((uint32_t)L.par[p]);
        flag[v] = DBSCAN_FLAG_CORE;
    }
    for (int p = s0 + (tid >> 6); p < s1; p += kW) {  // non-cores: a wave each
        if (L.core[p]) continue;
        const float2 me = L.rec[p];
        const int cc = (int)(L.info[p] & kCellMask);
        const int cy = cc / nx, cx = cc - cy * nx;
        const int x0 = max(cx - 1, 0), x1 = min(cx + 1, nx - 1);
        uint32_t best = 0xFFFFFFFFu;
        for (int d = 0; d < 3; ++d) {
            const int r = d == 0 ? cy : (d == 1 ? cy - 1 : cy + 1);
            if (r < 0 || r >= srows) continue;
            const int e = L.cst[r * nx + x1 + 1];
            for (int q = L.cst[r * nx + x0] + lane; q < e; q += 64) {
                if (!L.core[q]) continue;
                const uint32_t s = (uint32_t)L.par[q];
                if (s < best && sm_pair(L, c, p, me, q, L.rec[q])) best = s;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, 64));
        if (lane == 0) {
            const uint32_t v = L.info[p] >> 16;
            int cid = 0;
            uint8_t f = DBSCAN_FLAG_NOISE;
            if (best != 0xFFFFFFFFu && (mode != DBSCAN_MODE_NAIVE || best < v)) {
                cid = cluster_of(best);
                f = DBSCAN_FLAG_BORDER;
            }
            cluster[v] = cid;
            flag[v] = f;
        }
    }
    SM_STAMP(18);
    // ---- statistics (workgroup 0) and the barrier reset (the last workgroup to leave) ----
    if (g == 0 && tid == 0) {
        sm_set_stat(st, mirror, kStNf, nf);
        sm_set_stat(st, mirror, kStCore, __hip_atomic_load(&ba.cnt[0], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
        sm_set_stat(st, mirror, kStClusters, nclust);
        sm_set_stat(st, mirror, kStCells, nf > 0 ? __hip_atomic_load(&ba.cnt[1], __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_AGENT)
                                                 : 0);
        // (reported in the input's axes)
        GridParams gg{swp ? L.G.ymin2 : L.G.xmin2, swp ? L.G.xmin2 : L.G.ymin2,
                      swp ? L.G.invy : L.G.invx, swp ? L.G.invx : L.G.invy,
                      (uint32_t)(swp ? ny : nx), (uint32_t)(swp ? nx : ny), 1u, 1u, L.G.clique};
        *gp = gg;
        if (mirror) *reinterpret_cast<GridParams*>(mirror + kMiscGrid) = gg;
    }
    // The last workgroup to leave resets the barrier words.  After a barrier gave up (bar[2]
    // raised) workgroups that were not resident added to the row counts after others had
    // zeroed their shares: that workgroup zeroes them all (every other workgroup has left, and
    // the acq_rel departure orders their writes before its own), so the next band fit on the
    // handle starts from clean counters whatever this one's outcome.
    if (tid == 0) {
        const bool last = __hip_atomic_fetch_add(ba.bar + 1, 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)G - 1;
        L.meta[15] = last ? (sp_load(ba.bar + 2) != 0u ? 2 : 1) : 0;
    }
    __syncthreads();
    const int leave = L.meta[15];
    if (leave == 2 && !fullbox)
        for (int r = tid; r < kBandCap; r += kBandT) {
            __hip_atomic_store(ba.rowcnt + r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ba.rowcur + r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    if (leave && tid == 0) {
        __hip_atomic_store(ba.bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ba.bar + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ba.bar + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace

#if DBSCAN_AB_STAMPS
extern "C" int dbscan_ab_small_stamps(long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sm_stamps), 24 * sizeof(long long)) == hipSuccess
               ? 0 : -1;
}
extern "C" int dbscan_ab_band_wg(long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_band_wg), 64 * 12 * sizeof(long long)) ==
                   hipSuccess
               ? 0 : -1;
}
#endif

bool small_fit_eligible(int64_t n, double eps, int32_t mode) {
    const double eps2 = eps * eps;
    return n >= 0 && n <= kSmallMaxPoints && std::isfinite(eps2) &&
           (mode == DBSCAN_MODE_NAIVE || mode == DBSCAN_MODE_ARCHERY);
}

void enqueue_small_fits(hipStream_t s, Profiler* prof, const double* x, const double* y,
                        const int64_t* d_offs, const int32_t* d_list, int32_t nlist,
                        int64_t single_n, double eps, int32_t min_points, int32_t mode,
                        int32_t* cluster, uint8_t* flag, int32_t* d_nclusters, GridParams* gp,
                        int32_t* st, double* mirror) {
    const unsigned grid = d_offs ? (unsigned)nlist : 1u;
    if (grid == 0) return;
    klaunch(prof, "small_fit", small_fit_kernel, dim3(grid), dim3(kSmT), 0, s, x, y, d_offs,
            d_list, single_n, eps, eps * eps, (int)min_points, (int)mode, cluster, flag,
            d_nclusters, gp, st, mirror);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

// Workgroups of a spread fit: one per kSpreadPer points (at most kSpreadMaxWG; 128 and 512
// measured within a few microseconds of 256 per call, round 4)
constexpr int kSpreadPer = 256;
constexpr size_t kSpreadHead = 512;  // bar[2] at 0, npairs[kSpreadMaxWG] at 64

void enqueue_spread_fit(hipStream_t s, Profiler* prof, Workspace& ws, const double* x,
                        const double* y, int64_t n, double eps, int32_t min_points, int32_t mode,
                        int32_t* cluster, uint8_t* flag, GridParams* gp, int32_t* st,
                        double* mirror) {
    const size_t bytes = kSpreadHead + kSmN + (size_t)kSpreadMaxWG * kSmN * sizeof(uint32_t);
    if (ws.spread.bytes < bytes || !ws.spread_ready) {
        char* p = static_cast<char*>(ws.spread.ensure(bytes));
        DBSCAN_HIP_CHECK(hipMemsetAsync(p, 0, kSpreadHead, s));  // the barrier words, once
        ws.spread_ready = true;
    }
    char* base = static_cast<char*>(ws.spread.p);
    SpreadArgs sa;
    sa.bar = reinterpret_cast<uint32_t*>(base);
    sa.npairs = reinterpret_cast<int32_t*>(base + 64);
    sa.core = reinterpret_cast<uint8_t*>(base + kSpreadHead);
    sa.pairs = reinterpret_cast<uint32_t*>(base + kSpreadHead + kSmN);
    const int G = (int)std::min<int64_t>(kSpreadMaxWG, std::max<int64_t>(1, n / kSpreadPer));
    // (kStError of the fit's own stats block `mirror` is cleared by the caller, enqueue_fit:
    // the kernel never clears it, so a late workgroup 0 cannot erase another's barrier failure)
    if (!mirror) throw ArgError{"spread fit without a stats block"};
    klaunch(prof, "spread_fit", spread_fit_kernel, dim3(G), dim3(kSmT), 0, s, x, y, (int)n, eps,
            eps * eps, (int)min_points, (int)mode, cluster, flag, gp, st, mirror, sa,
            ws.spread_spin_limit);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

bool band_fit_eligible(int64_t n, double eps, int32_t mode, int32_t min_points) {
    const double eps2 = eps * eps;
    return n >= 1 && n <= kBandMaxPoints && std::isfinite(eps2) &&
           (mode == DBSCAN_MODE_NAIVE || mode == DBSCAN_MODE_ARCHERY) && min_points >= 1;
}

void enqueue_band_fit(hipStream_t s, Profiler* prof, Workspace& ws, const double* x,
                      const double* y, int64_t n, double eps, int32_t min_points, int32_t mode,
                      int32_t* cluster, uint8_t* flag, GridParams* gp, int32_t* st,
                      double* mirror) {
    // ~256 points per workgroup, 16..kBandMaxWG of them: fewer co-resident workgroups for the
    // smaller partitions when several executors' fits share the GPU (per-call latency within 1%
    // of 64 workgroups at every size from 3072 to 65536 points)
    const int G = (int)std::min<int64_t>(kBandMaxWG, std::max<int64_t>(16, (n + 255) / 256));
    // scratch: barrier words (zero between launches), counters, per input index core flags,
    // labels and the union-find, root words, the published pairs
    // (zeroed once, then by the kernel itself: bar[2] at 0, cnt[2] at 64, npairs[kBandMaxWG]
    // at 128, the row counts and claims; then the slices' boxes)
    constexpr size_t kHead = 512, kRows = (size_t)kBandCap * 4, kZero = kHead + 2 * kRows;
    constexpr size_t kBox = (size_t)kBandMaxWG * 5 * 8;
    const size_t bytes = kZero + kBox + (size_t)kBandMaxPoints * (1 + 4 + 16 + 4) +
                         (size_t)kBandMaxWG * kBandCap * 4;
    if (ws.band.bytes < bytes || !ws.band_ready) {
        char* p = static_cast<char*>(ws.band.ensure(bytes));
        DBSCAN_HIP_CHECK(hipMemsetAsync(p, 0, kZero, s));
        ws.band_ready = true;
    }
    char* base = static_cast<char*>(ws.band.p);
    BandArgs ba;
    ba.bar = reinterpret_cast<uint32_t*>(base);
    ba.cnt = reinterpret_cast<int32_t*>(base + 64);
    ba.npairs = reinterpret_cast<int32_t*>(base + 128);
    ba.rowcnt = reinterpret_cast<uint32_t*>(base + kHead);
    ba.rowcur = reinterpret_cast<uint32_t*>(base + kHead + kRows);
    ba.box = reinterpret_cast<double*>(base + kZero);
    char* q = base + kZero + kBox;
    ba.rxy = reinterpret_cast<double2*>(q);
    q += (size_t)kBandMaxPoints * 16;
    ba.ridx = reinterpret_cast<int32_t*>(q);
    q += (size_t)kBandMaxPoints * 4;
    ba.core = reinterpret_cast<uint8_t*>(q);
    q += kBandMaxPoints;
    ba.par = reinterpret_cast<int32_t*>(q);
    q += (size_t)kBandMaxPoints * 4;
    ba.pairs = reinterpret_cast<uint32_t*>(q);
    // (kStError of the fit's own stats block: cleared by the caller, as for enqueue_spread_fit)
    if (!mirror) throw ArgError{"band fit without a stats block"};
    klaunch(prof, "band_fit", band_fit_kernel, dim3(G), dim3(kBandT), 0, s, x, y, (int)n, eps,
            eps * eps, (int)min_points, (int)mode, cluster, flag, gp, st, mirror, ba,
            ws.spread_spin_limit);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

}  // namespace dbscan
