// fit.hip -- the local DBSCAN fit on gfx950: eps grid in 8x8-cell tiles, neighbour counts,
// lock-free union-find, border/noise labelling and cluster numbering.
//
// Reference semantics restated here (src/main/scala/org/apache/spark/mllib/clustering/dbscan/):
//   DBSCANPoint.scala:26-30           the fp64 predicate dx*dx + dy*dy <= eps*eps, no FMA
//   LocalDBSCANNaive.scala:37-118     order-dependent fit, as its closed form:
//     core(p) <=> |N(p)| >= minPoints (N includes p);  clusters = components of the core-core
//     eps graph;  s(K) = smallest visit index of a core in K;  cluster id = rank of s(K);
//     non-core b with adjacent clusters A and m = min s(K) over A:
//       Naive  : Border of the cluster with s = m if A != {} and m < index(b), else Noise
//       Archery: Border of the cluster with s = m if A != {}, else Noise
//                                                    (LocalDBSCANArchery.scala:103-106 re-claim)
//
// Layout.  Cells of side >= eps are grouped in 8x8-cell tiles; the sort key is
//   tile (row-major over tiles) | cell in tile (row-major) | quadrant (2x2 quarter cells)
// so every tile is one contiguous slot range and every cell and quarter cell is a contiguous
// sub-range.  A dense per-tile table tslot[tile][0..64] gives the slot start of every local
// cell, so any cell's points are found in O(1).
//
// Kernels, in pipeline order (one HIP stream per handle; DESIGN.md has the rooflines):
//   bin          key per point, perm = input index            [radix sort: primitives.hip]
//   gather       sorted double2 coordinates (AoS)
//   groups       occupied cells / quarter cells / tiles from key head flags (3 scans)
//   tables       tmap (tile id -> occupied tile) and tslot (per-tile cell starts)
//   segs         per cell: up to 6 slot pieces of the 3x3 stencil (global-memory fallback)
//   count_tile   ONE WORKGROUP PER TILE: the tile and its 1-cell halo (<= 100 cells) are staged
//                in LDS; each point scans its 3 contiguous LDS stencil ranges, own cell first,
//                with early exit at minPoints -> core flag
//   quarter_init quarter cells (side ~eps/2, diagonal ~0.71 eps: cliques of the predicate):
//                every core points at the quarter's minimum-visit-index core
//   tile_union   ONE WORKGROUP PER TILE: union-find in LDS over the tile's quarter cells (one
//                core-core edge per quarter pair within reach), then each tile component's
//                quarter reps point at its minimum-visit-index core
//   edge_union   tile-crossing quarter pairs, one wave per pair of adjacent tiles: LDS union-find
//                over the facing strips, then one global union per joined pair of tile
//                components (lock-free, hooking the root with the larger visit index under the
//                smaller, so a root IS s(K)); quarter reps then point at their roots
//   final        root of every core -> lab = s(K); roots set in a bit array in input order
//   [scan of the bit words' popcounts -> cluster id of root o = 1 + roots before o]
//   output       cores cluster_of_root(lab); non-cores min lab over core neighbours +
//                Naive/Archery
//                rule; written in input order
#include "internal.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace dbscan {

enum GridMode { kGridEps = 0, kGridAllPairs = 1, kGridNoPairs = 2 };

namespace {

constexpr int kTslot = 65;        // per-tile cell-start table stride (64 cells + end)
constexpr int kQReg = 4;          // own-quarter core points kept in registers for pair tests
constexpr int64_t kTileGrid = 8192;  // workgroups of the per-tile kernels (grid stride)
constexpr int kMaxNbr = 11;  // neighbour lists of non-cores kept while minPoints - 1 <= this
constexpr int32_t kModeArcheryBox = 2;     // DBSCAN_MODE_ARCHERY_F32BOX
constexpr int64_t kBoxEdgeCap = 1 << 20;   // initial capacity for one-way core pairs (grows)

// DBSCAN_AB_STAMPS (timing builds only, never the shipped library): the per-tile kernels' wave 0
// records the constant-rate clock (100 MHz) at its phase boundaries, per workgroup, read back by
// dbscan_ab_stamps() (tools/stamps_probe.py).
#ifndef DBSCAN_AB_STAMPS
#define DBSCAN_AB_STAMPS 0
#endif
#if DBSCAN_AB_STAMPS
constexpr int kStamps = 12;  // slots per workgroup: 0..9 clock, 10..11 tile sizes
__device__ long long g_ab_stamps[kTileGrid * kStamps];
#define AB_STAMP(k)                                                                     \
    do {                                                                                \
        if (threadIdx.x == 0) g_ab_stamps[blockIdx.x * kStamps + (k)] = wall_clock64(); \
    } while (0)
#define AB_NOTE(k, v)                                                        \
    do {                                                                     \
        if (threadIdx.x == 0) g_ab_stamps[blockIdx.x * kStamps + (k)] = (v); \
    } while (0)
#else
#define AB_STAMP(k) \
    do {            \
    } while (0)
#define AB_NOTE(k, v) \
    do {              \
    } while (0)
#endif

// DBSCAN_AB_CHECK (checking builds only, never the shipped library): edge_union's indices and
// the pair tests' slot indices checked against their ranges; an index out of range is counted
// per site (with the lowest and highest value seen) and clamped into range, so the checking
// build never faults.  Read back (and cleared) by dbscan_ab_bounds() (tools/bounds_probe.py).
// DBSCAN_AB_PAIR4 rebuilds the round-5 pair-test variant "the other quarter's cores four at a
// time, their loads in flight together" (DESIGN_LOG round 5), the build that faulted once.
#ifndef DBSCAN_AB_CHECK
#define DBSCAN_AB_CHECK 0
#endif
#ifndef DBSCAN_AB_PAIR4
#define DBSCAN_AB_PAIR4 0
#endif
// DBSCAN_AB_COUNTDIV (counting builds only): count32's scan divergence -- per wave iteration
// of the count loop, the longest lane's candidate batches against all lanes' (g_div, read by
// dbscan_ab_countdiv(), tools/countdiv_probe.py)
#ifndef DBSCAN_AB_COUNTDIV
#define DBSCAN_AB_COUNTDIV 0
#endif
#if DBSCAN_AB_COUNTDIV
__device__ unsigned long long g_div[8];
#endif
#if DBSCAN_AB_CHECK
constexpr int kChkSites = 12;
__device__ unsigned long long g_chk_bad[kChkSites];
#define CHK_12(v) {v, v, v, v, v, v, v, v, v, v, v, v}
__device__ long long g_chk_lo[kChkSites] = CHK_12(INT64_MAX);
__device__ long long g_chk_hi[kChkSites] = CHK_12(INT64_MIN);
__device__ __forceinline__ int64_t chk_idx(int site, int64_t i, int64_t lo, int64_t hi) {
    if (i >= lo && i < hi) return i;
    atomicAdd(&g_chk_bad[site], 1ull);
    atomicMin(&g_chk_lo[site], (long long)i);
    atomicMax(&g_chk_hi[site], (long long)i);
    return hi > lo ? (i < lo ? lo : hi - 1) : lo;
}
#define CHK(site, i, lo, hi) ((std::remove_reference_t<decltype(i)>)chk_idx((site), (int64_t)(i), (int64_t)(lo), (int64_t)(hi)))
#else
#define CHK(site, i, lo, hi) (i)
#endif

// DBSCANPoint.scala:26-30 as used at LocalDBSCANNaive.scala:77.  Two rounded subtractions,
// two rounded multiplies, one rounded add, <=.  The whole library is built with
// -ffp-contract=off; the pragma pins it here as well.
__device__ __forceinline__ bool within_eps(double px, double py, double ox, double oy,
                                           double eps2) {
#pragma clang fp contract(off)
    const double dx = ox - px;
    const double dy = oy - py;
    const double a = dx * dx;
    const double b = dy * dy;
    return (a + b) <= eps2;
}

__device__ __forceinline__ void cell_xy(uint32_t ck, uint32_t ntx, uint32_t& cx, uint32_t& cy) {
    const uint32_t t = ck >> 6, l = ck & 63u;
    const uint32_t ty = t / ntx, tx = t - ty * ntx;
    cx = (tx << 3) | (l & 7u);
    cy = (ty << 3) | (l >> 3);
}

__device__ __forceinline__ int tile_occ(const int32_t* __restrict__ tmap, const GridParams& g,
                                        int tx, int ty) {
    if (tx < 0 || ty < 0 || tx >= (int)g.ntx || ty >= (int)g.nty) return -1;
    return tmap[(int64_t)ty * g.ntx + tx];
}

struct Seg {  // 64 B: stencil pieces (rows cy, cy-1, cy+1; <= 2 tiles each), own cell range
    int b[6], e[6], cs, ce, pad0, pad1;
};

__device__ __forceinline__ Seg load_seg(const Seg* seg, int c) {
    const int4* p = reinterpret_cast<const int4*>(seg + c);
    const int4 u0 = p[0], u1 = p[1], u2 = p[2], u3 = p[3];
    Seg s;
    s.b[0] = u0.x; s.b[1] = u0.y; s.b[2] = u0.z; s.b[3] = u0.w;
    s.b[4] = u1.x; s.b[5] = u1.y; s.e[0] = u1.z; s.e[1] = u1.w;
    s.e[2] = u2.x; s.e[3] = u2.y; s.e[4] = u2.z; s.e[5] = u2.w;
    s.cs = u3.x; s.ce = u3.y; s.pad0 = 0; s.pad1 = 0;
    return s;
}

// f(j) for every candidate slot j of the 3x3 stencil; f returns false to stop early.
template <class F>
__device__ __forceinline__ void for_candidates(const Seg& s, F f) {
#pragma unroll
    for (int r = 0; r < 6; ++r)
        for (int j = s.b[r]; j < s.e[r]; ++j)
            if (!f(j)) return;
}

// Batched fits: the partition holding batch index i (offs[0] <= i < offs[np]; empty partitions
// are skipped because their range is empty)
__device__ __forceinline__ int part_of(const int64_t* __restrict__ offs, int np, int64_t i) {
    int lo = 0, hi = np;  // offs[lo] <= i < offs[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (offs[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// The origin of a tile's fp32 cell-unit records: the grid origin and the tile's halo corner in
// cells (batched fits: the tile's partition's local grid; tpart = partition of each tile)
struct TileOrg {
    double xmin2, ymin2, ox, oy;
};
__device__ __forceinline__ TileOrg tile_org(const GridParams& g, const int32_t* __restrict__ tpart,
                                            int t, uint32_t tk) {
    const uint32_t ty = tk / g.ntx, tx = tk - ty * g.ntx;
    TileOrg o{g.xmin2, g.ymin2, (double)(8 * (int64_t)tx - 1), (double)(8 * (int64_t)ty - 1)};
    if (g.nparts > 0) {
        const PartGrid P = g.parts[tpart[t]];
        o.xmin2 = P.xmin2;
        o.ymin2 = P.ymin2;
        o.ox -= (double)P.cx0;
        o.oy -= (double)P.cy0;
    }
    return o;
}

__global__ __launch_bounds__(kBlock) void bin_kernel(const double* __restrict__ x,
                                                     const double* __restrict__ y, int64_t n,
                                                     const GridParams* __restrict__ gp,
                                                     uint32_t* __restrict__ key) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const GridParams g = *gp;
    const double a = x[i], b = y[i];
    if (g.nparts == 0) {  // the fit's own grid (the bucketed sort's MSD pass bins the same way)
        key[i] = grid_key(a, b, g.xmin2, g.ymin2, g.invx, g.invy, g.nx, g.ny, g.ntx);
        return;
    }
    uint32_t k = kSentinelKey;
    // batched fits: the point's partition's local grid at that partition's place in the
    // virtual tile grid
    double xmin2 = g.xmin2, ymin2 = g.ymin2, mx = 2.0 * (double)g.nx - 1.0,
           my = 2.0 * (double)g.ny - 1.0;
    uint32_t qx0 = 0, qy0 = 0;
    bool binned = true;
    if (g.nparts > 0) {
        const PartGrid P = g.parts[part_of(g.poffs, g.nparts, i)];
        xmin2 = P.xmin2;
        ymin2 = P.ymin2;
        mx = 2.0 * (double)P.nx - 1.0;
        my = 2.0 * (double)P.ny - 1.0;
        qx0 = 2u * (uint32_t)P.cx0;
        qy0 = 2u * (uint32_t)P.cy0;
        binned = P.nx > 0;
    }
    if (binned && __builtin_isfinite(a) && __builtin_isfinite(b)) {
        // quarter-grid coordinates: floor(2t) >> 1 == floor(t) exactly (2t is exact)
        double fx = floor(2.0 * ((a * 0.5 - xmin2) * g.invx));
        double fy = floor(2.0 * ((b * 0.5 - ymin2) * g.invy));
        fx = fx < 0 ? 0 : (fx > mx ? mx : fx);
        fy = fy < 0 ? 0 : (fy > my ? my : fy);
        const uint32_t qx = (uint32_t)fx + qx0, qy = (uint32_t)fy + qy0;
        const uint32_t cx = qx >> 1, cy = qy >> 1;
        const uint32_t tile = (cy >> 3) * g.ntx + (cx >> 3);
        const uint32_t local = ((cy & 7u) << 3) | (cx & 7u);
        k = (tile << 8) | (local << 2) | ((qy & 1u) << 1) | (qx & 1u);
    }
    key[i] = k;  // the index payload is implicit: the sort's first pass generates it
}

__global__ __launch_bounds__(kBlock) void iota_key_kernel(int64_t n, uint32_t kval,
                                                          uint32_t* __restrict__ key,
                                                          int32_t* __restrict__ perm) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    key[i] = kval;
    perm[i] = (int32_t)i;
}

// Sorted coordinates by scattered writes: inv[perm[p]] = p, then xy[inv[i]] = (x[i], y[i]) in
// input order.  A random 4-B or 16-B write moves one 32-B sector; a random 8-B read (gathering
// x[perm[p]]) moves a whole 128-B line: 0.39 -> 0.30 ms at 10^7 points (r02).  inv is kept for
// the output permutation.
__global__ __launch_bounds__(kBlock) void inverse_kernel(int64_t n,
                                                         const int32_t* __restrict__ perm,
                                                         int32_t* __restrict__ inv) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p < n) inv[perm[p]] = (int32_t)p;
}

__global__ __launch_bounds__(kBlock) void scatter_xy_kernel(const double* __restrict__ x,
                                                            const double* __restrict__ y,
                                                            int64_t n,
                                                            const int32_t* __restrict__ nf_p,
                                                            const int32_t* __restrict__ inv,
                                                            double2* __restrict__ xy) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int32_t p = inv[i];
    if (p < *nf_p) xy[p] = make_double2(x[i], y[i]);
}

// Bucketed sort (large fits): perm and the sorted coordinates from the padded places, in slot
// order: one 32-B record (x, y, input index) read per slot from inside its band's segment
// (cache-resident while the launch sweeps the bands in order), coalesced writes.
// Slab fits: zs[p] = the slot's zone (from the record), and for the listed shared points
// sinv[i] = their slot (a scattered write per shared point only).
// Block index giving each XCD a contiguous range of the grid (as xcd_block below), for the
// bucketed gathers: the slots of one tile-row band then run under one L2, so each band's
// records (a random order inside the band) are fetched into one L2, not eight.  gather_bucket
// 0.167 -> 0.154 ms and label_sorted (its packed[place] writes) 0.128 -> 0.106 ms per 10^7
// points (A/B on one box).
__device__ __forceinline__ int64_t gather_block() {
    const int G = gridDim.x, b = blockIdx.x;
    const int x = b & 7, j = b >> 3, q = G >> 3, r = G & 7;
    return x * q + (x < r ? x : r) + j;
}

__global__ __launch_bounds__(kBlock) void gather_bucket_kernel(int64_t n,
                                                               const int32_t* __restrict__ place,
                                                               const double4* __restrict__ rec,
                                                               const int32_t* __restrict__ nf_p,
                                                               int32_t* __restrict__ perm,
                                                               double2* __restrict__ xy,
                                                               uint8_t* __restrict__ zs,
                                                               int32_t* __restrict__ sinv) {
    const int64_t p = gather_block() * kBlock + threadIdx.x;
    if (p >= n) return;
    const double4 r = rec[place[p]];
    const int32_t i = (int32_t)__double_as_longlong(r.z);
    perm[p] = i;
    if (p < *nf_p) xy[p] = make_double2(r.x, r.y);
    if (zs) {
        const uint32_t z = (uint32_t)__double_as_longlong(r.w);
        zs[p] = (uint8_t)(z & 255u);
        if (sinv && (z >> 8)) sinv[i] = (int32_t)p;
    }
}

// Lean slab fits with the bucketed sort: the listed shared points flagged in slab order.
__global__ __launch_bounds__(kBlock) void shared_mark_kernel(int64_t m,
                                                             const int64_t* __restrict__ idx,
                                                             uint8_t* __restrict__ shm) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k < m) shm[idx[k]] = 1;
}

// Slab fits: the zone-2 points (count candidates, never core) marked in sorted order (zs,
// zeroed before), so the fused count kernels know them before their tile unions.  Zone 2 is a
// thin band: a coalesced zone read per point, a scattered write per zone-2 point only.
__global__ __launch_bounds__(kBlock) void zone_mark_kernel(int64_t n,
                                                           const uint8_t* __restrict__ zone,
                                                           const int32_t* __restrict__ inv,
                                                           uint8_t* __restrict__ zs) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n && zone[i] == 2) zs[inv[i]] = 2;
}

// Occupied tiles, eps cells and quarter cells in one pass over the sorted keys (they are
// nested prefixes of the key: tile = key >> 8, cell = key >> 2, quarter = key).  A head flag
// marks the first slot of each group; groups are numbered by an exclusive scan of the flags:
// heads_reduce counts the flags per 4096-slot tile, the three rows of counts are scanned, and
// heads_down ranks each slot within its tile with wave ballots and writes the group tables.
constexpr int kHeadTile = 4096;

// XCD-aware block order (edge_union_kernel): workgroups are dispatched round-robin over the 8
// XCDs (block b on XCD b % 8), each with its own L2.  The remapped index gives every XCD a
// contiguous range of tiles, so tiles that share halo cells run under the same L2: edge_union
// 0.208 -> 0.193 ms (r12).  The count kernels stay round-robin: their class lists put the dense
// tiles together, and contiguous ranges unbalanced the XCDs (count32 0.32 -> 0.42 ms).  A
// bijection of 0..gridDim.x-1 for any grid size.
__device__ __forceinline__ int xcd_block(int G = -1) {  // G: the first G blocks of the grid
    if (G < 0) G = gridDim.x;
    const int b = blockIdx.x;
    const int x = b & 7, j = b >> 3, q = G >> 3, r = G & 7;
    return x * q + (x < r ? x : r) + j;
}

struct Heads {
    bool c, q, t;
};

// heads_reduce: each thread takes kHeadPer consecutive slots (four 16-B key loads, and the key
// before them): 0.021 -> 0.012 ms per 10^7-point fit.  (heads_down in that form, with 16-B
// stores of cell/qidx per thread, measured slower, 0.047 -> 0.071 ms, and keeps its rounds.)
constexpr int kHeadPer = kHeadTile / kBlock;
static_assert(kHeadPer == 16, "four uint4 key loads per thread");

// keys p0 .. p0 + 15 (sentinel past nf) and the three head masks (bit j: slot p0 + j heads a
// cell / quarter / tile); p = 0 heads everything
__device__ __forceinline__ void heads16(const uint32_t* __restrict__ key, int64_t p0, int64_t nf,
                                        uint32_t (&k)[kHeadPer], uint32_t& mc, uint32_t& mq,
                                        uint32_t& mt) {
    if (p0 + kHeadPer <= nf) {
        const uint4* k4 = reinterpret_cast<const uint4*>(key + p0);
#pragma unroll
        for (int u = 0; u < kHeadPer / 4; ++u) {
            const uint4 v = k4[u];
            k[4 * u] = v.x;
            k[4 * u + 1] = v.y;
            k[4 * u + 2] = v.z;
            k[4 * u + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kHeadPer; ++j) {
            k[j] = kSentinelKey;
            if (p0 + j < nf) k[j] = key[p0 + j];
        }
    }
    // the key before p0 (cached: the previous thread's line); p0 = 0 heads everything
    uint32_t kp = 0u;
    if (p0 > 0 && p0 <= nf) kp = key[p0 - 1];
    const uint32_t prev = p0 == 0 ? ~k[0] : kp;
    mc = mq = mt = 0;
#pragma unroll
    for (int j = 0; j < kHeadPer; ++j) {
        const uint32_t km = j ? k[j - 1] : prev;
        const bool in = p0 + j < nf;
        mc |= (in && (k[j] >> 2) != (km >> 2)) ? 1u << j : 0u;
        mq |= (in && k[j] != km) ? 1u << j : 0u;
        mt |= (in && (k[j] >> 8) != (km >> 8)) ? 1u << j : 0u;
    }
}

__global__ __launch_bounds__(kBlock) void heads_reduce_kernel(const uint32_t* __restrict__ key,
                                                              const int32_t* __restrict__ nf_p,
                                                              int nb,
                                                              int32_t* __restrict__ partial,
                                                              const GridParams* __restrict__ gp,
                                                              int32_t* __restrict__ tmap) {
    __shared__ int wsum[3][kBlock / 64];
    {  // tmap = -1 over the whole tile grid (tmap_kernel fills it after this launch)
        const int64_t nt = (int64_t)gp->ntx * gp->nty;
        for (int64_t u = (int64_t)blockIdx.x * kBlock + threadIdx.x; u < nt;
             u += (int64_t)gridDim.x * kBlock)
            tmap[u] = -1;
    }
    const int64_t nf = *nf_p;
    const int64_t p0 = (int64_t)blockIdx.x * kHeadTile + (int64_t)threadIdx.x * kHeadPer;
    uint32_t k[kHeadPer], mc, mq, mt;
    heads16(key, p0, nf, k, mc, mq, mt);
    int c = __popc(mc), q = __popc(mq), t = __popc(mt);
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o, 64);
        q += __shfl_xor(q, o, 64);
        t += __shfl_xor(t, o, 64);
    }
    const int w = threadIdx.x >> 6;
    if (__lane_id() == 0) {
        wsum[0][w] = c;
        wsum[1][w] = q;
        wsum[2][w] = t;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        int s = 0;
        for (int k = 0; k < kBlock / 64; ++k) s += wsum[threadIdx.x][k];
        partial[threadIdx.x * nb + blockIdx.x] = s;
    }
}

// offs: the exclusive scans of the three rows of partial counts.  qidx == nullptr: no quarter
// tables (quarter cells are not cliques of the predicate).
__global__ __launch_bounds__(kBlock) void heads_down_kernel(
    const uint32_t* __restrict__ key, const int32_t* __restrict__ nf_p, int nb,
    const int32_t* __restrict__ offs,
    int32_t* __restrict__ cell, uint32_t* __restrict__ ckey, int32_t* __restrict__ cstart,
    int32_t* __restrict__ qidx, uint32_t* __restrict__ qkey, int32_t* __restrict__ qstart,
    uint32_t* __restrict__ tkey, int32_t* __restrict__ tstart, uint64_t* __restrict__ zero_words,
    int64_t nzw) {
    __shared__ int wcnt[2][3][kBlock / 64];
    // the root bits of direct fits (quarter_root / final set them), one 64-bit word per 64 of
    // this block's kHeadTile slots: zeroed here instead of by a fill launch
    if (zero_words && threadIdx.x < kHeadTile / 64) {
        const int64_t wd = (int64_t)blockIdx.x * (kHeadTile / 64) + threadIdx.x;
        if (wd < nzw) zero_words[wd] = 0ull;
    }
    const int64_t nf = *nf_p;
    const int64_t base = (int64_t)blockIdx.x * kHeadTile;
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int oc = offs[blockIdx.x], oq = offs[nb + blockIdx.x], ot = offs[2 * nb + blockIdx.x];
    // every round's key (and the key before it) loaded up front: the rounds below wait on
    // their barriers only, not on a load each
    constexpr int R = kHeadTile / kBlock;
    uint32_t kr[R], km[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t p = base + r * kBlock + threadIdx.x;
        kr[r] = kSentinelKey;
        if (p < nf) kr[r] = key[p];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t p = base + r * kBlock + threadIdx.x;
        km[r] = __shfl_up(kr[r], 1, 64);
        if (lane == 0 && p > 0 && p <= nf) km[r] = key[p - 1];
    }
    for (int r = 0; r < R; ++r) {
        const int64_t p = base + r * kBlock + threadIdx.x;
        const uint32_t k = kr[r], kmr = km[r];
        const bool in = p < nf, first = p == 0;
        const Heads h = {in && (first || (k >> 2) != (kmr >> 2)), in && (first || k != kmr),
                         in && (first || (k >> 8) != (kmr >> 8))};
        const uint64_t bc = __ballot(h.c), bq = __ballot(h.q), bt = __ballot(h.t);
        if (lane == 0) {
            wcnt[r & 1][0][w] = __popcll(bc);
            wcnt[r & 1][1][w] = __popcll(bq);
            wcnt[r & 1][2][w] = __popcll(bt);
        }
        __syncthreads();
        int wc = 0, wq = 0, wt = 0, tc = 0, tq = 0, tt = 0;
#pragma unroll
        for (int v = 0; v < kBlock / 64; ++v) {
            const int c = wcnt[r & 1][0][v], q = wcnt[r & 1][1][v], t = wcnt[r & 1][2][v];
            wc += v < w ? c : 0;
            wq += v < w ? q : 0;
            wt += v < w ? t : 0;
            tc += c;
            tq += q;
            tt += t;
        }
        if (p < nf) {
            const int ic = oc + wc + __popcll(bc & lt);  // heads before p
            const int iq = oq + wq + __popcll(bq & lt);
            const int it = ot + wt + __popcll(bt & lt);
            cell[p] = ic + h.c - 1;
            if (h.c) {
                ckey[ic] = k >> 2;
                cstart[ic] = (int32_t)p;
            }
            if (qidx) {
                qidx[p] = iq + h.q - 1;
                if (h.q) {
                    qkey[iq] = k;
                    qstart[iq] = (int32_t)p;
                }
            }
            if (h.t) {
                tkey[it] = k >> 8;
                tstart[it] = (int32_t)p;
            }
            if (p == nf - 1) {  // end sentinels
                cstart[ic + h.c] = (int32_t)nf;
                if (qidx) qstart[iq + h.q] = (int32_t)nf;
                tstart[it + h.t] = (int32_t)nf;
            }
        }
        oc += tc;
        oq += tq;
        ot += tt;
    }
}

__global__ __launch_bounds__(kBlock) void tmap_kernel(const uint32_t* __restrict__ tkey,
                                                      const int32_t* __restrict__ ntiles_p,
                                                      int32_t* __restrict__ tmap) {
    const int ntiles = *ntiles_p;
    for (int t = blockIdx.x * kBlock + threadIdx.x; t < ntiles; t += gridDim.x * kBlock)
        tmap[tkey[t]] = t;
}

// tslot[t][l] = first slot of the first occupied cell of tile t with local index >= l
// (tile end if none): the slots of local cells [l0, l1] are [tslot[l0], tslot[l1 + 1]).
// With quarter cells (qidx != nullptr) also tq[t][l], the same table over quarter indices, and
// tnb[t] = occupied index of the E, S, SE, SW neighbour tiles (-1: empty), for edge_union.
__global__ __launch_bounds__(kBlock) void tslot_kernel(
    const int32_t* __restrict__ tstart, const uint32_t* __restrict__ tkey,
    const int32_t* __restrict__ ntiles_p, const int32_t* __restrict__ cell,
    const uint32_t* __restrict__ ckey, const int32_t* __restrict__ cstart,
    const int32_t* __restrict__ ncells_p, const int32_t* __restrict__ qidx,
    int32_t* __restrict__ tslot, int32_t* __restrict__ tq) {
    // one wave per tile, one lane per local cell
    const int lane = threadIdx.x & 63;
    const int ntiles = *ntiles_p;
    for (int t = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); t < ntiles;
         t += gridDim.x * (kBlock / 64)) {  // wave-uniform; no block barriers below
        const uint32_t tk = tkey[t];
        const int ts0 = tstart[t], end = tstart[t + 1];
        const int c0 = cell[ts0];
        const int c = c0 + lane;
        const bool mine = c < *ncells_p && (ckey[c] >> 6) == tk;
        uint64_t occ = mine ? 1ull << (ckey[c] & 63u) : 0ull;  // occupied local cells
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) occ |= __shfl_xor(occ, o, 64);
        const uint64_t rest = occ >> lane;
        int st = end;
        // first occupied local cell >= lane: its rank in the tile (the tile's cell count if none)
        int rank = __popcll(occ);
        if (rest) {
            const int nl = lane + __builtin_ctzll(rest);
            rank = __popcll(occ & ((nl == 0) ? 0ull : (~0ull >> (64 - nl))));
            st = cstart[c0 + rank];
        }
        int32_t* ts = tslot + (int64_t)t * kTslot;
        ts[lane] = st;
        if (lane == 0) ts[64] = end;
        if (qidx) {
            int32_t* tqq = tq + (int64_t)t * kTslot;
            // the entry past the tile's last cell is the next tile's first quarter
            const int qend = qidx[end - 1] + 1;
            tqq[lane] = st < end ? qidx[st] : qend;
            if (lane == 0) tqq[64] = qend;
        }
    }
}

// tslot_kernel with kTslotU tiles per wave and trip, their dependent loads (tile -> its first
// slot -> that slot's cell -> the cells' keys and starts) issued together: at config 5's share
// (1.46 M tiles) the one-tile form walks ~45 tiles per wave, a chain of four loads each (fit
// 24.6 -> 24.45 ms there; at 10^7 points the one-tile form is 5 us faster: kTslotMultiPoints).
constexpr int kTslotU = 4;
constexpr int64_t kTslotMultiPoints = int64_t(1) << 25;
__global__ __launch_bounds__(kBlock) void tslot_multi_kernel(
    const int32_t* __restrict__ tstart, const uint32_t* __restrict__ tkey,
    const int32_t* __restrict__ ntiles_p, const int32_t* __restrict__ cell,
    const uint32_t* __restrict__ ckey, const int32_t* __restrict__ cstart,
    const int32_t* __restrict__ ncells_p, const int32_t* __restrict__ qidx,
    int32_t* __restrict__ tslot, int32_t* __restrict__ tq) {
    const int lane = threadIdx.x & 63;
    const int ntiles = *ntiles_p, ncells = *ncells_p;
    const int stride = gridDim.x * (kBlock / 64);
    for (int t0 = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); t0 < ntiles;
         t0 += kTslotU * stride) {  // wave-uniform; no block barriers below
        int t[kTslotU], ts0[kTslotU], end[kTslotU], c0[kTslotU];
        uint32_t tk[kTslotU], ck[kTslotU];
#pragma unroll
        for (int u = 0; u < kTslotU; ++u) {
            t[u] = t0 + u * stride;
            const bool live = t[u] < ntiles;
            tk[u] = live ? tkey[t[u]] : 0u;
            ts0[u] = live ? tstart[t[u]] : 0;
            end[u] = live ? tstart[t[u] + 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < kTslotU; ++u) c0[u] = t[u] < ntiles ? cell[ts0[u]] : 0;
#pragma unroll
        for (int u = 0; u < kTslotU; ++u) {
            const int c = c0[u] + lane;
            ck[u] = (t[u] < ntiles && c < ncells) ? ckey[c] : ~0u;
        }
        int st[kTslotU];
#pragma unroll
        for (int u = 0; u < kTslotU; ++u) {
            uint64_t occ = (ck[u] >> 6) == tk[u] ? 1ull << (ck[u] & 63u) : 0ull;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) occ |= __shfl_xor(occ, o, 64);
            const uint64_t rest = occ >> lane;
            st[u] = end[u];
            if (t[u] < ntiles && rest) {
                const int nl = lane + __builtin_ctzll(rest);  // first occupied local >= lane
                const int rank = __popcll(occ & ((nl == 0) ? 0ull : (~0ull >> (64 - nl))));
                st[u] = cstart[c0[u] + rank];
            }
        }
        int qs[kTslotU], qe[kTslotU];
        if (qidx) {
#pragma unroll
            for (int u = 0; u < kTslotU; ++u) {
                const bool live = t[u] < ntiles;
                qe[u] = live ? qidx[end[u] - 1] + 1 : 0;
                qs[u] = (live && st[u] < end[u]) ? qidx[st[u]] : qe[u];
            }
        }
#pragma unroll
        for (int u = 0; u < kTslotU; ++u) {
            if (t[u] >= ntiles) continue;
            int32_t* ts = tslot + (int64_t)t[u] * kTslot;
            ts[lane] = st[u];
            if (lane == 0) ts[64] = end[u];
            if (qidx) {
                int32_t* tqq = tq + (int64_t)t[u] * kTslot;
                tqq[lane] = qs[u];
                if (lane == 0) tqq[64] = qe[u];
            }
        }
    }
}

// Per cell: the stencil's slot pieces (rows cy, cy-1, cy+1; a row of 3 cells splits in two
// where it crosses a tile edge) and the cell's own range.  Used by the global-memory paths.
__global__ __launch_bounds__(kBlock) void segs_kernel(const uint32_t* __restrict__ ckey,
                                                      const int32_t* __restrict__ cstart,
                                                      const int32_t* __restrict__ ncells_p,
                                                      const int32_t* __restrict__ tmap,
                                                      const int32_t* __restrict__ tslot,
                                                      const GridParams* __restrict__ gp,
                                                      Seg* __restrict__ seg,
                                                      const uint8_t* __restrict__ tclass) {
    const int c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= *ncells_p) return;
    const GridParams g = *gp;
    // tclass (clique grids, neighbour lists kept): only the big tiles' cells read their pieces
    if (tclass && g.clique && tclass[tmap[ckey[c] >> 6]] != 2) return;
    uint32_t cx, cy;
    cell_xy(ckey[c], g.ntx, cx, cy);
    const uint32_t lox = cx > 0 ? cx - 1 : cx, hix = cx + 1 < g.nx ? cx + 1 : cx;
    Seg s;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        s.b[k] = 0;
        s.e[k] = 0;
    }
    const int rows[3] = {(int)cy, (int)cy - 1, (int)cy + 1};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int ry = rows[r];
        if (ry < 0 || ry >= (int)g.ny) continue;
        const int ty = ry >> 3, ly = ry & 7;
        const int txa = (int)(lox >> 3), txb = (int)(hix >> 3);
        int occ = tile_occ(tmap, g, txa, ty);
        if (occ >= 0) {
            const int l0 = ly * 8 + (int)(lox & 7u);
            const int l1 = ly * 8 + (txa == txb ? (int)(hix & 7u) : 7);
            s.b[2 * r] = tslot[(int64_t)occ * kTslot + l0];
            s.e[2 * r] = tslot[(int64_t)occ * kTslot + l1 + 1];
        }
        if (txb != txa) {
            occ = tile_occ(tmap, g, txb, ty);
            if (occ >= 0) {
                s.b[2 * r + 1] = tslot[(int64_t)occ * kTslot + ly * 8];
                s.e[2 * r + 1] = tslot[(int64_t)occ * kTslot + ly * 8 + (int)(hix & 7u) + 1];
            }
        }
    }
    s.cs = cstart[c];
    s.ce = cstart[c + 1];
    s.pad0 = 0;
    s.pad1 = 0;
    seg[c] = s;
}

// ---------------------------------------------------------------------------------------
// Tile staging: a tile and its 1-cell halo as a 10x10 "extended" cell grid in LDS.  Extended
// cell k = (ey+1)*10 + (ex+1), ex, ey in -1..8; cells are stored in k order, so extended row ey
// is contiguous and a point at local cell (lx, ly) finds each of its 3 stencil rows as ONE LDS
// range [off[(ey+1)*10 + lx], off[(ey+1)*10 + lx + 3]).  Tiles whose tile+halo exceeds the
// kernel's staging capacity (dense data) fall back to the global-memory path.
// The per-tile kernels loop over occupied tiles with a grid stride (the tile count is only
// known on the device); every loop trip ends in a barrier before the stage is overwritten.
// ---------------------------------------------------------------------------------------
struct TileStage {
    int ok, total, ts, te, t, q0, nq;
    int cb[100];   // global slot begin of each extended cell
    int off[101];  // LDS offset of each extended cell
    int cn[100];
};

// tstage[t][k] = (first slot, point count) of extended cell k of tile t: the staging table of
// the per-tile kernels, so that staging a tile is one coalesced load per extended cell.
// (One wave per tile with a grid stride was slower: at config 5's per-GPU share, 1.46 M tiles,
// ~178 per resident wave, each trip a chain of 3 dependent loads: tile key -> neighbour's
// occupied index -> its tslot row.)
// thalo_kernel: the 100 staging entries of each tile (tstage_entry: the own tile's and the
// neighbour tiles' tslot rows), tsz = their point count, and tnb (quarter grids).  One thread per
// entry of kHaloTiles tiles per trip; each thread handles kHaloU trips' tiles with their loads
// issued together, so a resident wave keeps kHaloU independent load chains in flight instead
// of one.
constexpr int kHaloTiles = kBlock / 100;  // 2 tiles per block and trip (200 threads busy)
constexpr int kHaloU = 4;
__global__ __launch_bounds__(kBlock) void thalo_kernel(const uint32_t* __restrict__ tkey,
                                                       const int32_t* __restrict__ ntiles_p,
                                                       const int32_t* __restrict__ tmap,
                                                       const int32_t* __restrict__ tslot,
                                                       const GridParams* __restrict__ gp,
                                                       int2* __restrict__ tstage,
                                                       int32_t* __restrict__ tsz,
                                                       int4* __restrict__ tnb) {
    __shared__ int sum[kHaloU * kHaloTiles];
    const GridParams g = *gp;
    const int ntiles = *ntiles_p;
    const int j = (int)threadIdx.x / 100, k = (int)threadIdx.x - j * 100;
    const int ey = k / 10 - 1, ex = k % 10 - 1;  // extended cell k
    const int l = (ey & 7) * 8 + (ex & 7);
    const int dx = ex < 0 ? -1 : (ex > 7 ? 1 : 0), dy = ey < 0 ? -1 : (ey > 7 ? 1 : 0);
    // the entries that also name tnb's E, S, SE, SW neighbour
    const int nbc = (dx == 1 && ey == 0) ? 0 : (dy == 1 && ex == 0) ? 1
                  : (dx == 1 && dy == 1) ? 2 : (dx == -1 && dy == 1) ? 3 : -1;
    const int64_t step = (int64_t)gridDim.x * kHaloTiles * kHaloU;
    for (int64_t t0 = (int64_t)blockIdx.x * kHaloTiles * kHaloU; t0 < ntiles; t0 += step) {
        if (threadIdx.x < kHaloU * kHaloTiles) sum[threadIdx.x] = 0;
        __syncthreads();
        if (j < kHaloTiles) {
            int64_t t[kHaloU];
            uint32_t tk[kHaloU];
            int occ[kHaloU];
#pragma unroll
            for (int u = 0; u < kHaloU; ++u) {
                t[u] = t0 + u * kHaloTiles + j;
                tk[u] = t[u] < ntiles ? tkey[t[u]] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kHaloU; ++u) {
                const int ty0 = (int)(tk[u] / g.ntx), tx0 = (int)(tk[u] - (uint32_t)ty0 * g.ntx);
                occ[u] = t[u] >= ntiles ? -1
                         : (dx == 0 && dy == 0) ? (int)t[u]
                                                : tile_occ(tmap, g, tx0 + dx, ty0 + dy);
            }
            int2 e[kHaloU];
#pragma unroll
            for (int u = 0; u < kHaloU; ++u) {
                e[u] = make_int2(0, 0);
                if (occ[u] >= 0) {
                    const int b = tslot[(int64_t)occ[u] * kTslot + l];
                    e[u] = make_int2(b, tslot[(int64_t)occ[u] * kTslot + l + 1] - b);
                }
            }
#pragma unroll
            for (int u = 0; u < kHaloU; ++u) {
                if (t[u] >= ntiles) continue;
                tstage[t[u] * 100 + k] = e[u];
                if (e[u].y) atomicAdd(&sum[u * kHaloTiles + j], e[u].y);
                if (tnb && nbc >= 0) reinterpret_cast<int32_t*>(tnb + t[u])[nbc] = occ[u];
            }
        }
        __syncthreads();
        if (threadIdx.x < kHaloU * kHaloTiles) {
            const int u = (int)threadIdx.x / kHaloTiles, jj = (int)threadIdx.x - u * kHaloTiles;
            const int64_t t = t0 + u * kHaloTiles + jj;
            if (t < ntiles) tsz[t] = sum[threadIdx.x];
        }
    }
}

// Clique grids: tiles by the size of their tile + halo stage (the tstage counts), listed for
// the three count paths: small (<= kSmallCap points: count_wave_kernel, one wave per tile),
// medium (<= CAP: count_tile32_kernel, one workgroup per tile) and big (over CAP:
// big_count_kernel + big_union_kernel, global memory).  One tile per lane; one atomic per
// class and workgroup of 1024 tiles.  tclass[t] keeps the class (segs_kernel builds stencil pieces for the big
// tiles only).
enum TileClass { kTileSmall = 0, kTileMedium = 1, kTileBig = 2, kTileNone = 3 };
constexpr int kSmallCap = 192;

// The small and medium tiles are listed in buckets by stage size, the largest first: the
// count kernels walk them in that order and workgroups are dispatched in index order, so the
// longest tiles start first and the last ones dispatched are the shortest (a
// longest-processing-time order, which shortens the kernels' tails), and the four waves of a
// count_wave_kernel workgroup get tiles of about the same size.  Each bucket has its own list
// of capacity cap and its own counter.  Measured (round 2, 10^7 points): four small buckets
// took count_wave from 0.127 to 0.094 ms; eight medium buckets slowed count_tile32 (0.308 ->
// 0.316-0.331 ms: within a bucket the tiles lose the list's spatial order), so the medium tiles
// stay one list in tile order.  Small-tile buckets hold stage sizes (kSmallEdge[b + 1],
// kSmallEdge[b]]; count_wave_kernel runs in two instances by lanes per tile: 64 lanes above
// kTinyCap, 32 up to it (32 lanes up to 64 points measured even; 16 lanes up to 16 points no
// gain).
constexpr int kMedBuckets = 1;
constexpr int kSmallBuckets = 5;
__device__ constexpr int kSmallEdge[kSmallBuckets + 1] = {kSmallCap, 144, 96, 64, 32, 0};
constexpr int kTinyCap = 32;     // the 32-lane instance: stages up to 32
constexpr int kTinyBucket0 = 4;  // its first bucket
static_assert(kSmallBuckets + kMedBuckets <= 16, "kStTileBuckets holds 16 counters");

struct TileLists {
    int32_t* n;       // [3] list lengths (device): small, medium, big
    int32_t* small;   // [kSmallBuckets][cap] occupied tile indices
    int32_t* medium;  // [kMedBuckets][cap]
    int32_t* big;     // [cap]
    int32_t* sb;      // [kSmallBuckets] small bucket lengths (device)
    int32_t* mb;      // [kMedBuckets] medium bucket lengths (device)
    int32_t cap;      // capacity of each list
};

// Bucketed list position k of the size-descending order (pre: the buckets' exclusive prefix).
template <int NB>
struct BucketWalk {
    int pre[NB + 1];
    __device__ __forceinline__ BucketWalk(const int32_t* counts) {
        pre[0] = 0;
#pragma unroll
        for (int b = 0; b < NB; ++b) pre[b + 1] = pre[b] + counts[b];
    }
    __device__ __forceinline__ int size() const { return pre[NB]; }
    __device__ __forceinline__ int at(const int32_t* lists, int64_t cap, int k) const {
        int b = 0;
#pragma unroll
        for (int j = 1; j < NB; ++j) b += k >= pre[j] ? 1 : 0;
        return lists[(int64_t)b * cap + (k - pre[b])];
    }
};

constexpr int kClassRounds = 4;  // tile_class_kernel: 64 tiles per lane round, 1024 per block

template <int CAP>
__global__ __launch_bounds__(kBlock) void tile_class_kernel(const int32_t* __restrict__ tsz,
                                                            const int32_t* __restrict__ tstart,
                                                            const int32_t* __restrict__ ntiles_p,
                                                            const GridParams* __restrict__ gp,
                                                            TileLists tl,
                                                            uint8_t* __restrict__ tclass,
                                                            int32_t* __restrict__ class_pts,
                                                            uint8_t* __restrict__ tcore) {
    if (!gp->clique) return;
    // categories: small bucket b (b = 0 the largest stages), big, medium bucket b
    constexpr int kCatBig = kSmallBuckets, kCatMed = kSmallBuckets + 1;
    constexpr int kCat = kCatMed + kMedBuckets;
    __shared__ int wcnt[kCat][kBlock / 64];
    __shared__ int wpts[3][kBlock / 64];
    __shared__ int bbase[kCat];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ntiles = *ntiles_p;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int base = blockIdx.x * kBlock * kClassRounds; base < ntiles;
         base += gridDim.x * kBlock * kClassRounds) {  // block-uniform loop
        int v[kClassRounds], cat[kClassRounds];
        int pts[3] = {0, 0, 0};
#pragma unroll
        for (int r = 0; r < kClassRounds; ++r) {  // tile = base + (r * 4 + w) * 64 + lane
            const int t = base + (r * (kBlock / 64) + w) * 64 + lane;
            v[r] = kTileNone;
            cat[r] = -1;
            int own = 0;
            if (t < ntiles) {
                const int c = tsz[t];
                v[r] = c <= kSmallCap ? kTileSmall : (c <= CAP ? kTileMedium : kTileBig);
                tclass[t] = (uint8_t)v[r];
                if (v[r] == kTileBig) tcore[t] = 3;  // (big_union's tiles: not tracked)
                own = tstart[t + 1] - tstart[t];
                if (v[r] == kTileSmall) {
                    cat[r] = 0;
#pragma unroll
                    for (int j = 1; j < kSmallBuckets; ++j) cat[r] += c <= kSmallEdge[j] ? 1 : 0;
                }
                else if (v[r] == kTileBig)
                    cat[r] = kCatBig;
                else
                    cat[r] = kCatMed + (kMedBuckets - 1) -
                             (int)((int64_t)(c - kSmallCap - 1) * kMedBuckets / (CAP - kSmallCap));
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) pts[k] += v[r] == k ? own : 0;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) pts[k] += __shfl_xor(pts[k], o, 64);
#pragma unroll
        for (int k = 0; k < kCat; ++k) {
            int cnt = 0;
#pragma unroll
            for (int r = 0; r < kClassRounds; ++r) cnt += __popcll(__ballot(cat[r] == k));
            if (lane == 0) wcnt[k][w] = cnt;
        }
        if (lane < 3) wpts[lane][w] = lane == 0 ? pts[0] : (lane == 1 ? pts[1] : pts[2]);
        __syncthreads();
        if (threadIdx.x < kCat) {  // one atomic per category and workgroup
            const int k = threadIdx.x;
            const int tot = wcnt[k][0] + wcnt[k][1] + wcnt[k][2] + wcnt[k][3];
            int32_t* ctr = k < kCatBig ? &tl.sb[k] : (k == kCatBig ? &tl.n[kTileBig] : &tl.mb[k - kCatMed]);
            bbase[k] = tot ? atomicAdd(ctr, tot) : 0;
            if (k != kCatBig && tot) atomicAdd(&tl.n[k < kCatBig ? kTileSmall : kTileMedium], tot);
        }
        if (threadIdx.x < 3) {
            const int k = threadIdx.x;
            const int p = wpts[k][0] + wpts[k][1] + wpts[k][2] + wpts[k][3];
            if (p) atomicAdd(&class_pts[k], p);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kCat; ++k) {
            int at = bbase[k];
            for (int q = 0; q < w; ++q) at += wcnt[k][q];
            int32_t* list = k < kCatBig ? tl.small + (int64_t)k * tl.cap
                                        : (k == kCatBig ? tl.big
                                                        : tl.medium + (int64_t)(k - kCatMed) * tl.cap);
#pragma unroll
            for (int r = 0; r < kClassRounds; ++r) {
                const uint64_t m = __ballot(cat[r] == k);
                if (cat[r] == k)
                    list[at + __popcll(m & lt)] = base + (r * (kBlock / 64) + w) * 64 + lane;
                at += __popcll(m);
            }
        }
        __syncthreads();
    }
}

struct StageMeta {  // one tile's staging table, held in registers (lanes < 100; lane 0: range
                    // and, with tq, the tile's quarter range)
    int b = 0, cnt = 0, ts = 0, te = 0, q0 = 0, q1 = 0;
};

__device__ __forceinline__ StageMeta stage_meta(int t, int ntiles,
                                                const int2* __restrict__ tstage,
                                                const int32_t* __restrict__ tstart,
                                                const int32_t* __restrict__ tq = nullptr) {
    StageMeta m;
    if (t >= ntiles) return m;
    const int tid = threadIdx.x;
    if (tid < 100) {
        const int2 v = tstage[(int64_t)t * 100 + tid];
        m.b = v.x;
        m.cnt = v.y;
    }
    if (tid == 0) {
        m.ts = tstart[t];
        m.te = tstart[t + 1];
        if (tq) {
            m.q0 = tq[(int64_t)t * kTslot];
            m.q1 = tq[(int64_t)t * kTslot + 64];
        }
    }
    return m;
}

template <int CAP>
__device__ bool stage_build(const StageMeta& m, const double2* __restrict__ xy, TileStage& st,
                            double2* buf) {
    const int tid = threadIdx.x;
    if (tid < 100) {
        st.cb[tid] = m.b;
        st.cn[tid] = m.cnt;
    }
    if (tid == 0) {
        st.ts = m.ts;
        st.te = m.te;
        st.q0 = m.q0;
        st.nq = m.q1 - m.q0;
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the 100 counts by wave 0 (2 chunks)
        int carry = 0;
        for (int base = 0; base < 100; base += 64) {
            const int i = base + tid;
            const int v = i < 100 ? st.cn[i] : 0;
            int incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int u = __shfl_up(incl, o, 64);
                if (tid >= o) incl += u;
            }
            if (i < 100) st.off[i] = carry + incl - v;
            carry += __shfl(incl, 63, 64);
        }
        if (tid == 0) {
            st.off[100] = carry;
            st.total = carry;
            st.ok = carry <= CAP;
        }
    }
    __syncthreads();
    if (st.ok) {
        // unrolled so that a thread's loads are in flight together
        constexpr int kPer = (CAP + kBlock - 1) / kBlock;
        const int total = st.total;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int i = tid + u * kBlock;
            if (i < total) {
                int lo = 0;  // largest k with off[k] <= i
#pragma unroll
                for (int s = 64; s > 0; s >>= 1)
                    if (lo + s < 100 && st.off[lo + s] <= i) lo += s;
                buf[i] = xy[st.cb[lo] + (i - st.off[lo])];
            }
        }
    }
    __syncthreads();
    return st.ok;
}

struct LdsRanges {  // a point's stencil in LDS: rows ly, ly-1, ly+1 and its own cell
    int b[3], e[3], cs, ce;
};

__device__ __forceinline__ LdsRanges lds_ranges(const TileStage& st, int l) {
    const int lx = l & 7, ly = l >> 3;
    LdsRanges r;
    const int rows[3] = {ly, ly - 1, ly + 1};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int base = (rows[k] + 1) * 10 + lx;
        r.b[k] = st.off[base];
        r.e[k] = st.off[base + 3];
    }
    const int own = (ly + 1) * 10 + lx + 1;
    r.cs = st.off[own];
    r.ce = st.off[own + 1];
    return r;
}

// ---------------------------------------------------------------------------------------
// Neighbour counts -> core flags (LocalDBSCANNaive.scala:52-54, :99-101), with early exit once
// minPoints neighbours are seen (the count itself is never an output).  Own cell first, then
// the rest of its row, then the rows below and above; 8 candidates per batch.
// ---------------------------------------------------------------------------------------
// REC: the first nbr_k hits (self included) are also noted as LDS indices in the thread's
// column of `lst` (stride kBlock), so a point that ends below minPoints has its complete
// neighbour list without a second scan.
template <bool REC, class Src>
__device__ __forceinline__ bool scan_count(const Src* __restrict__ src, int b, int e,
                                           double2 me, double eps2, int min_points, int& cnt,
                                           uint16_t* lst, int nbr_k, int tag = 0) {
    int j = b;
    for (; j + 8 <= e; j += 8) {
        double2 qq[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) qq[u] = src[j + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool hit = within_eps(me.x, me.y, qq[u].x, qq[u].y, eps2);
            if (REC && hit && cnt < nbr_k) lst[cnt * kBlock] = (uint16_t)((j + u) | tag);
            cnt += hit ? 1 : 0;
        }
        if (cnt >= min_points) return true;
    }
    for (; j < e; ++j) {
        const double2 q = src[j];
        const bool hit = within_eps(me.x, me.y, q.x, q.y, eps2);
        if (REC && hit && cnt < nbr_k) lst[cnt * kBlock] = (uint16_t)(j | tag);
        cnt += hit ? 1 : 0;
    }
    return cnt >= min_points;
}

// one count over ranges (b[k], e[k]) with the own cell [cs, ce) first and excluded after;
// recorded hits are tagged with their range: LDS index | k << 12
template <int K, bool REC = false>
__device__ __forceinline__ void count_pieces(const double2* __restrict__ src, const int* b,
                                             const int* e, int cs, int ce, double2 me,
                                             double eps2, int min_points, int& cnt,
                                             uint16_t* lst = nullptr, int nbr_k = 0) {
    if (scan_count<REC>(src, cs, ce, me, eps2, min_points, cnt, lst, nbr_k)) return;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int lo = b[k], hi = e[k];
        if (lo <= cs && ce <= hi) {  // the piece holding the own cell: around it
            if (scan_count<REC>(src, lo, cs, me, eps2, min_points, cnt, lst, nbr_k, k << 12))
                return;
            if (scan_count<REC>(src, ce, hi, me, eps2, min_points, cnt, lst, nbr_k, k << 12))
                return;
        } else if (scan_count<REC>(src, lo, hi, me, eps2, min_points, cnt, lst, nbr_k, k << 12)) {
            return;
        }
    }
}

// One point's core decision + (non-core, nbr != nullptr) its neighbour list.  Staged: the
// point sits at LDS index j of local cell l and global slot p.  Unstaged: global stencil pieces.
template <bool STAGED>
__device__ __forceinline__ bool count_point(const TileStage& st, const double2* __restrict__ buf,
                                            const double2* __restrict__ xy,
                                            const int32_t* __restrict__ cell,
                                            const Seg* __restrict__ seg, int j, int l, int p,
                                            double eps2, int min_points, uint16_t* lst,
                                            int32_t* __restrict__ nbr, int nbr_k) {
    int cnt = 0;
    if constexpr (STAGED) {
        const double2 me = buf[j];
        const LdsRanges r = lds_ranges(st, l);
        if (nbr)
            count_pieces<3, true>(buf, r.b, r.e, r.cs, r.ce, me, eps2, min_points, cnt, lst,
                                  nbr_k);
        else
            count_pieces<3>(buf, r.b, r.e, r.cs, r.ce, me, eps2, min_points, cnt);
        if (cnt >= min_points) return true;
        // A non-core has fewer than minPoints neighbours, every one of them noted by the count
        // (self included): keep their slots, -1 terminated, for the label pass.
        if (nbr) {
            int32_t* out = nbr + (int64_t)p * nbr_k;
            int w = 0;
            const int lx = l & 7, ly = l >> 3;
            for (int k = 0; k < cnt; ++k) {
                const int v = lst[k * kBlock];
                const int q = v & 4095, row = v >> 12;  // row: 0 own, 1 above, 2 below
                const int k0 = (ly + (row == 0 ? 0 : (row == 1 ? -1 : 1)) + 1) * 10 + lx;
                const int c = k0 + (q >= st.off[k0 + 1] ? 1 : 0) + (q >= st.off[k0 + 2] ? 1 : 0);
                const int sq = st.cb[c] + (q - st.off[c]);
                if (sq != p) out[w++] = sq;
            }
            if (w < nbr_k) out[w] = -1;
        }
        return false;
    } else {
        const double2 me = xy[p];
        const Seg s = load_seg(seg, cell[p]);
        count_pieces<6>(xy, s.b, s.e, s.cs, s.ce, me, eps2, min_points, cnt);
        if (cnt >= min_points) return true;
        if (nbr) {
            int32_t* out = nbr + (int64_t)p * nbr_k;
            int w = 0;
            for (int k = 0; k < 6; ++k)
                for (int q = s.b[k]; q < s.e[k]; ++q) {
                    const double2 v = xy[q];
                    if (q != p && within_eps(me.x, me.y, v.x, v.y, eps2) && w < nbr_k)
                        out[w++] = q;
                }
            if (w < nbr_k) out[w] = -1;
        }
        return false;
    }
}

// Does any core of quarter A (points in registers: px/py, n) lie within eps of a core of B?
// core(j): is slot (or LDS index) j a core point.
template <class Src, class CoreF>
__device__ __forceinline__ bool pair_found(const double* px, const double* py, int na,
                                           const Src* __restrict__ src, int b0, int b1,
                                           uint32_t bmask, CoreF core, int boff, double eps2) {
    if (b1 - b0 <= 32) {
        uint32_t m = bmask;
#if DBSCAN_AB_PAIR4
        // (the round-5 variant: four cores per trip, loads in flight together; at a tail of
        // fewer than four set bits __ffs(0) - 1 = -1 indexes the slot BEFORE the quarter)
        while (m) {
            int j[4];
            double2 pb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                j[u] = __ffs(m) - 1;
                m &= m - 1;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) pb[u] = src[b0 - boff + CHK(0, j[u], 0, b1 - b0)];
            bool f = false;
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int k = 0; k < kQReg; ++k)
                    f |= (j[u] >= 0) && (k < na) && within_eps(px[k], py[k], pb[u].x, pb[u].y, eps2);
            if (f) return true;
        }
        return false;
#endif
        while (m) {
            const int j = __ffs(m) - 1;
            m &= m - 1;
            const double2 pb = src[b0 - boff + CHK(0, j, 0, b1 - b0)];
            bool f = false;
#pragma unroll
            for (int k = 0; k < kQReg; ++k) f |= (k < na) && within_eps(px[k], py[k], pb.x, pb.y, eps2);
            if (f) return true;
        }
        return false;
    }
    for (int j = b0; j < b1; ++j) {
        if (!core(j)) continue;
        const double2 pb = src[j - boff];
        bool f = false;
#pragma unroll
        for (int k = 0; k < kQReg; ++k) f |= (k < na) && within_eps(px[k], py[k], pb.x, pb.y, eps2);
        if (f) return true;
    }
    return false;
}

// own quarter's cores into registers; returns the count, or -1 if > kQReg (generic path)
template <class Src>
__device__ __forceinline__ int load_own(const Src* __restrict__ src, int4 me, int off,
                                        double* px, double* py) {
#pragma unroll
    for (int k = 0; k < kQReg; ++k) {
        px[k] = 0.0;
        py[k] = 0.0;
    }
    if (me.y - me.x > 32) return -1;
    uint32_t m = (uint32_t)me.w;
    int na = 0;
#pragma unroll
    for (int k = 0; k < kQReg; ++k) {
        if (m) {
            const int j = __ffs(m) - 1;
            m &= m - 1;
            const double2 v = src[me.x - off + CHK(1, j, 0, me.y - me.x)];
            px[k] = v.x;
            py[k] = v.y;
            na = k + 1;
        }
    }
    return m ? -1 : na;
}

// generic pair test when a quarter holds more than kQReg cores (dense data)
template <class Src, class CoreF>
__device__ bool pair_found_generic(const Src* __restrict__ src, int off, int4 a, int4 b,
                                   CoreF core, double eps2) {
    for (int i = a.x; i < a.y; ++i) {
        if (!core(i)) continue;
        const double2 pa = src[i - off];
        for (int j = b.x; j < b.y; ++j) {
            if (!core(j)) continue;
            const double2 pb = src[j - off];
            if (within_eps(pa.x, pa.y, pb.x, pb.y, eps2)) return true;
        }
    }
    return false;
}

// Orders one wave's LDS accesses across its lanes (a wave executes in lockstep; this keeps the
// compiler from reordering LDS reads above another lane's earlier writes).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS union-find over the tile's quarter cells (local indices; hook larger under smaller).
__device__ __forceinline__ int lfind(int* lp, int x) {
    while (true) {
        const int p = lp[x];
        if (p == x) return x;
        const int gp = lp[p];
        if (gp != p) lp[x] = gp;
        x = gp;
    }
}
__device__ __forceinline__ bool lunite(int* lp, int a, int b) {  // true: this call merged
    for (;;) {
        a = lfind(lp, a);
        b = lfind(lp, b);
        if (a == b) return false;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(&lp[a], a, b) == a) return true;
    }
}

constexpr int kMaxTileQ = 256;  // 64 cells x 4 quarters

// ---------------------------------------------------------------------------------------
// Tile-local quarter union fused into the count (plain fits with clique quarters): once a
// tile's core flags are known the block that counted it builds the quarter records
// (quarter_init's job) and unions the tile's quarters (tile_union's job) against the
// coordinates it still holds in LDS, instead of two later kernels re-reading them from memory.
// Every core of the tile then points straight at its tile component's rep.
// ---------------------------------------------------------------------------------------
struct FuseArgs {
    const int32_t* tq;       // per tile: first quarter of each local cell (+ end)
    const int32_t* qstart;   // quarter slot ranges
    const uint32_t* qkey;    // quarter keys
    const int32_t* perm;     // visit index per slot
    const uint32_t* tkey;    // occupied tile ids
    const GridParams* gp;
    TileLists tl;            // f32: clique-grid tiles by stage size (tile_class_kernel)
    const uint8_t* zs;       // slab fits: zone per sorted slot (2: candidate only, never core)
    int4* qinfo;             // out: (begin, end, rep, core mask) per quarter
    int4* qg;                // out: (quarter-grid x, y, min visit index of its cores, 0)
    int32_t* qcomp;          // out: tile component rep per quarter (-1: no cores)
    uint8_t* tcore;          // out (f32): per tile, bit 0 its east cell column holds a core,
                             // bit 1 its south cell row does (edge_union skips the other sides)
    const int32_t* tpart = nullptr;  // batched fits: partition of each occupied tile
};

struct UnionLds {  // aliases the count's neighbour-list staging (the two never overlap in time)
    int lp[kMaxTileQ];           // LDS union-find over the tile's quarters
    uint32_t lrange[kMaxTileQ];  // staged: LDS begin | length << 11; local quarter-grid cell
                                 // (16 y + x) << 22; bit 31: holds cores
    uint32_t lmask[kMaxTileQ];   // cores among the first 32 points
    uint16_t qmap[kMaxTileQ];    // 16x16 local quarter grid -> local quarter (0xFFFF: none)
    unsigned long long cmin[kMaxTileQ];  // per component: min (visit index << 32 | rep)
};
static_assert(sizeof(UnionLds) <= kMaxNbr * kBlock * sizeof(uint16_t), "UnionLds must fit");

// Quarter-grid offsets to test from each quarter: one of each opposite pair (dy < 0, or dy == 0
// and dx < 0), so every unordered quarter pair within the 5x5 stencil is one item -- the 4
// adjacent offsets first, then the 8 at distance 2.
__constant__ int8_t kRingDx[12] = {-1, 0, 1, -1, -2, -1, 0, 1, 2, -2, 2, -2};
__constant__ int8_t kRingDy[12] = {-1, -1, -1, 0, -2, -2, -2, -2, -2, -1, -1, 0};

// Is there an eps pair between a core of quarter A and a core of quarter B?  Ranges are LDS
// indices (staged) or slots; masks hold the cores among each quarter's first 32 points.
template <class CoreF>
__device__ __forceinline__ bool quarters_touch(const double2* __restrict__ src, int ab, int ae,
                                               uint32_t am, int bb, int be, uint32_t bm,
                                               CoreF is_core, double eps2) {
    if (ae - ab <= 32 && be - bb <= 32) {
        for (uint32_t m1 = am; m1; m1 &= m1 - 1) {
            const double2 pa = src[ab + __ffs(m1) - 1];
            for (uint32_t m2 = bm; m2; m2 &= m2 - 1) {
                const double2 pb = src[bb + __ffs(m2) - 1];
                if (within_eps(pa.x, pa.y, pb.x, pb.y, eps2)) return true;
            }
        }
        return false;
    }
    for (int i = ab; i < ae; ++i) {
        if (!is_core(i)) continue;
        const double2 pa = src[i];
        for (int j = bb; j < be; ++j)
            if (is_core(j) && within_eps(pa.x, pa.y, src[j].x, src[j].y, eps2)) return true;
    }
    return false;
}

// A workgroup barrier that orders LDS only: unlike __syncthreads it does not wait for this
// wave's outstanding global loads (a perm load stays in flight across the pair tests).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The tile-local quarter union of a big tile (big_union_kernel: its points are not staged, so
// every range is a slot range and every core flag a global byte).  b, e, key: this thread's
// quarter (threadIdx.x < nq).
__device__ void global_tile_union(int q0, int nq, int b, int e, uint32_t key, const FuseArgs& fa,
                                  const GridParams& g, const double2* __restrict__ xy,
                                  const uint8_t* __restrict__ core, double eps2,
                                  int32_t* __restrict__ parent, UnionLds& u) {
    const int i = threadIdx.x;
    const auto is_core = [&](int j) { return core[j] != 0; };
    // every quarter's slot range and its rep's coordinates in LDS: a pair's first test (the two
    // reps, which most adjacent pairs pass) reads no global memory
    __shared__ int qs[kMaxTileQ + 1];
    __shared__ double2 rxy[kMaxTileQ];
    u.qmap[i] = 0xFFFF;
    u.cmin[i] = ~0ull;
    lds_barrier();
    // quarter records: quarter rep and core mask.  The sort is stable and the visit index is the
    // input index, so a quarter's slots are in visit order and its rep (the core with the
    // smallest visit index) is simply its first core.
    int rep = -1, best = 0x7FFFFFFF, gx = 0, gy = 0;
    if (i < nq) {
        uint32_t cx, cy;
        cell_xy(key >> 2, g.ntx, cx, cy);
        gx = (int)(2 * cx + (key & 1u));
        gy = (int)(2 * cy + ((key >> 1) & 1u));
        const int lq = (gy & 15) * 16 + (gx & 15);
        const int len = e - b;
        uint32_t mask = 0;
        int first = -1;
        {
            // the first 32 core flags by up to 9 aligned words, all loads in flight (a loop of
            // byte loads waited for each one); the last word may reach 3 bytes past the
            // quarter, inside the core array's 4 bytes of slack
            const int l32 = len < 32 ? len : 32;
            const int a0 = b >> 2, sh = (b & 3) * 8;
            const int last = l32 > 0 ? ((b + l32 - 1) >> 2) - a0 : -1;  // words needed: 0..last
            const uint32_t* cw = reinterpret_cast<const uint32_t*>(core);
            uint32_t w[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) w[k] = k <= last ? cw[a0 + k] : 0u;
            // one bit per nonzero byte (bits 7, 15, 23, 31), packed to a nibble per word
            uint64_t bits = 0;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const uint32_t x = w[k];
                const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
                const uint32_t nib = ((nz >> 7) & 1u) | ((nz >> 14) & 2u) | ((nz >> 21) & 4u) |
                                     ((nz >> 28) & 8u);
                bits |= (uint64_t)nib << (4 * k);
            }
            mask = (uint32_t)(bits >> (sh >> 3)) & (l32 == 32 ? ~0u : ((1u << l32) - 1u));
            first = mask ? __ffs(mask) - 1 : -1;
            for (int j = 32; j < len && first < 0; ++j)
                if (is_core(b + j)) first = j;
        }
        if (first >= 0) {
            rep = b + first;
            best = fa.perm[rep];
        }
        fa.qinfo[q0 + i] = make_int4(b, e, rep, (int)mask);
        u.lp[i] = i;
        u.lrange[i] = (rep >= 0 ? 0x80000000u : 0u) | ((uint32_t)lq << 22);
        u.lmask[i] = mask;
        u.qmap[lq] = (uint16_t)i;
        qs[i] = b;
        if (i == nq - 1) qs[nq] = e;
        rxy[i] = rep >= 0 ? xy[rep] : make_double2(0.0, 0.0);
    }
    lds_barrier();
    // pair tests, one (quarter, offset) item per thread, adjacent quarters first so that most
    // distance-2 pairs are found joined and skipped
    for (int sweep = 0; sweep < 2; ++sweep) {
        const int o0 = sweep ? 4 : 0, nofs = sweep ? 8 : 4;
        for (int k = i; k < nq * nofs; k += kBlock) {
            const int o = k / nq, qi = k - o * nq;
            const uint32_t ri = u.lrange[qi];
            if (!(ri >> 31)) continue;
            const int lq = (int)((ri >> 22) & 255u);
            const int ux = (lq & 15) + kRingDx[o0 + o], uy = (lq >> 4) + kRingDy[o0 + o];
            if (ux < 0 || uy < 0 || ux > 15 || uy > 15) continue;
            const int j = u.qmap[uy * 16 + ux];
            if (j == 0xFFFF) continue;
            const uint32_t rj = u.lrange[j];
            if (!(rj >> 31)) continue;
            // (adjacent items run all at once: a find before each would rarely prune)
            if (sweep && lfind(u.lp, qi) == lfind(u.lp, j)) continue;
            {
                const double2 pa = rxy[qi], pb = rxy[j];
                if (within_eps(pa.x, pa.y, pb.x, pb.y, eps2)) {
                    lunite(u.lp, qi, j);
                    continue;
                }
            }
            const int ab = qs[qi], ae = qs[qi + 1];
            const int bb = qs[j], be = qs[j + 1];
            if (quarters_touch(xy, ab, ae, u.lmask[qi], bb, be, u.lmask[j], is_core, eps2))
                lunite(u.lp, qi, j);
        }
        lds_barrier();
    }
    // tile components: rep = the quarter rep with the smallest visit index
    int r = -1;
    if (i < nq && rep >= 0) {
        r = lfind(u.lp, i);
        atomicMin(&u.cmin[r], ((unsigned long long)(uint32_t)best << 32) | (uint32_t)rep);
    }
    lds_barrier();
    if (i < nq) {
        const int crep = r >= 0 ? (int)(uint32_t)(u.cmin[r] & 0xFFFFFFFFull) : -1;
        fa.qg[q0 + i] = make_int4(gx, gy, best, 0);
        fa.qcomp[q0 + i] = crep;
        if (rep >= 0) parent[rep] = crep;  // cores reach it through their quarter's rep
    }
}

// The fp64 count for grids whose quarter cells are not cliques of the predicate (grown cells;
// the all-pairs grid): staged tiles count from LDS, the rest from global stencil pieces; every
// point is its own parent for union_kernel.  Clique grids exit at once: the fp32 count kernels
// (count_tile32 / count_wave / big_count) count them.
// slots [nf, n) (outside the grid: never core unless minPoints <= 0), block b of nb
__device__ __forceinline__ void count_rest_body(int b, int nb, const int32_t* __restrict__ nf_p,
                                                int64_t n, int32_t min_points,
                                                uint8_t* __restrict__ core,
                                                int32_t* __restrict__ parent,
                                                int32_t* __restrict__ block_cores) {
    __shared__ int rcores[kBlock / 64];
    int mine = 0;
    for (int64_t p = *nf_p + (int64_t)b * kBlock + threadIdx.x; p < n; p += (int64_t)nb * kBlock) {
        const bool is_core = min_points <= 0;
        parent[p] = (int32_t)p;
        core[p] = is_core ? 1 : 0;
        mine += is_core ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if (__lane_id() == 0) rcores[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += rcores[w];
        block_cores[b] = tot;
    }
}

template <int CAP, int MINW>
__global__ __launch_bounds__(kBlock, MINW) void count_tile_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, const int32_t* __restrict__ tstart,
    const int2* __restrict__ tstage, const int32_t* __restrict__ ntiles_p, double eps2,
    int32_t min_points, uint8_t* __restrict__ core, int32_t* __restrict__ parent,
    int32_t* __restrict__ block_cores, int32_t* __restrict__ nbr, int nbr_k,
    const GridParams* __restrict__ gp, int ntile_blocks, const int32_t* __restrict__ nf_p,
    int64_t n, int32_t* __restrict__ rest_cores) {
    // blocks from ntile_blocks: count_rest's job (the slots outside the grid) in this launch
    if ((int)blockIdx.x >= ntile_blocks) {
        count_rest_body((int)blockIdx.x - ntile_blocks, (int)gridDim.x - ntile_blocks, nf_p, n,
                        min_points, core, parent, rest_cores);
        return;
    }
    __shared__ TileStage st;
    __shared__ double2 buf[CAP];
    __shared__ int wcores[kBlock / 64];
    __shared__ int rowoff[9];
    __shared__ __attribute__((aligned(16))) uint16_t lsts[kMaxNbr * kBlock];
    uint16_t* lst = lsts + threadIdx.x;
    if (gp->clique) {
        if (threadIdx.x == 0) block_cores[blockIdx.x] = 0;
        return;
    }
    const int ntiles = *ntiles_p;
    int mine = 0;
    StageMeta meta = stage_meta(blockIdx.x, ntiles, tstage, tstart);
    for (int t = blockIdx.x; t < ntiles; t += ntile_blocks) {
        const bool staged = stage_build<CAP>(meta, xy, st, buf);
        meta = stage_meta(t + ntile_blocks, ntiles, tstage, tstart);  // in flight during the scans
        if (staged) {
            if (threadIdx.x == 0) {  // own points per row of the tile: prefix over rows
                int acc = 0;
                for (int r = 0; r < 8; ++r) {
                    rowoff[r] = acc;
                    acc += st.off[(r + 1) * 10 + 9] - st.off[(r + 1) * 10 + 1];
                }
                rowoff[8] = acc;
            }
            __syncthreads();
            const int own = rowoff[8];
            for (int i = (int)threadIdx.x; i < own; i += kBlock) {
                int r = 0;  // row: largest r with rowoff[r] <= i
#pragma unroll
                for (int s = 4; s > 0; s >>= 1)
                    if (r + s < 8 && rowoff[r + s] <= i) r += s;
                const int base = (r + 1) * 10 + 1;
                const int j = st.off[base] + (i - rowoff[r]);
                int ex = 0;  // cell in the row: largest ex with off[base + ex] <= j
#pragma unroll
                for (int s = 4; s > 0; s >>= 1)
                    if (ex + s < 8 && st.off[base + ex + s] <= j) ex += s;
                const int p = st.cb[base + ex] + (j - st.off[base + ex]);
                const bool is_core =
                    min_points <= 0 || count_point<true>(st, buf, xy, cell, seg, j, r * 8 + ex, p,
                                                         eps2, min_points, lst, nbr, nbr_k);
                parent[p] = p;
                core[p] = is_core ? 1 : 0;
                mine += is_core ? 1 : 0;
            }
        } else {
            for (int p = st.ts + (int)threadIdx.x; p < st.te; p += kBlock) {
                const bool is_core =
                    min_points <= 0 || count_point<false>(st, buf, xy, cell, seg, 0, 0, p, eps2,
                                                          min_points, lst, nbr, nbr_k);
                parent[p] = p;
                core[p] = is_core ? 1 : 0;
                mine += is_core ? 1 : 0;
            }
        }
        __syncthreads();
    }
    // per-block core count (same-address atomics from every wave cost ~1.7 ms at 10^7 points)
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if (__lane_id() == 0) wcores[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += wcores[w];
        block_cores[blockIdx.x] = tot;
    }
}

// ---------------------------------------------------------------------------------------
// The clique-grid count with fp32 tile coordinates (count_tile32_kernel).  A tile's staged
// points are held in LDS as float2 offsets from the tile's halo corner in CELL units,
//   r = fl32((v*0.5 - vmin*0.5) * inv - (8*tile - 1)),   |r| < 10 (+ grid rounding),
// the same cell coordinate the bin kernel floors, so F = fl32(dx*dx + dy*dy) approximates the
// exact squared distance over h^2 to within 1.6e-5 (fp32 rounding of |r| <= 16: 4.8e-7 per
// coordinate, |dx| <= 3 inside the 3x3 stencil; the fp64 cell coordinates are off by < 3e-8).
// With e2 = eps*eps / h^2 (the clique grid has hx = hy = h) and M = 2^-14:
//   F <= lo = rd(e2 - M)  =>  the reference's fp64 dx*dx + dy*dy <= eps*eps   (a neighbour)
//   F >  hi = ru(e2 + M)  =>  it is not
//   otherwise             =>  the fp64 predicate itself on the two points' coordinates
// so counts, flags and pair tests stay bit-exact, while the hot loop runs fp32 math on 8-byte
// LDS records (half the LDS and registers of the fp64 staging; one ambiguous candidate in
// ~10^5 takes the exact path).
// ---------------------------------------------------------------------------------------
struct F32Cut {
    float lo, hi;  // F <= lo: a neighbour; F > hi: not; otherwise the exact fp64 predicate
    float ne2;     // -fl32(e2), for the count's signed form (count_d below)
};

__device__ __forceinline__ F32Cut f32_cut(const GridParams& g, double eps2) {
    const double s = 0.5 * g.invx;  // 1 / h
    const double e2 = eps2 * s * s;
    return {__double2float_rd(e2 - 0x1p-14), __double2float_ru(e2 + 0x1p-14), -(float)e2};
}

// The count's signed form of the same test (count_tile32_kernel): D = fl(dx*dx + fl(dy*dy -
// fl32(e2))), two fused steps.  D differs from F - e2 by at most the two roundings (|dx|, |dy|
// <= 3 cells inside the stencil: 2^-21 each) plus |fl32(e2) - e2| <= 2^-24 (e2 ~ 1 on clique
// grids), all far below the margin M = 2^-14 around the F bound of 1.6e-5: |D| > M means F is
// outside [lo, hi] on the same side, so D < 0 <=> a neighbour, exactly as F <= lo; |D| <= M
// takes the exact fp64 predicate (a superset of the F band).
constexpr float kCountBand = 0x1p-14f;
typedef float pk2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float count_d(float2 me, float2 q, float ne2) {
    // (dx, dy) as one packed subtraction of the record pair (written per coordinate, the
    // compiler paired the candidates' x and y across records, six moves per batch of four)
    const pk2f d = pk2f{q.x, q.y} - pk2f{me.x, me.y};
    return __builtin_fmaf(d.x, d.x, __builtin_fmaf(d.y, d.y, ne2));
}

// LDS index -> global slot of a staged tile (largest extended cell k with off[k] <= q)
__device__ __forceinline__ int stage_slot(const TileStage& st, int q) {
    int k = 0;
#pragma unroll
    for (int s = 64; s > 0; s >>= 1)
        if (k + s < 100 && st.off[k + s] <= q) k += s;
    return st.cb[k] + (q - st.off[k]);
}

__device__ __forceinline__ float f32_d2(float2 a, float2 b) {
    const float dx = b.x - a.x, dy = b.y - a.y;
    return __builtin_fmaf(dx, dx, dy * dy);
}

// stage_build with the float2 cell-unit records (origin ox, oy: the tile's halo corner)
template <int CAP>
__device__ bool stage_build32(const StageMeta& m, const double2* __restrict__ xy, TileStage& st,
                              float2* buf, const GridParams& g, const TileOrg& o) {
    const int tid = threadIdx.x;
    if (tid < 100) {
        st.cb[tid] = m.b;
        st.cn[tid] = m.cnt;
    }
    if (tid == 0) {
        st.ts = m.ts;
        st.te = m.te;
        st.q0 = m.q0;
        st.nq = m.q1 - m.q0;
    }
    __syncthreads();
    if (tid < 64) {
        int carry = 0;
        for (int base = 0; base < 100; base += 64) {
            const int i = base + tid;
            const int v = i < 100 ? st.cn[i] : 0;
            int incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int u = __shfl_up(incl, o, 64);
                if (tid >= o) incl += u;
            }
            if (i < 100) st.off[i] = carry + incl - v;
            carry += __shfl(incl, 63, 64);
        }
        if (tid == 0) {
            st.off[100] = carry;
            st.total = carry;
            st.ok = carry <= CAP;
        }
    }
    __syncthreads();
    if (st.ok) {
        constexpr int kPer = (CAP + kBlock - 1) / kBlock;
        const int total = st.total;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int i = tid + u * kBlock;
            if (i < total) {
                int lo = 0;
#pragma unroll
                for (int s = 64; s > 0; s >>= 1)
                    if (lo + s < 100 && st.off[lo + s] <= i) lo += s;
                const double2 v = xy[st.cb[lo] + (i - st.off[lo])];
                buf[i] = make_float2((float)((v.x * 0.5 - o.xmin2) * g.invx - o.ox),
                                     (float)((v.y * 0.5 - o.ymin2) * g.invy - o.oy));
            }
        }
    }
    __syncthreads();
    return st.ok;
}

// Is there an eps pair between a core of quarter A and a core of quarter B (LDS ranges)?
template <class CoreF, class ExactF>
__device__ __forceinline__ bool quarters_touch32(const float2* __restrict__ buf, int ab, int ae,
                                                 uint32_t am, int bb, int be, uint32_t bm,
                                                 CoreF is_core, F32Cut cut, ExactF exact) {
    if (ae - ab <= 32 && be - bb <= 32) {
        for (uint32_t m1 = am; m1; m1 &= m1 - 1) {
            const int ia = ab + __ffs(m1) - 1;
            const float2 pa = buf[ia];
            for (uint32_t m2 = bm; m2; m2 &= m2 - 1) {
                const int ib = bb + __ffs(m2) - 1;
                const float F = f32_d2(pa, buf[ib]);
                if (F <= cut.lo) return true;
                if (F <= cut.hi && exact(ia, ib)) return true;
            }
        }
        return false;
    }
    for (int i = ab; i < ae; ++i) {
        if (!is_core(i)) continue;
        const float2 pa = buf[i];
        for (int j = bb; j < be; ++j) {
            if (!is_core(j)) continue;
            const float F = f32_d2(pa, buf[j]);
            if (F <= cut.lo) return true;
            if (F <= cut.hi && exact(i, j)) return true;
        }
    }
    return false;
}


// The 4 adjacent (backward) quarter pairs of core quarter qi, from qi's own lane: the four
// lookups, and the tests of each pair's first cores, are issued together; a pair whose first
// cores are not a sure hit takes the full quarters_touch32 test.  lp/lrange/lmask/qmap: the
// tile's LDS union-find and quarter records (UnionLds / WaveUnion).
template <class CoreF, class ExactF>
__device__ __forceinline__ void unite_adjacent32(int* lp, const uint32_t* lrange,
                                                 const uint32_t* lmask, const uint16_t* qmap,
                                                 int qi, const float2* __restrict__ buf,
                                                 CoreF is_core, F32Cut cut, ExactF exact) {
    constexpr int kDx[4] = {-1, 0, 1, -1}, kDy[4] = {-1, -1, -1, 0};
    const uint32_t ri = lrange[qi], am = lmask[qi];
    const int lq = (int)((ri >> 22) & 255u);
    const int ab = (int)(ri & 2047u), ae = ab + (int)((ri >> 11) & 2047u);
    int jn[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int ux = (lq & 15) + kDx[o], uy = (lq >> 4) + kDy[o];
        jn[o] = (ux >= 0 && ux <= 15 && uy >= 0) ? (int)qmap[uy * 16 + ux] : 0xFFFF;
    }
    uint32_t rj[4], mj[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int jj = jn[o] == 0xFFFF ? qi : jn[o];
        rj[o] = jn[o] == 0xFFFF ? 0u : lrange[jj];
        mj[o] = lmask[jj];
    }
    const float2 pa = buf[ab + (am ? __ffs(am) - 1 : 0)];
    bool t[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const float2 pb = buf[(int)(rj[o] & 2047u) + (mj[o] ? __ffs(mj[o]) - 1 : 0)];
        t[o] = (rj[o] >> 31) && am && mj[o] && f32_d2(pa, pb) <= cut.lo;
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        if ((rj[o] >> 31) && !t[o]) {
            const int bb = (int)(rj[o] & 2047u), be = bb + (int)((rj[o] >> 11) & 2047u);
            t[o] = quarters_touch32(buf, ab, ae, am, bb, be, mj[o], is_core, cut, exact);
        }
        if (t[o]) lunite(lp, qi, jn[o]);
    }
}

// One LDS range of candidates in batches of kScanBatch (the last batch masked).  Hits by the sign
// of D (count_d), candidates inside the band by the exact fp64 predicate (exact(q) for LDS index
// q).  REC: each batch with
// hits is noted as ONE record (first LDS index | range tag << 11 | hit bits << 16) in the
// thread's column of lst while fewer than nbr_k records exist; a point that ends below
// minPoints has at most minPoints - 1 hits, so its records are complete.
// Candidates per batch: 4, the batch's tail clamped and masked once (round 2: against 8 with
// a per-candidate select, count_wave + count_tiny 0.092 -> 0.087 ms at 10^7, 0.256 -> 0.236
// on config 3's share; 8 in this form spilled at 80 VGPRs).
constexpr int kScanBatch = 4;  // (8: equal, 0.283 -> 0.286 ms, with spills at 80 VGPRs)
template <bool REC, int STRIDE = kBlock, class ExactF>
__device__ __forceinline__ bool scan_count32(const float2* __restrict__ buf, int b, int e,
                                             float2 me, F32Cut cut, int min_points, int& cnt,
                                             uint32_t* lst, int& nrec, int nbr_k, int tag,
                                             ExactF exact, int* nbatch = nullptr) {
    for (int j = b; j < e; j += kScanBatch) {
        if (nbatch) ++*nbatch;
        const int nin = e - j;
        float2 qq[kScanBatch];
#pragma unroll
        // (stage buffers end in kScanBatch pad records: a tail batch reads past its range, the
        // extra candidates masked below; clamped reads measured 0.309 -> 0.299 ms in count32)
        for (int u = 0; u < kScanBatch; ++u) qq[u] = buf[j + u];
        // the signed form (count_d): hits from sign bits, one band test per batch (the F <= lo /
        // F <= hi compares per candidate measured 0.312 -> 0.307 ms in count32)
        const uint32_t valid = nin >= kScanBatch ? (1u << kScanBatch) - 1u : (1u << nin) - 1u;
        uint32_t hm = 0, am = 0;
        float d[kScanBatch];
#pragma unroll
        for (int u = 0; u < kScanBatch; ++u) d[u] = count_d(me, qq[u], cut.ne2);
        // hit bits by one funnel shift per candidate, last candidate first: (hm << 1) | sign
        // (with the packed difference above: count32 0.298 -> 0.285 ms)
#pragma unroll
        for (int u = kScanBatch - 1; u >= 0; --u)
            hm = __builtin_amdgcn_alignbit(hm, __float_as_uint(d[u]), 31);
        hm &= valid;
        float mn = fabsf(d[0]);
#pragma unroll
        for (int u = 1; u < kScanBatch; ++u) mn = fminf(mn, fabsf(d[u]));
        if (__builtin_expect(mn <= kCountBand, 0)) {  // band members: the exact predicate
#pragma unroll
            for (int u = 0; u < kScanBatch; ++u)
                if (((valid >> u) & 1u) && fabsf(d[u]) <= kCountBand) am |= 1u << u;
            hm &= ~am;
        }
        if (__builtin_expect(am != 0, 0)) {
            for (uint32_t m = am; m; m &= m - 1) {
                const int u = __ffs(m) - 1;
                if (exact(j + u)) hm |= 1u << u;
            }
        }
        if (REC && hm && nrec < nbr_k) {
            lst[nrec * STRIDE] = (uint32_t)j | ((uint32_t)tag << 11) | (hm << 16);
            ++nrec;
        }
        cnt += __popc(hm);
        if (cnt >= min_points) return true;
    }
    return cnt >= min_points;
}

// fused_tile_union over the float2 stage (see fused_tile_union for the structure)
__device__ void fused_tile_union32(int t, int q0, int nq, int b, int e, uint32_t key,
                                   const FuseArgs& fa,
                                   const GridParams& g, const TileStage& st,
                                   const float2* __restrict__ buf,
                                   const uint32_t* __restrict__ lcore,
                                   const double2* __restrict__ xy, double eps2, F32Cut cut,
                                   int32_t* __restrict__ parent, UnionLds& u) {
    const int i = threadIdx.x;
    const auto is_core = [&](int j) { return ((lcore[j >> 5] >> (j & 31)) & 1u) != 0; };
    const auto exact = [&](int qa, int qb) {
        const double2 pa = xy[stage_slot(st, qa)], pb = xy[stage_slot(st, qb)];
        return within_eps(pa.x, pa.y, pb.x, pb.y, eps2);
    };
    __shared__ int s_first;  // smallest local quarter holding a core
    __shared__ int s_tflags;  // the tile's edge strips holding cores (FuseArgs::tcore)
    if (i == 0) {
        s_first = 0x7FFFFFFF;
        s_tflags = 0;
    }
    u.qmap[i] = 0xFFFF;
    u.cmin[i] = ~0ull;
    lds_barrier();
    int rep = -1, best = 0x7FFFFFFF, gx = 0, gy = 0;
    if (i < nq) {
        uint32_t cx, cy;
        cell_xy(key >> 2, g.ntx, cx, cy);
        gx = (int)(2 * cx + (key & 1u));
        gy = (int)(2 * cy + ((key >> 1) & 1u));
        const int lq = (gy & 15) * 16 + (gx & 15);
        const int len = e - b;
        const int l = (int)((key >> 2) & 63u);
        const int k = ((l >> 3) + 1) * 10 + (l & 7) + 1;
        const int jb = st.off[k] + (b - st.cb[k]);
        uint32_t mask = 0;
        int first = -1;
        if (len <= 32) {
            const int w = jb >> 5, o = jb & 31;
            const uint64_t v = (uint64_t)lcore[w] | ((uint64_t)lcore[w + 1] << 32);
            mask = (uint32_t)(v >> o) & (len == 32 ? ~0u : ((1u << len) - 1u));
            first = mask ? __ffs(mask) - 1 : -1;
        } else {
            for (int j = 0; j < len && (j < 32 || first < 0); ++j)
                if (is_core(jb + j)) {
                    if (j < 32) mask |= 1u << j;
                    if (first < 0) first = j;
                }
        }
        if (first >= 0) {
            rep = b + first;
            best = fa.perm[rep];
        }
        if (rep >= 0) {
            atomicMin(&s_first, i);
            // east cell column: local quarter x 14, 15; south cell row: local quarter y 14, 15
            const int tf = ((gx & 15) >= 14 ? 1 : 0) | ((gy & 15) >= 14 ? 2 : 0);
            if (tf) atomicOr(&s_tflags, tf);
        }
        fa.qinfo[q0 + i] = make_int4(b, e, rep, (int)mask);
        u.lp[i] = i;
        u.lrange[i] = (rep >= 0 ? 0x80000000u : 0u) | ((uint32_t)lq << 22) | (uint32_t)jb |
                      ((uint32_t)len << 11);
        u.lmask[i] = mask;
        u.qmap[lq] = (uint16_t)i;
    }
    lds_barrier();
    if (i == 0) fa.tcore[t] = (uint8_t)s_tflags;
    AB_STAMP(5);
    {
        // adjacent quarters (the 4 backward offsets) from each core quarter's own thread
        if (i < nq && rep >= 0)
            unite_adjacent32(u.lp, u.lrange, u.lmask, u.qmap, i, buf, is_core, cut, exact);
        lds_barrier();
        AB_STAMP(6);
        // the adjacent pairs joined every core of the tile: no distance-2 pair can add an edge
        // inside it
        const int f = s_first;
        const bool split = i < nq && rep >= 0 && lfind(u.lp, i) != lfind(u.lp, f);
        if (__syncthreads_or(split)) {
            for (int k = i; k < nq * 8; k += kBlock) {
                const int o = k / nq, qi = k - o * nq;
                const uint32_t ri = u.lrange[qi];
                if (!(ri >> 31)) continue;
                const int lq = (int)((ri >> 22) & 255u);
                const int ux = (lq & 15) + kRingDx[4 + o], uy = (lq >> 4) + kRingDy[4 + o];
                if (ux < 0 || uy < 0 || ux > 15 || uy > 15) continue;
                const int j = u.qmap[uy * 16 + ux];
                if (j == 0xFFFF) continue;
                const uint32_t rj = u.lrange[j];
                if (!(rj >> 31)) continue;
                if (lfind(u.lp, qi) == lfind(u.lp, j)) continue;
                const int ab = (int)(ri & 2047u), ae = ab + (int)((ri >> 11) & 2047u);
                const int bb = (int)(rj & 2047u), be = bb + (int)((rj >> 11) & 2047u);
                if (quarters_touch32(buf, ab, ae, u.lmask[qi], bb, be, u.lmask[j], is_core, cut,
                                     exact))
                    lunite(u.lp, qi, j);
            }
            lds_barrier();
        }
        AB_STAMP(7);
    }
    int r = -1;
    if (i < nq && rep >= 0) {
        r = lfind(u.lp, i);
        atomicMin(&u.cmin[r], ((unsigned long long)(uint32_t)best << 32) | (uint32_t)rep);
    }
    lds_barrier();
    AB_STAMP(8);
    if (i < nq) {
        const int crep = r >= 0 ? (int)(uint32_t)(u.cmin[r] & 0xFFFFFFFFull) : -1;
        fa.qg[q0 + i] = make_int4(gx, gy, best, 0);
        fa.qcomp[q0 + i] = crep;
        if (rep >= 0) parent[rep] = crep;
    }
}

// Count + fused tile union on clique grids with the fp32 tile records above (the fp64
// count_tile_kernel<.., true> runs the other grids; each exits at once on the other's).
template <int CAP, int MINW>
__global__ __launch_bounds__(kBlock, MINW) void count_tile32_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ tstart,
    const int2* __restrict__ tstage, const int32_t* __restrict__ ntiles_p, double eps2,
    int32_t min_points, uint8_t* __restrict__ core, int32_t* __restrict__ parent,
    int32_t* __restrict__ block_cores, int32_t* __restrict__ nbr, int nbr_k, FuseArgs fa) {
    const GridParams g = *fa.gp;
    if (!g.clique) {  // count_tile_kernel counts this grid
        if (threadIdx.x == 0) block_cores[blockIdx.x] = 0;
        return;
    }
    __shared__ TileStage st;
    __shared__ float2 buf[CAP + kScanBatch];
    __shared__ int wcores[kBlock / 64];
    __shared__ int rowoff[9];
    __shared__ __attribute__((aligned(16))) uint32_t lsts[kMaxNbr * kBlock];
    __shared__ uint32_t lcore[(CAP + 31) / 32 + 1];
    static_assert(CAP < 2048, "LDS ranges are packed in 11 bits");
    static_assert(sizeof(UnionLds) <= sizeof(lsts), "UnionLds must fit");
    uint32_t* lst = lsts + threadIdx.x;
    const int ntiles = *ntiles_p;
    const F32Cut cut = f32_cut(g, eps2);
    int mine = 0;
    // the medium tiles (tile_class_kernel): each fits the staging capacity
    const BucketWalk<kMedBuckets> order(fa.tl.mb);  // largest stages first (tile_class_kernel)
    const int nt = order.size();
    const auto tile_at = [&](int k) { return k < nt ? order.at(fa.tl.medium, fa.tl.cap, k) : ntiles; };
    StageMeta meta = stage_meta(tile_at(blockIdx.x), ntiles, tstage, tstart, fa.tq);
    for (int k = blockIdx.x; k < nt; k += gridDim.x) {
        AB_STAMP(0);
        const int t = tile_at(k);
        if (threadIdx.x < (CAP + 31) / 32 + 1) lcore[threadIdx.x] = 0u;
        stage_build32<CAP>(meta, xy, st, buf, g, tile_org(g, fa.tpart, t, fa.tkey[t]));
        AB_STAMP(1);
        AB_NOTE(10, st.total);
        meta = stage_meta(tile_at(k + gridDim.x), ntiles, tstage, tstart, fa.tq);
        const int q0 = st.q0, nq = st.nq;
        int qb = 0, qe = 0;
        uint32_t qk = 0;
        if ((int)threadIdx.x < nq) {
            qb = fa.qstart[q0 + threadIdx.x];
            qe = fa.qstart[q0 + threadIdx.x + 1];
            qk = fa.qkey[q0 + threadIdx.x];
        }
        {
            if (threadIdx.x == 0) {
                int acc = 0;
                for (int r = 0; r < 8; ++r) {
                    rowoff[r] = acc;
                    acc += st.off[(r + 1) * 10 + 9] - st.off[(r + 1) * 10 + 1];
                }
                rowoff[8] = acc;
            }
            __syncthreads();
            AB_STAMP(2);
            const int own = rowoff[8];
            AB_NOTE(11, own);
            for (int i = (int)threadIdx.x; i < own; i += kBlock) {
                int r = 0;
#pragma unroll
                for (int s = 4; s > 0; s >>= 1)
                    if (r + s < 8 && rowoff[r + s] <= i) r += s;
                const int base = (r + 1) * 10 + 1;
                const int j = st.off[base] + (i - rowoff[r]);
                int ex = 0;
#pragma unroll
                for (int s = 4; s > 0; s >>= 1)
                    if (ex + s < 8 && st.off[base + ex + s] <= j) ex += s;
                const int p = st.cb[base + ex] + (j - st.off[base + ex]);
                bool is_core = true;
                if (min_points > 0) {
                    const int l = r * 8 + ex;
                    const float2 me = buf[j];
                    const LdsRanges rg = lds_ranges(st, l);
                    const auto exact = [&](int q) {
                        const double2 a = xy[p], o = xy[stage_slot(st, q)];
                        return within_eps(a.x, a.y, o.x, o.y, eps2);
                    };
                    int cnt = 0, nrec = 0;
                    const int k_rec = nbr_k;
#if DBSCAN_AB_COUNTDIV
                    int nbt = 0;
                    int* const nbp = &nbt;
#else
                    int* const nbp = nullptr;
#endif
                    bool done = scan_count32<true>(buf, rg.cs, rg.ce, me, cut, min_points, cnt,
                                                   lst, nrec, k_rec, 0, exact, nbp);
#pragma unroll
                    for (int k = 0; k < 3 && !done; ++k) {
                        const int lo = rg.b[k], hi = rg.e[k];
                        if (lo <= rg.cs && rg.ce <= hi) {
                            done = scan_count32<true>(buf, lo, rg.cs, me, cut, min_points, cnt,
                                                      lst, nrec, k_rec, k, exact, nbp) ||
                                   scan_count32<true>(buf, rg.ce, hi, me, cut, min_points, cnt,
                                                      lst, nrec, k_rec, k, exact, nbp);
                        } else {
                            done = scan_count32<true>(buf, lo, hi, me, cut, min_points, cnt, lst,
                                                      nrec, k_rec, k, exact, nbp);
                        }
                    }
                    is_core = cnt >= min_points;
#if DBSCAN_AB_COUNTDIV
                    {  // per wave: the longest lane's batches, all lanes' batches, lanes, cores
                        const uint64_t act = __ballot(1);
                        int mx = nbt, sm = nbt;
                        for (int o = 32; o > 0; o >>= 1) {
                            mx = max(mx, __shfl_xor(mx, o, 64));
                            sm += __shfl_xor(sm, o, 64);
                        }
                        const uint64_t cm = __ballot(is_core);
                        if (__lane_id() == __builtin_ctzll(act)) {
                            atomicAdd(&g_div[0], (unsigned long long)mx);
                            atomicAdd(&g_div[1], (unsigned long long)sm);
                            atomicAdd(&g_div[2], (unsigned long long)__popcll(act));
                            atomicAdd(&g_div[3], (unsigned long long)__popcll(cm));
                            atomicAdd(&g_div[4], 1ull);
                        }
                    }
#endif
                    if (!is_core && k_rec > 0) {  // (a complete list: cnt < minPoints)
                        // the non-core's neighbours (self excluded), -1 terminated
                        int32_t* out = nbr + (int64_t)p * nbr_k;
                        int w = 0;
                        for (int rr = 0; rr < nrec; ++rr) {
                            const uint32_t v = lst[rr * kBlock];
                            const int q = (int)(v & 2047u), row = (int)((v >> 11) & 3u);
                            const int k0 = (r + (row == 0 ? 0 : (row == 1 ? -1 : 1)) + 1) * 10 + ex;
                            for (uint32_t m = v >> 16; m; m &= m - 1) {
                                const int qq = q + __ffs(m) - 1;
                                const int c = k0 + (qq >= st.off[k0 + 1] ? 1 : 0) +
                                              (qq >= st.off[k0 + 2] ? 1 : 0);
                                const int sq = st.cb[c] + (qq - st.off[c]);
                                if (sq != p) out[w++] = sq;
                            }
                        }
                        if (w < nbr_k) out[w] = -1;
                    }
                }
                if (fa.zs && fa.zs[p] == 2) is_core = false;  // slab halo: candidate only
                if (is_core) atomicOr(&lcore[j >> 5], 1u << (j & 31));
                core[p] = is_core ? 1 : 0;
                mine += is_core ? 1 : 0;
            }
            AB_STAMP(3);
            __syncthreads();
            AB_STAMP(4);
            fused_tile_union32(t, q0, nq, qb, qe, qk, fa, g, st, buf, lcore, xy, eps2, cut, parent,
                               *reinterpret_cast<UnionLds*>(lsts));
        }
        __syncthreads();
        AB_STAMP(9);
    }
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if (__lane_id() == 0) wcores[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += wcores[w];
        block_cores[blockIdx.x] = tot;
    }
}


// Small clique-grid tiles (tile + halo <= kSmallCap points; most tiles of a clustered set are
// sparse ones at cluster edges): ONE WAVE per tile, the same stage / count / quarter union as
// count_tile32_kernel with wave syncs instead of workgroup barriers, so the four waves of a
// workgroup work on four tiles independently and a tile's latency chain (stage loads, scans,
// union) never waits for a slower tile.
// SEG: lanes per tile.  SEG = 64 is one tile per wave; SEG = 32 (stages of at most kTinyCap
// points) packs 64 / SEG tiles into a wave, which divides the per-tile instruction stream: a
// tile that small is bound by that stream (its count is a few candidates), not by its loads.
// SCAP: the stage capacity; a tile's quarters (each holds >= 1 own point) are at most SCAP.
template <int SCAP>
struct WaveUnion {  // per tile, aliases the count's neighbour records
    int lp[SCAP];
    uint32_t lrange[SCAP];
    uint32_t lmask[SCAP];
    unsigned long long cmin[SCAP];
    uint16_t qmap[kMaxTileQ];
};

template <int SCAP>
struct WaveSeg {  // one tile of a wave
    TileStage st;
    int rowoff[9];
    uint32_t lcore[SCAP / 32 + 1];
    float2 buf[SCAP + kScanBatch];
};

template <int SCAP, int NSEG>
struct WaveTile {
    WaveSeg<SCAP> sg[NSEG];
    union {
        uint32_t rec[kMaxNbr * 64];  // the count's neighbour records, one column per lane
        WaveUnion<SCAP> u[NSEG];
    };
};

// Walks the small-tile buckets [B0, B0 + NB) (tile_class_kernel), largest stages first.
template <int MINW, int SEG, int SCAP, int B0, int NB, int WAVES>
__global__ __launch_bounds__(64 * WAVES, MINW) void count_wave_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ tstart,
    const int2* __restrict__ tstage, double eps2, int32_t min_points,
    uint8_t* __restrict__ core, int32_t* __restrict__ parent,
    int32_t* __restrict__ block_cores, int32_t* __restrict__ nbr, int nbr_k, FuseArgs fa) {
    constexpr int NSEG = 64 / SEG, NQ = SCAP / SEG;
    static_assert(B0 + NB <= kSmallBuckets && 64 % SEG == 0 && SEG >= 8 && SCAP % SEG == 0,
                  "small-tile buckets / segments");
    __shared__ WaveTile<SCAP, NSEG> wt[WAVES];
    __shared__ int wcores[WAVES];
    const GridParams g = *fa.gp;
    const int lane = __lane_id(), w = threadIdx.x >> 6;
    const int sgi = lane / SEG, sl = lane - sgi * SEG;  // the lane's tile and its lane in it
    const uint64_t smask = SEG == 64 ? ~0ull : (((1ull << SEG) - 1) << (sgi * SEG));
    WaveSeg<SCAP>& T = wt[w].sg[sgi];
    TileStage& st = T.st;
    WaveUnion<SCAP>& u = wt[w].u[sgi];
    int mine = 0;
    if (g.clique) {
        const F32Cut cut = f32_cut(g, eps2);
        const BucketWalk<NB> order(fa.tl.sb + B0);  // largest stages first
        const int32_t* lists = fa.tl.small + (int64_t)B0 * fa.tl.cap;
        const int nt = order.size();
        const int ngroups = (nt + NSEG - 1) / NSEG;
        for (int kg = blockIdx.x * WAVES + w; kg < ngroups; kg += gridDim.x * WAVES) {
            // a segment without a tile runs the same steps over an empty stage
            const int k = kg * NSEG + sgi;
            const bool live = k < nt;
            const int t = live ? order.at(lists, fa.tl.cap, k) : 0;
            // stage table: extended cells sl, sl + SEG, ..., scanned across the segment
            constexpr int kRounds = (100 + SEG - 1) / SEG;
            int2 m[kRounds];
#pragma unroll
            for (int r = 0; r < kRounds; ++r) {
                const int e = r * SEG + sl;
                m[r] = (live && e < 100) ? tstage[(int64_t)t * 100 + e] : make_int2(0, 0);
            }
            const uint32_t tk = live ? fa.tkey[t] : 0u;
            const int q0 = live ? fa.tq[(int64_t)t * kTslot] : 0;
            const int nq = live ? fa.tq[(int64_t)t * kTslot + 64] - q0 : 0;
            int incl[kRounds];
#pragma unroll
            for (int r = 0; r < kRounds; ++r) incl[r] = m[r].y;
#pragma unroll
            for (int o = 1; o < SEG; o <<= 1) {
#pragma unroll
                for (int r = 0; r < kRounds; ++r) {
                    const int v = __shfl_up(incl[r], o, SEG);
                    if (sl >= o) incl[r] += v;
                }
            }
            int carry = 0;
#pragma unroll
            for (int r = 0; r < kRounds; ++r) {
                const int e = r * SEG + sl;
                if (e < 100) {
                    st.cb[e] = m[r].x;
                    st.off[e] = carry + incl[r] - m[r].y;
                }
                carry += __shfl(incl[r], SEG - 1, SEG);
            }
            const int total = carry;
            if (sl == 0) st.off[100] = total;
            if (sl < SCAP / 32 + 1) T.lcore[sl] = 0u;
            wave_sync();
            {
                const TileOrg o = live ? tile_org(g, fa.tpart, t, tk) : TileOrg{0, 0, 0, 0};
#pragma unroll
                for (int uu = 0; uu < SCAP / SEG; ++uu) {
                    const int e = sl + uu * SEG;
                    if (e < total) {
                        int c = 0;
#pragma unroll
                        for (int sh = 64; sh > 0; sh >>= 1)
                            if (c + sh < 100 && st.off[c + sh] <= e) c += sh;
                        const double2 v = xy[st.cb[c] + (e - st.off[c])];
                        T.buf[e] = make_float2((float)((v.x * 0.5 - o.xmin2) * g.invx - o.ox),
                                               (float)((v.y * 0.5 - o.ymin2) * g.invy - o.oy));
                    }
                }
            }
            if (sl < 8) {  // own points per tile row, prefix over the rows
                const int rs = st.off[(sl + 1) * 10 + 9] - st.off[(sl + 1) * 10 + 1];
                int rincl = rs;
#pragma unroll
                for (int o = 1; o < 8; o <<= 1) {
                    const int v = __shfl_up(rincl, o, SEG);
                    if (sl >= o) rincl += v;
                }
                T.rowoff[sl] = rincl - rs;
                if (sl == 7) T.rowoff[8] = rincl;
            }
            wave_sync();
            const int own = T.rowoff[8];
            int tflags = 0;
            for (int i = sl; i < own; i += SEG) {
                int r = 0;
#pragma unroll
                for (int sh = 4; sh > 0; sh >>= 1)
                    if (r + sh < 8 && T.rowoff[r + sh] <= i) r += sh;
                const int base = (r + 1) * 10 + 1;
                const int j = st.off[base] + (i - T.rowoff[r]);
                int ex = 0;
#pragma unroll
                for (int sh = 4; sh > 0; sh >>= 1)
                    if (ex + sh < 8 && st.off[base + ex + sh] <= j) ex += sh;
                const int p = st.cb[base + ex] + (j - st.off[base + ex]);
                bool is_core = true;
                if (min_points > 0) {
                    const float2 me = T.buf[j];
                    const LdsRanges rg = lds_ranges(st, r * 8 + ex);
                    const auto exact = [&](int q) {
                        const double2 a = xy[p], o = xy[stage_slot(st, q)];
                        return within_eps(a.x, a.y, o.x, o.y, eps2);
                    };
                    uint32_t* lst = wt[w].rec + lane;
                    int cnt = 0, nrec = 0;
                    bool done = scan_count32<true, 64>(T.buf, rg.cs, rg.ce, me, cut, min_points,
                                                       cnt, lst, nrec, nbr_k, 0, exact);
#pragma unroll
                    for (int kk = 0; kk < 3 && !done; ++kk) {
                        const int lo = rg.b[kk], hi = rg.e[kk];
                        if (lo <= rg.cs && rg.ce <= hi) {
                            done = scan_count32<true, 64>(T.buf, lo, rg.cs, me, cut, min_points,
                                                          cnt, lst, nrec, nbr_k, kk, exact) ||
                                   scan_count32<true, 64>(T.buf, rg.ce, hi, me, cut, min_points,
                                                          cnt, lst, nrec, nbr_k, kk, exact);
                        } else {
                            done = scan_count32<true, 64>(T.buf, lo, hi, me, cut, min_points, cnt,
                                                          lst, nrec, nbr_k, kk, exact);
                        }
                    }
                    is_core = cnt >= min_points;
                    if (!is_core && nbr_k > 0) {
                        int32_t* out = nbr + (int64_t)p * nbr_k;
                        int wn = 0;
                        for (int rr = 0; rr < nrec; ++rr) {
                            const uint32_t v = lst[rr * 64];
                            const int q = (int)(v & 2047u), row = (int)((v >> 11) & 3u);
                            const int k0 = (r + (row == 0 ? 0 : (row == 1 ? -1 : 1)) + 1) * 10 + ex;
                            for (uint32_t mm = v >> 16; mm; mm &= mm - 1) {
                                const int qq = q + __ffs(mm) - 1;
                                const int c = k0 + (qq >= st.off[k0 + 1] ? 1 : 0) +
                                              (qq >= st.off[k0 + 2] ? 1 : 0);
                                const int sq = st.cb[c] + (qq - st.off[c]);
                                if (sq != p) out[wn++] = sq;
                            }
                        }
                        if (wn < nbr_k) out[wn] = -1;
                    }
                }
                if (fa.zs && fa.zs[p] == 2) is_core = false;  // slab halo: candidate only
                if (is_core) atomicOr(&T.lcore[j >> 5], 1u << (j & 31));
                if (is_core) tflags |= (ex == 7 ? 1 : 0) | (r == 7 ? 2 : 0);
                core[p] = is_core ? 1 : 0;
                mine += is_core ? 1 : 0;
            }
            {
                const uint64_t b0 = __ballot(tflags & 1) & smask, b1 = __ballot(tflags & 2) & smask;
                if (live && sl == 0) fa.tcore[t] = (uint8_t)((b0 ? 1 : 0) | (b1 ? 2 : 0));
            }
            wave_sync();
            // quarter records + union over the tile's quarters (fused_tile_union32, per tile)
            for (int idx = sl; idx < kMaxTileQ; idx += SEG) u.qmap[idx] = 0xFFFF;
            for (int idx = sl; idx < SCAP; idx += SEG) u.cmin[idx] = ~0ull;
            wave_sync();
            int rep[NQ], best[NQ];
#pragma unroll
            for (int pp = 0; pp < NQ; ++pp) {
                const int qi = sl + pp * SEG;
                rep[pp] = -1;
                best[pp] = 0x7FFFFFFF;
                if (qi < nq) {
                    const int b = fa.qstart[q0 + qi], e = fa.qstart[q0 + qi + 1];
                    const uint32_t key = fa.qkey[q0 + qi];
                    uint32_t cx, cy;
                    cell_xy(key >> 2, g.ntx, cx, cy);
                    const int gx = (int)(2 * cx + (key & 1u)), gy = (int)(2 * cy + ((key >> 1) & 1u));
                    const int lq = (gy & 15) * 16 + (gx & 15);
                    const int len = e - b;
                    const int l = (int)((key >> 2) & 63u);
                    const int kc = ((l >> 3) + 1) * 10 + (l & 7) + 1;
                    const int jb = st.off[kc] + (b - st.cb[kc]);
                    // len <= 32: a small tile's quarter rarely holds more; else scan the bits
                    uint32_t mask = 0;
                    int first = -1;
                    for (int jj = 0; jj < len && (jj < 32 || first < 0); ++jj)
                        if ((T.lcore[(jb + jj) >> 5] >> ((jb + jj) & 31)) & 1u) {
                            if (jj < 32) mask |= 1u << jj;
                            if (first < 0) first = jj;
                        }
                    if (first >= 0) {
                        rep[pp] = b + first;
                        best[pp] = fa.perm[rep[pp]];
                    }
                    fa.qinfo[q0 + qi] = make_int4(b, e, rep[pp], (int)mask);
                    fa.qg[q0 + qi] = make_int4(gx, gy, best[pp], 0);
                    u.lp[qi] = qi;
                    u.lrange[qi] = (rep[pp] >= 0 ? 0x80000000u : 0u) | ((uint32_t)lq << 22) |
                                   (uint32_t)jb | ((uint32_t)len << 11);
                    u.lmask[qi] = mask;
                    u.qmap[lq] = (uint16_t)qi;
                }
            }
            wave_sync();
            const auto is_core_l = [&](int j) { return ((T.lcore[j >> 5] >> (j & 31)) & 1u) != 0; };
            const auto exact2 = [&](int qa, int qb) {
                const double2 pa = xy[stage_slot(st, qa)], pb = xy[stage_slot(st, qb)];
                return within_eps(pa.x, pa.y, pb.x, pb.y, eps2);
            };
            for (int qi = sl; qi < nq; qi += SEG)
                if (u.lrange[qi] >> 31)
                    unite_adjacent32(u.lp, u.lrange, u.lmask, u.qmap, qi, T.buf, is_core_l, cut,
                                     exact2);
            wave_sync();
            // the adjacent pairs joined every core of the tile: no distance-2 pair can add an
            // edge inside it
            int f = 0x7FFFFFFF;
#pragma unroll
            for (int pp = NQ - 1; pp >= 0; --pp)
                if (sl + pp * SEG < nq && rep[pp] >= 0) f = sl + pp * SEG;
#pragma unroll
            for (int o = SEG / 2; o > 0; o >>= 1) f = min(f, __shfl_xor(f, o, SEG));
            bool split = false;
#pragma unroll
            for (int pp = 0; pp < NQ; ++pp) {
                const int qi = sl + pp * SEG;
                if (qi < nq && rep[pp] >= 0 && lfind(u.lp, qi) != lfind(u.lp, f)) split = true;
            }
            if (__ballot(split) & smask) {
                wave_sync();
                for (int it = sl; it < nq * 8; it += SEG) {
                    const int o = it / nq, qi = it - o * nq;
                    const uint32_t ri = u.lrange[qi];
                    if (!(ri >> 31)) continue;
                    const int lq = (int)((ri >> 22) & 255u);
                    const int ux = (lq & 15) + kRingDx[4 + o], uy = (lq >> 4) + kRingDy[4 + o];
                    if (ux < 0 || uy < 0 || ux > 15 || uy > 15) continue;
                    const int j = u.qmap[uy * 16 + ux];
                    if (j == 0xFFFF) continue;
                    const uint32_t rj = u.lrange[j];
                    if (!(rj >> 31)) continue;
                    if (lfind(u.lp, qi) == lfind(u.lp, j)) continue;
                    const int ab = (int)(ri & 2047u), ae = ab + (int)((ri >> 11) & 2047u);
                    const int bb = (int)(rj & 2047u), be = bb + (int)((rj >> 11) & 2047u);
                    if (quarters_touch32(T.buf, ab, ae, u.lmask[qi], bb, be, u.lmask[j],
                                         is_core_l, cut, exact2))
                        lunite(u.lp, qi, j);
                }
            }
            wave_sync();
            int rr[NQ];
#pragma unroll
            for (int pp = 0; pp < NQ; ++pp) {
                const int qi = sl + pp * SEG;
                rr[pp] = -1;
                if (qi < nq && rep[pp] >= 0) {
                    rr[pp] = lfind(u.lp, qi);
                    atomicMin(&u.cmin[rr[pp]],
                              ((unsigned long long)(uint32_t)best[pp] << 32) | (uint32_t)rep[pp]);
                }
            }
            wave_sync();
#pragma unroll
            for (int pp = 0; pp < NQ; ++pp) {
                const int qi = sl + pp * SEG;
                if (qi < nq) {
                    const int crep =
                        rr[pp] >= 0 ? (int)(uint32_t)(u.cmin[rr[pp]] & 0xFFFFFFFFull) : -1;
                    fa.qcomp[q0 + qi] = crep;
                    if (rep[pp] >= 0) parent[rep[pp]] = crep;
                }
            }
            wave_sync();
        }
    }
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if (lane == 0) wcores[w] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int v = 0; v < WAVES; ++v) tot += wcores[v];
        block_cores[blockIdx.x] = tot;
    }
}

// Clique-grid tiles over the fp32 staging capacity (big_tiles_kernel's list): their points'
// counts from global memory, spread over kBigChunks workgroups per tile (such tiles are the
// dense cores of clusters: thousands of points each), then each tile's quarter union.
constexpr int kBigChunks = 8;
template <int MINW, int WAVES>
__global__ __launch_bounds__(64 * WAVES, MINW) void big_count_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, const int32_t* __restrict__ tstart,
    const int32_t* __restrict__ qidx, double eps2, int32_t min_points,
    uint8_t* __restrict__ core, int32_t* __restrict__ block_cores, int32_t* __restrict__ nbr,
    int nbr_k, FuseArgs fa) {
    // WAVES waves per workgroup: a tile's points in chunks of 64 * WAVES, kBigChunks * kBlock
    // apart (the same coverage whatever WAVES)
    constexpr int CS = 64 * WAVES, NC = kBigChunks * kBlock / CS;
    __shared__ int wcores[WAVES];
    __shared__ TileStage st;  // (unused by the global-memory count)
    int mine = 0;
    if (fa.gp->clique) {
        const int nb = fa.tl.n[kTileBig];
        for (int k = blockIdx.x; k < nb * NC; k += gridDim.x) {
            const int t = fa.tl.big[k / NC], c = k % NC;
            const int te = tstart[t + 1];
            for (int p = tstart[t] + c * CS + (int)threadIdx.x; p < te;
                 p += kBigChunks * kBlock) {
                // a quarter cell is a clique on these grids: one holding minPoints points makes
                // each of them core without a count (a third of the big tiles' points at 10^7)
                const int q = qidx[p];
                const int lb = fa.qstart[q + 1] - fa.qstart[q];  // a lower bound of |N(p)|
                const bool is_core =
                    (min_points <= 0 || lb >= min_points ||
                     count_point<false>(st, nullptr, xy, cell, seg, 0, 0, p, eps2, min_points,
                                        nullptr, nbr, nbr_k)) &&
                    !(fa.zs && fa.zs[p] == 2);  // slab halo: candidate only
                core[p] = is_core ? 1 : 0;
                mine += is_core ? 1 : 0;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if (__lane_id() == 0) wcores[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < WAVES; ++w) tot += wcores[w];
        block_cores[blockIdx.x] = tot;
    }
}

__global__ __launch_bounds__(kBlock) void big_union_kernel(const double2* __restrict__ xy,
                                                           const uint8_t* __restrict__ core,
                                                           double eps2,
                                                           int32_t* __restrict__ parent,
                                                           FuseArgs fa) {
    const GridParams g = *fa.gp;
    if (!g.clique) return;
    __shared__ UnionLds u;
    const int nb = fa.tl.n[kTileBig];
    for (int k = blockIdx.x; k < nb; k += gridDim.x) {
        const int t = fa.tl.big[k];
        const int q0 = fa.tq[(int64_t)t * kTslot], nq = fa.tq[(int64_t)t * kTslot + 64] - q0;
        int qb = 0, qe = 0;
        uint32_t qk = 0;
        if ((int)threadIdx.x < nq) {
            qb = fa.qstart[q0 + threadIdx.x];
            qe = fa.qstart[q0 + threadIdx.x + 1];
            qk = fa.qkey[q0 + threadIdx.x];
        }
        global_tile_union(q0, nq, qb, qe, qk, fa, g, xy, core, eps2, parent, u);
        __syncthreads();
    }
}

// Slab fits: outer-halo points (zone 2) are count candidates only, never core.  The count
// kernels treat every point alike; this clears the zone-2 core flags afterwards, reading the
// zones coalesced in slab order (a random write only per zone-2 point, a thin band) instead of
// a random zone read per point inside the count.
__global__ __launch_bounds__(kBlock) void zone_fix_kernel(int64_t n,
                                                          const uint8_t* __restrict__ zone,
                                                          const int32_t* __restrict__ inv,
                                                          uint8_t* __restrict__ core) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n && zone[i] == 2) core[inv[i]] = 0;
}

// The same from the zones in sorted order (bucketed sort: zs holds every slot's zone).
__global__ __launch_bounds__(kBlock) void zone_fix_sorted_kernel(int64_t n,
                                                                 const uint8_t* __restrict__ zs,
                                                                 uint8_t* __restrict__ core) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p < n && zs[p] == 2) core[p] = 0;
}

// Slots outside the grid (non-finite coordinates, or every slot when eps*eps is NaN): no
// neighbours, not even themselves.
__global__ __launch_bounds__(kBlock) void count_rest_kernel(const int32_t* __restrict__ nf_p,
                                                            int64_t n,
                                                            int32_t min_points,
                                                            uint8_t* __restrict__ core,
                                                            int32_t* __restrict__ parent,
                                                            int32_t* __restrict__ block_cores) {
    count_rest_body(blockIdx.x, gridDim.x, nf_p, n, min_points, core, parent, block_cores);
}

// ---------------------------------------------------------------------------------------
// Lock-free union-find over slots.  parent pointers always lead to a strictly smaller visit
// index (perm), so there are no cycles and a root is the minimum-index core of its set.
// Only CAS hooks write roots; stale reads only ever show an older ancestor (still an
// ancestor), so plain loads are safe.
// V = 0: agent-scope atomic loads (L1-bypassing) with path-halving stores (per-point fallback);
// V = 1: plain L1-cacheable loads, no stores (quarter unions; measured faster, r01 notes).
// ---------------------------------------------------------------------------------------
template <int V>
__device__ __forceinline__ int ld_par(int* par, int i) {
    if constexpr (V == 1) {
        return par[i];
    } else {
        return __hip_atomic_load(par + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__device__ __forceinline__ void st_par(int* par, int i, int v) {
    __hip_atomic_store(par + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int V = 0>
__device__ int uf_find(int* par, int x) {
    int cur = ld_par<V>(par, x);
    if (cur == x) return x;
    int prev = x;
    for (;;) {
        const int next = ld_par<V>(par, cur);
        if (next == cur) return cur;
        if constexpr (V == 0) st_par(par, prev, next);  // path halving (prev is a non-root)
        prev = cur;
        cur = next;
    }
}

// Walk x's chain; stop early (returning `target`) when the walk meets `target`, which then
// need not be a root any more: the two are in one set.  Avoids re-reading a hot root's line.
template <int V = 0>
__device__ int uf_find_until(int* par, int x, int target) {
    if (x == target) return target;
    int cur = ld_par<V>(par, x);
    if (cur == x || cur == target) return cur;
    int prev = x;
    for (;;) {
        const int next = ld_par<V>(par, cur);
        if (next == cur || next == target) return next;
        if constexpr (V == 0) st_par(par, prev, next);
        prev = cur;
        cur = next;
    }
}

// Merge the sets of believed roots ra, rb; returns the believed root of the union.
template <int V = 0>
__device__ int uf_unite_roots(int* par, const int32_t* __restrict__ prio, int ra, int rb) {
    while (ra != rb) {
        const bool swap = prio[ra] < prio[rb];
        const int hi = swap ? rb : ra;  // larger visit index: hooked
        const int lo = swap ? ra : rb;
        int expected = hi;
        if (__hip_atomic_compare_exchange_strong(par + hi, &expected, lo, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return lo;
        ra = uf_find<V>(par, expected);  // hi was hooked meanwhile: continue from its new parent
        rb = uf_find<V>(par, lo);
    }
    return ra;
}

// Per-point union (used when quarter cells are not cliques: grown grid, all-pairs mode).
// Each core-core edge once: from the endpoint with the larger slot.
__device__ __forceinline__ void union_body(int b, int nb, const double2* __restrict__ xy,
                                           const int32_t* __restrict__ cell,
                                           const Seg* __restrict__ seg,
                                           const int32_t* __restrict__ nf_p,
                                           const GridParams* __restrict__ gp, double eps2,
                                           const int32_t* __restrict__ perm,
                                           const uint8_t* __restrict__ core,
                                           int32_t* __restrict__ parent) {
    if (gp->clique) return;  // quarter-cell unions instead (a small grid: exits at once)
    const int64_t nf = *nf_p;
    const int bs = (int)blockDim.x;
    for (int64_t p = (int64_t)b * bs + threadIdx.x; p < nf; p += (int64_t)nb * bs) {
        if (!core[p]) continue;
        const double2 me = xy[p];
        const Seg s = load_seg(seg, cell[p]);
        int rp = uf_find(parent, (int)p);
        for_candidates(s, [&](int j) {
            if (j >= (int)p) return true;
            const double2 q = xy[j];
            if (within_eps(me.x, me.y, q.x, q.y, eps2) && core[j]) {
                const int rj = uf_find(parent, j);
                if (rj != rp) rp = uf_unite_roots(parent, perm, rp, rj);
            }
            return true;
        });
    }
}

__global__ __launch_bounds__(kBlock) void union_kernel(const double2* __restrict__ xy,
                                                       const int32_t* __restrict__ cell,
                                                       const Seg* __restrict__ seg,
                                                       const int32_t* __restrict__ nf_p,
                                                       const GridParams* __restrict__ gp,
                                                       double eps2,
                                                       const int32_t* __restrict__ perm,
                                                       const uint8_t* __restrict__ core,
                                                       int32_t* __restrict__ parent) {
    union_body(blockIdx.x, gridDim.x, xy, cell, seg, nf_p, gp, eps2, perm, core, parent);
}

// ---------------------------------------------------------------------------------------
// Clique-quarter union (cell side <= eps*(1+2^-14)).  A quarter cell has side ~eps/2 and
// diagonal ~0.71*eps, so any two of its points satisfy the fp64 predicate: its cores are one
// connected set without a single distance test.  Two quarter cells can hold an eps pair only
// if their quarter-grid offsets are <= 2 (inside the 3x3 eps-cell stencil); ONE core-core
// edge per such pair suffices.
// ---------------------------------------------------------------------------------------
// Quarter pairs that cross a tile edge.  One wave per (tile, side), each wave looping on its
// own (no block barriers): side 0 pairs the tile's
// east cell column with the E tile's west column plus the SE tile's corner cell; side 1 its
// south row with the S tile's north row plus the SW tile's corner cell.  With the mirrored
// sides of the other tiles, every pair of adjacent cells in different tiles is covered once.
// The wave loads the quarter cells of the facing strips (<= 32 + 36) into LDS, tags each with
// its tile component (qcomp, from the count kernels' tile unions), pre-joins equal tags in an LDS union-find, then
// pair-tests facing quarters within quarter distance 2 (adjacent first) only while the two are
// not yet joined in LDS.  A found edge is one global union of the two tile components, so the
// global union-find sees about one operation per component pair per tile side.
constexpr int kEdgeNodes = 72;
// DBSCAN_AB_EDGE_STOP (timing builds only): 1 ends each trip after the node loads, 2 after the
// LDS pre-join, 3 skips the global unions
// edge_union_kernel's launch bound, waves per SIMD: 5 (96 VGPRs, no scratch) measured 0.166 ->
// 0.153 ms at config 2 against 6 (80 VGPRs, 48 B of scratch); 4: 0.178
#ifndef DBSCAN_AB_EDGE_W
#define DBSCAN_AB_EDGE_W 5
#endif
// (launch bound 8 -- 64 VGPRs, 72 B of scratch -- is a broken build of this kernel: round 5's
// four-at-a-time pair-test variant faulted with it once (illegal address), round 6's rebuild of
// that variant faulted again, and the SHIPPED source at bound 8 with every global index checked
// and clamped (DBSCAN_AB_CHECK, tools/bounds_probe.py) hung in its union loops, while the same
// checked source at bound 5 ran configs 2, 3's share and 4 with 0 indices out of range: the
// fault follows the 64-VGPR code generation, not the strip / quarter indexing.  DESIGN_LOG r6.)
static_assert(DBSCAN_AB_EDGE_W <= 6, "edge_union_kernel misbehaves at launch bound 8");
// big_count_kernel's launch bound, waves per SIMD: 7 (71 VGPRs, no scratch) measured 0.113 ->
// 0.103 ms at config 2 against 5 (81 VGPRs); 6: 0.111; 8 spills
#ifndef DBSCAN_AB_BIGC_W
#define DBSCAN_AB_BIGC_W 7
#endif
// waves per workgroup of big_count and of count_wave / count_tiny (each wave on work of its own;
// a workgroup's slot is released only when its last wave ends): big_count 1 wave 0.105 -> 0.099
// ms at config 2, 0.44 -> 0.42 at config 4 (2 waves: 0.102, 0.428); count_wave 1 wave 0.058 ->
// 0.057 ms at config 2, 0.124 -> 0.118 on config 3's share (round 6, A/B on one box)
#ifndef DBSCAN_AB_BIGC_WAVES
#define DBSCAN_AB_BIGC_WAVES 1
#endif
#ifndef DBSCAN_AB_CW_WAVES
#define DBSCAN_AB_CW_WAVES 1
#endif
#ifndef DBSCAN_AB_EDGE_STOP
#define DBSCAN_AB_EDGE_STOP 0
#endif
// edge_union's waves per workgroup: 2 (or 1) measured 0.154 -> 0.146 ms at config 2 and 0.184 ->
// 0.172 on config 3's share against 4: a workgroup's slot is freed only when its last wave ends
#ifndef DBSCAN_AB_EDGE_WAVES
#define DBSCAN_AB_EDGE_WAVES 2
#endif
// DBSCAN_AB_EDGE_COUNT (counting builds only): edge_union's pair-test outcomes, summed over the
// fit, read back (and cleared) by dbscan_ab_edge_counts() (tools/edge_probe.py)
#ifndef DBSCAN_AB_EDGE_COUNT
#define DBSCAN_AB_EDGE_COUNT 0
#endif
#if DBSCAN_AB_EDGE_COUNT
__device__ unsigned long long g_edge_cnt[8];
#define EDGE_CNT(k) atomicAdd(&g_edge_cnt[(k)], 1ull)
#else
#define EDGE_CNT(k) \
    do {            \
    } while (0)
#endif

// edge_union's full pair test (the reps were not within eps) and its global union.
__device__ __forceinline__ bool edge_pair_full(const double2* __restrict__ xy, int4 me, int4 o,
                                               const uint8_t* __restrict__ core, double eps2) {
    const auto gcore = [core](int j) { return core[j] != 0; };
    double px[kQReg], py[kQReg];
    const int na = load_own(xy, me, 0, px, py);
    EDGE_CNT(na >= 0 ? 3 : 4);
    return na >= 0 ? pair_found(px, py, na, xy, o.x, o.y, (uint32_t)o.w, gcore, 0, eps2)
                   : pair_found_generic(xy, 0, me, o, gcore, eps2);
}
__device__ __forceinline__ void edge_unite(int32_t* __restrict__ parent,
                                           const int32_t* __restrict__ perm, int ca, int cb,
                                           int nf) {
#if DBSCAN_AB_CHECK
    // (checking builds: every parent-chain index in [0, nf), checked and clamped)
    const auto find = [&](int x) {
        x = CHK(9, x, 0, nf);
        for (int k = 0; k < (1 << 20); ++k) {
            const int p = CHK(9, ld_par<0>(parent, x), 0, nf);
            if (p == x) break;
            x = p;
        }
        return x;
    };
    int ra = find(ca), rb = find(cb);
    for (int k = 0; k < (1 << 20) && ra != rb; ++k) {
        const bool swap = perm[ra] < perm[rb];
        const int hi = swap ? rb : ra, lo = swap ? ra : rb;
        int expected = hi;
        if (__hip_atomic_compare_exchange_strong(parent + hi, &expected, lo, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
        ra = find(expected);
        rb = find(lo);
    }
#else
    (void)nf;
    const int ra = uf_find(parent, ca);
    const int rb = uf_find(parent, cb);
    if (ra != rb) uf_unite_roots(parent, perm, ra, rb);
#endif
}

// WAVES: waves per workgroup, each on its own (tile, side) tasks.  (A workgroup's slot is freed
// only when its last wave ends, so waves of uneven task lists hold each other's slots.)
template <int MINW, int WAVES>
__global__ __launch_bounds__(64 * WAVES, MINW) void edge_union_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ ntiles_p,
    const int32_t* __restrict__ tq, const int4* __restrict__ tnb,
    const int4* __restrict__ qinfo, const int4* __restrict__ qg,
    const int32_t* __restrict__ qcomp, double eps2, const int32_t* __restrict__ perm,
    const uint8_t* __restrict__ core, int32_t* __restrict__ parent,
    const GridParams* __restrict__ gp, const uint8_t* __restrict__ tcore, int edge_blocks,
    const int32_t* __restrict__ cell, const Seg* __restrict__ seg,
    const int32_t* __restrict__ nf_p) {
    // blocks from edge_blocks: union_kernel's job in this launch (the per-point union of grids
    // whose quarters are not cliques; the edge blocks then exit, and vice versa)
    if ((int)blockIdx.x >= edge_blocks) {
        union_body((int)blockIdx.x - edge_blocks, (int)gridDim.x - edge_blocks, xy, cell, seg,
                   nf_p, gp, eps2, perm, core, parent);
        return;
    }
    if (!gp->clique) return;
    __shared__ int4 nqi[WAVES][kEdgeNodes];
    __shared__ int2 ngq[WAVES][kEdgeNodes];
    __shared__ int ncomp[WAVES][kEdgeNodes];
    __shared__ int nlp[WAVES][kEdgeNodes];
    // facing nodes by position along the strip: facing cell f (0..7; the corner cell is f = 8
    // on side 0, f = -1 on side 1) holds nodes [fnb[f + 1], fne[f + 1])
    __shared__ int fnb[WAVES][10], fne[WAVES][10];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ntiles = *ntiles_p;
    int* lp = nlp[w];
    // one (tile, side) per wave and loop trip: waves never wait for each other
    for (int tw = xcd_block(edge_blocks) * WAVES + w; tw < 2 * ntiles;
         tw += edge_blocks * WAVES) {
        const int t = tw >> 1, side = tw & 1;
        int nA = 0, ntot = 0;
        {
            const int4 nb = tnb[t];
            // an own strip without cores has no pair to test (tcore: the count kernels')
            if (tcore && !((tcore[t] >> side) & 1)) continue;
            const int occB = side ? nb.y : nb.x, occC = side ? nb.w : nb.z;
            const int k = lane & 7;
            int occ = -1, l = 0;
            if (lane < 8) {  // own strip
                occ = t;
                l = side ? 56 + k : k * 8 + 7;
            } else if (lane < 16) {  // facing strip
                occ = occB;
                l = side ? k : k * 8;
            } else if (lane == 16) {  // corner cell
                occ = occC;
                l = side ? 7 : 0;
            }
            int cnt = 0, q0 = 0;
            if (occ >= 0) {
                occ = CHK(7, occ, 0, ntiles);
                q0 = tq[(int64_t)occ * kTslot + l];
                cnt = tq[(int64_t)occ * kTslot + l + 1] - q0;
            }
            int incl = cnt;  // own nodes first, then facing + corner
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) {
                const int u = __shfl_up(incl, o, 64);
                if (lane >= o) incl += u;
            }
            nA = __shfl(incl, 7, 64);
            ntot = __shfl(incl, 16, 64);
            if (lane < 10) {
                fnb[w][lane] = 0;
                fne[w][lane] = 0;
            }
            wave_sync();
            if (lane >= 8 && lane <= 16) {
                const int f = lane < 16 ? k : (side ? -1 : 8);
                fnb[w][f + 1] = incl - cnt;
                fne[w][f + 1] = incl;
            }
            // node -> quarter index in LDS (lp, free until the pre-join), then a lane per node:
            // the quarter loads of all nodes in flight at once, not one cell's per trip
            for (int j = 0; j < cnt; ++j) lp[incl - cnt + j] = q0 + j;
            wave_sync();
            for (int i = lane; i < ntot; i += 64) {
                const int q = CHK(8, lp[CHK(2, i, 0, kEdgeNodes)], 0,
                                  ntiles_p[kStQuarters - kStTiles]);
                const int4 qi = qinfo[q];
                const int4 gq = qg[q];
                const int qc = qcomp[q];  // tile component rep (a member of the set)
                nqi[w][i] = qi;
                ngq[w][i] = make_int2(gq.x, gq.y);
                ncomp[w][i] = qc;
            }
        }
        wave_sync();
        if (lane == 0) EDGE_CNT(0);
        if (lane == 0 && ntot > 64) EDGE_CNT(7);
        if (DBSCAN_AB_EDGE_STOP == 1) continue;
        {
            // pre-join nodes sharing a tile component (own nodes among themselves, facing nodes
            // among themselves): lp[i] = the first such node.  Nodes 0..63 sit in the lanes, one
            // ballot per distinct component (a per-lane scan of the earlier nodes cost ~40 us of
            // the launch at 10^7); nodes 64.. (corner quarters) against the lanes, then each other
            const int c = lane < ntot ? ncomp[w][lane] : -1;
            const bool own = lane < nA;
            int r = lane;
            unsigned long long todo = __ballot(c >= 0);
            while (todo) {
                const int ld = __builtin_ctzll(todo);
                const int lc = __shfl(c, ld, 64);
                const unsigned long long m = __ballot(c == lc && own == (ld < nA)) & todo;
                if ((m >> lane) & 1ull) r = ld;
                todo &= ~m;
            }
            if (lane < ntot) lp[lane] = r;
            for (int i = 64; i < ntot; ++i) {  // (wave-uniform; node i >= nA: a facing node)
                const int ci = ncomp[w][i];
                const unsigned long long m = __ballot(ci >= 0 && c == ci && !own);
                int ri = m ? __builtin_ctzll(m) : i;
                if (!m && ci >= 0)
                    for (int j = 64; j < i; ++j)
                        if (ncomp[w][j] == ci) {
                            ri = j;
                            break;
                        }
                if (lane == 0) lp[i] = ri;
            }
        }
        wave_sync();
        if (DBSCAN_AB_EDGE_STOP == 2) continue;
        const int a = lane & 31, half = lane >> 5;  // two lanes per own-strip quarter
        if (a < nA) {
            const int4 me = nqi[w][a];
            const int2 mg = ngq[w][a];
            if (me.z >= 0) {
                // only facing cells within quarter distance 2 along the strip: three cells, at
                // most two of each cell's quarters per lane (two lanes per own quarter)
                const int ua = (side ? mg.x : mg.y) & 15;
                const int flo = (ua - 2) >> 1;
                int sb[6], sd[6];
#pragma unroll
                for (int c = 0; c < 6; ++c) {
                    const int f = CHK(3, flo + (c >> 1) + 1, 0, 10) - 1;
                    const int b = fnb[w][f + 1] + half + 2 * (c & 1);
                    sb[c] = -1;
                    sd[c] = 0;
                    if (b < fne[w][f + 1]) {
                        const int2 og = ngq[w][CHK(4, b, 0, ntot)];
                        const int d = max(abs(og.x - mg.x), abs(og.y - mg.y));
                        if (d <= 2 && nqi[w][b].z >= 0) {
                            sb[c] = b;
                            sd[c] = d;
                        }
                    }
                }
                // each pair's first test: the two quarters' reps (cores), all loads in flight
                // together; the full test only where the reps are not within eps
                const double2 pr = xy[CHK(5, me.z, 0, *nf_p)];
                double2 po[6];
#pragma unroll
                for (int c = 0; c < 6; ++c)
                    po[c] = sb[c] >= 0 ? xy[CHK(5, nqi[w][sb[c]].z, 0, *nf_p)] : make_double2(0.0, 0.0);
#pragma unroll 1
                for (int sweep = 1; sweep <= 2; ++sweep)
#pragma unroll
                    for (int c = 0; c < 6; ++c) {
                        if (sb[c] < 0 || sd[c] != sweep) continue;
                        const int b = sb[c];
                        if (lfind(lp, a) == lfind(lp, b)) continue;
                        EDGE_CNT(sweep);
#if DBSCAN_AB_CHECK
                        {  // the two quarters' slot ranges inside [0, nf]
                            const int4 ob = nqi[w][b];
                            (void)CHK(10, me.x, 0, *nf_p + 1);
                            (void)CHK(10, me.y, me.x, *nf_p + 1);
                            (void)CHK(10, ob.x, 0, *nf_p + 1);
                            (void)CHK(10, ob.y, ob.x, *nf_p + 1);
                        }
#endif
                        if (!within_eps(pr.x, pr.y, po[c].x, po[c].y, eps2) &&
                            !edge_pair_full(xy, me, nqi[w][b], core, eps2))
                            continue;
                        EDGE_CNT(5);
                        // one global union per merge of two LDS sets: a lane that finds its
                        // pair already joined (another lane's merge) leaves the global sets alone
                        if (lunite(lp, a, b) && DBSCAN_AB_EDGE_STOP != 3) {
                            EDGE_CNT(6);
                            edge_unite(parent, perm, CHK(6, ncomp[w][a], 0, *nf_p),
                                       CHK(6, ncomp[w][b], 0, *nf_p), *nf_p);
                        }
                    }
            }
        }
        wave_sync();
    }
}

// After all unions: every quarter rep points straight at its root, so the per-point walk in
// final_kernel is core -> rep -> root.  qlab (direct fits): also the root's visit index per
// quarter, and the root flag (every root is a quarter rep: the rep of exactly one quarter), so
// that final_kernel's grid cores only read their quarter's qlab.
// Quarters per thread (quarter base + k * kBlock): their rep loads, then their parent chains one
// step per trip with the steps' loads in flight together; 1 quarter per thread 0.035 ms per
// 10^7 points, 4: 0.031 (A/B on one box, round 6).
constexpr int kQrootPer = 4;  // (2 and 8: the same)

__global__ __launch_bounds__(kBlock) void quarter_root_kernel(
    const int4* __restrict__ qinfo, const int32_t* __restrict__ nq_p,
    const GridParams* __restrict__ gp, int32_t* __restrict__ parent,
    const int32_t* __restrict__ perm, int32_t* __restrict__ qlab,
    unsigned long long* __restrict__ root_bits) {
    if (!gp->clique) return;
    constexpr int K = kQrootPer;
    const int nq = *nq_p;
    const int base = blockIdx.x * (K * kBlock) + threadIdx.x;
    int rep[K], r[K], nx[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int q = base + k * kBlock;
        rep[k] = q < nq ? qinfo[q].z : -1;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        r[k] = rep[k];
        nx[k] = rep[k] >= 0 ? parent[rep[k]] : rep[k];
    }
    for (;;) {  // every open chain one step per trip, their loads in flight together
        bool open = false;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (nx[k] != r[k]) {
                r[k] = nx[k];
                nx[k] = parent[r[k]];
                open = true;
            }
        if (!open) break;
    }
    int32_t o[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (rep[k] < 0) continue;
        parent[rep[k]] = r[k];
        if (qlab) o[k] = perm[r[k]];
    }
    if (qlab) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (rep[k] < 0) continue;
            qlab[base + k * kBlock] = o[k];
            if (r[k] == rep[k]) atomicOr(root_bits + (o[k] >> 6), 1ull << (o[k] & 63));
        }
    }
}

// qidx/qinfo (fused union: core parents were never written): a grid core's walk starts at its
// quarter's rep (slots >= nf are outside the grid and their own parents).
__device__ __forceinline__ void final_point(int64_t p, const int32_t* __restrict__ nf_p,
                                            const GridParams* __restrict__ gp,
                                            const int32_t* __restrict__ perm,
                                            const uint8_t* __restrict__ core,
                                            const int32_t* __restrict__ parent,
                                            const int32_t* __restrict__ qidx,
                                            const int4* __restrict__ qinfo,
                                            int32_t* __restrict__ lab,
                                            unsigned long long* __restrict__ root_bits,
                                            int32_t* __restrict__ root_out,
                                            const int32_t* __restrict__ qlab) {
    if (!core[p]) {
        lab[p] = -1;
        return;
    }
    int r = (int)p;
    const int64_t nf = *nf_p;
    if (qlab && gp->clique && p < nf) {  // quarter_root_kernel resolved the quarter's root
        lab[p] = qlab[qidx[p]];
        return;
    }
    if (qidx && gp->clique && nf > 0) {
        // Branch-free on purpose: the divergent form `p < nf ? qinfo[qidx[p]].z : p` was
        // miscompiled (ROCm 7.2 clang, gfx950: the else value was never moved into place for
        // the lanes with p >= nf).  Clamp the index, load, select.
        const int rq = qinfo[qidx[p < nf ? p : nf - 1]].z;
        r = p < nf ? rq : r;
    }
    for (int nx = parent[r]; nx != r; nx = parent[r]) r = nx;
    const int32_t o = perm[r];
    lab[p] = o;
    if (r == (int)p && root_bits) atomicOr(root_bits + (o >> 6), 1ull << (o & 63));
    if (r == (int)p && root_out) root_out[o] = o;  // lean slab output: the local roots
}

// Four consecutive slots per thread: on direct clique fits (every grid slot's label is its
// quarter's root label, qlab) one 4-B core load, one 16-B quarter-index load, four qlab loads
// in flight and one 16-B store; 0.040 -> 0.022 ms per 10^7 points (A/B on one box, round 6).
constexpr int kFinalPer = 4;

__global__ __launch_bounds__(kBlock) void final_kernel(int64_t n, const int32_t* __restrict__ nf_p,
                                                       const GridParams* __restrict__ gp,
                                                       const int32_t* __restrict__ perm,
                                                       const uint8_t* __restrict__ core,
                                                       const int32_t* __restrict__ parent,
                                                       const int32_t* __restrict__ qidx,
                                                       const int4* __restrict__ qinfo,
                                                       int32_t* __restrict__ lab,
                                                       unsigned long long* __restrict__ root_bits,
                                                       int32_t* __restrict__ root_out,
                                                       const int32_t* __restrict__ qlab) {
    const int64_t p0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kFinalPer;
    if (p0 >= n) return;
    if (qlab && gp->clique && p0 + 3 < *nf_p) {
        // four consecutive grid slots: core bytes and quarter indices by one load each, their
        // quarters' root labels in flight together, one 16-B store
        const uchar4 c = *reinterpret_cast<const uchar4*>(core + p0);
        const int4 qi = *reinterpret_cast<const int4*>(qidx + p0);
        int4 out;
        out.x = c.x ? qlab[qi.x] : -1;
        out.y = c.y ? qlab[qi.y] : -1;
        out.z = c.z ? qlab[qi.z] : -1;
        out.w = c.w ? qlab[qi.w] : -1;
        *reinterpret_cast<int4*>(lab + p0) = out;
        return;
    }
    for (int64_t p = p0; p < p0 + kFinalPer && p < n; ++p)
        final_point(p, nf_p, gp, perm, core, parent, qidx, qinfo, lab, root_bits, root_out, qlab);
}

// Lean slab output for the listed (shared) slab points: core flag and local root.
__global__ __launch_bounds__(kBlock) void slab_shared_kernel(int64_t m,
                                                             const int64_t* __restrict__ idx,
                                                             const int32_t* __restrict__ inv,
                                                             const uint8_t* __restrict__ core,
                                                             const int32_t* __restrict__ lab,
                                                             uint8_t* __restrict__ core_out,
                                                             int32_t* __restrict__ root_out) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= m) return;
    const int64_t i = idx[k];
    const int32_t p = inv[i];
    const bool c = core[p] != 0;
    core_out[i] = c ? 1 : 0;
    root_out[i] = c ? lab[p] : -1;
}

// Cluster id of the component whose root (s(K)) is input point o: 1 + number of roots before o
// in input order, from the root bit words and their scanned popcounts (L2-resident: n/8 +
// n/16 bytes, where a per-point rank array would be 4n bytes of scattered reads).
__device__ __forceinline__ uint32_t cluster_of_root(const uint64_t* __restrict__ root_bits,
                                                    const int32_t* __restrict__ word_rank,
                                                    int32_t o) {
    const uint64_t below = root_bits[o >> 6] & ((1ull << (o & 63)) - 1ull);
    return (uint32_t)(word_rank[o >> 6] + __popcll(below)) + 1u;
}

// Labels, one thread per sorted slot: cores rank[lab]+1 (or the merged label for slab fits);
// non-cores the minimum lab over their core neighbours, read from the neighbour lists the
// count pass kept (nbr != nullptr: minPoints <= kMaxNbr + 1), else by a stencil scan.  The
// result is packed per slot as (cluster << 1) | core, coalesced; permute_out_kernel then moves
// it to input order with one random 4-B read per point (the packed array was just written and
// is cache-resident), instead of two scattered partial-line writes (cluster 4 B + flag 1 B).
// Slab fits (SLAB) label zone-0 points from the merged global component ids.  Slots >= nf are
// outside the grid: never anyone's neighbour.  ROOTS (slab fits only): the numbering is not
// known yet, so the packed value names the local root instead, ((root + 1) << 1) | core, and
// slab_map_kernel turns it into a cluster id once the roots are numbered.
template <bool SLAB, bool ROOTS = false>
__global__ __launch_bounds__(kBlock) void label_sorted_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, const int32_t* __restrict__ nbr, int nbr_k,
    const int32_t* __restrict__ nf_p, int64_t n, double eps2, int32_t mode, const int32_t* __restrict__ perm,
    const uint8_t* __restrict__ core, const int32_t* __restrict__ lab,
    const uint64_t* __restrict__ root_bits, const int32_t* __restrict__ word_rank,
    const uint8_t* __restrict__ zone,
    const int64_t* __restrict__ gid, const int64_t* __restrict__ gs_of_root,
    const int32_t* __restrict__ label_of_root, uint32_t* __restrict__ packed,
    const int32_t* __restrict__ place) {
    // bucketed fits: XCD-contiguous slot ranges (gather_block: the packed[place] writes of a band
    // merge in one L2)
    const int64_t blk = place ? gather_block() : (int64_t)blockIdx.x;
    const int64_t p = blk * kBlock + threadIdx.x;
    if (p >= n) return;
    const int64_t nf = *nf_p;
    uint32_t v = 0;  // Noise
    if (core[p]) {
        const uint32_t cl = ROOTS ? (uint32_t)lab[p] + 1u
                            : SLAB ? (uint32_t)label_of_root[lab[p]]
                                   : cluster_of_root(root_bits, word_rank, lab[p]);
        v = (cl << 1) | 1u;
    } else if (p < nf) {
        const int32_t o = perm[p];
        if (SLAB && zone[o] != 0) {
            packed[place ? place[p] : p] = 0;
            return;  // zone 2 has no neighbour list; zones 1/2 are not labelled here
        }
        int64_t m = 0x7FFFFFFFFFFFFFFFll;
        int32_t mr = -1;
        auto visit = [&](int j) {
            if (!core[j]) return;
            const int32_t lj = lab[j];
            const int64_t w = SLAB ? gs_of_root[lj] : (int64_t)lj;
            if (w < m) {
                m = w;
                mr = lj;
            }
        };
        if (nbr) {
            // the whole list, then every neighbour's core flag, then the cores' labs: three
            // rounds of loads in flight instead of a dependent pair per neighbour (the non-core
            // lanes are each wave's longest chains)
            const int32_t* l = nbr + p * nbr_k;
            int js[kMaxNbr];
            bool live = true;
#pragma unroll
            for (int k = 0; k < kMaxNbr; ++k) {
                js[k] = -1;
                if (k < nbr_k) js[k] = l[k];
            }
#pragma unroll
            for (int k = 0; k < kMaxNbr; ++k) {  // -1 ends the list; later entries are stale
                live = live && js[k] >= 0;
                if (!live) js[k] = -1;
            }
            bool cj[kMaxNbr];
#pragma unroll
            for (int k = 0; k < kMaxNbr; ++k) {
                cj[k] = false;
                if (js[k] >= 0) cj[k] = core[js[k]] != 0;
            }
            int32_t lj[kMaxNbr];
#pragma unroll
            for (int k = 0; k < kMaxNbr; ++k) {
                lj[k] = 0;
                if (cj[k]) lj[k] = lab[js[k]];
            }
#pragma unroll
            for (int k = 0; k < kMaxNbr; ++k) {
                if (!cj[k]) continue;
                const int64_t w = SLAB ? gs_of_root[lj[k]] : (int64_t)lj[k];
                if (w < m) {
                    m = w;
                    mr = lj[k];
                }
            }
        } else {
            const double2 me = xy[p];
            const Seg s = load_seg(seg, cell[p]);
            for (int k = 0; k < 6; ++k)
                for (int j = s.b[k]; j < s.e[k]; ++j) {
                    const double2 q = xy[j];
                    if (within_eps(me.x, me.y, q.x, q.y, eps2)) visit(j);
                }
        }
        const int64_t self = SLAB ? gid[o] : (int64_t)o;
        if (mr >= 0 && (mode != 0 || m < self)) {
            const uint32_t cl = ROOTS ? (uint32_t)mr + 1u
                                : SLAB ? (uint32_t)label_of_root[mr]
                                       : cluster_of_root(root_bits, word_rank, mr);
            v = cl << 1;  // Border
        }
    }
    packed[place ? place[p] : p] = v;  // (bucketed sort: at the slot's padded place)
}

// Input order: cluster = packed >> 1; flag Core (odd), Border (even, nonzero), Noise (0).
// Slab fits leave zone 1/2 entries untouched.
template <bool SLAB>
__global__ __launch_bounds__(kBlock) void permute_out_kernel(
    int64_t n, const int32_t* __restrict__ inv, const uint32_t* __restrict__ packed,
    const uint8_t* __restrict__ zone, int32_t* __restrict__ cluster_out,
    uint8_t* __restrict__ flag_out, const int32_t* __restrict__ nk_src,
    int32_t* __restrict__ nk_out) {
    if (nk_out && blockIdx.x == 0 && threadIdx.x == 0) *nk_out = *nk_src;  // (the cluster count)
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (SLAB && zone[i] != 0) return;
    const uint32_t v = packed[inv[i]];
    cluster_out[i] = (int32_t)(v >> 1);
    flag_out[i] = v == 0 ? 2 : (uint8_t)(v & 1u);
}

// Batched fits: clusters numbered per partition (LocalDBSCANNaive.scala:58 counts from 0 in every
// fit): roots(o) = roots with a visit (batch) index below o, so partition p's ids are the batch
// ids minus roots(offs[p]).
__device__ __forceinline__ int32_t roots_before(const uint64_t* __restrict__ root_bits,
                                                const int32_t* __restrict__ word_rank,
                                                int64_t o) {
    return word_rank[o >> 6] + __popcll(root_bits[o >> 6] & ((1ull << (o & 63)) - 1ull));
}

__global__ __launch_bounds__(kBlock) void permute_out_batch_kernel(
    int64_t n, const int32_t* __restrict__ inv, const uint32_t* __restrict__ packed,
    const int64_t* __restrict__ poffs, int np, const uint64_t* __restrict__ root_bits,
    const int32_t* __restrict__ word_rank, int32_t* __restrict__ cluster_out,
    uint8_t* __restrict__ flag_out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = packed[inv[i]];
    const int32_t c = (int32_t)(v >> 1);
    cluster_out[i] = c ? c - roots_before(root_bits, word_rank, poffs[part_of(poffs, np, i)]) : 0;
    flag_out[i] = v == 0 ? 2 : (uint8_t)(v & 1u);
}

// Clusters of every partition of a batch (n = the batch's span; the total is st[kStClusters]).
__global__ __launch_bounds__(kBlock) void batch_nclusters_kernel(
    int64_t n, const int64_t* __restrict__ poffs, int np, const uint64_t* __restrict__ root_bits,
    const int32_t* __restrict__ word_rank, const int32_t* __restrict__ st,
    int32_t* __restrict__ nclusters) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= np) return;
    const int64_t a = poffs[p], b = poffs[p + 1];
    const int32_t ra = a >= n ? st[kStClusters] : roots_before(root_bits, word_rank, a);
    const int32_t rb = b >= n ? st[kStClusters] : roots_before(root_bits, word_rank, b);
    nclusters[p] = rb - ra;
}

// Batched fits: the partition of every occupied tile (all of a tile's points belong to one
// partition: each partition's grid holds its own tiles), from its first slot's batch index.
__global__ __launch_bounds__(kBlock) void tile_part_kernel(const int32_t* __restrict__ tstart,
                                                           const int32_t* __restrict__ ntiles_p,
                                                           const int32_t* __restrict__ perm,
                                                           const GridParams* __restrict__ gp,
                                                           int32_t* __restrict__ tpart) {
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= *ntiles_p) return;
    tpart[t] = part_of(gp->poffs, gp->nparts, perm[tstart[t]]);
}

// Bucketed sort: input order from the labels at the padded places (pos: input -> place); pos
// reads are coalesced, and a block's points read from the 256 bands' segments where they
// stand in input order (runs that advance together).  kPermPer points per thread (point
// base + k * kBlock): their pos loads, then their packed reads, in flight together.  One point
// per thread: 0.059 ms per 10^7 points; 4: 0.058; 8: 0.052-0.053 (config 3's share 0.071 ->
// 0.057); 16: 0.052 (A/B on one box, round 6).
constexpr int kPermPer = 8;
__global__ __launch_bounds__(kBlock) void permute_out_bucket_kernel(
    int64_t n, const int32_t* __restrict__ pos, const uint32_t* __restrict__ packed,
    int32_t* __restrict__ cluster_out, uint8_t* __restrict__ flag_out,
    const int32_t* __restrict__ nk_src, int32_t* __restrict__ nk_out) {
    if (nk_out && blockIdx.x == 0 && threadIdx.x == 0) *nk_out = *nk_src;  // (the cluster count)
    const int64_t base = (int64_t)blockIdx.x * (kPermPer * kBlock) + threadIdx.x;
    int32_t ps[kPermPer];
#pragma unroll
    for (int k = 0; k < kPermPer; ++k) {
        const int64_t i = base + k * kBlock;
        ps[k] = i < n ? pos[i] : 0;
    }
    uint32_t v[kPermPer];
#pragma unroll
    for (int k = 0; k < kPermPer; ++k)
        if (base + k * kBlock < n) v[k] = packed[ps[k]];
#pragma unroll
    for (int k = 0; k < kPermPer; ++k) {
        const int64_t i = base + k * kBlock;
        if (i >= n) break;
        cluster_out[i] = (int32_t)(v[k] >> 1);
        flag_out[i] = v[k] == 0 ? 2 : (uint8_t)(v[k] & 1u);
    }
}

// ---------------------------------------------------------------------------------------
// LocalDBSCANArchery with its float32 R-tree search box (DBSCAN_MODE_ARCHERY_F32BOX).
// The tree stores Point(p.x.toFloat, p.y.toFloat) (LocalDBSCANArchery.scala:38-41) and a
// query searches Box((x-eps).toFloat, (y-eps).toFloat, (x+eps).toFloat, (y+eps).toFloat)
// (:118-124), filtered by the fp64 predicate (:114-116).  So o is a neighbour of p iff
// d2 <= eps2 AND o's float point lies in p's float box -- a DIRECTED relation: near the box
// edge one of the two directions can fail.  Containment is taken inclusive on all four sides
// (archery 0.3.0's source is absent: the one unpinned assumption).
//   core(p)  <=> |N(p)| >= minPoints (N(p) from p's own box)
//   clusters: components of the core-core pairs that hold in BOTH directions, plus the
//             one-way core-core pairs, recorded here and resolved on the host exactly as the
//             sequential expansion does (components in s order; a new cluster claims every
//             component reachable over one-way pairs that no earlier cluster claimed)
//   non-core b: Border of the smallest cluster number among cores c with b in N(c), else Noise
// (the archery re-claim rule, :103-106).  One thread per point over the global stencil
// pieces: this mode is a parity path, not the bench path.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool in_f32_box(double px, double py, double ox, double oy,
                                           double eps) {
#pragma clang fp contract(off)
    const float x1 = (float)(px - eps), y1 = (float)(py - eps);
    const float x2 = (float)(px + eps), y2 = (float)(py + eps);
    const float fx = (float)ox, fy = (float)oy;
    return x1 <= fx && fx <= x2 && y1 <= fy && fy <= y2;
}

__global__ __launch_bounds__(kBlock) void box_count_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, const int32_t* __restrict__ nf_p, double eps, double eps2,
    int32_t min_points, uint8_t* __restrict__ core, int32_t* __restrict__ parent,
    int32_t* __restrict__ block_cores) {
    __shared__ int wcores[kBlock / 64];
    const int64_t nf = *nf_p;
    int mine = 0;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < nf;
         p += (int64_t)gridDim.x * kBlock) {
        const double2 me = xy[p];
        const Seg s = load_seg(seg, cell[p]);
        int cnt = 0;
        if (min_points > 0)
            for_candidates(s, [&](int j) {
                const double2 q = xy[j];
                cnt += (within_eps(me.x, me.y, q.x, q.y, eps2) &&
                        in_f32_box(me.x, me.y, q.x, q.y, eps)) ? 1 : 0;
                return cnt < min_points;
            });
        const bool is_core = cnt >= min_points;
        parent[p] = (int32_t)p;
        core[p] = is_core ? 1 : 0;
        mine += is_core ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if (__lane_id() == 0) wcores[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += wcores[w];
        block_cores[blockIdx.x] = tot;
    }
}

// Core-core pairs that hold in both directions -> union (once, from the larger slot).
__global__ __launch_bounds__(kBlock) void box_union_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, const int32_t* __restrict__ nf_p, double eps, double eps2,
    const int32_t* __restrict__ perm, const uint8_t* __restrict__ core,
    int32_t* __restrict__ parent) {
    const int64_t nf = *nf_p;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < nf;
         p += (int64_t)gridDim.x * kBlock) {
        if (!core[p]) continue;
        const double2 me = xy[p];
        const Seg s = load_seg(seg, cell[p]);
        int rp = uf_find(parent, (int)p);
        for_candidates(s, [&](int j) {
            if (j >= (int)p || !core[j]) return true;
            const double2 q = xy[j];
            if (!within_eps(me.x, me.y, q.x, q.y, eps2)) return true;
            if (in_f32_box(me.x, me.y, q.x, q.y, eps) && in_f32_box(q.x, q.y, me.x, me.y, eps)) {
                const int rj = uf_find(parent, j);
                if (rj != rp) rp = uf_unite_roots(parent, perm, rp, rj);
            }
            return true;
        });
    }
}

// After the components are final (lab = s(K) of every core): the one-way core-core pairs
// (q in N(p), p not in N(q)) whose two ends lie in DIFFERENT components -- the only ones that
// carry information -- recorded as (source slot, target slot) while fewer than `cap` exist.
// The 64-bit count keeps growing past cap, so the host can size the buffer and run this again.
__global__ __launch_bounds__(kBlock) void box_pairs_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, const int32_t* __restrict__ nf_p, double eps, double eps2,
    const uint8_t* __restrict__ core, const int32_t* __restrict__ lab, int2* __restrict__ edges,
    unsigned long long* __restrict__ n_edges, unsigned long long cap) {
    const int64_t nf = *nf_p;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < nf;
         p += (int64_t)gridDim.x * kBlock) {
        if (!core[p]) continue;
        const double2 me = xy[p];
        const Seg s = load_seg(seg, cell[p]);
        const int32_t lp = lab[p];
        for_candidates(s, [&](int j) {
            if (j == (int)p || !core[j] || lab[j] == lp) return true;
            const double2 q = xy[j];
            if (!within_eps(me.x, me.y, q.x, q.y, eps2)) return true;
            if (in_f32_box(me.x, me.y, q.x, q.y, eps) && !in_f32_box(q.x, q.y, me.x, me.y, eps)) {
                const unsigned long long k = atomicAdd(n_edges, 1ull);
                if (k < cap) edges[k] = make_int2((int)p, j);
            }
            return true;
        });
    }
}

// The recorded pairs as (component number of the source, of the target), 0-based in s order.
__global__ __launch_bounds__(kBlock) void box_edge_ranks_kernel(
    const int2* __restrict__ edges, int32_t m, const int32_t* __restrict__ lab,
    const uint64_t* __restrict__ root_bits, const int32_t* __restrict__ word_rank,
    int2* __restrict__ out) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= m) return;
    const int2 e = edges[k];
    out[k] = make_int2((int)cluster_of_root(root_bits, word_rank, lab[e.x]) - 1,
                       (int)cluster_of_root(root_bits, word_rank, lab[e.y]) - 1);
}

// Labels (packed per sorted slot like label_sorted_kernel): cores their component's cluster
// number; non-cores the smallest cluster number among cores c whose box holds them.  cmap
// (one-way pairs present): component number -> cluster number; else the identity.
__global__ __launch_bounds__(kBlock) void box_label_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, const int32_t* __restrict__ nf_p, int64_t n, double eps,
    double eps2, const uint8_t* __restrict__ core, const int32_t* __restrict__ lab,
    const uint64_t* __restrict__ root_bits, const int32_t* __restrict__ word_rank,
    const int32_t* __restrict__ cmap, uint32_t* __restrict__ packed,
    const int32_t* __restrict__ place) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    auto number = [&](int j) -> uint32_t {
        const uint32_t c = cluster_of_root(root_bits, word_rank, lab[j]);
        return cmap ? (uint32_t)cmap[c - 1] : c;
    };
    uint32_t v = 0;  // Noise
    if (core[p]) {
        v = (number((int)p) << 1) | 1u;
    } else if (p < *nf_p) {
        const double2 me = xy[p];
        const Seg s = load_seg(seg, cell[p]);
        uint32_t best = 0xFFFFFFFFu;
        for_candidates(s, [&](int j) {
            if (!core[j]) return true;
            const double2 q = xy[j];
            if (within_eps(q.x, q.y, me.x, me.y, eps2) && in_f32_box(q.x, q.y, me.x, me.y, eps)) {
                const uint32_t c = number(j);
                best = c < best ? c : best;
            }
            return true;
        });
        if (best != 0xFFFFFFFFu) v = best << 1;  // Border
    }
    packed[place ? place[p] : p] = v;  // (bucketed sort: at the slot's padded place)
}

// The finish of a prepared slab label: each zone-0 point reads its packed label through
// to_packed (its sorted slot or padded place) and maps its local root to the cluster id
// (label_of_root), flag Core / Border / Noise as permute_out_kernel.  (Copying the packed
// labels to slab order first and mapping them there cost 0.076 + 0.038 ms on config 3's share.)
__global__ __launch_bounds__(kBlock) void slab_map_packed_kernel(
    int64_t n, const int32_t* __restrict__ to_packed, const uint32_t* __restrict__ packed,
    const uint8_t* __restrict__ zone, const int32_t* __restrict__ label_of_root,
    int32_t* __restrict__ cluster_out, uint8_t* __restrict__ flag_out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || zone[i] != 0) return;
    const uint32_t v = packed[to_packed[i]];
    cluster_out[i] = v == 0 ? 0 : label_of_root[(v >> 1) - 1u];
    flag_out[i] = v == 0 ? 2 : (uint8_t)(v & 1u);
}

// Slab fit, phase 1 output (multi-GPU node path): per sorted slot, the slab index of the
// minimum-index core of its local component (lab) or -1 for a non-core, packed coalesced, then
// moved to slab order through inv (one random read per point): root_out, core_out = root >= 0.
__global__ __launch_bounds__(kBlock) void slab_pack_kernel(int64_t n,
                                                           const uint8_t* __restrict__ core,
                                                           const int32_t* __restrict__ lab,
                                                           int32_t* __restrict__ packed,
                                                           const int32_t* __restrict__ place) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p < n) packed[place ? place[p] : p] = core[p] ? lab[p] : -1;
}

__global__ __launch_bounds__(kBlock) void slab_roots_kernel(int64_t n,
                                                            const int32_t* __restrict__ inv,
                                                            const int32_t* __restrict__ packed,
                                                            uint8_t* __restrict__ core_out,
                                                            int32_t* __restrict__ root_out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int32_t v = packed[inv[i]];
    core_out[i] = v >= 0 ? 1 : 0;
    root_out[i] = v;
}

// Slab label, phase 2 prologue: the global cluster id of every local root r (a sorted slot whose
// lab is its own visit index): 1 + rank of its global s(K) among all ranks' global roots
// (all_roots sorted ascending; every s(K) is in it).
__global__ __launch_bounds__(kBlock) void slab_root_labels_kernel(
    int64_t n, const int32_t* __restrict__ perm, const uint8_t* __restrict__ core,
    const int32_t* __restrict__ lab, const int64_t* __restrict__ gs_of_root,
    const int64_t* __restrict__ all_roots, int64_t n_roots, int32_t* __restrict__ label_of_root) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n || !core[p] || lab[p] != perm[p]) return;
    const int32_t r = lab[p];
    const int64_t g = gs_of_root[r];
    int64_t lo = 0, hi = n_roots;  // first index with all_roots[idx] >= g
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (all_roots[mid] < g) lo = mid + 1; else hi = mid;
    }
    label_of_root[r] = (int32_t)(lo + 1);
}

// The same from the list of local roots the prepare compacted (slab indices): one thread per
// root instead of one per sorted slot.
__global__ __launch_bounds__(kBlock) void slab_root_labels_list_kernel(
    int64_t m, const int32_t* __restrict__ lroots, const int64_t* __restrict__ gs_of_root,
    const int64_t* __restrict__ all_roots, int64_t n_roots, int32_t* __restrict__ label_of_root) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    const int32_t r = lroots[i];
    const int64_t g = gs_of_root[r];
    int64_t lo = 0, hi = n_roots;  // first index with all_roots[idx] >= g
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (all_roots[mid] < g) lo = mid + 1; else hi = mid;
    }
    label_of_root[r] = (int32_t)(lo + 1);
}

// Grid sizing (see DESIGN.md "grid soundness"), on the device so a fit needs no host sync: cell side >= R*(1+2^-16) with
// R = max(|eps|*(1+2^-40), 2^-500) bounds |x'-x| for every pair the fp64 predicate accepts;
// at most 2^23 tiles of 8x8 cells (u32 keys = tile*256 + cell*4 + quadrant, below the
// sentinel), growing the side (never shrinking it) when the extent would need more.  Quarter
// cells are cliques only while the side was not grown: clique = side <= |eps|*(1+2^-14).
__device__ bool make_grid(const double* bb, double eps, GridParams* g) {
    const double xmin = bb[0], xmax = bb[1], ymin = bb[2], ymax = bb[3];
    double R = fabs(eps) * (1.0 + 0x1p-40);
    if (R < 0x1p-500) R = 0x1p-500;
    double hx = R * (1.0 + 0x1p-16), hy = hx;
    const double limit = 8388608.0;  // 2^23 tiles
    auto cells = [](double vmax, double vmin, double h) {
        const double t = (vmax * 0.5 - vmin * 0.5) * (2.0 / h);
        return floor(t) + 1.0;  // may be +inf for absurd extents
    };
    for (int it = 0; it < 4096; ++it) {
        const double cx = cells(xmax, xmin, hx), cy = cells(ymax, ymin, hy);
        const double tx = ceil(cx / 8.0), ty = ceil(cy / 8.0);
        if (tx <= limit && ty <= limit && tx * ty <= limit) {
            g->invx = 2.0 / hx;
            g->invy = 2.0 / hy;
            g->xmin2 = xmin * 0.5;
            g->ymin2 = ymin * 0.5;
            g->nx = (uint32_t)cx;
            g->ny = (uint32_t)cy;
            g->ntx = (uint32_t)tx;
            g->nty = (uint32_t)ty;
            const double cl = fabs(eps) * (1.0 + 0x1p-14);
            g->clique = (hx <= cl && hy <= cl) ? 1 : 0;
            return true;
        }
        if (cx >= cy) hx *= 2.0; else hy *= 2.0;
    }
    return false;
}

// One thread: the grid from the bbox of the finite points (bb = xmin, xmax, ymin, ymax, count),
// the finite count nf, the radix key width and a sizing error flag.  No finite point: nf = 0
// and a 1x1 dummy grid (every slot is outside the grid).
// bbox_finite's final reduction of the per-block partials + grid_kernel + the fit state's
// zeroing, in one single-workgroup launch (three launches before)
__device__ __forceinline__ double bg_wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double bg_wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ void grid_state(const double* bb, double eps, GridParams* __restrict__ gp,
                           int32_t* __restrict__ st);

__global__ __launch_bounds__(kBlock) void bbox_grid_kernel(const double* __restrict__ partial,
                                                           int nb, double* __restrict__ bb,
                                                           double eps, GridParams* __restrict__ gp,
                                                           int32_t* __restrict__ st) {
    __shared__ double sm[kBlock / 64][5];
    if (threadIdx.x < kStCount) st[threadIdx.x] = 0;
    double r0 = INFINITY, r1 = -INFINITY, r2 = INFINITY, r3 = -INFINITY, r4 = 0;
    for (int b = threadIdx.x; b < nb; b += kBlock) {
        r0 = fmin(r0, partial[b * 5 + 0]);
        r1 = fmax(r1, partial[b * 5 + 1]);
        r2 = fmin(r2, partial[b * 5 + 2]);
        r3 = fmax(r3, partial[b * 5 + 3]);
        r4 += partial[b * 5 + 4];
    }
    r0 = bg_wave_min(r0);
    r1 = bg_wave_max(r1);
    r2 = bg_wave_min(r2);
    r3 = bg_wave_max(r3);
    for (int o = 32; o > 0; o >>= 1) r4 += __shfl_xor(r4, o, 64);
    const int w = threadIdx.x >> 6;
    if (__lane_id() == 0) {
        sm[w][0] = r0;
        sm[w][1] = r1;
        sm[w][2] = r2;
        sm[w][3] = r3;
        sm[w][4] = r4;
    }
    __syncthreads();  // (st zeroed by this workgroup before thread 0 writes it below)
    if (threadIdx.x == 0) {
        for (int k = 1; k < kBlock / 64; ++k) {
            sm[0][0] = fmin(sm[0][0], sm[k][0]);
            sm[0][1] = fmax(sm[0][1], sm[k][1]);
            sm[0][2] = fmin(sm[0][2], sm[k][2]);
            sm[0][3] = fmax(sm[0][3], sm[k][3]);
            sm[0][4] += sm[k][4];
        }
        double v[5];
        for (int c = 0; c < 5; ++c) v[c] = bb[c] = sm[0][c];
        grid_state(v, eps, gp, st);
    }
}

__device__ void grid_state(const double* bb, double eps, GridParams* __restrict__ gp,
                           int32_t* __restrict__ st) {
    GridParams g{0, 0, 1, 1, 1, 1, 1, 1, 0};
    const int nf = (int)bb[4];
    int bits = 0;
    if (nf > 0) {
        if (!make_grid(bb, eps, &g)) {
            st[kStError] = 1;
            g = GridParams{0, 0, 1, 1, 1, 1, 1, 1, 0};
        }
        const uint64_t nkeys = 256ull * g.ntx * g.nty;  // valid keys < nkeys <= 2^31
        bits = 1;
        while (bits < 32 && (1ull << bits) <= nkeys) ++bits;  // keys < 2^bits - 1 (sentinel)
    }
    *gp = g;
    st[kStNf] = nf;
    st[kStBits] = bits;
}

// Batched fits: the virtual grid planned on the host (plan_batch_grid).
__global__ void batch_grid_kernel(GridParams g, int32_t nf, int32_t bits,
                                  GridParams* __restrict__ gp, int32_t* __restrict__ st) {
    *gp = g;
    st[kStNf] = nf;
    st[kStBits] = bits;
}

// All-pairs (eps*eps = +inf: one cell holding every point) and no-pairs (eps*eps NaN) fits.
__global__ void grid_fixed_kernel(int32_t nf, GridParams* __restrict__ gp,
                                  int32_t* __restrict__ st) {
    *gp = GridParams{0, 0, 1, 1, 1, 1, 1, 1, 0};
    st[kStNf] = nf;
    st[kStBits] = 0;
}


// The cluster count of a fit into caller memory (asynchronous API).
__global__ void nclusters_kernel(const int32_t* __restrict__ st, int32_t* __restrict__ out) {
    *out = st[kStClusters];
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

// ---------------------------------------------------------------------------------------
// Host orchestration
// ---------------------------------------------------------------------------------------

// Waves per SIMD of the packed count_wave instance (count_tiny) and the staging capacity of
// count_tile32 (tiles over it take the big-tile path; 1024 / 1280 / 1792 measured slower).
static constexpr int kTinyWaves = 5;
constexpr int kCap32 = 1536;

// Archery float32 box, after the rank scan: the one-way core-core pairs decide which component
// a cluster's expansion claims beyond its own.  Usually there are none (returns nullptr: the
// cluster number is the component number).  Otherwise the sequential rule on the component
// graph: components in s order; an unclaimed one opens the next cluster, which then claims every
// unclaimed component reachable over one-way pairs (LocalDBSCANArchery.scala:45-63, 82-110).
// The only host synchronization of a fit, and only in this mode.
static const int32_t* resolve_box_pairs(hipStream_t s, Workspace& ws, int32_t* st,
                                        const int32_t* lab, const uint64_t* root_bits,
                                        const int32_t* word_rank, const double2* xy,
                                        const int32_t* cell, const Seg* seg,
                                        const int32_t* nf_p, int64_t n, double eps, double eps2,
                                        const uint8_t* core) {
    // what the buffer already holds (edges + ranks behind a 64-B count): ensure() must not grow it
    const int64_t held = ws.box_edges.bytes > 64
                             ? (int64_t)((ws.box_edges.bytes - 64) / (2 * sizeof(int2))) : 0;
    int64_t cap = std::max<int64_t>(kBoxEdgeCap, held);
    unsigned long long m = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        char* buf = static_cast<char*>(ws.box_edges.ensure(2 * cap * sizeof(int2) + 64));
        auto* cnt = reinterpret_cast<unsigned long long*>(buf);
        int2* edges = reinterpret_cast<int2*>(buf + 64);
        DBSCAN_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(*cnt), s));
        hipLaunchKernelGGL(box_pairs_kernel, dim3(std::min(nblk(n), 4096u)), dim3(kBlock), 0, s,
                           xy, cell, seg, nf_p, eps, eps2, core, lab, edges, cnt,
                           (unsigned long long)cap);
        DBSCAN_HIP_CHECK(hipGetLastError());
        DBSCAN_HIP_CHECK(hipMemcpyAsync(&m, cnt, sizeof(m), hipMemcpyDeviceToHost, s));
        DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
        if (m <= (unsigned long long)cap) break;
        if (m > (unsigned long long)INT32_MAX)
            throw ArgError{"archery float32 box: more than 2^31 one-way core pairs"};
        cap = (int64_t)m;  // one more pass records every pair (the count is exact)
    }
    int32_t hst[kStCount];
    DBSCAN_HIP_CHECK(hipMemcpyAsync(hst, st, sizeof(hst), hipMemcpyDeviceToHost, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    const int64_t k = hst[kStClusters];
    if (m == 0) return nullptr;
    char* buf = static_cast<char*>(ws.box_edges.p);
    int2* edges = reinterpret_cast<int2*>(buf + 64);
    int2* ranks = edges + cap;
    hipLaunchKernelGGL(box_edge_ranks_kernel, dim3(nblk((int64_t)m)), dim3(kBlock), 0, s, edges,
                       (int32_t)m, lab, root_bits, word_rank, ranks);
    DBSCAN_HIP_CHECK(hipGetLastError());
    std::vector<int2> e((size_t)m);
    DBSCAN_HIP_CHECK(hipMemcpyAsync(e.data(), ranks, m * sizeof(int2), hipMemcpyDeviceToHost, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    // CSR of the component graph (self pairs inside a component carry no information)
    std::vector<int32_t> head((size_t)k + 1, 0), adj;
    for (const int2& v : e)
        if (v.x != v.y) ++head[(size_t)v.x + 1];
    for (int64_t c = 0; c < k; ++c) head[(size_t)c + 1] += head[(size_t)c];
    adj.resize((size_t)head[(size_t)k]);
    {
        std::vector<int32_t> fill(head.begin(), head.end() - 1);
        for (const int2& v : e)
            if (v.x != v.y) adj[(size_t)fill[(size_t)v.x]++] = v.y;
    }
    std::vector<int32_t> cmap((size_t)k, 0), stack;
    int32_t next = 0;
    for (int64_t c = 0; c < k; ++c) {
        if (cmap[(size_t)c]) continue;
        cmap[(size_t)c] = ++next;
        stack.assign(1, (int32_t)c);
        while (!stack.empty()) {
            const int32_t u = stack.back();
            stack.pop_back();
            for (int32_t q = head[(size_t)u]; q < head[(size_t)u + 1]; ++q) {
                const int32_t w = adj[(size_t)q];
                if (!cmap[(size_t)w]) {
                    cmap[(size_t)w] = next;
                    stack.push_back(w);
                }
            }
        }
    }
    int32_t* d_map = static_cast<int32_t*>(ws.box_map.ensure((size_t)k * sizeof(int32_t) + 4));
    DBSCAN_HIP_CHECK(hipMemcpyAsync(d_map, cmap.data(), (size_t)k * sizeof(int32_t),
                                    hipMemcpyHostToDevice, s));
    DBSCAN_HIP_CHECK(hipMemcpyAsync(&st[kStClusters], &next, sizeof(int32_t),
                                    hipMemcpyHostToDevice, s));
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));  // (the host vectors go out of scope)
    return d_map;
}

// Enqueues one whole fit on stream s and never waits on the device: the grid, the finite count
// nf and every table size live in device memory (ws.misc), so launch sizes derive from n alone
// and kernels bound themselves by the device-side counts.  The grid is sized by grid_kernel
// from the device bbox (no host readback), the radix sort skips the key digits the grid does
// not use, and the clique (quarter-cell) and per-point union paths are both enqueued, each
// exiting at once when the grid selects the other.
// The handle's pinned stats block (the tiled pipeline's stats are copied there).
static void stats_block(Workspace& ws) {
    if (!ws.stats_host)
        DBSCAN_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ws.stats_host),
                                       kFitStatsDoubles * sizeof(double), hipHostMallocDefault));
}

// A stats block of the ring for one LDS fit (Workspace::ring_host), its kStError cleared by the
// host: the block belongs to this fit alone, and no earlier fit still queued can write it (a
// block is reused only after the stream has drained since it was taken: a full ring drains
// the stream and the queued fits' recalls first).  Returns the device address.
static double* take_stat_block(hipStream_t s, Profiler* prof, Workspace& ws) {
    if (!ws.ring_host) {
        DBSCAN_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&ws.ring_host),
                                       (size_t)Workspace::kStatRing * Workspace::kStatBlock *
                                           sizeof(double),
                                       hipHostMallocMapped | hipHostMallocCoherent));
        DBSCAN_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ws.ring_dev),
                                                 ws.ring_host, 0));
        ws.ring_next = ws.ring_used = 0;
    }
    if (ws.ring_used >= Workspace::kStatRing) {
        DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
        drain_recalls(s, prof, ws);  // (resets ring_used)
        ws.ring_used = 0;
    }
    const int k = ws.ring_next;
    ws.ring_next = (k + 1) % Workspace::kStatRing;
    ++ws.ring_used;
    double* host = ws.ring_host + (size_t)k * Workspace::kStatBlock;
    reinterpret_cast<int32_t*>(host + kMiscState)[kStError] = 0;
    ws.fit_block = host;
    return ws.ring_dev + (size_t)k * Workspace::kStatBlock;
}

void enqueue_fit(hipStream_t s, Workspace& ws, Profiler* prof, const FitArgs& a,
                 SlabState* slab) {
    // Which form: partition-sized full fits (the seam's usual call, DBSCAN.scala:150-155) take
    // one launch with everything in LDS (small.hip), one workgroup or several; larger ones the
    // tiled pipeline below.
    const bool lds_small = !a.zone && a.n > 0 && a.n <= std::min<int64_t>(a.small_max, kSmallMaxPoints) &&
                           small_fit_eligible(a.n, a.eps, a.mode);
    const bool lds_band = !lds_small && !a.zone && !a.batch && a.n > 0 &&
                          a.small_max >= kSmallMaxPoints && a.n <= a.band_max &&
                          band_fit_eligible(a.n, a.eps, a.mode, a.min_points);
    // Queued spread / band fits not yet checked are re-run (if they must be) in the tiled
    // pipeline's buffers: settled before a tiled fit uses those buffers (its slab state must
    // survive until the label phase).  (Mixing the forms on one handle without a sync is rare.)
    if (!lds_small && !lds_band && !ws.recalls.empty()) {
        DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
        drain_recalls(s, prof, ws);
    }
    if (slab) slab->valid = false;
    ws.fit_mirrored = false;
    ws.out_direct = false;
    ws.nk_written = false;
    const int64_t n = a.n;
    const double eps2 = a.eps * a.eps;  // LocalDBSCANNaive.scala:33
    const int mode =
        std::isnan(eps2) ? kGridNoPairs : (std::isinf(eps2) ? kGridAllPairs : kGridEps);
    ws.fit_n = n;
    ws.fit_mode = mode;
    double* misc = static_cast<double*>(ws.misc.ensure(64 * sizeof(double)));
    GridParams* gp = reinterpret_cast<GridParams*>(misc + kMiscGrid);
    int32_t* st = reinterpret_cast<int32_t*>(misc + kMiscState);
    if (n == 0) {
        DBSCAN_HIP_CHECK(hipMemsetAsync(st, 0, kStCount * sizeof(int32_t), s));
        if (slab) {
            slab->valid = a.zone != nullptr;
            slab->nlroots = -1;
            slab->n = 0;
        }
        return;
    }
    const int32_t* nf_p = &st[kStNf];
    if (lds_small || lds_band) {
        // (from band_min points the band form: its cooperative staging and quarter unions
        // measured faster than the spread form from ~3000 points (133 -> 121 us at 8192) in its
        // first form, from ~400 points since: 2000 / 600 points 77 / 64 us against 82 / 73)
        const bool band = lds_band || (n >= a.band_min && n <= a.band_max && !a.batch &&
                                       band_fit_eligible(n, a.eps, a.mode, a.min_points));
        const bool spread = !band && n >= a.spread_min;  // two grid barriers (spread_fit_kernel)
        StageTimer t(prof, s, band ? "band_fit" : "small_fit");
        // (LDS fits write their stats into a pinned block of their own: no copy back)
        double* mirror = take_stat_block(s, prof, ws);
        // (and their labels into pinned host buffers when the caller passes them: one launch,
        // no copy back; a re-run writes the device twins and copies them there in one DMA)
        ws.out_direct = a.cluster_host != nullptr;
        int32_t* const cl = ws.out_direct ? a.cluster_host : a.cluster;
        uint8_t* const fl = ws.out_direct ? a.flag_host : a.flag;
        if (band || spread) {  // a grid barrier may give up, a band overflow: a recall record
            Workspace::Recall r;
            r.band = band;
            r.x = a.x;
            r.y = a.y;
            r.n = n;
            r.eps = a.eps;
            r.min_points = a.min_points;
            r.mode = a.mode;
            r.cluster = cl;
            r.flag = fl;
            r.dev_cluster = ws.out_direct ? a.cluster : nullptr;
            r.dev_flag = ws.out_direct ? a.flag : nullptr;
            r.block_host = ws.fit_block;
            r.block_dev = mirror;
            ws.recalls.push_back(r);
        }
        if (band)
            enqueue_band_fit(s, prof, ws, a.x, a.y, n, a.eps, a.min_points, a.mode, cl, fl, gp,
                             st, mirror);
        else if (spread)
            enqueue_spread_fit(s, prof, ws, a.x, a.y, n, a.eps, a.min_points, a.mode, cl, fl, gp,
                               st, mirror);
        else
            enqueue_small_fits(s, prof, a.x, a.y, nullptr, nullptr, 1, n, a.eps, a.min_points,
                               a.mode, cl, fl, nullptr, gp, st, mirror);
        ws.fit_mirrored = true;
        return;
    }
    if (mode != kGridEps || a.batch)  // (eps grids of direct fits: bbox_grid_kernel zeroes it)
        DBSCAN_HIP_CHECK(hipMemsetAsync(st, 0, kStCount * sizeof(int32_t), s));

    // large direct fits sort through the padded bands (bucket_sort: cache-resident random writes)
    const bool bucketed = !a.batch && mode == kGridEps && n >= kBucketMinPoints &&
                          n + 256 * 2048 < (int64_t)INT32_MAX;
    uint32_t* key = static_cast<uint32_t*>(ws.key.ensure(n * sizeof(uint32_t)));
    uint32_t* key2 = static_cast<uint32_t*>(ws.key2.ensure(n * sizeof(uint32_t)));
    int32_t* inv = static_cast<int32_t*>(ws.inv.ensure(n * sizeof(int32_t)));
    int32_t* perm = static_cast<int32_t*>(ws.perm.ensure(n * sizeof(int32_t)));
    int32_t* perm2 = static_cast<int32_t*>(ws.perm2.ensure(n * sizeof(int32_t)));
    if (mode == kGridEps) {
        if (a.batch) {  // batched fits: the virtual grid of the partitions' local grids
            klaunch(prof, "grid", batch_grid_kernel, dim3(1), dim3(1), 0, s, a.batch->g,
                    a.batch->nf, a.batch->bits, gp, st);
            DBSCAN_HIP_CHECK(hipGetLastError());
        } else {
            StageTimer t(prof, s, "bbox");
            double* partial = nullptr;
            const int nbb = bbox_partials(s, a.x, a.y, n, ws.scan_tmp, &partial);
            // (the fit state zeroed here as well: no fill ahead of this path)
            klaunch(prof, "grid", bbox_grid_kernel, dim3(1), dim3(kBlock), 0, s,
                    (const double*)partial, nbb, misc, a.eps, gp, st);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        if (!bucketed) {  // (bucketed: the MSD pass bins x, y itself)
            StageTimer t(prof, s, "bin");
            klaunch(prof, "bin", bin_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, a.x, a.y, n, gp, key);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        if (bucketed) {  // large fits: MSD band split, then LSD inside the bands
            uint8_t* shm = nullptr;  // lean slab fits: the listed shared points, in slab order
            if (a.zone && a.shared_idx && a.n_shared > 0) {
                shm = static_cast<uint8_t*>(ws.shm.ensure(n));
                DBSCAN_HIP_CHECK(hipMemsetAsync(shm, 0, n, s));
                klaunch(prof, "shared_mark", shared_mark_kernel, dim3(nblk(a.n_shared)),
                        dim3(kBlock), 0, s, a.n_shared, a.shared_idx, shm);
            }
            bucket_sort(s, a.x, a.y, nullptr, n, &st[kStBits], ws.bucket,
                        ws.hist, ws.scan, prof, a.zone, shm, gp);
            key = ws.bucket.key_fin;  // (perm: written by scatter_bucket_kernel below)
        } else {
            uint32_t* key3 = static_cast<uint32_t*>(ws.key3.ensure(n * sizeof(uint32_t)));
            int32_t* perm3 = static_cast<int32_t*>(ws.perm3.ensure(n * sizeof(int32_t)));
            radix_sort_pairs(s, key, perm, key2, perm2, key3, perm3, n, &st[kStBits], ws.hist,
                             ws.scan, prof, inv, /*iota=*/true);
        }
    } else {
        StageTimer t(prof, s, "bin");
        // all pairs: one cell holding every point, the predicate decides (incl. non-finite)
        klaunch(prof, "grid_fixed", grid_fixed_kernel, dim3(1), dim3(1), 0, s,
                           mode == kGridAllPairs ? (int32_t)n : 0, gp, st);
        klaunch(prof, "iota_key", iota_key_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n,
                           mode == kGridAllPairs ? 0u : kSentinelKey, key, perm);
        DBSCAN_HIP_CHECK(hipGetLastError());
    }
    ws.perm_sorted = perm;
    ws.key_sorted = key;
    // direct fits: the root bits (quarter_root / final), zeroed by heads_down on eps grids
    uint64_t* root_words =
        (!a.zone && mode != kGridNoPairs)
            ? static_cast<uint64_t*>(ws.is_root.ensure(((n + 63) / 64) * sizeof(uint64_t)))
            : nullptr;

    // Sizes: every nf-sized table is allocated for n; the tile grid holds <= 2^23 tiles.
    const int64_t ntile_bound = std::min<int64_t>(n, kMaxGridTiles);
    double2* xy = static_cast<double2*>(ws.xy.ensure(n * sizeof(double2)));
    int32_t* cell = static_cast<int32_t*>(ws.cell.ensure(n * sizeof(int32_t)));
    uint32_t* ckey = static_cast<uint32_t*>(ws.ckey.ensure(n * sizeof(uint32_t)));
    int32_t* cstart = static_cast<int32_t*>(ws.cstart.ensure((n + 1) * sizeof(int32_t)));
    Seg* seg = static_cast<Seg*>(ws.seg.ensure(n * sizeof(Seg)));
    uint32_t* tkey = static_cast<uint32_t*>(ws.tkey.ensure(n * sizeof(uint32_t)));
    int32_t* tstart = static_cast<int32_t*>(ws.tstart.ensure((n + 1) * sizeof(int32_t)));
    int32_t* tmap = static_cast<int32_t*>(ws.tmap.ensure(kMaxGridTiles * sizeof(int32_t)));
    int32_t* tslot =
        static_cast<int32_t*>(ws.tslot.ensure((size_t)ntile_bound * kTslot * sizeof(int32_t)));
    int2* tstage = static_cast<int2*>(ws.tstage.ensure((size_t)ntile_bound * 100 * sizeof(int2)));
    // (+4: big_union reads a quarter's first core flags as whole 4-B words)
    uint8_t* core = static_cast<uint8_t*>(ws.core.ensure(n + 4));
    int32_t* parent = static_cast<int32_t*>(ws.parent.ensure(n * sizeof(int32_t)));
    int32_t* lab = static_cast<int32_t*>(ws.lab.ensure(n * sizeof(int32_t)));
    int32_t* tq = static_cast<int32_t*>(ws.tq.ensure((size_t)ntile_bound * kTslot * sizeof(int32_t)));
    int4* tnb = static_cast<int4*>(ws.tnb.ensure((size_t)ntile_bound * sizeof(int4)));
    int32_t* qcomp = static_cast<int32_t*>(ws.qcomp.ensure(n * sizeof(int32_t)));
    int32_t* qidx = static_cast<int32_t*>(ws.qidx.ensure(n * sizeof(int32_t)));
    uint32_t* qkey = static_cast<uint32_t*>(ws.qkey.ensure(n * sizeof(uint32_t)));
    int32_t* qstart = static_cast<int32_t*>(ws.qstart.ensure((n + 1) * sizeof(int32_t)));
    int4* qinfo = static_cast<int4*>(ws.qrep.ensure(n * sizeof(int4)));
    int4* qg = static_cast<int4*>(ws.qmask.ensure(n * sizeof(int4)));
    // the tile-local quarter union runs inside the count kernels (slab fits: the fp32 count
    // kernels, which read the sorted zones; the fp64 fused kernel would union zone-2 points)
    // archery's float32 search box (mode 2): its own count / union / label kernels over the
    // global stencil pieces; none of the clique-quarter or fp32-record paths
    const bool box = a.mode == kModeArcheryBox;
    const bool fuse = !box && mode == kGridEps;
    uint8_t* zs =
        (a.zone && (fuse || bucketed)) ? static_cast<uint8_t*>(ws.zs.ensure(n)) : nullptr;
    // eps grids: the fp32-record count kernels by tile class (tile_class_kernel) when the
    // grid's quarter cells are cliques, count_tile_kernel (fp64) when not
    const bool f32 = fuse;
    const int nbr_k =
        (!box && a.min_points >= 2 && a.min_points - 1 <= kMaxNbr) ? a.min_points - 1 : 0;
    TileLists tl{};
    uint8_t* tclass = nullptr;
    uint8_t* tcore = nullptr;  // f32: per tile, its edge strips hold cores (count kernels)
    if (f32) {
        int32_t* lists = static_cast<int32_t*>(
            ws.bigt.ensure((1 + kSmallBuckets + kMedBuckets) * ntile_bound * sizeof(int32_t)));
        tl = TileLists{&st[kStTileLists],
                       lists + ntile_bound,
                       lists + (1 + kSmallBuckets) * ntile_bound,
                       lists,
                       &st[kStTileBuckets],
                       &st[kStTileBuckets + kSmallBuckets],
                       (int32_t)ntile_bound};
        tclass = static_cast<uint8_t*>(ws.tclass.ensure(ntile_bound));
        tcore = static_cast<uint8_t*>(ws.tcore.ensure(ntile_bound));
    }
    int32_t* tsz = static_cast<int32_t*>(ws.tsz.ensure(ntile_bound * sizeof(int32_t)));
    int32_t* tpart =
        a.batch ? static_cast<int32_t*>(ws.tpart.ensure(ntile_bound * sizeof(int32_t))) : nullptr;

    {
        StageTimer t(prof, s, "gather");
        if (mode != kGridEps)  // (eps grids: the radix sort's final pass wrote inv)
            klaunch(prof, "inverse", inverse_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n, perm,
                    inv);
        if (bucketed)  // (slab fits: zs from the records, inv only for the shared points)
            klaunch(prof, "gather_bucket", gather_bucket_kernel,
                    dim3(nblk(n)), dim3(kBlock), 0, s,
                    n, (const int32_t*)ws.bucket.slot_place, (const double4*)ws.bucket.rec, nf_p,
                    perm, xy, zs, (a.zone && a.shared_idx) ? inv : (int32_t*)nullptr);
        else if (mode != kGridNoPairs)
            klaunch(prof, "scatter_xy", scatter_xy_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, a.x, a.y, n,
                               nf_p, inv, xy);
        if (zs && !bucketed) {
            DBSCAN_HIP_CHECK(hipMemsetAsync(zs, 0, n, s));
            klaunch(prof, "zone_mark", zone_mark_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n,
                    a.zone, inv, zs);
        }
        DBSCAN_HIP_CHECK(hipGetLastError());
    }
    if (mode != kGridNoPairs) {
        {
            StageTimer t(prof, s, "cells");
            const int nb = (int)((n + kHeadTile - 1) / kHeadTile);
            int32_t* part =
                static_cast<int32_t*>(ws.heads.ensure(6 * (size_t)nb * sizeof(int32_t)));
            int32_t* offs = part + 3 * nb;
            klaunch(prof, "heads_reduce", heads_reduce_kernel, dim3(nb), dim3(kBlock), 0, s, key, nf_p, nb,
                    part, (const GridParams*)gp, tmap);
            DBSCAN_HIP_CHECK(hipGetLastError());
            if (nb <= 4096) {  // (n <= 2^24: the three head counts in one launch)
                scan3(s, part, nb, nb, offs, &st[kStCells], &st[kStQuarters], &st[kStTiles]);
            } else {
                exclusive_scan(s, 0, part, offs, nb, &st[kStCells], ws.scan);
                exclusive_scan(s, 0, part + nb, offs + nb, nb, &st[kStQuarters], ws.scan);
                exclusive_scan(s, 0, part + 2 * nb, offs + 2 * nb, nb, &st[kStTiles], ws.scan);
            }
            klaunch(prof, "heads_down", heads_down_kernel, dim3(nb), dim3(kBlock), 0, s, key, nf_p, nb,
                    offs, cell, ckey, cstart, qidx, qkey, qstart, tkey, tstart, root_words,
                    root_words ? (n + 63) / 64 : (int64_t)0);
            DBSCAN_HIP_CHECK(hipGetLastError());
            if (tpart)
                klaunch(prof, "tile_part", tile_part_kernel, dim3(nblk(ntile_bound)),
                        dim3(kBlock), 0, s, tstart, &st[kStTiles], perm, gp, tpart);
        }
        {
            StageTimer t(prof, s, "tables");
            const unsigned tgrid = (unsigned)std::min<int64_t>(nblk(ntile_bound), 1024);
            klaunch(prof, "tmap", tmap_kernel, dim3(tgrid), dim3(kBlock), 0, s, tkey,
                               &st[kStTiles], tmap);
            DBSCAN_HIP_CHECK(hipGetLastError());
            const dim3 tsgrid((unsigned)std::min<int64_t>((ntile_bound + 3) / 4, kTileGrid));
            if (n >= kTslotMultiPoints)
                klaunch(prof, "tslot", tslot_multi_kernel, tsgrid, dim3(kBlock), 0, s, tstart, tkey,
                        &st[kStTiles], cell, ckey, cstart, &st[kStCells], qidx, tslot, tq);
            else
                klaunch(prof, "tslot", tslot_kernel, tsgrid, dim3(kBlock), 0, s, tstart, tkey,
                        &st[kStTiles], cell, ckey, cstart, &st[kStCells], qidx, tslot, tq);
            DBSCAN_HIP_CHECK(hipGetLastError());
            klaunch(prof, "tstage", thalo_kernel,
                    dim3((unsigned)std::min<int64_t>(
                        (ntile_bound + kHaloTiles * kHaloU - 1) / (kHaloTiles * kHaloU), kTileGrid)),
                    dim3(kBlock), 0, s, tkey, &st[kStTiles], tmap, tslot, gp, tstage, tsz, tnb);
            DBSCAN_HIP_CHECK(hipGetLastError());
            if (f32)  // clique grids: small / medium / big tile lists
                klaunch(prof, "tile_class", tile_class_kernel<kCap32>,
                        dim3((unsigned)std::min<int64_t>(
                            (ntile_bound + kBlock * kClassRounds - 1) / (kBlock * kClassRounds),
                            1024)),
                        dim3(kBlock), 0, s, tsz, tstart, &st[kStTiles], gp, tl, tclass,
                        &st[kStClassPts], tcore);
        }
        {
            StageTimer t(prof, s, "segs");
            klaunch(prof, "segs", segs_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, ckey, cstart,
                               &st[kStCells], tmap, tslot, gp, seg,
                               (f32 && nbr_k > 0) ? (const uint8_t*)tclass : nullptr);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
    }
    // per-tile kernels: grid stride over occupied tiles (their count stays on the device)
    const unsigned tile_grid = (unsigned)std::min<int64_t>(ntile_bound, kTileGrid);
    // slots [nf, n): outside the grid (usually none: a small grid, since every block's count
    // enters the core scan)
    const unsigned rest_grid = std::min(nblk(n), 256u);
    // per-block core counts: (f32: count32 | big_count |) count (| f32: count_wave) |
    // count_rest, then their scan
    int32_t* block_cores = static_cast<int32_t*>(
        ws.blockcnt.ensure(2 * ((size_t)(2 + 4 / DBSCAN_AB_BIGC_WAVES + 8 / DBSCAN_AB_CW_WAVES) *
                                    tile_grid + rest_grid + 1) * sizeof(int32_t)));
    int32_t* nbr = nbr_k > 0
                       ? static_cast<int32_t*>(ws.nbr.ensure((size_t)n * nbr_k * sizeof(int32_t)))
                       : nullptr;
    // per-block core counts: count32 [0, G), big_count [G, G + BG), count (fp64) [G + BG,
    // 2G + BG), count_wave and count_tiny CG each after it; G = tile_grid, BG and CG the grids of
    // the kernels whose workgroups are smaller than kBlock
    const int64_t big_grid = (int64_t)tile_grid * (4 / DBSCAN_AB_BIGC_WAVES);
    const int64_t cw_grid = (int64_t)tile_grid * (4 / DBSCAN_AB_CW_WAVES);  // count_wave, _tiny
    const int64_t nmain =
        f32 ? 2 * (int64_t)tile_grid + big_grid + 2 * cw_grid : (int64_t)tile_grid;
    bool rest_done = false;  // count_rest's blocks ran inside the fp64 count launch
    {
        StageTimer t(prof, s, "count");
        if (mode != kGridNoPairs) {
            const FuseArgs fa{tq, qstart, qkey, perm, tkey, gp, tl, zs, qinfo, qg, qcomp, tcore,
                              tpart};
            if (box) {
                klaunch(prof, "box_count", box_count_kernel, dim3(tile_grid), dim3(kBlock), 0, s,
                        xy, cell, seg, nf_p, a.eps, eps2, a.min_points, core, parent,
                        block_cores);
            } else if (f32) {
                // clique grids by tile stage size: small tiles one wave each (count_wave: 64
                // lanes per tile over kTinyCap points; count_tiny: tiles packed 2 to a wave),
                // medium one workgroup each (count32), big from global memory (big_count +
                // big_union); other eps grids: count (fp64, exits at once on clique grids)
                int32_t* bc = block_cores + 2 * tile_grid + big_grid;
                constexpr int CW = DBSCAN_AB_CW_WAVES;
                klaunch(prof, "count_wave",
                        count_wave_kernel<5, 64, kSmallCap, 0, kTinyBucket0, CW>,
                        dim3((unsigned)cw_grid), dim3(64 * CW), 0, s, xy, tstart, tstage, eps2,
                        a.min_points, core, parent, bc, nbr, nbr_k, fa);
                klaunch(prof, "count_tiny",
                        count_wave_kernel<kTinyWaves, 32, kTinyCap, kTinyBucket0,
                                          kSmallBuckets - kTinyBucket0, CW>,
                        dim3((unsigned)cw_grid), dim3(64 * CW), 0, s, xy, tstart, tstage, eps2,
                        a.min_points, core, parent, bc + cw_grid, nbr, nbr_k, fa);
                klaunch(prof, "count32", count_tile32_kernel<kCap32, 6>, dim3(tile_grid),
                        dim3(kBlock), 0, s, xy, tstart, tstage, &st[kStTiles], eps2,
                        a.min_points, core, parent, block_cores, nbr, nbr_k, fa);
                klaunch(prof, "big_count", big_count_kernel<DBSCAN_AB_BIGC_W, DBSCAN_AB_BIGC_WAVES>,
                        dim3((unsigned)big_grid), dim3(64 * DBSCAN_AB_BIGC_WAVES), 0,
                        s, xy, cell, seg, tstart, qidx, eps2, a.min_points, core,
                        block_cores + tile_grid, nbr, nbr_k, fa);
                // one workgroup per big tile up to kTileGrid (a grid of 2048 gave the tiles past
                // it a second serial turn)
                klaunch(prof, "big_union", big_union_kernel, dim3(tile_grid), dim3(kBlock), 0, s, xy,
                        (const uint8_t*)core, eps2, parent, fa);
                klaunch(prof, "count", count_tile_kernel<1536, 5>, dim3(tile_grid + rest_grid),
                        dim3(kBlock), 0, s, xy, cell, seg, tstart, tstage, &st[kStTiles], eps2,
                        a.min_points, core, parent, block_cores + tile_grid + big_grid, nbr, nbr_k,
                        (const GridParams*)gp, (int)tile_grid, nf_p, n, block_cores + nmain);
                rest_done = true;
            } else {
                klaunch(prof, "count", count_tile_kernel<1536, 5>, dim3(tile_grid + rest_grid),
                        dim3(kBlock), 0, s, xy, cell, seg, tstart, tstage, &st[kStTiles], eps2,
                        a.min_points, core, parent, block_cores, nbr, nbr_k, (const GridParams*)gp,
                        (int)tile_grid, nf_p, n, block_cores + nmain);
                rest_done = true;
            }
        } else {
            DBSCAN_HIP_CHECK(hipMemsetAsync(block_cores, 0, tile_grid * sizeof(int32_t), s));
        }
        if (!rest_done)
            klaunch(prof, "count_rest", count_rest_kernel, dim3(rest_grid), dim3(kBlock), 0, s,
                    nf_p, n, a.min_points, core, parent, block_cores + nmain);
        DBSCAN_HIP_CHECK(hipGetLastError());
        const int64_t nb = nmain + rest_grid;
        exclusive_scan(s, 0, block_cores, block_cores + nb + 1, nb, &st[kStCore], ws.scan);
        if (a.zone && bucketed)  // (the core count above then includes zone-2 points: a statistic)
            klaunch(prof, "zone_fix", zone_fix_sorted_kernel, dim3(nblk(n)), dim3(kBlock), 0, s,
                    n, (const uint8_t*)zs, core);
        else if (a.zone)
            klaunch(prof, "zone_fix", zone_fix_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n, a.zone, inv,
                               core);
    }
    // direct fits with fused quarter unions: quarter_root_kernel flags the roots (root bits)
    uint64_t* qlab_bits =
        (!a.zone && fuse)
            ? static_cast<uint64_t*>(ws.is_root.ensure(((n + 63) / 64) * sizeof(uint64_t)))
            : nullptr;
    if (fuse) {  // quarter-cell unions across tiles (no-ops unless the grid made them cliques)
        {
            StageTimer t(prof, s, "union_edge");
            // (+ union_kernel's blocks: a no-op on clique grids, the only union on the others)
            constexpr int EW = DBSCAN_AB_EDGE_WAVES;
            const unsigned ug = std::min(nblk(n), 2048u) * (kBlock / (64 * EW));
            const unsigned eg = tile_grid * (kBlock / (64 * EW));  // (the same waves in all)
            klaunch(prof, "edge_union", edge_union_kernel<DBSCAN_AB_EDGE_W, EW>, dim3(eg + ug),
                    dim3(64 * EW), 0, s, xy, &st[kStTiles], tq, tnb, qinfo, qg, qcomp, eps2, perm,
                    core, parent, gp, (const uint8_t*)tcore, (int)eg, cell, seg, nf_p);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        StageTimer t(prof, s, "union_root");
        // direct fits (fused quarter unions): the roots' visit indices per quarter (into the
        // dead qcomp) and the root flags, for final_kernel
        // (qlab_bits: zeroed by heads_down)
        klaunch(prof, "quarter_root", quarter_root_kernel,
                dim3((unsigned)((n + kQrootPer * kBlock - 1) / (kQrootPer * kBlock))), dim3(kBlock), 0, s, qinfo,
                &st[kStQuarters], gp, parent, perm, qlab_bits ? qcomp : (int32_t*)nullptr,
                reinterpret_cast<unsigned long long*>(qlab_bits));
        DBSCAN_HIP_CHECK(hipGetLastError());
    }
    if (mode != kGridNoPairs && !fuse) {  // per-point union (fuse: inside the edge_union launch)
        StageTimer t(prof, s, "union");
        if (box) {
            klaunch(prof, "box_union", box_union_kernel, dim3(std::min(nblk(n), 4096u)),
                    dim3(kBlock), 0, s, xy, cell, seg, nf_p, a.eps, eps2, perm, core, parent);
        } else {
            // (a no-op on clique grids: a grid that just fills the GPU once)
            klaunch(prof, "union", union_kernel, dim3(std::min(nblk(n), 2048u)), dim3(kBlock), 0,
                    s, xy, cell, seg, nf_p, gp, eps2, perm, core, parent);
        }
        DBSCAN_HIP_CHECK(hipGetLastError());
    }
    if (!a.zone) {
        const int64_t nw = (n + 63) / 64;
        uint64_t* root_bits = static_cast<uint64_t*>(ws.is_root.ensure(nw * sizeof(uint64_t)));
        int32_t* word_rank = static_cast<int32_t*>(ws.rank.ensure(nw * sizeof(int32_t)));
        {
            StageTimer t(prof, s, "final");
            if (!root_words)  // (eps grids: zeroed by heads_down)
                DBSCAN_HIP_CHECK(hipMemsetAsync(root_bits, 0, nw * sizeof(uint64_t), s));
            klaunch(prof, "final", final_kernel, dim3(nblk((n + kFinalPer - 1) / kFinalPer)), dim3(kBlock), 0, s, n, nf_p, gp, perm, core,
                               parent, fuse ? qidx : nullptr, qinfo, lab,
                               reinterpret_cast<unsigned long long*>(root_bits), (int32_t*)nullptr,
                               qlab_bits ? (const int32_t*)qcomp : (const int32_t*)nullptr);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        {
            StageTimer t(prof, s, "rank");
            exclusive_scan(s, 2, root_bits, word_rank, nw, &st[kStClusters], ws.scan);
        }
        if (box) {
            StageTimer t(prof, s, "output");
            const int32_t* cmap = resolve_box_pairs(s, ws, st, lab, root_bits, word_rank, xy,
                                                    cell, seg, nf_p, n, a.eps, eps2, core);
            uint32_t* packed = static_cast<uint32_t*>(
                ws.packed.ensure((bucketed ? ws.bucket.np : n) * sizeof(uint32_t)));
            klaunch(prof, "box_label", box_label_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, xy,
                    cell, seg, nf_p, n, a.eps, eps2, core, lab, root_bits, word_rank, cmap,
                    packed, bucketed ? (const int32_t*)ws.bucket.slot_place : nullptr);
            if (bucketed)
                klaunch(prof, "permute_out", permute_out_bucket_kernel,
                        dim3((unsigned)((n + kPermPer * kBlock - 1) / (kPermPer * kBlock))), dim3(kBlock),
                        0, s, n, (const int32_t*)ws.bucket.pos, (const uint32_t*)packed, a.cluster,
                        a.flag, (const int32_t*)&st[kStClusters], a.n_clusters_dev);
            else
                klaunch(prof, "permute_out", permute_out_kernel<false>, dim3(nblk(n)), dim3(kBlock),
                        0, s, n, inv, packed, (const uint8_t*)nullptr, a.cluster, a.flag,
                        (const int32_t*)&st[kStClusters], a.n_clusters_dev);
            DBSCAN_HIP_CHECK(hipGetLastError());
            ws.nk_written = a.n_clusters_dev != nullptr;
        } else {
            StageTimer t(prof, s, "output");
            uint32_t* packed = static_cast<uint32_t*>(
                ws.packed.ensure((bucketed ? ws.bucket.np : n) * sizeof(uint32_t)));
            klaunch(prof, "label_sorted", label_sorted_kernel<false>, dim3(nblk(n)), dim3(kBlock), 0, s, xy,
                               cell, seg, nbr, nbr_k, nf_p, n, eps2, a.mode, perm, core, lab,
                               root_bits, word_rank, (const uint8_t*)nullptr, (const int64_t*)nullptr,
                               (const int64_t*)nullptr, (const int32_t*)nullptr, packed,
                               bucketed ? (const int32_t*)ws.bucket.slot_place : nullptr);
            if (a.batch) {  // cluster ids per partition, and each partition's count
                const GridParams& bg = a.batch->g;
                klaunch(prof, "permute_out", permute_out_batch_kernel, dim3(nblk(n)), dim3(kBlock),
                        0, s, n, inv, packed, bg.poffs, bg.nparts, (const uint64_t*)root_bits,
                        (const int32_t*)word_rank, a.cluster, a.flag);
                klaunch(prof, "batch_nclusters", batch_nclusters_kernel,
                        dim3(nblk(bg.nparts)), dim3(kBlock), 0, s, n, bg.poffs, bg.nparts,
                        (const uint64_t*)root_bits, (const int32_t*)word_rank,
                        (const int32_t*)st, a.batch->nclusters);
            } else if (bucketed) {
                klaunch(prof, "permute_out", permute_out_bucket_kernel,
                        dim3((unsigned)((n + kPermPer * kBlock - 1) / (kPermPer * kBlock))), dim3(kBlock),
                        0, s, n, (const int32_t*)ws.bucket.pos, (const uint32_t*)packed, a.cluster,
                        a.flag, (const int32_t*)&st[kStClusters], a.n_clusters_dev);
            } else {
                klaunch(prof, "permute_out", permute_out_kernel<false>, dim3(nblk(n)), dim3(kBlock),
                        0, s, n, inv, packed, (const uint8_t*)nullptr, a.cluster, a.flag,
                        (const int32_t*)&st[kStClusters], a.n_clusters_dev);
            }
            DBSCAN_HIP_CHECK(hipGetLastError());
            ws.nk_written = a.n_clusters_dev != nullptr && !a.batch;
        }
    } else {
        {
            StageTimer t(prof, s, "final");
            const bool lean = a.shared_idx != nullptr;
            if (lean) DBSCAN_HIP_CHECK(hipMemsetAsync(a.root_out, 0xFF, n * sizeof(int32_t), s));
            klaunch(prof, "final", final_kernel, dim3(nblk((n + kFinalPer - 1) / kFinalPer)), dim3(kBlock), 0, s, n, nf_p, gp, perm, core,
                               parent, fuse ? qidx : nullptr, qinfo, lab,
                               (unsigned long long*)nullptr, lean ? a.root_out : (int32_t*)nullptr,
                               (const int32_t*)nullptr);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        {
            StageTimer t(prof, s, "output");
            if (a.shared_idx) {
                if (a.n_shared > 0)
                    klaunch(prof, "slab_shared", slab_shared_kernel, dim3(nblk(a.n_shared)),
                            dim3(kBlock), 0, s, a.n_shared, a.shared_idx, inv, core, lab,
                            a.core_out, a.root_out);
            } else {  // (bucketed sort: packed at the slots' places, read back through pos)
                int32_t* packed = static_cast<int32_t*>(
                    ws.packed.ensure((bucketed ? ws.bucket.np : n) * sizeof(int32_t)));
                klaunch(prof, "slab_pack", slab_pack_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n,
                        core, lab, packed,
                        bucketed ? (const int32_t*)ws.bucket.slot_place : nullptr);
                klaunch(prof, "slab_roots", slab_roots_kernel, dim3(nblk(n)), dim3(kBlock), 0, s,
                        n, bucketed ? (const int32_t*)ws.bucket.pos : (const int32_t*)inv,
                        (const int32_t*)packed, a.core_out, a.root_out);
            }
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
    }
    if (slab) {
        slab->valid = a.zone != nullptr;
        slab->nlroots = -1;
        slab->n = n;
        slab->eps2 = eps2;
        slab->to_packed = bucketed ? ws.bucket.pos : inv;
        slab->place = bucketed ? ws.bucket.slot_place : nullptr;
        slab->npacked = bucketed ? ws.bucket.np : n;
        slab->nbr = nbr;
        slab->nbr_k = nbr_k;
    }
}

#if DBSCAN_AB_COUNTDIV
extern "C" int dbscan_ab_countdiv(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_div), 8 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_div), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

#if DBSCAN_AB_CHECK
// checking builds: per site {count, lowest, highest} out-of-range indices since the last read
extern "C" int dbscan_ab_bounds(long long* out) {
    unsigned long long bad[kChkSites];
    long long lo[kChkSites], hi[kChkSites];
    if (hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_chk_bad), sizeof(bad)) != hipSuccess ||
        hipMemcpyFromSymbol(lo, HIP_SYMBOL(g_chk_lo), sizeof(lo)) != hipSuccess ||
        hipMemcpyFromSymbol(hi, HIP_SYMBOL(g_chk_hi), sizeof(hi)) != hipSuccess)
        return -1;
    for (int k = 0; k < kChkSites; ++k) {
        out[3 * k] = (long long)bad[k];
        out[3 * k + 1] = bad[k] ? lo[k] : 0;
        out[3 * k + 2] = bad[k] ? hi[k] : 0;
        bad[k] = 0;
        lo[k] = INT64_MAX;
        hi[k] = INT64_MIN;
    }
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_chk_bad), bad, sizeof(bad)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_chk_lo), lo, sizeof(lo)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_chk_hi), hi, sizeof(hi)) != hipSuccess)
        return -1;
    return kChkSites;
}
#endif

void write_nclusters(hipStream_t s, Workspace& ws, int32_t* d_out) {
    if (ws.nk_written) return;  // (the fit's output kernel wrote it: FitArgs::n_clusters_dev)
    if (ws.fit_n == 0) {
        DBSCAN_HIP_CHECK(hipMemsetAsync(d_out, 0, sizeof(int32_t), s));
        return;
    }
    const int32_t* st = reinterpret_cast<const int32_t*>(static_cast<double*>(ws.misc.p) + kMiscState);
    hipLaunchKernelGGL(nclusters_kernel, dim3(1), dim3(1), 0, s, st, d_out);
    DBSCAN_HIP_CHECK(hipGetLastError());
    // (a re-run of this fit rewrites the word: drain_recalls)
    if (ws.fit_mirrored && !ws.recalls.empty() && ws.recalls.back().block_host == ws.fit_block)
        ws.recalls.back().nk = d_out;
}

void enqueue_fit_stats_copy(hipStream_t s, Workspace& ws, double* dst) {
    if (ws.fit_n == 0 || ws.fit_mirrored) return;  // (mirrored: parse reads the fit's block)
    DBSCAN_HIP_CHECK(
        hipMemcpyAsync(dst, ws.misc.p, kFitStatsDoubles * sizeof(double), hipMemcpyDeviceToHost, s));
}

bool drain_recalls(hipStream_t s, Profiler* prof, Workspace& ws) {
    ws.ring_used = 0;  // (the stream has drained: every block taken so far is free)
    if (ws.recalls.empty()) return false;
    std::vector<Workspace::Recall> list;
    list.swap(ws.recalls);
    // the last fit's state (a re-run below enqueues fits of its own)
    const int64_t fit_n = ws.fit_n;
    const int fit_mode = ws.fit_mode;
    const bool mirrored = ws.fit_mirrored, direct = ws.out_direct;
    double* const block = ws.fit_block;
    bool last = false, any = false;
    int32_t* const st = reinterpret_cast<int32_t*>(static_cast<double*>(ws.misc.p) + kMiscState);
    GridParams* const gp = reinterpret_cast<GridParams*>(static_cast<double*>(ws.misc.p) + kMiscGrid);
    for (const Workspace::Recall& r : list) {
        const int32_t e = reinterpret_cast<const int32_t*>(r.block_host + kMiscState)[kStError];
        if (!(e == 2 || (r.band && e == 3))) continue;
        any = true;
        int32_t* cl = r.dev_cluster ? r.dev_cluster : r.cluster;
        uint8_t* fl = r.dev_cluster ? r.dev_flag : r.flag;
        if (r.band) {  // the tiled pipeline (no LDS fit, no band fit); its stats to the block
            FitArgs b{r.x, r.y, nullptr, r.n, r.eps, r.min_points, r.mode, cl, fl, nullptr,
                      nullptr};
            b.small_max = 0;
            enqueue_fit(s, ws, prof, b, nullptr);
            enqueue_fit_stats_copy(s, ws, r.block_host);
        } else {  // the one-workgroup kernel: no grid barrier, every label and statistic
            enqueue_small_fits(s, prof, r.x, r.y, nullptr, nullptr, 1, r.n, r.eps, r.min_points,
                               r.mode, cl, fl, nullptr, gp, st, r.block_dev);
        }
        if (r.dev_cluster) {  // direct fits: the labels to the caller's pinned block, one DMA each
            DBSCAN_HIP_CHECK(hipMemcpyAsync(r.cluster, cl, (size_t)r.n * sizeof(int32_t),
                                            hipMemcpyDeviceToDevice, s));
            DBSCAN_HIP_CHECK(hipMemcpyAsync(r.flag, fl, (size_t)r.n, hipMemcpyDeviceToDevice, s));
        }
        if (r.nk) {
            hipLaunchKernelGGL(nclusters_kernel, dim3(1), dim3(1), 0, s, st, r.nk);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        ++ws.spread_fallbacks;
        if (r.block_host == block) last = true;
    }
    if (any) {
        // (a barrier that gave up left the band scratch to its last workgroup's cleanup; zeroed
        // again ahead of the next band fit all the same)
        ws.band_ready = false;
        DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    }
    ws.fit_n = fit_n;
    ws.fit_mode = fit_mode;
    ws.fit_mirrored = mirrored;
    ws.out_direct = direct;
    ws.fit_block = block;
    ws.ring_used = 0;
    return last;
}

FitStats read_fit_stats(hipStream_t s, Workspace& ws, Profiler* prof) {
    stats_block(ws);  // (pinned: a pageable copy costs a staging pass per fit)
    enqueue_fit_stats_copy(s, ws, ws.stats_host);
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    // queued spread / band fits whose workgroups were not all resident (or whose band
    // overflowed): re-run, each into its own outputs
    ws.spread_recovered = drain_recalls(s, prof, ws);
    return parse_fit_stats(ws, ws.stats_host);
}

FitStats parse_fit_stats(const Workspace& ws, const double* buf) {
    if (ws.fit_mirrored) buf = ws.fit_block;  // (an LDS fit wrote it; no copy was made)
    FitStats stats;
    stats.n = ws.fit_n;
    stats.grid_mode = ws.fit_mode;
    if (ws.fit_n == 0) return stats;
    GridParams g;
    memcpy(&g, buf + kMiscGrid, sizeof(g));
    int32_t v[kStTileBuckets];  // (the stats copy holds the states before the buckets)
    memcpy(v, buf + kMiscState, sizeof(v));
    if (v[kStError] == 2)  // (spread_fit_kernel: its workgroups were not all resident)
        throw HipError(hipErrorLaunchTimeOut, "spread_fit_kernel grid barrier (workgroups not resident)",
                       __FILE__, __LINE__);
    if (v[kStError]) throw ArgError{"cannot size the eps grid"};
    stats.nf = v[kStNf];
    if (ws.fit_mode == kGridEps && stats.nf == 0) stats.grid_mode = kGridNoPairs;
    const bool grid = stats.nf > 0 && ws.fit_mode != kGridNoPairs;
    stats.nx = grid ? g.nx : 0;
    stats.ny = grid ? g.ny : 0;
    stats.clique = grid ? g.clique : 0;
    stats.bits = v[kStBits];
    stats.ncells = grid ? v[kStCells] : 0;
    stats.ntiles = grid ? v[kStTiles] : 0;
    stats.ncore = v[kStCore];
    stats.nclusters = v[kStClusters];
    stats.pts_small = grid ? v[kStClassPts] : 0;
    stats.pts_medium = grid ? v[kStClassPts + 1] : 0;
    stats.pts_big = grid ? v[kStClassPts + 2] : 0;
    return stats;
}

int64_t run_fit(hipStream_t s, Workspace& ws, Profiler* prof, const FitArgs& a, FitStats* st,
                SlabState* slab) {
    enqueue_fit(s, ws, prof, a, slab);
    const FitStats stats = read_fit_stats(s, ws, prof);
    if (slab) slab->nf = stats.nf;
    if (st) *st = stats;
    return a.zone ? 0 : stats.nclusters;
}

void run_slab_label(hipStream_t s, Workspace& ws, Profiler* prof, const SlabState& st,
                    const uint8_t* zone, const int64_t* gid, const int64_t* gs_of_root,
                    const int64_t* all_roots, int64_t n_roots, int32_t mode, int32_t* cluster,
                    uint8_t* flag) {
    if (!st.valid) throw ArgError{"dbscan_slab_label_device: no slab fit on this handle"};
    if (st.n == 0) return;
    StageTimer t(prof, s, "slab_label");
    const int32_t* perm = static_cast<const int32_t*>(ws.perm_sorted);
    const uint8_t* core = static_cast<const uint8_t*>(ws.core.p);
    const int32_t* lab = static_cast<const int32_t*>(ws.lab.p);
    int32_t* label_of_root = static_cast<int32_t*>(ws.slab_lor.ensure(st.n * sizeof(int32_t)));
    klaunch(prof, "slab_root_labels", slab_root_labels_kernel, dim3(nblk(st.n)), dim3(kBlock), 0, s, st.n, perm,
                       core, lab, gs_of_root, all_roots, n_roots, label_of_root);
    uint32_t* packed = static_cast<uint32_t*>(ws.packed.ensure(st.npacked * sizeof(uint32_t)));
    klaunch(prof, "label_sorted", label_sorted_kernel<true>, dim3(nblk(st.n)), dim3(kBlock), 0, s,
                       static_cast<const double2*>(ws.xy.p), static_cast<const int32_t*>(ws.cell.p),
                       static_cast<const Seg*>(ws.seg.p), st.nbr, st.nbr_k,
                       reinterpret_cast<const int32_t*>(static_cast<double*>(ws.misc.p) + kMiscState) +
                           kStNf,
                       st.n, st.eps2, mode, perm, core, lab, (const uint64_t*)nullptr,
                       (const int32_t*)nullptr, zone, gid,
                       gs_of_root, label_of_root, packed, st.place);
    klaunch(prof, "permute_out", permute_out_kernel<true>, dim3(nblk(st.n)), dim3(kBlock), 0, s, st.n,
                       st.to_packed, packed, zone, cluster, flag, (const int32_t*)nullptr,
                       (int32_t*)nullptr);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

void enqueue_slab_label_prepare(hipStream_t s, Workspace& ws, Profiler* prof,
                                const SlabState& st, const uint8_t* zone, const int64_t* gid,
                                const int64_t* gs_of_root, int32_t mode) {
    if (!st.valid) throw ArgError{"dbscan_slab_roots_prepare_device: no slab fit on this handle"};
    if (st.n == 0) return;
    StageTimer t(prof, s, "slab_label");
    uint32_t* packed = static_cast<uint32_t*>(ws.packed.ensure(st.npacked * sizeof(uint32_t)));
    klaunch(prof, "label_sorted", label_sorted_kernel<true, true>, dim3(nblk(st.n)), dim3(kBlock), 0,
            s, static_cast<const double2*>(ws.xy.p), static_cast<const int32_t*>(ws.cell.p),
            static_cast<const Seg*>(ws.seg.p), st.nbr, st.nbr_k,
            reinterpret_cast<const int32_t*>(static_cast<double*>(ws.misc.p) + kMiscState) + kStNf, st.n,
            st.eps2, mode, static_cast<const int32_t*>(ws.perm_sorted),
            static_cast<const uint8_t*>(ws.core.p), static_cast<const int32_t*>(ws.lab.p),
            (const uint64_t*)nullptr, (const int32_t*)nullptr, zone, gid, gs_of_root,
            (const int32_t*)nullptr, packed, st.place);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

void run_slab_label_finish(hipStream_t s, Workspace& ws, Profiler* prof, const SlabState& st,
                           const uint8_t* zone, const int64_t* gs_of_root,
                           const int64_t* all_roots, int64_t n_roots, int32_t* cluster,
                           uint8_t* flag) {
    if (!st.valid) throw ArgError{"dbscan_slab_label_finish_device_async: no slab fit on this handle"};
    if (st.n == 0) return;
    StageTimer t(prof, s, "slab_label");
    int32_t* label_of_root = static_cast<int32_t*>(ws.slab_lor.ensure(st.n * sizeof(int32_t)));
    if (st.nlroots >= 0) {
        if (st.nlroots > 0)
            klaunch(prof, "slab_root_labels", slab_root_labels_list_kernel, dim3(nblk(st.nlroots)),
                    dim3(kBlock), 0, s, st.nlroots, static_cast<const int32_t*>(ws.lroots.p),
                    gs_of_root, all_roots, n_roots, label_of_root);
    } else {
        klaunch(prof, "slab_root_labels", slab_root_labels_kernel, dim3(nblk(st.n)), dim3(kBlock), 0,
                s, st.n, static_cast<const int32_t*>(ws.perm_sorted),
                static_cast<const uint8_t*>(ws.core.p), static_cast<const int32_t*>(ws.lab.p),
                gs_of_root, all_roots, n_roots, label_of_root);
    }
    // (the packed labels of the prepare, still in the workspace)
    klaunch(prof, "slab_map", slab_map_packed_kernel, dim3(nblk(st.n)), dim3(kBlock), 0, s, st.n,
            st.to_packed, static_cast<const uint32_t*>(ws.packed.p), zone, label_of_root, cluster,
            flag);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

}  // namespace dbscan

#if DBSCAN_AB_STAMPS
// Timing builds: out = NULL clears the stamps; else copies n <= kTileGrid * kStamps of them.
extern "C" int dbscan_ab_stamps(long long* out, int n) {
    using namespace dbscan;
    const size_t bytes = sizeof(long long) * (size_t)kTileGrid * kStamps;
    if (!out) {
        std::vector<long long> z((size_t)kTileGrid * kStamps, 0);
        return hipMemcpyToSymbol(HIP_SYMBOL(g_ab_stamps), z.data(), bytes) == hipSuccess ? 0 : -1;
    }
    const size_t want = sizeof(long long) * (size_t)n;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ab_stamps), want < bytes ? want : bytes) ==
                   hipSuccess ? 0 : -1;
}
#endif

#if DBSCAN_AB_EDGE_COUNT
// Counting builds: copies edge_union's eight counters into out and clears them.
extern "C" int dbscan_ab_edge_counts(unsigned long long* out) {
    using namespace dbscan;
    unsigned long long z[8] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_edge_cnt), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_edge_cnt), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
