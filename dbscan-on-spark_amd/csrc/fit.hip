// fit.hip -- the local DBSCAN fit on gfx950: eps grid, neighbour counts, lock-free
// union-find, border/noise labelling and cluster numbering.
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
// Kernels, in pipeline order (one HIP stream per handle; see DESIGN.md for the rooflines):
//   bin        key = cy*nx + cx (u32) per point, perm = input index
//   [radix sort (primitives.hip)]
//   gather     sorted double2 coordinates (AoS) -- one global_load_dwordx4 per candidate test
//   cells      occupied cells from the key head flags (scan) -> ckey, cstart, cell-of-slot
//   segs       per cell: slot ranges of the 3 stencil rows (row-major keys make the 3 cells of a
//              stencil row one contiguous slot range)
//   count      thread per slot: candidate loop with early exit at minPoints -> core flag
//   union      thread per core slot: candidates with smaller slot only (rows cy-1 and the
//              head of row cy); lock-free union-find hooking the root with the larger visit
//              index under the smaller (CAS, agent scope), so every root is s(K) directly
//   final      root of every core -> lab = visit index of its root; roots flagged in input order
//   [scan of root flags in input order -> rank = cluster id - 1]
//   output     cores: rank[lab]+1; non-cores: min lab over core neighbours + Naive/Archery rule;
//              written in input order
#include "internal.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace dbscan {

enum GridMode { kGridEps = 0, kGridAllPairs = 1, kGridNoPairs = 2 };

struct GridParams {
    double xmin2, ymin2, invx, invy;  // cell = floor((v*0.5 - vmin*0.5) * inv)
    uint32_t nx, ny;
    int clique;  // cell side <= eps*(1+2^-14): quarter cells are cliques of the predicate
};

namespace {

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

struct Seg {  // 32 B: rows dy = -1, 0, +1 as [b, e) slot ranges, then the cell's own range
    int b0, e0, b1, e1, b2, e2, cs, ce;
};

__device__ __forceinline__ Seg load_seg(const Seg* seg, int c) {
    const int4* p = reinterpret_cast<const int4*>(seg + c);
    const int4 u = p[0];
    const int4 v = p[1];
    Seg s;
    s.b0 = u.x; s.e0 = u.y; s.b1 = u.z; s.e1 = u.w; s.b2 = v.x; s.e2 = v.y;
    s.cs = v.z; s.ce = v.w;
    return s;
}

// Candidate iteration over up to three slot ranges [b0,e0) [b1,e1) [b2,e2) (the stencil rows).
// f(j) returns false to stop early.
template <class F>
__device__ __forceinline__ void for_candidates(const Seg& s, F f) {
    const int b[3] = {s.b0, s.b1, s.b2};
    const int e[3] = {s.e0, s.e1, s.e2};
#pragma unroll
    for (int r = 0; r < 3; ++r)
        for (int j = b[r]; j < e[r]; ++j)
            if (!f(j)) return;
}

__global__ __launch_bounds__(kBlock) void bin_kernel(const double* __restrict__ x,
                                                     const double* __restrict__ y, int64_t n,
                                                     GridParams g, uint32_t* __restrict__ key,
                                                     int32_t* __restrict__ perm) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double a = x[i], b = y[i];
    uint32_t k = kSentinelKey;
    if (__builtin_isfinite(a) && __builtin_isfinite(b)) {
        // quarter-grid coordinates: floor(2t) >> 1 == floor(t) exactly (2t is exact)
        double fx = floor(2.0 * ((a * 0.5 - g.xmin2) * g.invx));
        double fy = floor(2.0 * ((b * 0.5 - g.ymin2) * g.invy));
        const double mx = 2.0 * (double)g.nx - 1.0, my = 2.0 * (double)g.ny - 1.0;
        fx = fx < 0 ? 0 : (fx > mx ? mx : fx);
        fy = fy < 0 ? 0 : (fy > my ? my : fy);
        const uint32_t qx = (uint32_t)fx, qy = (uint32_t)fy;
        const uint64_t cellk = (uint64_t)(qy >> 1) * g.nx + (qx >> 1);
        k = (uint32_t)((cellk << 2) | ((qy & 1u) << 1) | (qx & 1u));
    }
    key[i] = k;
    perm[i] = (int32_t)i;
}

__global__ __launch_bounds__(kBlock) void iota_key_kernel(int64_t n, uint32_t kval,
                                                          uint32_t* __restrict__ key,
                                                          int32_t* __restrict__ perm) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    key[i] = kval;
    perm[i] = (int32_t)i;
}

__global__ __launch_bounds__(kBlock) void gather_kernel(const double* __restrict__ x,
                                                        const double* __restrict__ y, int64_t nf,
                                                        const int32_t* __restrict__ perm,
                                                        double2* __restrict__ xy) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= nf) return;
    const int32_t o = perm[p];
    xy[p] = make_double2(x[o], y[o]);
}

// cell[p] holds the exclusive scan of head flags on entry; converted to the group index.
// shift = 2: eps cells (key >> 2); shift = 0: quarter cells (full key).
__global__ __launch_bounds__(kBlock) void cells_kernel(const uint32_t* __restrict__ key,
                                                       int shift, int64_t nf,
                                                       int32_t* __restrict__ cell,
                                                       uint32_t* __restrict__ ckey,
                                                       int32_t* __restrict__ cstart,
                                                       const int32_t* __restrict__ ncells) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= nf) {
        if (p == nf) cstart[*ncells] = (int32_t)nf;
        return;
    }
    const int32_t ex = cell[p];
    const bool head = (p == 0) || (key[p] >> shift) != (key[p - 1] >> shift);
    if (head) {
        ckey[ex] = key[p] >> shift;
        cstart[ex] = (int32_t)p;
    }
    cell[p] = ex + (head ? 1 : 0) - 1;
}

__device__ __forceinline__ int lower_bound_u32(const uint32_t* a, int n, uint32_t k) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = lo + ((hi - lo) >> 1);
        if (a[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) void segs_kernel(const uint32_t* __restrict__ ckey,
                                                      const int32_t* __restrict__ cstart,
                                                      const int32_t* __restrict__ ncells_p,
                                                      GridParams g, Seg* __restrict__ seg) {
    const int c = blockIdx.x * kBlock + threadIdx.x;
    const int C = *ncells_p;
    if (c >= C) return;
    const uint32_t key = ckey[c];
    const uint32_t cy = key / g.nx, cx = key - cy * g.nx;
    const uint32_t lox = cx > 0 ? cx - 1 : cx;
    const uint32_t hix = cx + 1 < g.nx ? cx + 1 : cx;
    int rb[3], re[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        rb[r] = 0;
        re[r] = 0;
        const int64_t ry = (int64_t)cy + r - 1;
        if (ry < 0 || ry >= (int64_t)g.ny) continue;
        const uint32_t klo = (uint32_t)ry * g.nx + lox, khi = (uint32_t)ry * g.nx + hix;
        int a, z;
        if (r == 1) {  // own row: neighbours are adjacent entries of ckey
            a = (c > 0 && ckey[c - 1] == klo && lox != cx) ? c - 1 : c;
            z = (c + 1 < C && ckey[c + 1] == khi && hix != cx) ? c + 2 : c + 1;
        } else {
            a = lower_bound_u32(ckey, C, klo);
            z = a;
            while (z < C && ckey[z] <= khi) ++z;
        }
        rb[r] = cstart[a];
        re[r] = cstart[z];
    }
    Seg s;
    s.b0 = rb[0]; s.e0 = re[0]; s.b1 = rb[1]; s.e1 = re[1]; s.b2 = rb[2]; s.e2 = re[2];
    s.cs = cstart[c]; s.ce = cstart[c + 1];
    seg[c] = s;
}

// ---------------------------------------------------------------------------------------
// Block staging of stencil candidates in LDS.  Slots are in row-major cell-key order, so the
// 256 slots of a block usually cover a run of cells [c0, c1] of ONE cell row; the candidates
// of all of them are then the three contiguous slot ranges of rows cy-1, cy, cy+1 spanning
// cells cx0-1 .. cx1+1.  Those are loaded once (coalesced 16-B loads) into LDS and every
// thread's candidate loop reads LDS instead of issuing dependent global gathers.  Blocks that
// straddle two cell rows, or whose candidates exceed the LDS budget, read global memory.
// ---------------------------------------------------------------------------------------
constexpr int kStageCap = 3072;  // points (48 KB of double2)

struct StageInfo {
    int ok;          // 1: the block's candidates are in LDS
    int B[3], E[3];  // global slot range of each stencil row
    int off[3];      // LDS offset of each row's first point
};

__device__ __forceinline__ int row_of(uint32_t ck, uint32_t nx) { return (int)(ck / nx); }

// Fills `st` (LDS) and stages candidates into `buf` (LDS).  All threads must call it.
__device__ void stage_block(const double2* __restrict__ xy, const int32_t* __restrict__ cell,
                            const uint32_t* __restrict__ ckey, const int32_t* __restrict__ cstart,
                            int C, int64_t p0, int64_t p1, GridParams g, StageInfo& st,
                            double2* buf) {
    if (threadIdx.x < 3) {
        const int r = threadIdx.x;
        const int c0 = cell[p0], c1 = cell[p1 - 1];
        const uint32_t k0 = ckey[c0], k1 = ckey[c1];
        const int cy = row_of(k0, g.nx);
        int ok = row_of(k1, g.nx) == cy;
        int B = 0, E = 0;
        const int64_t ry = (int64_t)cy + r - 1;
        if (ok && ry >= 0 && ry < (int64_t)g.ny) {
            const uint32_t cx0 = k0 - (uint32_t)cy * g.nx, cx1 = k1 - (uint32_t)cy * g.nx;
            const uint32_t lo = (uint32_t)ry * g.nx + (cx0 > 0 ? cx0 - 1 : 0);
            const uint32_t hi = (uint32_t)ry * g.nx + (cx1 + 1 < g.nx ? cx1 + 1 : cx1);
            int a = lower_bound_u32(ckey, C, lo);
            int z = lower_bound_u32(ckey, C, hi + 1);
            B = cstart[a];
            E = cstart[z];
        }
        st.B[r] = B;
        st.E[r] = E;
        if (r == 0) st.ok = ok;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int n0 = st.E[0] - st.B[0], n1 = st.E[1] - st.B[1], n2 = st.E[2] - st.B[2];
        st.off[0] = 0;
        st.off[1] = n0;
        st.off[2] = n0 + n1;
        if (n0 + n1 + n2 > kStageCap) st.ok = 0;
    }
    __syncthreads();
    if (st.ok) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int B = st.B[r], n = st.E[r] - B, o = st.off[r];
            for (int t = threadIdx.x; t < n; t += kBlock) buf[o + t] = xy[B + t];
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------------------
// Neighbour counts -> core flags (LocalDBSCANNaive.scala:52-54, :99-101), with early exit
// once minPoints neighbours are seen (the count itself is never an output).
// zone (optional, slab fits): zone-2 points are halo-only candidates -> never core.
// ---------------------------------------------------------------------------------------
template <bool STAGED>
__device__ __forceinline__ bool count_ranges(const double2* __restrict__ src, const Seg& s,
                                             const StageInfo& st, double2 me, double eps2,
                                             int min_points, int& cnt) {
    // own cell first (most likely neighbours -> earliest exit), then the rest of its row,
    // then the rows below and above; 8 candidates per batch
    auto map = [&](int j, int r) -> int { return STAGED ? j - st.B[r] + st.off[r] : j; };
    auto scan = [&](int b, int e, int r) -> bool {
        int j = b;
        for (; j + 8 <= e; j += 8) {
            const int m0 = map(j, r);
            double2 qq[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) qq[u] = src[m0 + u];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                cnt += within_eps(me.x, me.y, qq[u].x, qq[u].y, eps2) ? 1 : 0;
            if (cnt >= min_points) return true;
        }
        for (; j < e; ++j) {
            const double2 q = src[map(j, r)];
            cnt += within_eps(me.x, me.y, q.x, q.y, eps2) ? 1 : 0;
        }
        return cnt >= min_points;
    };
    return scan(s.cs, s.ce, 1) || scan(s.b1, s.cs, 1) || scan(s.ce, s.e1, 1) ||
           scan(s.b0, s.e0, 0) || scan(s.b2, s.e2, 2);
}

__global__ __launch_bounds__(kBlock) void count_kernel(const double2* __restrict__ xy,
                                                       const int32_t* __restrict__ cell,
                                                       const Seg* __restrict__ seg,
                                                       const uint32_t* __restrict__ ckey,
                                                       const int32_t* __restrict__ cstart,
                                                       const int32_t* __restrict__ ncells_p,
                                                       GridParams g, int64_t n, int64_t nf,
                                                       double eps2, int32_t min_points,
                                                       const int32_t* __restrict__ perm,
                                                       const uint8_t* __restrict__ zone,
                                                       const int32_t* __restrict__ qidx,
                                                       const int32_t* __restrict__ qstart,
                                                       uint8_t* __restrict__ core,
                                                       int32_t* __restrict__ parent,
                                                       int32_t* __restrict__ block_cores) {
    __shared__ StageInfo st;
    __shared__ int wcores[kBlock / 64];
    __shared__ double2 buf[kStageCap];
    const int64_t p0 = (int64_t)blockIdx.x * kBlock;
    const int64_t p = p0 + threadIdx.x;
    // stage only blocks entirely inside the grid (block-uniform condition)
    const bool stage = min_points > 0 && p0 + kBlock <= nf;
    if (stage) stage_block(xy, cell, ckey, cstart, *ncells_p, p0, p0 + kBlock, g, st, buf);
    bool is_core = false;
    if (p >= n) {
        // no neighbours to count
    } else if (zone && zone[perm[p]] == 2) {
        is_core = false;
    } else if (min_points <= 0) {
        is_core = true;
    } else if (p >= nf) {
        is_core = false;  // outside the grid: no neighbours, not even itself
    } else {
        const int32_t c = cell[p];
        const double2 me = xy[p];
        const int32_t q = qidx ? qidx[p] : 0;
        const Seg s = load_seg(seg, c);
        // a clique quarter holding >= minPoints points (a dense box): core without a test
        const bool dense = qidx && (qstart[q + 1] - qstart[q] >= min_points);
        int cnt = dense ? min_points : 0;
        if (!dense) {
            if (stage && st.ok)
                count_ranges<true>(buf, s, st, me, eps2, min_points, cnt);
            else
                count_ranges<false>(xy, s, st, me, eps2, min_points, cnt);
        }
        is_core = cnt >= min_points;
    }
    if (p < n) {
        parent[p] = (int32_t)p;
        core[p] = is_core ? 1 : 0;
    }
    // per-block core count (no same-address atomics: 156K of them cost ~1.7 ms at 10^7 points)
    const uint64_t cm = __ballot(is_core);
    if (__lane_id() == 0) wcores[threadIdx.x >> 6] = (int)__popcll(cm);
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += wcores[w];
        block_cores[blockIdx.x] = t;
    }
}

// ---------------------------------------------------------------------------------------
// Lock-free union-find over slots.  parent pointers always lead to a strictly smaller visit
// index (perm), so there are no cycles and a root is the minimum-index core of its set.
// Loads/stores are agent-scope relaxed atomics (L1-bypassing), hooks are CAS on roots only;
// stale reads only ever show an older ancestor, which is still an ancestor.
// ---------------------------------------------------------------------------------------
// UF load policy (template parameter V): 0 = agent-scope atomic loads (L1-bypassing) with
// path-halving stores (per-point fallback union); 1 = plain L1-cacheable loads, no stores
// (quarter union; measured 2.4 vs 5.0 ms, tools/uf_variants.sh).  Stale copies are older
// ancestors, which are still ancestors, so both are correct; only CAS hooks write roots.
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

__global__ __launch_bounds__(kBlock) void union_kernel(const double2* __restrict__ xy,
                                                       const int32_t* __restrict__ cell,
                                                       const Seg* __restrict__ seg, int64_t nf,
                                                       double eps2,
                                                       const int32_t* __restrict__ perm,
                                                       const uint8_t* __restrict__ core,
                                                       int32_t* __restrict__ parent) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= nf || !core[p]) return;
    const double2 me = xy[p];
    Seg s = load_seg(seg, cell[p]);
    // only slots < p: row cy-1 entirely, row cy up to p, row cy+1 never
    s.e1 = (int)p;
    s.b2 = 0;
    s.e2 = 0;
    int rp = uf_find(parent, (int)p);
    for_candidates(s, [&](int j) {
        const double2 q = xy[j];
        if (within_eps(me.x, me.y, q.x, q.y, eps2) && core[j]) {
            const int rj = uf_find(parent, j);
            if (rj != rp) rp = uf_unite_roots(parent, perm, rp, rj);
        }
        return true;
    });
}

// ---------------------------------------------------------------------------------------
// Clique-quarter union (cell side <= eps*(1+2^-14)).  A quarter cell has side ~eps/2 and
// diagonal ~0.71*eps, so any two of its points satisfy the fp64 predicate: its cores are one
// connected set without a single distance test.  quarter_init points every core of a quarter at
// the quarter's minimum-visit-index core (a valid union-find state: pointers go to a smaller
// visit index); quarter_union then needs ONE core-core edge per pair of quarter cells within
// reach (offsets <= 2 on the quarter grid, i.e. inside the 3x3 eps-cell stencil), examined once
// by the later quarter in sorted order, and one union per connected pair.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void quarter_init_kernel(const int32_t* __restrict__ qstart,
                                                              const uint32_t* __restrict__ qkey,
                                                              const int32_t* __restrict__ nq_p,
                                                              const int32_t* __restrict__ perm,
                                                              const uint8_t* __restrict__ core,
                                                              int4* __restrict__ qinfo,
                                                              uint32_t* __restrict__ qmask,
                                                              int32_t* __restrict__ parent) {
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= *nq_p) return;
    const int b = qstart[q], e = qstart[q + 1];
    int rep = -1, best = 0x7FFFFFFF;
    uint32_t mask = 0;  // cores among the first 32 slots (quarters rarely hold more)
    for (int j = b; j < e; ++j)
        if (core[j]) {
            if (j - b < 32) mask |= 1u << (j - b);
            if (perm[j] < best) {
                best = perm[j];
                rep = j;
            }
        }
    qinfo[q] = make_int4(b, e, rep, (int)qkey[q]);  // one 16-B record per quarter cell
    qmask[q] = mask;
    if (rep < 0) return;
    for (int j = b; j < e; ++j)
        if (core[j]) parent[j] = rep;
}

// ABL: timing ablations for attribution only (1 no union, 2 no pair test, 3 metadata only).
constexpr int kQReg = 8;  // own-quarter core points kept in registers for the pair tests

// ABL: timing ablations for attribution only (1 no union, 2 no pair test, 3 metadata only).
template <int ABL = 0>
__global__ __launch_bounds__(kBlock) void quarter_union_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, const int32_t* __restrict__ qidx,
    const int4* __restrict__ qinfo, const uint32_t* __restrict__ qmask,
    const int32_t* __restrict__ nq_p, GridParams g, double eps2,
    const int32_t* __restrict__ perm, const uint8_t* __restrict__ core,
    int32_t* __restrict__ parent) {
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= *nq_p) return;
    const int4 me = qinfo[q];
    if (me.z < 0) return;
    const uint32_t key = (uint32_t)me.w, ck = key >> 2;
    const uint32_t cy = ck / g.nx, cx = ck - cy * g.nx;
    const int gx = (int)(2 * cx + (key & 1u)), gy = (int)(2 * cy + ((key >> 1) & 1u));
    const Seg s = load_seg(seg, cell[me.x]);
    // own cores in registers (the same set is tested against every neighbour quarter)
    double px[kQReg], py[kQReg];
    int nmine = 0;
    const bool small = me.y - me.x <= 32;
    {
        uint32_t m = qmask[q];
        const uint32_t m0 = small ? m : 0u;
#pragma unroll
        for (int k = 0; k < kQReg; ++k) {
            px[k] = 0.0;
            py[k] = 0.0;
        }
        uint32_t mm = m0;
#pragma unroll
        for (int k = 0; k < kQReg; ++k) {
            if (mm) {
                const int j = me.x + (__ffs(mm) - 1);
                mm &= mm - 1;
                const double2 v = xy[j];
                px[k] = v.x;
                py[k] = v.y;
                nmine = k + 1;
            }
        }
        if (mm) nmine = -1;  // more than kQReg cores: generic loop below
    }
    const bool inreg = small && nmine >= 0;
    int rp = uf_find<1>(parent, me.z);
    // two sweeps: adjacent quarters (Chebyshev distance 1) first so most merges happen early
    // and the far (distance-2) candidates are usually skipped by the find-first check
#pragma unroll
    for (int sweep = 0; sweep < 2; ++sweep) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {  // rows cy-1 and cy: every quarter there with a smaller key
            const int rb = r == 0 ? s.b0 : s.b1, re = r == 0 ? s.e0 : s.e1;
            if (rb >= re) continue;
            const int ry = (int)cy + r - 1;
            const int64_t rowbase = (int64_t)ry * g.nx;
            const int q_lo = qidx[rb], q_hi = qidx[re - 1];
            for (int q2 = q_lo; q2 <= q_hi && q2 < q; ++q2) {
                const int4 o = qinfo[q2];
                if (o.z < 0) continue;
                const uint32_t k2 = (uint32_t)o.w;
                const int gx2 = (int)(2 * ((int64_t)(k2 >> 2) - rowbase)) + (int)(k2 & 1u);
                const int gy2 = 2 * ry + (int)((k2 >> 1) & 1u);
                const int d = max(abs(gx2 - gx), abs(gy2 - gy));
                if (d > 2 || (sweep == 0) != (d <= 1)) continue;
                if constexpr (ABL == 3) {
                    asm volatile("" ::"v"(gx2));
                    continue;
                }
                const int rr = uf_find_until<1>(parent, o.z, rp);
                if (rr == rp) continue;  // already one set: skip the pair test
                bool found = ABL == 2;
                if (!found && inreg && o.y - o.x <= 32) {
                    uint32_t om = qmask[q2];
                    while (om && !found) {
                        const int b2 = o.x + (__ffs(om) - 1);
                        om &= om - 1;
                        const double2 pb = xy[b2];
#pragma unroll
                        for (int k = 0; k < kQReg; ++k)
                            found |= (k < nmine) && within_eps(px[k], py[k], pb.x, pb.y, eps2);
                    }
                } else if (!found) {
                    for (int a = me.x; a < me.y && !found; ++a) {
                        if (!core[a]) continue;
                        const double2 pa = xy[a];
                        for (int b2 = o.x; b2 < o.y; ++b2) {
                            if (!core[b2]) continue;
                            const double2 pb = xy[b2];
                            if (within_eps(pa.x, pa.y, pb.x, pb.y, eps2)) {
                                found = true;
                                break;
                            }
                        }
                    }
                }
                if (!found) continue;
                if constexpr (ABL == 1) {
                    asm volatile("" ::"v"(rr));
                    continue;
                }
                rp = uf_unite_roots<1>(parent, perm, rp, rr);
            }
        }
    }
}

__global__ __launch_bounds__(kBlock) void final_kernel(int64_t n,
                                                       const int32_t* __restrict__ perm,
                                                       const uint8_t* __restrict__ core,
                                                       const int32_t* __restrict__ parent,
                                                       int32_t* __restrict__ lab,
                                                       uint8_t* __restrict__ is_root) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    if (!core[p]) {
        lab[p] = -1;
        return;
    }
    int r = (int)p;
    for (int nx = parent[r]; nx != r; nx = parent[r]) r = nx;
    lab[p] = perm[r];
    if (r == (int)p && is_root) is_root[perm[p]] = 1;
}

// Border / noise rule + cluster numbering, written in input order.
__global__ __launch_bounds__(kBlock) void output_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, int64_t n, int64_t nf, double eps2, int32_t mode,
    const int32_t* __restrict__ perm, const uint8_t* __restrict__ core,
    const int32_t* __restrict__ lab, const int32_t* __restrict__ rank,
    int32_t* __restrict__ cluster_out, uint8_t* __restrict__ flag_out) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const int32_t o = perm[p];
    int32_t cl = 0;
    uint8_t fl = 2;  // Noise
    if (core[p]) {
        cl = rank[lab[p]] + 1;
        fl = 1;  // Core
    } else if (p < nf) {
        const double2 me = xy[p];
        const Seg s = load_seg(seg, cell[p]);
        int32_t m = 0x7FFFFFFF;
        for_candidates(s, [&](int j) {
            const double2 q = xy[j];
            if (within_eps(me.x, me.y, q.x, q.y, eps2) && core[j]) {
                const int32_t lj = lab[j];
                m = lj < m ? lj : m;
            }
            return true;
        });
        if (m != 0x7FFFFFFF && (mode != 0 || m < o)) {
            cl = rank[m] + 1;
            fl = 0;  // Border
        }
    }
    cluster_out[o] = cl;
    flag_out[o] = fl;
}

// Slab fit, phase 1 output (multi-GPU node path): core flag and local root (slab index of the
// minimum-index core of the local component), in slab order.
__global__ __launch_bounds__(kBlock) void slab_roots_kernel(int64_t n,
                                                            const int32_t* __restrict__ perm,
                                                            const uint8_t* __restrict__ core,
                                                            const int32_t* __restrict__ lab,
                                                            uint8_t* __restrict__ core_out,
                                                            int32_t* __restrict__ root_out) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const int32_t o = perm[p];
    core_out[o] = core[p];
    root_out[o] = core[p] ? lab[p] : -1;
}

// Slab fit, phase 2 (after the global merge): labels of the owned (zone 0) points.
//   gs_of_root[r]    global s(K) (a global visit index) of local root r (slab index)
//   label_of_root[r] global cluster id of that component
// Border rule on global visit indices: m = min over core neighbours of gs_of_root[root];
// Naive: Border iff m < gid(b); Archery: Border iff a core neighbour exists.
__global__ __launch_bounds__(kBlock) void slab_label_kernel(
    const double2* __restrict__ xy, const int32_t* __restrict__ cell,
    const Seg* __restrict__ seg, int64_t n, int64_t nf, double eps2, int32_t mode,
    const int32_t* __restrict__ perm, const uint8_t* __restrict__ zone,
    const uint8_t* __restrict__ core, const int32_t* __restrict__ lab,
    const int64_t* __restrict__ gid, const int64_t* __restrict__ gs_of_root,
    const int32_t* __restrict__ label_of_root, int32_t* __restrict__ cluster_out,
    uint8_t* __restrict__ flag_out) {
    const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const int32_t o = perm[p];
    if (zone[o] != 0) return;
    int32_t cl = 0;
    uint8_t fl = 2;
    if (core[p]) {
        cl = label_of_root[lab[p]];
        fl = 1;
    } else if (p < nf) {
        const double2 me = xy[p];
        const Seg s = load_seg(seg, cell[p]);
        int64_t m = 0x7FFFFFFFFFFFFFFFll;
        int32_t mr = -1;
        for_candidates(s, [&](int j) {
            const double2 q = xy[j];
            if (within_eps(me.x, me.y, q.x, q.y, eps2) && core[j]) {
                const int32_t r = lab[j];
                const int64_t v = gs_of_root[r];
                if (v < m) {
                    m = v;
                    mr = r;
                }
            }
            return true;
        });
        if (mr >= 0 && (mode != 0 || m < gid[o])) {
            cl = label_of_root[mr];
            fl = 0;
        }
    }
    cluster_out[o] = cl;
    flag_out[o] = fl;
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

// ---------------------------------------------------------------------------------------
// Host orchestration
// ---------------------------------------------------------------------------------------

// Grid sizing on the host (see DESIGN.md "grid soundness"): cell side >= R*(1+2^-16) with
// R = max(|eps|*(1+2^-40), 2^-500) bounds |x'-x| for every pair the fp64 predicate accepts;
// nx*ny <= 2^29 (u32 keys = cell*4 + quadrant, below the sentinel), growing the side (never
// shrinking it) when the extent would need more cells.  Quarter cells are cliques only while
// the side was not grown: clique = side <= |eps|*(1+2^-14).
static bool make_grid(const double bb[5], double eps, GridParams* g) {
    const double xmin = bb[0], xmax = bb[1], ymin = bb[2], ymax = bb[3];
    double R = std::fabs(eps) * (1.0 + 0x1p-40);
    if (R < 0x1p-500) R = 0x1p-500;
    double hx = R * (1.0 + 0x1p-16), hy = hx;
    const double limit = 536870912.0;  // 2^29 cells
    auto cells = [](double vmax, double vmin, double h) {
        const double t = (vmax * 0.5 - vmin * 0.5) * (2.0 / h);
        return std::floor(t) + 1.0;  // may be +inf for absurd extents
    };
    for (int it = 0; it < 4096; ++it) {
        const double cx = cells(xmax, xmin, hx), cy = cells(ymax, ymin, hy);
        if (cx <= limit && cy <= limit && cx * cy <= limit) {
            g->invx = 2.0 / hx;
            g->invy = 2.0 / hy;
            g->xmin2 = xmin * 0.5;
            g->ymin2 = ymin * 0.5;
            g->nx = (uint32_t)cx;
            g->ny = (uint32_t)cy;
            const double cl = std::fabs(eps) * (1.0 + 0x1p-14);
            g->clique = (hx <= cl && hy <= cl) ? 1 : 0;
            return true;
        }
        if (cx >= cy) hx *= 2.0; else hy *= 2.0;
    }
    return false;
}

int64_t run_fit(hipStream_t s, Workspace& ws, Profiler* prof, const FitArgs& a, FitStats* st,
                SlabState* slab) {
    if (slab) slab->valid = false;
    const int64_t n = a.n;
    FitStats stats;
    stats.n = n;
    if (n == 0) {
        if (st) *st = stats;
        if (slab) {
            slab->valid = a.zone != nullptr;
            slab->n = 0;
            slab->nf = 0;
        }
        return 0;
    }
    const double eps2 = a.eps * a.eps;  // LocalDBSCANNaive.scala:33
    int mode = std::isnan(eps2) ? kGridNoPairs : (std::isinf(eps2) ? kGridAllPairs : kGridEps);

    uint32_t* key = static_cast<uint32_t*>(ws.key.ensure(n * sizeof(uint32_t)));
    uint32_t* key2 = static_cast<uint32_t*>(ws.key2.ensure(n * sizeof(uint32_t)));
    int32_t* perm = static_cast<int32_t*>(ws.perm.ensure(n * sizeof(int32_t)));
    int32_t* perm2 = static_cast<int32_t*>(ws.perm2.ensure(n * sizeof(int32_t)));
    double* misc = static_cast<double*>(ws.misc.ensure(64 * sizeof(double)));
    int32_t* misc_i = reinterpret_cast<int32_t*>(misc + 16);  // [0] ncells, [1] nclusters

    DBSCAN_HIP_CHECK(hipMemsetAsync(misc_i, 0, 4 * sizeof(int32_t), s));
    GridParams g{0, 0, 0, 0, 1, 1, 0};
    int64_t nf = 0;
    int bits = 0;
    if (mode == kGridEps) {
        double bb[5];
        {
            StageTimer t(prof, s, "bbox");
            bbox_finite(s, a.x, a.y, n, misc, ws.scan_tmp);
        }
        DBSCAN_HIP_CHECK(hipMemcpyAsync(bb, misc, sizeof(bb), hipMemcpyDeviceToHost, s));
        DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
        nf = (int64_t)bb[4];
        if (nf > 0 && !make_grid(bb, a.eps, &g)) throw ArgError{"cannot size the eps grid"};
        if (nf == 0) mode = kGridNoPairs;
    } else if (mode == kGridAllPairs) {
        nf = n;  // one cell holding every point; the predicate decides (incl. non-finite)
    }
    stats.grid_mode = mode;
    stats.nf = nf;
    stats.nx = g.nx;
    stats.ny = g.ny;

    if (mode == kGridEps) {
        {
            StageTimer t(prof, s, "bin");
            hipLaunchKernelGGL(bin_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, a.x, a.y, n, g, key,
                               perm);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        const uint64_t qcells = 4ull * g.nx * g.ny;  // valid keys < qcells <= 2^31
        bits = 1;
        while (bits < 32 && (1ull << bits) <= qcells) ++bits;  // keys < 2^bits - 1 (sentinel)
        radix_sort_pairs(s, key, perm, key2, perm2, n, bits, ws.hist, ws.scan_tmp, prof);
    } else {
        StageTimer t(prof, s, "bin");
        hipLaunchKernelGGL(iota_key_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n,
                           mode == kGridAllPairs ? 0u : kSentinelKey, key, perm);
        DBSCAN_HIP_CHECK(hipGetLastError());
    }
    stats.bits = bits;
    ws.perm_sorted = perm;

    const int64_t nfa = nf > 0 ? nf : 1;
    double2* xy = static_cast<double2*>(ws.xy.ensure(nfa * sizeof(double2)));
    int32_t* cell = static_cast<int32_t*>(ws.cell.ensure(nfa * sizeof(int32_t)));
    uint32_t* ckey = static_cast<uint32_t*>(ws.ckey.ensure(nfa * sizeof(uint32_t)));
    int32_t* cstart = static_cast<int32_t*>(ws.cstart.ensure((nfa + 1) * sizeof(int32_t)));
    Seg* seg = static_cast<Seg*>(ws.seg.ensure(nfa * sizeof(Seg)));
    uint8_t* core = static_cast<uint8_t*>(ws.core.ensure(n));
    int32_t* parent = static_cast<int32_t*>(ws.parent.ensure(n * sizeof(int32_t)));
    int32_t* lab = static_cast<int32_t*>(ws.lab.ensure(n * sizeof(int32_t)));
    const bool clique = mode == kGridEps && g.clique;
    int32_t* qidx = nullptr;
    uint32_t* qkey = nullptr;
    int32_t* qstart = nullptr;
    int4* qinfo = nullptr;
    uint32_t* qmask = nullptr;
    if (clique) {
        qidx = static_cast<int32_t*>(ws.qidx.ensure(nfa * sizeof(int32_t)));
        qkey = static_cast<uint32_t*>(ws.qkey.ensure(nfa * sizeof(uint32_t)));
        qstart = static_cast<int32_t*>(ws.qstart.ensure((nfa + 1) * sizeof(int32_t)));
        qinfo = static_cast<int4*>(ws.qrep.ensure(nfa * sizeof(int4)));
        qmask = static_cast<uint32_t*>(ws.qmask.ensure(nfa * sizeof(uint32_t)));
    }

    if (nf > 0) {
        {
            StageTimer t(prof, s, "gather");
            hipLaunchKernelGGL(gather_kernel, dim3(nblk(nf)), dim3(kBlock), 0, s, a.x, a.y, nf,
                               perm, xy);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        {
            StageTimer t(prof, s, "cells");
            exclusive_scan(s, 3, key, cell, nf, &misc_i[0], ws.scan_tmp);
            hipLaunchKernelGGL(cells_kernel, dim3(nblk(nf + 1)), dim3(kBlock), 0, s, key, 2, nf,
                               cell, ckey, cstart, &misc_i[0]);
            DBSCAN_HIP_CHECK(hipGetLastError());
            if (clique) {
                exclusive_scan(s, 2, key, qidx, nf, &misc_i[3], ws.scan_tmp);
                hipLaunchKernelGGL(cells_kernel, dim3(nblk(nf + 1)), dim3(kBlock), 0, s, key, 0,
                                   nf, qidx, qkey, qstart, &misc_i[3]);
                DBSCAN_HIP_CHECK(hipGetLastError());
            }
        }
        {
            StageTimer t(prof, s, "segs");
            hipLaunchKernelGGL(segs_kernel, dim3(nblk(nf)), dim3(kBlock), 0, s, ckey, cstart,
                               &misc_i[0], g, seg);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
    }
    int32_t* block_cores =
        static_cast<int32_t*>(ws.blockcnt.ensure(2 * (nblk(n) + 1) * sizeof(int32_t)));
    {
        StageTimer t(prof, s, "count");
        hipLaunchKernelGGL(count_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, xy, cell, seg, ckey,
                           cstart, &misc_i[0], g, n, nf, eps2, a.min_points, perm, a.zone, qidx,
                           qstart, core, parent, block_cores);
        DBSCAN_HIP_CHECK(hipGetLastError());
        exclusive_scan(s, 0, block_cores, block_cores + nblk(n) + 1, nblk(n), &misc_i[2],
                       ws.scan_tmp);
    }
    if (clique) {
        {
            StageTimer t(prof, s, "quarter_init");
            hipLaunchKernelGGL(quarter_init_kernel, dim3(nblk(nf)), dim3(kBlock), 0, s, qstart,
                               qkey, &misc_i[3], perm, core, qinfo, qmask, parent);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        StageTimer t(prof, s, "union");
        static const int ablate = [] {
            const char* e = getenv("DBSCAN_UF_ABLATE");
            return e ? atoi(e) : 0;
        }();
        auto* kq = ablate == 1   ? quarter_union_kernel<1>
                   : ablate == 2 ? quarter_union_kernel<2>
                   : ablate == 3 ? quarter_union_kernel<3>
                                 : quarter_union_kernel<0>;
        hipLaunchKernelGGL(kq, dim3(nblk(nf)), dim3(kBlock), 0, s, xy, cell, seg, qidx, qinfo,
                           qmask, &misc_i[3], g, eps2, perm, core, parent);
        DBSCAN_HIP_CHECK(hipGetLastError());
    } else if (nf > 0) {
        StageTimer t(prof, s, "union");
        hipLaunchKernelGGL(union_kernel, dim3(nblk(nf)), dim3(kBlock), 0, s, xy, cell, seg, nf,
                           eps2, perm, core, parent);
        DBSCAN_HIP_CHECK(hipGetLastError());
    }
    int64_t k = 0;
    if (!a.zone) {
        uint8_t* is_root = static_cast<uint8_t*>(ws.is_root.ensure(n));
        int32_t* rank = static_cast<int32_t*>(ws.rank.ensure(n * sizeof(int32_t)));
        {
            StageTimer t(prof, s, "final");
            DBSCAN_HIP_CHECK(hipMemsetAsync(is_root, 0, n, s));
            hipLaunchKernelGGL(final_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n, perm, core,
                               parent, lab, is_root);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        {
            StageTimer t(prof, s, "rank");
            exclusive_scan(s, 1, is_root, rank, n, &misc_i[1], ws.scan_tmp);
        }
        {
            StageTimer t(prof, s, "output");
            hipLaunchKernelGGL(output_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, xy, cell, seg, n,
                               nf, eps2, a.mode, perm, core, lab, rank, a.cluster, a.flag);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        int32_t hv[3];
        DBSCAN_HIP_CHECK(hipMemcpyAsync(hv, misc_i, sizeof(hv), hipMemcpyDeviceToHost, s));
        DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
        k = hv[1];
        stats.ncells = nf > 0 ? hv[0] : 0;
        stats.ncore = hv[2];
    } else {
        {
            StageTimer t(prof, s, "final");
            hipLaunchKernelGGL(final_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n, perm, core,
                               parent, lab, (uint8_t*)nullptr);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        {
            StageTimer t(prof, s, "output");
            hipLaunchKernelGGL(slab_roots_kernel, dim3(nblk(n)), dim3(kBlock), 0, s, n, perm,
                               core, lab, a.core_out, a.root_out);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        int32_t hv[3];
        DBSCAN_HIP_CHECK(hipMemcpyAsync(hv, misc_i, sizeof(hv), hipMemcpyDeviceToHost, s));
        DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
        stats.ncells = nf > 0 ? hv[0] : 0;
        stats.ncore = hv[2];
    }
    stats.nclusters = k;
    if (st) *st = stats;
    if (slab) {
        slab->valid = a.zone != nullptr;
        slab->n = n;
        slab->nf = nf;
        slab->eps2 = eps2;
    }
    return k;
}

void run_slab_label(hipStream_t s, Workspace& ws, Profiler* prof, const SlabState& st,
                    const uint8_t* zone, const int64_t* gid, const int64_t* gs_of_root,
                    const int32_t* label_of_root, int32_t mode, int32_t* cluster,
                    uint8_t* flag) {
    if (!st.valid) throw ArgError{"dbscan_slab_label_device: no slab fit on this handle"};
    if (st.n == 0) return;
    StageTimer t(prof, s, "slab_label");
    hipLaunchKernelGGL(slab_label_kernel, dim3(nblk(st.n)), dim3(kBlock), 0, s,
                       static_cast<const double2*>(ws.xy.p), static_cast<const int32_t*>(ws.cell.p),
                       static_cast<const Seg*>(ws.seg.p), st.n, st.nf, st.eps2, mode,
                       static_cast<const int32_t*>(ws.perm_sorted),
                       zone, static_cast<const uint8_t*>(ws.core.p),
                       static_cast<const int32_t*>(ws.lab.p), gid, gs_of_root, label_of_root,
                       cluster, flag);
    DBSCAN_HIP_CHECK(hipGetLastError());
    DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace dbscan
