// batch.hip -- an executor's partitions fitted as ONE tiled fit (dbscan_fit_batch*).
//
// DBSCAN.scala:150-155 runs `new LocalDBSCANNaive(eps, minPoints).fit(points)` once per spatial
// partition (<= maxPointsPerPartition points plus the eps halo of DBSCAN.scala:116-137).  One
// tiled fit per partition is ~45 launches for a few thousand points; instead every partition of
// a batch gets its own eps grid -- origin at its bbox minimum, the cell side a single fit would
// use (make_grid in fit.hip, never grown) -- and the grids are placed side by side in one virtual
// tile grid (shelves of tile rectangles).  Each rectangle is tile-aligned and holds at least one
// empty cell column and row after its cells, so no cell of one partition is in another's 3x3
// stencil and no pair across partitions is ever tested.  The fit then runs once over the whole
// batch: the sort key is the virtual tile | cell | quadrant, the fp32 cell-unit records of a tile
// are taken against its partition's origin (tile_org), visit order is the batch order (each
// partition's own order, partitions in sequence), and cluster ids are numbered per partition
// (permute_out_batch_kernel).  Results equal one fit per partition bit for bit.
#include "internal.h"

#include <algorithm>
#include <cmath>

namespace dbscan {
namespace {

constexpr int kBoxBlock = 256;

__device__ __forceinline__ double bmin(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double bmax(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

// One workgroup per partition (grid stride): min/max of the finite points and their count.
__global__ __launch_bounds__(kBoxBlock) void part_bbox_kernel(const double* __restrict__ x,
                                                              const double* __restrict__ y,
                                                              const int64_t* __restrict__ offs,
                                                              int np, double* __restrict__ out) {
    __shared__ double red[5][kBoxBlock / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int p = blockIdx.x; p < np; p += gridDim.x) {
        const int64_t a = offs[p], b = offs[p + 1];
        double mnx = INFINITY, mxx = -INFINITY, mny = INFINITY, mxy = -INFINITY, c = 0;
        for (int64_t i = a + threadIdx.x; i < b; i += kBoxBlock) {
            const double u = x[i], v = y[i];
            if (__builtin_isfinite(u) && __builtin_isfinite(v)) {
                mnx = fmin(mnx, u);
                mxx = fmax(mxx, u);
                mny = fmin(mny, v);
                mxy = fmax(mxy, v);
                c += 1.0;
            }
        }
        mnx = bmin(mnx);
        mxx = bmax(mxx);
        mny = bmin(mny);
        mxy = bmax(mxy);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if (lane == 0) {
            red[0][w] = mnx;
            red[1][w] = mxx;
            red[2][w] = mny;
            red[3][w] = mxy;
            red[4][w] = c;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double r[5] = {red[0][0], red[1][0], red[2][0], red[3][0], red[4][0]};
            for (int k = 1; k < kBoxBlock / 64; ++k) {
                r[0] = fmin(r[0], red[0][k]);
                r[1] = fmax(r[1], red[1][k]);
                r[2] = fmin(r[2], red[2][k]);
                r[3] = fmax(r[3], red[3][k]);
                r[4] += red[4][k];
            }
            for (int k = 0; k < 5; ++k) out[(int64_t)p * 5 + k] = r[k];
        }
        __syncthreads();
    }
}

}  // namespace

void enqueue_batch_bbox(hipStream_t s, const double* x, const double* y, const int64_t* d_offs,
                        int32_t n_parts, double* d_box) {
    if (n_parts <= 0) return;
    hipLaunchKernelGGL(part_bbox_kernel, dim3((unsigned)std::min<int32_t>(n_parts, 8192)),
                       dim3(kBoxBlock), 0, s, x, y, d_offs, (int)n_parts, d_box);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

bool plan_batch_grid(const double* box, const int64_t* offs, int32_t n_parts, double eps,
                     PartGrid* table, BatchFit* bf, std::vector<int32_t>* alone) {
    alone->clear();
    // the cell side of make_grid (fit.hip) before any growth: h >= R*(1+2^-16) bounds every
    // accepted pair's offset; quarter cells are cliques while h <= |eps|*(1+2^-14)
    double R = std::fabs(eps) * (1.0 + 0x1p-40);
    if (R < 0x1p-500) R = 0x1p-500;
    const double h = R * (1.0 + 0x1p-16);
    const double inv = 2.0 / h;
    const bool clique = h <= std::fabs(eps) * (1.0 + 0x1p-14);
    const double eps2 = eps * eps;
    if (!clique || !std::isfinite(eps2) || !std::isfinite(inv)) {
        for (int32_t p = 0; p < n_parts; ++p) alone->push_back(p);
        return false;
    }
    // each partition's local grid and its tile rectangle (cells + one empty column / row)
    std::vector<int64_t> tw((size_t)n_parts, 0), th((size_t)n_parts, 0);
    int64_t area = 0, widest = 1;
    int64_t nf = 0;
    for (int32_t p = 0; p < n_parts; ++p) {
        const double* b = box + (size_t)p * 5;
        PartGrid& P = table[p];
        P = PartGrid{0, 0, 0, 0, 0, 0};
        const int64_t m = offs[p + 1] - offs[p];
        if (b[4] <= 0) continue;  // no finite point: every point is outside the grid
        const double cx = std::floor((b[1] * 0.5 - b[0] * 0.5) * inv) + 1.0;
        const double cy = std::floor((b[3] * 0.5 - b[2] * 0.5) * inv) + 1.0;
        // a sparse extent (outliers far from the rest) would spend a big empty rectangle of
        // the virtual grid: such a partition is fitted on its own (its grid may grow there)
        const double tiles = std::ceil((cx + 1.0) / 8.0) * std::ceil((cy + 1.0) / 8.0);
        if (!(cx <= 65536.0 && cy <= 65536.0) || tiles > std::max(4096.0, (double)m)) {
            alone->push_back(p);
            continue;
        }
        P.xmin2 = b[0] * 0.5;
        P.ymin2 = b[2] * 0.5;
        P.nx = (int32_t)cx;
        P.ny = (int32_t)cy;
        tw[(size_t)p] = (int64_t)std::ceil((cx + 1.0) / 8.0);
        th[(size_t)p] = (int64_t)std::ceil((cy + 1.0) / 8.0);
        area += tw[(size_t)p] * th[(size_t)p];
        widest = std::max(widest, tw[(size_t)p]);
        nf += (int64_t)b[4];
    }
    if (nf == 0) {  // nothing to place: every partition (empty, all non-finite, sparse) alone
        alone->clear();
        for (int32_t p = 0; p < n_parts; ++p) alone->push_back(p);
        return false;
    }
    // shelves: rows of rectangles, a row as wide as the square root of the total area
    const int64_t W = std::max<int64_t>(widest, (int64_t)std::ceil(std::sqrt((double)area)));
    int64_t x = 0, y = 0, row_h = 0;
    for (int32_t p = 0; p < n_parts; ++p) {
        if (tw[(size_t)p] == 0) continue;
        if (x + tw[(size_t)p] > W) {
            y += row_h;
            x = 0;
            row_h = 0;
        }
        table[p].cx0 = (int32_t)(8 * x);
        table[p].cy0 = (int32_t)(8 * y);
        x += tw[(size_t)p];
        row_h = std::max(row_h, th[(size_t)p]);
    }
    const int64_t ntx = W, nty = y + row_h;
    if (ntx * nty > kMaxGridTiles || 8 * std::max(ntx, nty) > (int64_t)INT32_MAX / 4) {
        alone->clear();
        for (int32_t p = 0; p < n_parts; ++p) alone->push_back(p);
        return false;
    }
    GridParams g{0, 0, inv, inv, (uint32_t)(8 * ntx), (uint32_t)(8 * nty), (uint32_t)ntx,
                 (uint32_t)nty, 1};
    g.nparts = n_parts;
    bf->g = g;
    bf->nf = (int32_t)nf;
    const uint64_t nkeys = 256ull * (uint64_t)ntx * (uint64_t)nty;
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= nkeys) ++bits;
    bf->bits = bits;
    return true;
}

}  // namespace dbscan
