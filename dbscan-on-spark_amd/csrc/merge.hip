// merge.hip -- the exact cross-slab merge of the multi-GPU node path (dbscan_amd/node.py), as
// device kernels on the caller's stream.  Replaces the reference's driver-side merge:
//   DBSCAN.scala:158-222   band points, findAdjacencies, DBSCANGraph connected components,
//                          global cluster ids
// with a lock-free union-find over GLOBAL visit indices (gids).  Every rank gathers the records
// (a, b) = (gid of a shared core point, gid of its local root on the emitting rank; b < 0: the
// shared point is not core there) of all ranks and runs the same union on its own GPU:
//   merge_init      parent[a] = a, parent[b] = b for every valid record
//   merge_union     unite(a, b): CAS hook of the larger root under the smaller, so a root is
//                   the smallest gid of its component = s(K), the reference's opening order
//   merge_compress  parent[x] = root(x) for every node
// parent is a dense int32 array over gids (the job's n_total points), -1 = untouched; the
// touched entries are reset after use (merge_reset), so a step costs O(records), not O(n_total).
// run_slab_merge_roots then gives every local root its global s(K) and lists the zone-0 ones
// that are global roots (owned by this rank) for the cluster numbering.
#include "../../include/dbscan_hip.h"
#include "internal.h"

namespace dbscan {
namespace {

__device__ __forceinline__ int32_t mfind(const int32_t* __restrict__ par, int32_t x) {
    for (int32_t p = par[x]; p != x; p = par[x]) x = p;
    return x;
}

__global__ __launch_bounds__(kBlock) void merge_init_kernel(const int64_t* __restrict__ a,
                                                            const int64_t* __restrict__ b,
                                                            int64_t m, int32_t* __restrict__ par) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m || b[i] < 0) return;
    par[a[i]] = (int32_t)a[i];
    par[b[i]] = (int32_t)b[i];
}

__global__ __launch_bounds__(kBlock) void merge_union_kernel(const int64_t* __restrict__ a,
                                                             const int64_t* __restrict__ b,
                                                             int64_t m, int32_t* __restrict__ par) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m || b[i] < 0) return;
    int32_t ra = (int32_t)a[i], rb = (int32_t)b[i];
    for (;;) {
        ra = mfind(par, ra);
        rb = mfind(par, rb);
        if (ra == rb) return;
        const int32_t hi = ra > rb ? ra : rb, lo = ra > rb ? rb : ra;
        int32_t expected = hi;
        if (__hip_atomic_compare_exchange_strong(par + hi, &expected, lo, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
        ra = expected;  // hi was hooked meanwhile: retry from its new parent
        rb = lo;
    }
}

__global__ __launch_bounds__(kBlock) void merge_compress_kernel(const int64_t* __restrict__ a,
                                                                const int64_t* __restrict__ b,
                                                                int64_t m,
                                                                int32_t* __restrict__ par) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m || b[i] < 0) return;
    const int32_t x = (int32_t)a[i], y = (int32_t)b[i];
    par[x] = mfind(par, x);
    par[y] = mfind(par, y);
}

__global__ __launch_bounds__(kBlock) void merge_reset_kernel(const int64_t* __restrict__ a,
                                                             const int64_t* __restrict__ b,
                                                             int64_t m, int32_t* __restrict__ par) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m || b[i] < 0) return;
    par[a[i]] = -1;
    par[b[i]] = -1;
}

// Local roots of a slab fit (root[p] == p: a zone 0/1 core that is the minimum-index core of
// its local component): gs_of_root[p] = global s(K), the merged root of gid[p] (or gid[p] when
// no record touched it).  Zone-0 local roots whose s(K) is their own gid are the global roots
// owned by this rank; they are compacted in slab order (= increasing gid) by an ordered
// three-kernel compaction -- per-block counts, a scan, a ballot-ranked write -- since the few
// thousand same-address atomics of an append would serialize (~25 ns each).
constexpr int kRootTile = 4096;  // slab points per block (16 rounds of 256)

// 0: not a local root; 1: a local root (gs_of_root[p] written when given); 3: also a zone-0
// global root owned here (g = its gid).
__device__ __forceinline__ int root_kind_at(int64_t p, int64_t n, const uint8_t* __restrict__ zone,
                                            const int64_t* __restrict__ gid,
                                            const int32_t* __restrict__ root,
                                            const int32_t* __restrict__ par,
                                            int64_t* __restrict__ gs_of_root, int64_t& g) {
    if (p >= n || root[p] != (int32_t)p) return 0;
    g = gid[p];
    const int32_t pg = par[g];
    const int64_t gs = pg >= 0 ? (int64_t)pg : g;
    if (gs_of_root) gs_of_root[p] = gs;
    return zone[p] == 0 && gs == g ? 3 : 1;
}

// Per block: the owned global roots (blockcnt[b]) and all local roots (blockcnt[nb + b]); one
// scan over both rows gives the two compactions' offsets (the second row's shifted by the
// owned total, offs[nb]).
__global__ __launch_bounds__(kBlock) void roots_count_kernel(
    int64_t n, const uint8_t* __restrict__ zone, const int64_t* __restrict__ gid,
    const int32_t* __restrict__ root, const int32_t* __restrict__ par,
    int64_t* __restrict__ gs_of_root, int32_t* __restrict__ blockcnt) {
    __shared__ int wsum[2][kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kRootTile;
    int c = 0, a = 0;
    for (int r = 0; r < kRootTile / kBlock; ++r) {
        int64_t g;
        const int k = root_kind_at(base + r * kBlock + threadIdx.x, n, zone, gid, root, par,
                                   gs_of_root, g);
        c += k >> 1;
        a += k & 1;
    }
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o, 64);
        a += __shfl_xor(a, o, 64);
    }
    if (__lane_id() == 0) {
        wsum[0][threadIdx.x >> 6] = c;
        wsum[1][threadIdx.x >> 6] = a;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        int t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += wsum[threadIdx.x][w];
        blockcnt[threadIdx.x * gridDim.x + blockIdx.x] = t;
    }
}

// Ballot-ranked ordered writes of both lists (lroots == nullptr: the owned list only); block 0
// also copies the two totals next to each other (totals[0] owned, totals[1] owned + local).
__global__ __launch_bounds__(kBlock) void roots_write_kernel(
    int64_t n, const uint8_t* __restrict__ zone, const int64_t* __restrict__ gid,
    const int32_t* __restrict__ root, const int32_t* __restrict__ par,
    const int32_t* __restrict__ blockoff, int64_t* __restrict__ own_roots,
    int32_t* __restrict__ lroots, int32_t* __restrict__ totals) {
    __shared__ int wcnt[2][2][kBlock / 64];
    const int nb = gridDim.x;
    const int64_t base = (int64_t)blockIdx.x * kRootTile;
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (blockIdx.x == 0 && threadIdx.x < 2) totals[threadIdx.x] = blockoff[(threadIdx.x + 1) * nb];
    int off = blockoff[blockIdx.x], offl = blockoff[nb + blockIdx.x] - blockoff[nb];
    for (int r = 0; r < kRootTile / kBlock; ++r) {
        int64_t g = 0;
        const int64_t p = base + r * kBlock + threadIdx.x;
        const int k = root_kind_at(p, n, zone, gid, root, par, nullptr, g);
        const uint64_t b = __ballot(k == 3), bl = __ballot(k != 0);
        if (lane == 0) {
            wcnt[r & 1][0][w] = __popcll(b);
            wcnt[r & 1][1][w] = __popcll(bl);
        }
        __syncthreads();
        int before = 0, total = 0, beforel = 0, totall = 0;
#pragma unroll
        for (int v = 0; v < kBlock / 64; ++v) {
            const int c = wcnt[r & 1][0][v], cl = wcnt[r & 1][1][v];
            before += v < w ? c : 0;
            total += c;
            beforel += v < w ? cl : 0;
            totall += cl;
        }
        if (k == 3) own_roots[off + before + __popcll(b & lt)] = g;
        if (k != 0 && lroots) lroots[offl + beforel + __popcll(bl & lt)] = (int32_t)p;
        off += total;
        offl += totall;
    }
}

inline unsigned blocks(int64_t m) { return (unsigned)((m + kBlock - 1) / kBlock); }

}  // namespace
}  // namespace dbscan

namespace dbscan {

int64_t run_slab_merge_roots(hipStream_t s, Workspace& ws, int64_t n, const uint8_t* zone,
                             const int64_t* gid, const int32_t* root, const int32_t* parent,
                             int64_t* gs_of_root, int64_t* own_roots) {
    int32_t total = 0;
    enqueue_slab_merge_roots(s, ws, n, zone, gid, root, parent, gs_of_root, own_roots, &total,
                             nullptr);
    if (n > 0) DBSCAN_HIP_CHECK(hipStreamSynchronize(s));
    return total;
}

void enqueue_slab_merge_roots(hipStream_t s, Workspace& ws, int64_t n, const uint8_t* zone,
                              const int64_t* gid, const int32_t* root, const int32_t* parent,
                              int64_t* gs_of_root, int64_t* own_roots, int32_t* total_dst,
                              int32_t* lroots) {
    if (n == 0) {
        total_dst[0] = 0;
        if (lroots) total_dst[1] = 0;
        return;
    }
    const int64_t nb = (n + kRootTile - 1) / kRootTile;
    int32_t* cnt = static_cast<int32_t*>(ws.own_flag.ensure((4 * nb + 4) * sizeof(int32_t)));
    int32_t* off = cnt + 2 * nb + 1;
    int32_t* totals = off + 2 * nb + 1;
    hipLaunchKernelGGL(roots_count_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, n, zone, gid,
                       root, parent, gs_of_root, cnt);
    DBSCAN_HIP_CHECK(hipGetLastError());
    exclusive_scan(s, 0, cnt, off, 2 * nb, off + 2 * nb, ws.scan);
    hipLaunchKernelGGL(roots_write_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, n, zone, gid,
                       root, parent, off, own_roots, lroots, totals);
    DBSCAN_HIP_CHECK(hipGetLastError());
    DBSCAN_HIP_CHECK(hipMemcpyAsync(total_dst, totals, (lroots ? 2 : 1) * sizeof(int32_t),
                                    hipMemcpyDeviceToHost, s));
}

}  // namespace dbscan

namespace {
template <class F>
int32_t run_guarded(F&& f) {
    dbscan::set_last_error("");
    try {
        f();
        return DBSCAN_OK;
    } catch (const dbscan::HipError& e) {
        dbscan::set_last_error(e.what);
        return DBSCAN_EHIP;
    }
}
}  // namespace

extern "C" {

int32_t dbscan_merge_union_device(const int64_t* d_a, const int64_t* d_b, int64_t m,
                                  int32_t* d_parent, void* stream) {
    if (m < 0 || (m > 0 && (!d_a || !d_b || !d_parent))) return DBSCAN_EARG;
    if (m == 0) return DBSCAN_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    return run_guarded([&] {
        using namespace dbscan;
        hipLaunchKernelGGL(merge_init_kernel, dim3(blocks(m)), dim3(kBlock), 0, s, d_a, d_b, m,
                           d_parent);
        hipLaunchKernelGGL(merge_union_kernel, dim3(blocks(m)), dim3(kBlock), 0, s, d_a, d_b, m,
                           d_parent);
        hipLaunchKernelGGL(merge_compress_kernel, dim3(blocks(m)), dim3(kBlock), 0, s, d_a, d_b,
                           m, d_parent);
        DBSCAN_HIP_CHECK(hipGetLastError());
    });
}

int32_t dbscan_merge_reset_device(const int64_t* d_a, const int64_t* d_b, int64_t m,
                                  int32_t* d_parent, void* stream) {
    if (m < 0 || (m > 0 && (!d_a || !d_b || !d_parent))) return DBSCAN_EARG;
    if (m == 0) return DBSCAN_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    return run_guarded([&] {
        using namespace dbscan;
        hipLaunchKernelGGL(merge_reset_kernel, dim3(blocks(m)), dim3(kBlock), 0, s, d_a, d_b, m,
                           d_parent);
        DBSCAN_HIP_CHECK(hipGetLastError());
    });
}

}  // extern "C"
