// internal.h -- shared declarations of libdbscan_hip.so (gfx950 only).
//
// Device data layout (one fit, n points, nf finite points in the eps grid):
//   key[n]   u32 tile<<8 | cell-in-tile<<2 | quadrant, tiles of 8x8 eps cells row-major over
//            the grid (0xFFFFFFFF for points outside the grid)                -> radix sorted
//   perm[n]  i32 input index of each sorted slot (the reference's visit index)
//   xy[nf]   double2 sorted coordinates, SoA->AoS so one 16-B load feeds a candidate test
//   cell[nf] i32 occupied-cell index of each sorted slot
//   ckey[C], cstart[C+1]  occupied cells (key >> 2) and their first slot
//   tkey[T], tstart[T+1]  occupied tiles (key >> 8) and their first slot
//   tmap[ntx*nty]  occupied-tile index of every tile of the grid (-1: empty)
//   tslot[T][65]   first slot of the first occupied cell with local index >= l
//   tstage[T][100]  (first slot, count) of the 10x10 cells of each tile + its 1-cell halo
//   tq[T][65], tnb[T]  the tslot table over quarter indices; E/S/SE/SW neighbour tiles
//   seg[C]   64 B: <= 6 slot pieces of the 3x3 stencil + the own cell range
//   qidx[nf], qkey[Q], qstart[Q+1]  quarter cells (2x2 per eps cell; key low 2 bits =
//            quadrant): side ~eps/2, so each is a clique under the exact predicate
//   qrep[Q]  int4 (begin, end, minimum-visit-index core or -1, core mask); qmask[Q] int2
//            quarter-grid coordinates
//   nbr[nf][minPoints-1]  slots of each non-core's neighbours (-1 terminated), minPoints <= 12
//   core[n]  u8, parent[n] i32 (union-find over slots, hooked by visit index), lab[n] i32
//   is_root[ceil(n/64)] u64 root bits over INPUT order and rank[ceil(n/64)] i32 their per-word
//   exclusive popcount prefix: rank(o) = rank[o>>6] + popc(is_root[o>>6] below bit o&63)
//   inv[n]   i32 sorted slot of each input index (inverse of perm)
//   packed[n] u32 per sorted slot: (cluster << 1) | core, moved to input order through inv
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dbscan_hip.h"

#include <string>
#include <vector>

namespace dbscan {

constexpr uint32_t kSentinelKey = 0xFFFFFFFFu;
constexpr int kBlock = 256;
constexpr int64_t kMaxGridTiles = int64_t(1) << 23;  // 8x8-cell tiles per grid (u32 keys)
// Partitions of at most this many points are fitted by ONE workgroup in LDS (small.hip)
constexpr int64_t kSmallMaxPoints = 8192;

// Device-side fit state (ints after the grid in the handle's misc buffer), written by kernels
// and read back by the host only when it synchronizes.
enum FitState {
    kStCells = 0,     // occupied eps cells
    kStClusters = 1,  // clusters of a full fit
    kStCore = 2,      // core points
    kStQuarters = 3,  // occupied quarter cells
    kStTiles = 4,     // occupied tiles
    kStNf = 6,        // points inside the grid (finite coordinates)
    kStBits = 7,      // radix key width
    kStError = 8,     // the eps grid could not be sized
    kStTileLists = 9,  // [3] clique-grid tiles per count path: small, medium, big
    kStClassPts = 12,  // [3] their own points (what each count kernel processes)
    kStBoxEdges = 15,  // archery float32 box: one-way core-core pairs recorded
    kStTileBuckets = 16,  // [<= 16] small, medium tiles per stage-size bucket (tile_class_kernel)
    kStCount = 32
};

#define DBSCAN_HIP_CHECK(expr)                                                              \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) throw ::dbscan::HipError(_e, #expr, __FILE__, __LINE__);     \
    } while (0)

struct HipError {
    hipError_t err;
    std::string what;
    HipError(hipError_t e, const char* expr, const char* file, int line);
};

struct ArgError {
    std::string what;
};

// The thread-local message behind dbscan_last_error().
void set_last_error(const std::string& s);

// Grow-only device buffer (owned by one handle; never copied).
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    void* ensure(size_t need);
    void release();
    ~DevBuf() { release(); }
};

// Timing with events on the fit stream.  mode 1 (stages): an event pair brackets every pipeline
// stage (each hipEventRecord between kernels costs ~10 us of idle GPU: 26 stage boundaries add
// 0.24 ms to a 2.65 ms fit).  mode 2 (kernels): the events ride on the dispatch packets of the
// kernels themselves (hipExtLaunchKernelGGL), one pair per kernel launch, with no extra packets
// between kernels -- the form bench.py times with.
struct Profiler {
    bool on = false;
    int mode = 0;
    std::string only;  // kernel mode: time only the launches of this kernel ("" = all)
    struct Stage {
        std::string name;
        double ms = 0;
        int64_t launches = 0;
    };
    std::vector<Stage> stages;
    struct Pending {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    hipEvent_t take();
    int stage_index(const char* name);
    void flush();  // after the stream is synchronized: accumulate and recycle events
    void flush_ready();  // the same for the completed pairs only (the stream may still run)
    void destroy();
};

// A kernel launch, timed by packet events in kernel-profiling mode.
template <typename F, typename... Args>
void klaunch(Profiler* prof, const char* name, F kernel, dim3 grid, dim3 block, uint32_t shmem,
             hipStream_t s, Args... args) {
    if (prof && prof->on && prof->mode == 2 && (prof->only.empty() || prof->only == name)) {
        hipEvent_t a = prof->take(), b = prof->take();
        hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, a, b, 0, args...);
        prof->pending.push_back({prof->stage_index(name), a, b});
    } else {
        hipLaunchKernelGGL(kernel, grid, block, shmem, s, args...);
    }
}

// RAII bracket around one stage's launches (stage-profiling mode only).
struct StageTimer {
    Profiler* prof;
    hipStream_t s;
    int stage = -1;
    hipEvent_t a = nullptr;
    StageTimer(Profiler* p, hipStream_t st, const char* name);
    ~StageTimer();
};

// Look-back state of the single-pass scan: state[0] a watchdog flag, then one status word per
// tile; the epoch distinguishes successive scans so the words need clearing only on fresh
// memory or when the 30-bit epoch wraps.
struct ScanState {
    DevBuf buf;
    uint32_t epoch = 0;
    uint64_t* prepare(hipStream_t s, int64_t ntiles);  // also advances the epoch
};

// Bucketed sort (fits of >= kBucketMinPoints points, whose arrays outgrow the Infinity Cache):
// one MSD pass on the top 8 key bits into padded per-band segments, each point's record (x, y,
// input index) moved to its padded place, then LSD passes inside the segments.  Outputs:
// key_fin[n] sorted keys, slot_place[n] the padded place of each sorted slot, rec[place] the
// record there, pos[i] the padded place of input i; np padded places.
// Threshold 2^23 (A/B against 2^20 and 2^24: at 10^7 points a wash, at config 3's share
// 2.63 -> 2.52 ms).
constexpr int64_t kBucketMinPoints = int64_t(1) << 23;
struct BucketSort {
    DevBuf ka, kb, jb, kc, jc, recb, posb, kf, jf, tab;
    uint32_t* key_fin = nullptr;
    int32_t* slot_place = nullptr;
    double4* rec = nullptr;
    int32_t* pos = nullptr;
    int64_t np = 0;
    void release() {
        for (DevBuf* b : {&ka, &kb, &jb, &kc, &jc, &recb, &posb, &kf, &jf, &tab}) b->release();
    }
};

struct GridParams;

struct Workspace {
    DevBuf key, key2, perm, perm2, hist, scan_tmp, xy, cell, ckey, cstart, seg, core, parent, lab,
        is_root, rank, misc, qidx, qkey, qstart, qrep, qmask, blockcnt, heads, tkey, tstart, tmap,
        tslot, qcomp, nbr, tq, tnb, tstage, inv, packed, slab_lor, own_flag, bigt, zs, tclass, tsz,
        key3, perm3, lroots, box_edges, box_map, tcore, tpart, pbox, ptab, shm, route, route_tab,
        spread, band;
    bool spread_ready = false;  // spread.p holds zeroed barrier words (small.hip)
    double* stats_host = nullptr;  // pinned: the stats block read_fit_stats copies back
    bool fit_mirrored = false;     // the last fit (an LDS form) wrote its stats into fit_block
    bool out_direct = false;       // ... and its labels into FitArgs::cluster_host / flag_host
    bool nk_written = false;       // the last fit (tiled) wrote its count to FitArgs::n_clusters_dev
    // Every LDS fit (small.hip: one-workgroup, spread and band forms) writes its statistics,
    // kStError included, into a pinned block of its OWN, taken from a ring: fits queued back to
    // back on the stream never share one, so each one's outcome survives until the host reads
    // it.  A block is reused only after the stream has drained since it was taken.
    static constexpr int kStatRing = 64;
    // block stride, doubles: the misc block's layout up to the whole FitState (kStCount ints
    // from kMiscState, which the LDS kernels zero: 320 B, past a 32-double copy's 256 B)
    static constexpr int kStatBlock = 64;
    double* ring_host = nullptr;   // kStatRing blocks of kStatBlock doubles
    double* ring_dev = nullptr;    // ... their device address
    int ring_next = 0;             // the next block to take
    int ring_used = 0;             // blocks taken since the stream last drained
    double* fit_block = nullptr;   // the last LDS fit's block (host address)
    // A spread or band fit queued and not checked yet: when a grid barrier of it gave up
    // (kStError 2: its workgroups were not all resident) or a band overflowed its staging (3),
    // drain_recalls re-runs it (one-workgroup kernel / tiled pipeline: the same results bit for
    // bit) into its own outputs.  Every queued fit has its own record, checked in stream order.
    struct Recall {
        bool band = false;
        const double *x = nullptr, *y = nullptr;
        int64_t n = 0;
        double eps = 0.0;
        int32_t min_points = 0, mode = 0;
        int32_t* cluster = nullptr;  // where the fit wrote its labels (may be host-mapped)
        uint8_t* flag = nullptr;
        int32_t* dev_cluster = nullptr;  // direct fits: device twins a re-run writes into, then
        uint8_t* dev_flag = nullptr;     // ... copied to cluster / flag in one DMA (or nullptr)
        int32_t* nk = nullptr;           // device word its cluster count was copied to
        double* block_host = nullptr;    // its stats block
        double* block_dev = nullptr;
    };
    std::vector<Recall> recalls;
    bool band_ready = false;                // band.p holds zeroed barrier words (small.hip)
    uint32_t spread_spin_limit = 1u << 21;  // barrier polls before giving up (0: at once; tests)
    int64_t spread_fallbacks = 0;           // spread / band fits re-run (drain_recalls)
    bool spread_recovered = false;          // the last read_fit_stats re-ran the last fit
    Workspace() = default;
    ~Workspace() {
        if (stats_host) (void)hipHostFree(stats_host);
        if (ring_host) (void)hipHostFree(ring_host);
    }
    ScanState scan;
    BucketSort bucket;  // the bucketed sort's buffers (large fits only)
    int64_t fit_n = 0;               // the last enqueued fit
    int fit_mode = 0;
    int32_t* perm_sorted = nullptr;  // perm or perm2, whichever holds the sorted order
    uint32_t* key_sorted = nullptr;  // key or key2, likewise
    void release() {
        scan.buf.release();
        bucket.release();
        for (DevBuf* b : {&key, &key2, &perm, &perm2, &hist, &scan_tmp, &xy, &cell, &ckey, &cstart,
                          &seg, &core, &parent, &lab, &is_root, &rank, &misc, &qidx, &qkey,
                          &qstart, &qrep, &qmask, &blockcnt, &heads, &tkey, &tstart, &tmap, &tslot,
                          &qcomp, &nbr, &tq, &tnb, &tstage, &inv, &packed, &slab_lor,
                          &own_flag, &bigt, &zs, &tclass, &tsz, &key3, &perm3, &lroots,
                          &box_edges, &box_map, &tcore, &tpart, &pbox, &ptab, &shm, &route,
                          &route_tab, &spread, &band})
            b->release();
        spread_ready = false;
        band_ready = false;
        if (stats_host) (void)hipHostFree(stats_host);
        stats_host = nullptr;
        if (ring_host) (void)hipHostFree(ring_host);
        ring_host = ring_dev = fit_block = nullptr;
        ring_next = ring_used = 0;
        recalls.clear();
    }
};

// Batched fits (batch.hip): each partition of a batch gets its own eps grid (origin at its bbox
// minimum, the common cell side), placed in one virtual tile grid at a tile-aligned cell offset
// with at least one empty cell row and column after it, so no 3x3 stencil ever reaches another
// partition and ONE tiled fit serves the whole batch.
struct PartGrid {
    double xmin2, ymin2;  // local origin: cell = floor((v*0.5 - vmin2) * inv) + c0
    int32_t cx0, cy0;     // virtual cell offset of the partition's local cell (0, 0)
    int32_t nx, ny;       // local cells per axis; 0: the partition's points are not binned
};

struct GridParams {
    double xmin2, ymin2, invx, invy;  // cell = floor((v*0.5 - vmin*0.5) * inv)
    uint32_t nx, ny;                  // eps cells per axis
    uint32_t ntx, nty;                // 8x8-cell tiles per axis
    int clique;  // cell side <= eps*(1+2^-14): quarter cells are cliques of the predicate
    // batched fits: nparts > 0 partitions [poffs[p], poffs[p+1]) each binned on parts[p]'s grid
    // (xmin2/ymin2 above unused)
    int32_t nparts = 0;
    const PartGrid* parts = nullptr;
    const int64_t* poffs = nullptr;
};

// The sort key of a point on a fit's own grid (not batched): tile << 8 | cell-in-tile << 2 |
// quadrant, the sentinel for a non-finite point.  bin_kernel and the bucketed sort's MSD pass
// (which bins on the fly instead of reading bin_kernel's keys) share it.
// (Scalars, not a GridParams reference: a reference to a kernel's local copy of the struct put
// that copy in scratch memory, bin_kernel 0.035 -> 0.18 ms per 10^7 points.)
__device__ __forceinline__ uint32_t grid_key(double a, double b, double xmin2, double ymin2,
                                             double invx, double invy, uint32_t nx, uint32_t ny,
                                             uint32_t ntx) {
    if (!__builtin_isfinite(a) || !__builtin_isfinite(b)) return kSentinelKey;
    const double mx = 2.0 * (double)nx - 1.0, my = 2.0 * (double)ny - 1.0;
    // quarter-grid coordinates: floor(2t) >> 1 == floor(t) exactly (2t is exact)
    double fx = floor(2.0 * ((a * 0.5 - xmin2) * invx));
    double fy = floor(2.0 * ((b * 0.5 - ymin2) * invy));
    fx = fx < 0 ? 0 : (fx > mx ? mx : fx);
    fy = fy < 0 ? 0 : (fy > my ? my : fy);
    const uint32_t qx = (uint32_t)fx, qy = (uint32_t)fy;
    const uint32_t cx = qx >> 1, cy = qy >> 1;
    const uint32_t tile = (cy >> 3) * ntx + (cx >> 3);
    const uint32_t local = ((cy & 7u) << 3) | (cx & 7u);
    return (tile << 8) | (local << 2) | ((qy & 1u) << 1) | (qx & 1u);
}

// What enqueue_fit needs for a batched fit (planned on the host by plan_batch_grid).
struct BatchFit {
    GridParams g;                // the virtual grid (nparts, parts, poffs set)
    int32_t nf = 0, bits = 0;    // points inside the grid, radix key width
    int32_t* nclusters = nullptr;  // out (device): cluster count per partition
};

struct FitStats {
    int64_t n = 0, nf = 0, ncells = 0, ncore = 0, nclusters = 0, nx = 0, ny = 0, bits = 0,
            grid_mode = 0, ntiles = 0, clique = 0, pts_small = 0, pts_medium = 0, pts_big = 0;
};

// One fit.  Full fits (zone == nullptr) write cluster/flag in input order and return the
// cluster count; slab fits (zone != nullptr) write core_out/root_out and keep their grid in the
// workspace for run_slab_label.
struct FitArgs {
    const double* x;
    const double* y;
    const uint8_t* zone;
    int64_t n;
    double eps;
    int32_t min_points;
    int32_t mode;
    int32_t* cluster;
    uint8_t* flag;
    uint8_t* core_out;
    int32_t* root_out;
    // slab fits with shared_idx: only what the merge reads -- root_out[r] = r for every local
    // root r, root/core of the n_shared listed points, -1 / undefined elsewhere (no full
    // permutation of the per-point roots to slab order)
    const int64_t* shared_idx = nullptr;
    int64_t n_shared = 0;
    // full fits of n <= small_max points (and a mode / eps the one-workgroup kernel serves) run
    // small.hip's single-launch fit; 0 keeps every fit on the tiled pipeline
    int64_t small_max = 0;  // (0: the tiled pipeline; entry points opt in from the handle)
    // ... of which fits of >= spread_min points spread over several workgroups of one launch
    int64_t spread_min = INT64_MAX;
    // ... and, when small_max covers the LDS capacity, fits up to band_max points run the band
    // form (small.hip band_fit_kernel)
    int64_t band_max = 0;
    int64_t band_min = 0;  // (LDS-sized fits of >= band_min points also take the band form)
    // batched fit (n = the batch's span, cluster ids numbered per partition): see BatchFit
    const BatchFit* batch = nullptr;
    // device pointers of pinned host buffers for cluster / flag: the LDS forms (one launch)
    // write the labels there themselves, no copy back (Workspace::out_direct tells)
    int32_t* cluster_host = nullptr;
    uint8_t* flag_host = nullptr;
    // device word for the cluster count (asynchronous API): the tiled pipeline's output kernel
    // writes it (Workspace::nk_written; write_nclusters then launches nothing)
    int32_t* n_clusters_dev = nullptr;
};

// What a slab fit leaves on its handle for the label phase (dbscan_slab_label_device).
struct SlabState {
    bool valid = false;
    int64_t n = 0, nf = 0;
    double eps2 = 0;
    GridParams g{};
    const int32_t* nbr = nullptr;  // non-core neighbour lists (nullptr: label by stencil scan)
    int nbr_k = 0;
    int64_t nlroots = -1;  // local roots listed in ws.lroots by the last prepare (-1: none)
    // where a point's packed label lives: packed[to_packed[i]] for slab index i, written at
    // place[slot] (bucketed sort: pos / slot_place) or at the slot (plain sort: inv / none)
    const int32_t* to_packed = nullptr;
    const int32_t* place = nullptr;
    int64_t npacked = 0;  // entries of the packed array
};

int64_t run_fit(hipStream_t s, Workspace& ws, Profiler* prof, const FitArgs& a, FitStats* st,
                SlabState* slab);
// The same fit, enqueued without any host synchronization; read_fit_stats (which synchronizes)
// returns its stats, write_nclusters enqueues a copy of its cluster count to device memory.
void enqueue_fit(hipStream_t s, Workspace& ws, Profiler* prof, const FitArgs& a,
                 SlabState* slab);
FitStats read_fit_stats(hipStream_t s, Workspace& ws, Profiler* prof = nullptr);
// read_fit_stats in two halves: an asynchronous copy of the stats block to dst (pinned host
// memory, kFitStatsDoubles doubles), and its parse once the copy has completed.
constexpr int kFitStatsDoubles = 32;
// The handle's misc block (doubles): [0, 8) bbox scratch, [kMiscGrid, kMiscState) the device
// GridParams, then the FitState ints.
constexpr int kMiscGrid = 8, kMiscState = 24;
static_assert(sizeof(GridParams) <= (kMiscState - kMiscGrid) * sizeof(double),
              "GridParams overlaps the fit state");
static_assert(kMiscState * sizeof(double) + kStTileBuckets * sizeof(int32_t) <=
                  kFitStatsDoubles * sizeof(double), "the stats copy must hold the states");
// (an LDS fit writes the whole FitState into its stats block: the ring's stride must hold it)
static_assert(kMiscState * sizeof(double) + kStCount * sizeof(int32_t) <=
                  Workspace::kStatBlock * sizeof(double) &&
              kFitStatsDoubles <= Workspace::kStatBlock, "LDS fits' stats blocks");
void enqueue_fit_stats_copy(hipStream_t s, Workspace& ws, double* dst);
FitStats parse_fit_stats(const Workspace& ws, const double* buf);
void write_nclusters(hipStream_t s, Workspace& ws, int32_t* d_out);
// Batched fits (batch.hip).  enqueue_batch_bbox: per-partition {xmin, xmax, ymin, ymax, finite
// count} of [d_offs[p], d_offs[p+1]) into d_box (5 doubles each).  plan_batch_grid: from those
// boxes (host), the virtual grid and the partition table (host, nparts entries); partitions it
// cannot place (no clique grid, absurd extents) are listed in *alone, to be fitted on their own.
// Returns false when no partition is placed.
void enqueue_batch_bbox(hipStream_t s, const double* x, const double* y, const int64_t* d_offs,
                        int32_t n_parts, double* d_box);
bool plan_batch_grid(const double* box, const int64_t* offs, int32_t n_parts, double eps,
                     PartGrid* table, BatchFit* bf, std::vector<int32_t>* alone);
// The slab label in two parts around the cluster numbering: prepare (labels in terms of local
// roots, moved to slab order; needs only gs_of_root) and finish (roots numbered, one map pass).
void enqueue_slab_label_prepare(hipStream_t s, Workspace& ws, Profiler* prof,
                                const SlabState& st, const uint8_t* zone, const int64_t* gid,
                                const int64_t* gs_of_root, int32_t mode);
void run_slab_label_finish(hipStream_t s, Workspace& ws, Profiler* prof, const SlabState& st,
                           const uint8_t* zone, const int64_t* gs_of_root,
                           const int64_t* all_roots, int64_t n_roots, int32_t* cluster,
                           uint8_t* flag);
void run_slab_label(hipStream_t s, Workspace& ws, Profiler* prof, const SlabState& st,
                    const uint8_t* zone, const int64_t* gid, const int64_t* gs_of_root,
                    const int64_t* all_roots, int64_t n_roots, int32_t mode, int32_t* cluster,
                    uint8_t* flag);
// The reference's spatial partitioner (partition.hip): DBSCAN.scala:91-97 cell histogram on
// the GPU, EvenSplitPartitioner.scala:44-209 splits on the host.
constexpr double kMaxPartitionCells = 4e8;  // dense 2*eps cell window limit
struct Partition {
    double x, y, x2, y2;
    int64_t count;
};
int64_t run_partition(hipStream_t s, Workspace& ws, const double* d_x, const double* d_y,
                      int64_t n, double eps, int64_t max_points, std::vector<Partition>* out);
int64_t partition_cells(const double* cell_x, const double* cell_y, const int64_t* counts,
                        int64_t ncells, int64_t max_points, double mrs,
                        std::vector<Partition>* out);
int64_t split_partitions(double mrs, int64_t imin, int64_t jmin, int64_t W, int64_t H,
                         const std::vector<uint32_t>& hist, int64_t max_points,
                         std::vector<Partition>* out);

// Text I/O of the reference (csv.hip): DBSCANSuite/DBSCANSample input and output formats.
int64_t csv_read(const char* path, double* x_out, double* y_out, int64_t capacity);
void csv_write(const char* path, const double* x, const double* y, const int32_t* cluster,
               int64_t n);
// javanum.hip: java.lang.Double.toString as JDK 7/8 print it (NUL-terminated, returns the
// length) and Scala 2.10's NumericRange.count for Double ranges
int jdk8_double_string(double d, char* buf);
int64_t scala_range_count(double start, double end, double step, bool inclusive);

// Whole-node fit in one process (node.hip): n_shards slabs over the visible GPUs.
int32_t train_node(const double* x, const double* y, int64_t n, double eps, int32_t min_points,
                   int32_t mode, int32_t n_shards, int32_t* cluster_out, uint8_t* flag_out,
                   int64_t* n_clusters_out, std::string* err);
int32_t worker_selftest(int32_t* rcs, int32_t n);
// dbscan_train_node_shards / dbscan_selftest_node_plan (node.hip): see include/dbscan_hip.h.
int32_t node_record(int32_t* device_out, int64_t* points_out, int64_t* shared_out, int32_t max);
int32_t node_plan_selftest(int32_t n_shards, int32_t ndev, int32_t fail_device, int32_t* ran_on,
                           int32_t* rc_of_device);
// Node-path slab selection, label rows and scatter (node.hip): see include/dbscan_hip.h.
int64_t select_slab(hipStream_t s, DevBuf& scratch, ScanState& scan, const double* x,
                    const double* y, int64_t n, const double* cuts, int32_t n_cuts, int32_t rank,
                    double eps, double* sx, double* sy, uint8_t* sz, int64_t* sgid,
                    int64_t* sshared, int64_t capacity, int64_t* ns_out);
int64_t owned_rows(hipStream_t s, DevBuf& scratch, ScanState& scan, const uint8_t* zone,
                   const int64_t* gid, const int32_t* cl, const uint8_t* fl, int64_t m,
                   int64_t* rows, int64_t capacity);
void label_scatter(hipStream_t s, const int64_t* rows, int64_t k, int64_t start, int64_t m,
                   int32_t* cl, uint8_t* fl);
int64_t unpack_rows(hipStream_t s, DevBuf& scratch, ScanState& scan, const int64_t* rows,
                    int64_t k, double* sx, double* sy, uint8_t* sz, int64_t* sgid,
                    int64_t* sshared);
// Node-path routing (node.hip, dbscan_route_slabs_device): see include/dbscan_hip.h.
int64_t route_slabs(hipStream_t s, DevBuf& scratch, DevBuf& tabbuf, const double* x,
                    const double* y, int64_t m, int64_t start, const double* cuts, int32_t n_cuts,
                    double eps, int64_t* rows, int64_t capacity, int64_t* counts_out);
// Node-path merge (merge.hip): every local root's global s(K) (gs_of_root, slab index) and the
// zone-0 global roots owned here, compacted in slab (= gid) order; returns their count (syncs).
int64_t run_slab_merge_roots(hipStream_t s, Workspace& ws, int64_t n, const uint8_t* zone,
                             const int64_t* gid, const int32_t* root, const int32_t* parent,
                             int64_t* gs_of_root, int64_t* own_roots);
// The same without waiting: the count is copied to total_dst[0] (pinned host memory) on s.
// lroots != nullptr: every local root's slab index too, in slab order (the label's root
// numbering reads only these), and total_dst[1] = total_dst[0] + their count.
void enqueue_slab_merge_roots(hipStream_t s, Workspace& ws, int64_t n, const uint8_t* zone,
                              const int64_t* gid, const int32_t* root, const int32_t* parent,
                              int64_t* gs_of_root, int64_t* own_roots, int32_t* total_dst,
                              int32_t* lroots);

// ---- one-workgroup fits (small.hip) ----
// Can small_fit_kernel fit n points with this eps / mode (finite eps*eps, Naive or Archery)?
bool small_fit_eligible(int64_t n, double eps, int32_t mode);
// d_offs == nullptr: one fit of single_n points (x, y, cluster, flag from index 0), its cluster
// count and statistics into st / gp (the handle's fit state).  Else one workgroup per listed
// partition: d_list[i] indexes d_offs (partition p = points [d_offs[p], d_offs[p+1]), each of
// <= kSmallMaxPoints), cluster counts into d_nclusters[p].
void enqueue_small_fits(hipStream_t s, Profiler* prof, const double* x, const double* y,
                        const int64_t* d_offs, const int32_t* d_list, int32_t nlist,
                        int64_t single_n, double eps, int32_t min_points, int32_t mode,
                        int32_t* cluster, uint8_t* flag, int32_t* d_nclusters, GridParams* gp,
                        int32_t* st, double* mirror = nullptr);
// One fit of n <= kSmallMaxPoints points spread over several workgroups of one launch
// (small.hip, spread_fit_kernel): the same results as the one-workgroup fit; statistics into
// st / gp (the handle's fit state) and the fit's own stats block `mirror` (whose kStError the
// caller has cleared), kStError = 2 there if a grid barrier gave up.
void enqueue_spread_fit(hipStream_t s, Profiler* prof, Workspace& ws, const double* x,
                        const double* y, int64_t n, double eps, int32_t min_points, int32_t mode,
                        int32_t* cluster, uint8_t* flag, GridParams* gp, int32_t* st,
                        double* mirror);
// Partitions of kSmallMaxPoints < n <= kBandMaxPoints in ONE launch, each of G workgroups
// staging a band of cell rows (small.hip band_fit_kernel); statistics as the spread fit,
// kStError = 2 (barrier gave up) or 3 (a band over the staging capacity): drain_recalls then
// re-runs the fit through the tiled pipeline.
constexpr int64_t kBandMaxPoints = 65536;
bool band_fit_eligible(int64_t n, double eps, int32_t mode, int32_t min_points);
void enqueue_band_fit(hipStream_t s, Profiler* prof, Workspace& ws, const double* x,
                      const double* y, int64_t n, double eps, int32_t min_points, int32_t mode,
                      int32_t* cluster, uint8_t* flag, GridParams* gp, int32_t* st,
                      double* mirror);
// After the stream has drained: every spread / band fit queued since the last check whose
// barrier gave up or whose band overflowed is re-run, in stream order, into its own outputs
// (its stats block and cluster-count word rewritten), synchronously; counted in
// ws.spread_fallbacks.  Returns true when the LAST fit was re-run.
bool drain_recalls(hipStream_t s, Profiler* prof, Workspace& ws);
// DBSCAN.scala:116-137 on the host: the points every partition's outer rectangle (main grown
// by eps, inclusive) holds, in input order (partition.hip)
int64_t duplicate_points(const double* x, const double* y, int64_t n, const double* rects,
                         int64_t n_parts, double eps, int64_t* offsets_out, int64_t* index_out,
                         int64_t capacity);

// ---- primitives (primitives.hip) ----
// Exclusive scan of int32 values produced by `mode`:
//   0: in = const int32_t* values
//   1: in = const uint8_t* flags (nonzero counts 1)
//   2: in = const uint64_t* bit words (each counts its popcount)
// Writes out[0..n) (out may equal in) and, if total_dev != nullptr, the total at *total_dev.
// One launch; successive scans on one ScanState must be stream-ordered.
void exclusive_scan(hipStream_t s, int mode, const void* in, int32_t* out, int64_t n,
                    int32_t* total_dev, ScanState& ss);

// LSD radix sort of (key, val) pairs: four passes of 8, 8, 9 and 7 bits; bits_dev holds the
// key width on the device and passes at or beyond it return at once (keys of <= 25 bits: three
// passes).  The input is (key, val); the passes ping-pong through (key2, val2) and the last
// sorting pass writes (key3, val3), whose pointers are then swapped into key/val.  Stable.
// inv (optional): the inverse permutation of the sorted vals (a permutation of 0..n-1),
// inv[val] = sorted position, written by the last pass.  iota: the input vals are the identity
// 0..n-1 and are not read (the first pass generates them; val is then only a ping-pong buffer).
void radix_sort_pairs(hipStream_t s, uint32_t*& key, int32_t*& val, uint32_t*& key2,
                      int32_t*& val2, uint32_t*& key3, int32_t*& val3, int64_t n,
                      const int32_t* bits_dev, DevBuf& hist, ScanState& scan, Profiler* prof,
                      int32_t* inv = nullptr, bool iota = false);

int64_t bucket_padded(int64_t n);
// zone (slab fits): each point's zone rides in its record (gather_bucket writes zs from it);
// shm (lean slab fits): the listed shared points, whose slots gather_bucket writes by input index
// key == nullptr: the MSD pass bins x, y on *gp itself (grid_key), so bin_kernel's key pass
// and its 4 B/point key array are skipped.
void bucket_sort(hipStream_t s, const double* x, const double* y, const uint32_t* key, int64_t n,
                 const int32_t* bits_dev, BucketSort& b, DevBuf& hist, ScanState& scan,
                 Profiler* prof, const uint8_t* zone = nullptr, const uint8_t* shm = nullptr,
                 const GridParams* gp = nullptr);

// Per-block partials of the bbox (xmin, xmax, ymin, ymax, count of finite points; 5 doubles
// per block) for fit.hip's bbox_grid_kernel; returns the block count.
int bbox_partials(hipStream_t s, const double* x, const double* y, int64_t n, DevBuf& tmp,
                  double** partial_out);
// Three independent exclusive scans of n <= 4096 int32 values each (arrays at in + b * stride,
// results at out + b * stride, totals t0..t2) in one launch.
void scan3(hipStream_t s, const int32_t* in, int64_t n, int64_t stride, int32_t* out,
           int32_t* t0, int32_t* t1, int32_t* t2);

}  // namespace dbscan
