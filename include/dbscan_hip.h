/*
 * dbscan_hip.h -- C-ABI of libdbscan_hip.so, the MI355X (gfx950) local DBSCAN fit.
 *
 * The reference has no FFI: its seam is the Scala expression
 *     new LocalDBSCANNaive(eps, minPoints).fit(points)           DBSCAN.scala:153-154
 * with  fit(points: Iterable[DBSCANPoint]): Iterable[DBSCANLabeledPoint]
 *                                                                 LocalDBSCANNaive.scala:37
 * and its variant LocalDBSCANArchery(eps, minPoints).fit          LocalDBSCANArchery.scala:36
 * (paths relative to src/main/scala/org/apache/spark/mllib/clustering/dbscan/).  Every entry
 * point below is what a JNI binding of that seam binds (INTEGRATION.md shows the JNI stub and
 * the Scala `LocalDBSCANHip` wrapper).  Plain pointers and sizes only; no torch types.
 *
 * Semantics (bit-exact with the reference for mode NAIVE, visit order = array order):
 *   neighbour(p, o)  <=>  dx = o.x - p.x; dy = o.y - p.y; dx*dx + dy*dy <= eps*eps   in fp64,
 *                        never fused into FMA                       DBSCANPoint.scala:26-30,
 *                                                                   LocalDBSCANNaive.scala:33,77
 *   |N(p)| counts p itself; core <=> |N(p)| >= min_points          LocalDBSCANNaive.scala:54,101
 *   clusters are numbered 1..k in the order the reference's outer loop would open them
 *   (rank of the smallest core index of each core-core component)  LocalDBSCANNaive.scala:45-64
 *   NAIVE:   a non-core point is Border of the first-opened adjacent cluster if that cluster
 *            opens before the point's own index, else Noise           LocalDBSCANNaive.scala:94
 *   ARCHERY: a non-core point with any core neighbour is Border of the first-opened adjacent
 *            cluster (Noise re-claimed)                              LocalDBSCANArchery.scala:103-106
 *            (archery visits in R-tree entry order; callers pass the order they want as the
 *            array order -- raw archery numbering is not reproducible)
 * Outputs are in INPUT order: cluster (0 = Unknown/Noise) and flag (Flag ordinals below).
 * Non-finite coordinates are never anyone's neighbour (not even their own) while eps*eps is
 * finite; eps*eps = +inf makes every pair whose d2 is not NaN a neighbour (all-pairs, O(n^2));
 * eps*eps = NaN has no pairs.
 */
#ifndef DBSCAN_HIP_H
#define DBSCAN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* DBSCANLabeledPoint.Flag ordinals, DBSCANLabeledPoint.scala:28-31 */
#define DBSCAN_FLAG_BORDER 0
#define DBSCAN_FLAG_CORE 1
#define DBSCAN_FLAG_NOISE 2
#define DBSCAN_FLAG_NOT_FLAGGED 3

#define DBSCAN_MODE_NAIVE 0   /* LocalDBSCANNaive   (used by DBSCAN.train, DBSCAN.scala:154) */
#define DBSCAN_MODE_ARCHERY 1 /* LocalDBSCANArchery (LocalDBSCANArcherySuite)               */
/* LocalDBSCANArchery with its float32 R-tree search box applied before the fp64 filter
 * (LocalDBSCANArchery.scala:38-41,114-124): a directed neighbour relation.  Local fits only
 * (dbscan_fit, dbscan_fit_h, dbscan_fit_device, dbscan_fit_device_async -- the async form waits
 * on the device once, to resolve one-way pairs); slab and node entry points reject it. */
#define DBSCAN_MODE_ARCHERY_F32BOX 2

/* return codes */
#define DBSCAN_OK 0
#define DBSCAN_EARG (-1) /* bad argument: n < 0, n > DBSCAN_MAX_POINTS, NULL pointer, bad mode */
#define DBSCAN_EHIP (-2) /* HIP runtime error (details in dbscan_last_error) */
#define DBSCAN_EOOM (-3) /* device allocation failed */

#define DBSCAN_MAX_POINTS 2147483000LL /* int32 point indices on device */

typedef struct dbscan_handle dbscan_handle;

/* Thread-local description of the last error on this thread ("" if none). */
const char* dbscan_last_error(void);
/* ABI version (major*100 + minor). */
int32_t dbscan_version(void);
/* Number of visible HIP devices (0 when none; never fails). */
int32_t dbscan_device_count(void);

/* A handle owns one HIP stream and grow-only device work buffers on `device`; one handle per
 * thread (Spark local[N] runs N concurrent fits).  NULL on failure (see dbscan_last_error). */
dbscan_handle* dbscan_create(int32_t device);
void dbscan_destroy(dbscan_handle* h);

/* Host arrays in, host arrays out (input order).  Replaces LocalDBSCANNaive.fit /
 * LocalDBSCANArchery.fit (LocalDBSCANNaive.scala:37, LocalDBSCANArchery.scala:36).
 * n == 0 returns DBSCAN_OK with *n_clusters_out = 0.  The handle-less form uses a
 * thread-local handle on device 0. */
int32_t dbscan_fit(const double* x, const double* y, int64_t n, double eps, int32_t min_points,
                   int32_t mode, int32_t* cluster_out, uint8_t* flag_out,
                   int32_t* n_clusters_out);
int32_t dbscan_fit_h(dbscan_handle* h, const double* x, const double* y, int64_t n, double eps,
                     int32_t min_points, int32_t mode, int32_t* cluster_out, uint8_t* flag_out,
                     int32_t* n_clusters_out);

/* Device-resident form: d_x, d_y, d_cluster, d_flag are device pointers on the handle's
 * device.  All work is enqueued on the handle's stream; the call returns after the stream has
 * drained (the cluster count is read back). */
int32_t dbscan_fit_device(dbscan_handle* h, const double* d_x, const double* d_y, int64_t n,
                          double eps, int32_t min_points, int32_t mode, int32_t* d_cluster,
                          uint8_t* d_flag, int32_t* n_clusters_out);

/* Asynchronous device-resident form: enqueues the whole fit on the handle's stream and returns
 * without waiting (no host synchronization anywhere inside a fit: the eps grid is sized on the
 * device).  The cluster count is written to DEVICE memory at d_n_clusters (may be NULL).
 * dbscan_sync waits for the stream, then makes the fit's statistics available and reports
 * device-side errors (an eps grid that cannot be sized) as DBSCAN_EARG.  Any synchronous entry
 * point on the same handle settles a pending asynchronous fit first.  Several fits may be queued
 * back to back (inputs and outputs kept alive until dbscan_sync): each partition-sized fit
 * (the LDS forms) records its outcome in a stats block of its own, and dbscan_sync re-runs, in
 * order and into their own outputs and cluster-count words, every queued spread or band fit
 * whose grid barrier gave up or whose band overflowed -- not only the last one -- so no queued
 * fit ever keeps wrong labels; the statistics reported are the last fit's.  bench.py times this
 * form: K fits back to back, one synchronization. */
int32_t dbscan_fit_device_async(dbscan_handle* h, const double* d_x, const double* d_y,
                                int64_t n, double eps, int32_t min_points, int32_t mode,
                                int32_t* d_cluster, uint8_t* d_flag, int32_t* d_n_clusters);
int32_t dbscan_sync(dbscan_handle* h);

/* The handle's hipStream_t (as void*), for callers that order their own work around it. */
void* dbscan_stream(dbscan_handle* h);
/* Run the handle's work on the caller's stream (a hipStream_t of the handle's device, as void*;
 * NULL is the device's null stream) from now on, so a caller whose own work is on that stream
 * needs no cross-stream waits; own != 0 returns to the handle's own stream (stream ignored).
 * Waits for the work already enqueued.  The handle never destroys a caller's stream: the caller
 * must keep it alive while it is bound (until dbscan_set_stream(h, NULL, 1) or dbscan_destroy). */
int32_t dbscan_set_stream(dbscan_handle* h, void* stream, int32_t own);

/* Statistics of the handle's last fit:
 *   [0] n  [1] finite points in the grid  [2] occupied cells  [3] core points
 *   [4] clusters  [5] grid nx  [6] grid ny  [7] radix key bits  [8] grid mode
 *   (0 = eps grid, 1 = all pairs, 2 = no pairs)  [9] occupied 8x8-cell tiles
 *   [10] 1 if quarter cells are cliques of the predicate (tile union path)
 *   [11..13] clique grids: points in the small / medium / big tiles (the three count paths)
 * Returns the number of values written (<= max).                               */
int32_t dbscan_last_stats(dbscan_handle* h, int64_t* out, int32_t max);

/* Timing with HIP events on the handle's stream.  dbscan_profile_enable(h, 1): every pipeline
 * stage of each fit is bracketed by event records (each costs ~10 us of GPU idle); (h, 2): every
 * kernel launch carries its own start/stop events on its dispatch packet (hipExtLaunchKernel; no
 * added gaps); 0 turns timing off.  read accumulates (name, total ms, launches).
 * `names` receives NUL-separated stage names.  Returns the number of stages written. */
int32_t dbscan_profile_enable(dbscan_handle* h, int32_t on);
/* Kernel mode: time only the launches of the named kernel (its profile name; NULL = all). */
int32_t dbscan_profile_only(dbscan_handle* h, const char* kernel);
int32_t dbscan_profile_reset(dbscan_handle* h);
int32_t dbscan_profile_read(dbscan_handle* h, char* names, int32_t names_cap, double* total_ms,
                            int64_t* launches, int32_t max);

/* The reference's spatial partitioner: DBSCAN.scala:91-97 maps every point
 * to its 2*eps cell (corner = (shiftIfNegative(p) / (2*eps)).intValue * 2*eps,
 * DBSCAN.scala:345-356) and counts points per cell -- a histogram on the GPU here -- then
 * EvenSplitPartitioner.partition(cells, maxPointsPerPartition, 2*eps)
 * (EvenSplitPartitioner.scala:44-209) splits the bounding rectangle until every partition holds
 * at most maxPointsPerPartition points or cannot be split (host, summed-area table).
 * Partitions are written as (x, y, x2, y2) quadruples + point counts in the reference's list
 * order, at most max_parts of them; the return value is the full partition count (call again
 * with a larger buffer if it exceeds max_parts) or a negative error code.  Exact fp semantics
 * of the reference, including its split-line/cell-corner defect; equal-cost
 * splits are broken by candidate order (x splits, then y), where the reference iterates a
 * Scala HashSet.  dbscan_partition_cells is EvenSplitPartitioner.partition over an explicit
 * cell set (cells given by lower corners on the min_rect_size grid), as
 * EvenSplitPartitionerSuite calls it. */
int64_t dbscan_partition(dbscan_handle* h, const double* x, const double* y, int64_t n,
                         double eps, int64_t max_points_per_partition, double* rects_out,
                         int64_t* counts_out, int64_t max_parts);
int64_t dbscan_partition_device(dbscan_handle* h, const double* d_x, const double* d_y, int64_t n,
                                double eps, int64_t max_points_per_partition, double* rects_out,
                                int64_t* counts_out, int64_t max_parts);
int64_t dbscan_partition_cells(const double* cell_x, const double* cell_y,
                               const int64_t* cell_counts, int64_t ncells,
                               int64_t max_points_per_partition, double min_rect_size,
                               double* rects_out, int64_t* counts_out, int64_t max_parts);

/* Text I/O of the reference, host code.
 * dbscan_csv_read: the input of DBSCANSuite.scala:31-33 / DBSCANSample.scala:21,
 *   sc.textFile(path).map(s => Vectors.dense(s.split(',').map(_.toDouble))): one point per
 *   line, every field a java.lang.Double.parseDouble number (trailing empty fields dropped, as
 *   String.split does), x = field 0, y = field 1 (DBSCANPoint reads only those two; a label
 *   column is parsed and ignored).  With x_out == y_out == NULL returns the record count;
 *   otherwise fills up to `capacity` records and returns the count; a malformed record is
 *   DBSCAN_EARG naming its 1-based line.  Memory-mapped, parsed by host threads.
 * dbscan_csv_write: the output of DBSCANSample.scala:35, "x,y,cluster" per point with x and y
 *   in java.lang.Double.toString form as the reference's runtime prints it (Spark 2.1.0 on JDK
 *   7/8, pom.xml:30-37): sun.misc.FloatingDecimal's digits (dbscan_format_double; buf >= 32
 *   bytes, returns the length) -- usually the shortest round-trip digits, but e.g.
 *   2.82879384806159E17 prints as 2.82879384806159008E17; plain for 1e-3 <= |v| < 1e7, else
 *   d.dddE[-]n.
 * dbscan_scala_range_count: the element count of the Scala 2.10 Double range
 *   `start until end by step` (inclusive != 0: `to`), NumericRange.count with
 *   Numeric.DoubleAsIfIntegral (BigDecimal(Double.toString) quot/rem at DECIMAL128): the
 *   EvenSplitPartitioner's candidate splits (EvenSplitPartitioner.scala:150-152).  Negative on
 *   the reference's exceptions (step 0, more than Int.MaxValue elements). */
int64_t dbscan_csv_read(const char* path, double* x_out, double* y_out, int64_t capacity);
int32_t dbscan_csv_write(const char* path, const double* x, const double* y,
                         const int32_t* cluster, int64_t n);
int32_t dbscan_format_double(double v, char* buf);
int64_t dbscan_scala_range_count(double start, double end, double step, int32_t inclusive);

/* ---------------------------------------------------------------------------------------
 * Partition-sized fits: the seam's real call pattern.  DBSCAN.scala:150-155 runs one
 * LocalDBSCANNaive(eps, minPoints).fit per spatial partition -- at most maxPointsPerPartition
 * points (EvenSplitPartitioner.scala:44-209) plus the eps halo (DBSCAN.scala:116-137).
 * Full fits of at most dbscan_set_small_max(h, ...) points (default
 * DBSCAN_SMALL_DEFAULT_POINTS = the ceiling DBSCAN_SMALL_MAX_POINTS: the LDS fits beat the tiled
 * pipeline on a single call at every size up to it) with a finite eps*eps in mode NAIVE or
 * ARCHERY run ONE kernel in which a workgroup holds the whole partition in LDS (same results
 * bit for bit as the tiled pipeline; dbscan_fit / dbscan_fit_h / dbscan_fit_device /
 * dbscan_fit_device_async all route there).  dbscan_set_small_max returns the previous value (0
 * sends every fit through the tiled pipeline). */
#define DBSCAN_SMALL_MAX_POINTS 8192
#define DBSCAN_SMALL_DEFAULT_POINTS 8192
int64_t dbscan_set_small_max(dbscan_handle* h, int64_t max_points);

/* Of those LDS fits, the ones of at least dbscan_set_spread_min(h, ...) points (default
 * DBSCAN_SPREAD_DEFAULT_POINTS) run spread over several workgroups of the one launch: each
 * workgroup stages the whole partition, counts and walks the unions of ~256 of its points, and two
 * grid-wide barriers exchange the core flags and the union forests (same results bit for bit).
 * A value above DBSCAN_SMALL_MAX_POINTS keeps every LDS fit on one workgroup.  Returns the
 * previous value.  A spread fit whose workgroups cannot all be resident (the GPU filled by other
 * work, e.g. many executors' spread fits at once) gives up its grid barrier after a bounded poll
 * instead of waiting forever, and the fit is then re-run by the one-workgroup kernel in the same
 * call (for dbscan_fit_device_async: in dbscan_sync), with the same results; the fit never
 * fails for it.  Such re-runs are counted (dbscan_spread_fallbacks).  With the defaults the
 * band form below takes every eligible fit from DBSCAN_BAND_MIN_DEFAULT_POINTS points, so the
 * spread form serves the fits the band form does not take (minPoints <= 0, the float32-box
 * Archery mode) or a handle whose dbscan_set_band_min is raised. */
#define DBSCAN_SPREAD_DEFAULT_POINTS 512
int64_t dbscan_set_spread_min(dbscan_handle* h, int64_t min_points);
/* Full fits above the LDS fits' capacity (DBSCAN_SMALL_MAX_POINTS, with small_max at that
 * ceiling) and up to dbscan_set_band_max(h, ...) points (default and ceiling
 * DBSCAN_BAND_MAX_POINTS; 0: never) in modes NAIVE and ARCHERY with minPoints >= 1 run in ONE
 * launch instead of the tiled pipeline's ~45: 64 workgroups, each owning a range of eps cells of
 * ~1/64 of the estimated work and staging those cells' rows (plus one row either side) in its
 * LDS, meeting at six grid barriers, the clusters merged in a union-find over input indices
 * -- same results bit for bit.  A range over the staging capacity (very dense rows) or a
 * barrier that gives up re-runs the fit through the tiled pipeline in the same call (counted
 * by dbscan_spread_fallbacks).  Returns the previous value. */
#define DBSCAN_BAND_MAX_POINTS 65536
#define DBSCAN_BAND_DEFAULT_POINTS 65536
int64_t dbscan_set_band_max(dbscan_handle* h, int64_t max_points);
/* Fits inside the LDS fits' capacity of >= min_points points (default
 * DBSCAN_BAND_MIN_DEFAULT_POINTS; measured faster than the one-workgroup and spread forms from
 * ~400 points) take the band form too, with the same eligibility (and up to the band maximum
 * above).  Returns the previous value. */
#define DBSCAN_BAND_MIN_DEFAULT_POINTS 400
int64_t dbscan_set_band_min(dbscan_handle* h, int64_t min_points);
/* Test hook: the spread fit's barrier poll bound (default 2^21 polls, ~seconds); 0 makes every
 * barrier give up at once, so every spread fit takes the one-workgroup re-run.  Returns the
 * previous bound (negative: an error code). */
int64_t dbscan_set_spread_spin_limit(dbscan_handle* h, int64_t polls);
/* Spread and band fits of this handle re-run by the fallback (the one-workgroup kernel, the
 * tiled pipeline) so far (negative: an error). */
int64_t dbscan_spread_fallbacks(dbscan_handle* h);

/* A batch of independent local fits -- an executor's partitions -- in one call: partition p is
 * points [offsets[p], offsets[p+1]) of x, y (host array offsets, n_parts + 1 non-decreasing
 * values >= 0), each fitted exactly as dbscan_fit would fit it alone: cluster_out / flag_out at
 * the same indices (partition-local cluster ids 1..k_p, 0 = Noise), k_p in n_clusters_out[p].
 * Partitions the one-workgroup kernel serves run in ONE launch, one workgroup each; the others
 * run the tiled pipeline one after another on the handle's stream.  Replaces the per-partition
 * flatMapValues(LocalDBSCANNaive.fit) of DBSCAN.scala:153-154 for a whole batch.
 * dbscan_fit_batch: host arrays, synchronous.  dbscan_fit_batch_device_async: device arrays
 * (n_clusters too; offsets stay a host array), enqueued on the handle's stream; dbscan_sync waits. */
int32_t dbscan_fit_batch(dbscan_handle* h, const double* x, const double* y,
                         const int64_t* offsets, int32_t n_parts, double eps, int32_t min_points,
                         int32_t mode, int32_t* cluster_out, uint8_t* flag_out,
                         int32_t* n_clusters_out);
int32_t dbscan_fit_batch_device_async(dbscan_handle* h, const double* d_x, const double* d_y,
                                      const int64_t* offsets, int32_t n_parts, double eps,
                                      int32_t min_points, int32_t mode, int32_t* d_cluster,
                                      uint8_t* d_flag, int32_t* d_n_clusters);

/* DBSCAN.scala:116-137 on the host: every point goes to every partition whose outer rectangle
 * (the partition's rectangle (x, y, x2, y2) from dbscan_partition, grown by eps with the
 * reference's arithmetic, shrink(-eps)) contains it, borders included; each partition's points
 * in input order, as groupByKey hands them to the local fit.  Returns the total number of
 * (partition, point) records; fills offsets_out[n_parts + 1] and, when index_out is not NULL and
 * capacity >= the total, index_out (input indices) -- ready for dbscan_fit_batch after a gather. */
int64_t dbscan_duplicate(const double* x, const double* y, int64_t n, const double* rects,
                         int64_t n_parts, double eps, int64_t* offsets_out, int64_t* index_out,
                         int64_t capacity);

/* Whole-node entry: DBSCAN.train(points, eps, minPoints, ...).labeledPoints
 * (DBSCAN.scala:91-283) for one node, from host arrays, in ONE process.  The points are cut
 * into n_shards x-slabs at count quantiles snapped to the 2*eps grid (n_shards <= 0: one per
 * visible GPU; shard s runs on device s % device_count, each with its own stream), every slab
 * is fitted with its eps halos, and the slabs are merged exactly: the outputs equal one
 * LocalDBSCANNaive / LocalDBSCANArchery fit of all n points in input order, global cluster ids
 * 1..k (0 = Noise) -- not the reference merge's approximations.  The
 * multi-process form of the same plan is dbscan_amd/node.py (one rank per GPU, RCCL). */
int32_t dbscan_train_node(const double* x, const double* y, int64_t n, double eps,
                          int32_t min_points, int32_t mode, int32_t n_shards,
                          int32_t* cluster_out, uint8_t* flag_out, int64_t* n_clusters_out);

/* Self-test of dbscan_train_node's per-device worker error handling, on the host alone (no
 * device is touched): worker w of n throws failure kind w % 9 (none; a HIP OOM; another HIP
 * failure; a C-ABI status; a HIP check; an argument error; std::bad_alloc; std::exception;
 * an unknown type) and rcs[w] receives the status it maps to (DBSCAN_OK, EOOM, EHIP, EARG,
 * EHIP, EARG, EOOM, EHIP, EHIP) -- never a process abort. */
int32_t dbscan_selftest_worker_errors(int32_t* rcs, int32_t n);
/* What the calling thread's last dbscan_train_node ran, per shard s < the returned shard count
 * (up to max entries written; any pointer may be NULL): device_out[s] the device its worker ran
 * on (hipGetDevice inside the worker: s % device_count), points_out[s] its points with halos,
 * shared_out[s] its points shared with a neighbouring slab.  Negative: an error code. */
int32_t dbscan_train_node_shards(int32_t* device_out, int64_t* points_out, int64_t* shared_out,
                                 int32_t max);
/* Self-test of dbscan_train_node's shard plan and per-device status on the host alone (no
 * device is touched): ndev mocked devices and n_shards shards through the same plan and worker
 * pool; ran_on[s] = the device whose worker ran shard s; the worker of device fail_device (-1:
 * none) fails with a HIP error on its first shard; rc_of_device[d] = each device worker's status
 * (min(n_shards, ndev) entries).  Returns the call's status as dbscan_train_node would report it
 * (the first failed device's, else DBSCAN_OK). */
int32_t dbscan_selftest_node_plan(int32_t n_shards, int32_t ndev, int32_t fail_device,
                                  int32_t* ran_on, int32_t* rc_of_device);

/* ---------------------------------------------------------------------------------------
 * Slab fits for the multi-GPU node path (dbscan_amd/node.py).  The caller
 * passes the points of one spatial slab grown by halos, in increasing global visit order, with
 * a zone per point:
 *   0 = owned (inside this rank's slab), 1 = inner halo (within eps of the slab: exact counts,
 *   joins the local union-find), 2 = outer halo (within 2*eps: neighbour-count candidate only).
 * Phase 1, dbscan_slab_fit_device: exact core flags for zones 0/1 and, per core, the slab
 *   index of the minimum-index core of its local component (d_root; -1 for non-cores).
 *   This mirrors the per-partition LocalDBSCANNaive.fit of DBSCAN.scala:150-155 with the
 *   partition's eps-grown rectangle (DBSCAN.scala:116-137).
 * The caller merges local components across slabs (RCCL all-gather of shared core points,
 * global min-label union; replaces DBSCAN.scala:158-222) and numbers global clusters.
 * Phase 2, dbscan_slab_label_device (same handle, no fit in between): labels of the zone-0
 *   points in slab order.  d_gid[i] = global visit index of slab point i; for every local root
 *   r: d_gs_of_root[r] = global s(K) of its component (dbscan_slab_merge_roots_device);
 *   d_all_roots = the s(K) of every global component, all ranks, sorted ascending: a cluster
 *   id is 1 + the rank of s(K) in it.  Cores get the id of their root's component; a non-core
 *   takes the neighbour root with the smallest gs_of_root (Naive: only if that is < its own
 *   gid).  Zone 1/2 entries are left untouched.  Replaces the relabel of DBSCAN.scala:232-270. */
int32_t dbscan_slab_fit_device(dbscan_handle* h, const double* d_x, const double* d_y,
                               const uint8_t* d_zone, int64_t n, double eps,
                               int32_t min_points, uint8_t* d_core, int32_t* d_root);
int32_t dbscan_slab_label_device(dbscan_handle* h, const uint8_t* d_zone, const int64_t* d_gid,
                                 const int64_t* d_gs_of_root, const int64_t* d_all_roots,
                                 int64_t n_all_roots, int32_t mode, int32_t* d_cluster,
                                 uint8_t* d_flag);
/* The same two phases enqueued on the handle's stream without waiting (order the caller's own
 * streams around dbscan_stream(h)); the fit's statistics settle at the next synchronizing call. */
int32_t dbscan_slab_fit_device_async(dbscan_handle* h, const double* d_x, const double* d_y,
                                     const uint8_t* d_zone, int64_t n, double eps,
                                     int32_t min_points, uint8_t* d_core, int32_t* d_root);
/* dbscan_slab_fit_device_async with only the outputs the merge reads (dbscan_amd/node.py):
 * d_root[r] = r for every local root r; for the n_shared slab indices d_shared[k] (the points
 * this rank shares with a neighbour rank) d_core and d_root as in dbscan_slab_fit_device; every
 * other d_root entry is -1 and every other d_core entry is left unwritten.  Skips moving every
 * point's root to slab order (one random read per point). */
int32_t dbscan_slab_fit_shared_device_async(dbscan_handle* h, const double* d_x,
                                            const double* d_y, const uint8_t* d_zone, int64_t n,
                                            double eps, int32_t min_points,
                                            const int64_t* d_shared, int64_t n_shared,
                                            uint8_t* d_core, int32_t* d_root);
int32_t dbscan_slab_label_device_async(dbscan_handle* h, const uint8_t* d_zone,
                                       const int64_t* d_gid, const int64_t* d_gs_of_root,
                                       const int64_t* d_all_roots, int64_t n_all_roots,
                                       int32_t mode, int32_t* d_cluster, uint8_t* d_flag);

/* Cross-slab merge of the node path (replaces DBSCAN.scala:158-222: band points,
 * findAdjacencies, DBSCANGraph components, global ids), enqueued on the CALLER's stream
 * (a hipStream_t passed as void*; the caller's current device).  Records (d_a[i], d_b[i]) are
 * (gid of a shared core point, gid of its local root on the emitting rank), gathered from all
 * ranks; d_b[i] < 0 marks a record to skip.  d_parent is a dense int32 array over all gids of
 * the job, initialised to -1 once; the union leaves parent[x] = s(K) (smallest gid of x's
 * global component) for every node x of a valid record, and dbscan_merge_reset_device restores
 * those entries to -1 (O(records) per step).
 * dbscan_slab_merge_roots_device (handle stream; synchronizes), after a slab fit and the union
 * (d_root as returned by the slab fit: a local root p has d_root[p] == p): for every local root
 * p, d_gs_of_root[p] = the global s(K) of its component; the zone-0 local roots whose s(K) is
 * their own gid -- the global roots owned by this rank -- are written to d_own_roots in
 * increasing gid order, their count to *n_own_out (host). */
int32_t dbscan_merge_union_device(const int64_t* d_a, const int64_t* d_b, int64_t m,
                                  int32_t* d_parent, void* stream);
int32_t dbscan_merge_reset_device(const int64_t* d_a, const int64_t* d_b, int64_t m,
                                  int32_t* d_parent, void* stream);
int32_t dbscan_slab_merge_roots_device(dbscan_handle* h, int64_t n, const uint8_t* d_zone,
                                       const int64_t* d_gid, const int32_t* d_root,
                                       const int32_t* d_parent, int64_t* d_gs_of_root,
                                       int64_t* d_own_roots, int64_t* n_own_out);

/* dbscan_slab_merge_roots_device and dbscan_slab_label_device_async split around the cluster
 * numbering, so the host's wait for the owned-root count (and the caller's all-gather of the
 * roots) overlaps GPU work (dbscan_amd/node.py):
 * dbscan_slab_roots_prepare_device (after a slab fit on this handle, n = its point count):
 *   everything dbscan_slab_merge_roots_device does, then enqueues the part of the label that
 *   needs only d_gs_of_root (each zone-0 point's local root, moved to slab order); returns once
 *   the count is known (*n_own_out), while that label work is still running.
 * dbscan_slab_label_finish_device_async (same handle, no fit in between): numbers the local
 *   roots from d_all_roots (as dbscan_slab_label_device) and writes d_cluster / d_flag of the
 *   zone-0 points; zone 1/2 entries are left untouched.  Outputs equal
 *   dbscan_slab_label_device's.  Both replace the relabel of DBSCAN.scala:232-270. */
int32_t dbscan_slab_roots_prepare_device(dbscan_handle* h, int64_t n, const uint8_t* d_zone,
                                         const int64_t* d_gid, const int32_t* d_root,
                                         const int32_t* d_parent, int64_t* d_gs_of_root,
                                         int32_t mode, int64_t* d_own_roots,
                                         int64_t* n_own_out);
int32_t dbscan_slab_label_finish_device_async(dbscan_handle* h, const uint8_t* d_zone,
                                              const int64_t* d_gs_of_root,
                                              const int64_t* d_all_roots, int64_t n_all_roots,
                                              int32_t* d_cluster, uint8_t* d_flag);

/* Host-to-slab routing of the node path (dbscan_amd/node.py NodeJob.from_chunk; the point
 * duplication of DBSCAN.scala:116-137 for x-slabs): a rank holds the chunk [start, start + m)
 * of the global input (device arrays, global visit order); every point goes to each of the
 * n_cuts + 1 slabs (x < cuts[0], [cuts[0], cuts[1]), ...; at most 64) whose zone 0/1/2 holds it
 * (node.py zones(): owned, within eps-reach of the slab, within twice that).  Rows of three
 * int64: (x bits, y bits, gid * 8 + zone * 2 + shared), grouped by destination slab, ascending
 * gid within each.  counts_out[d] (host, n_cuts + 1 entries) = rows for slab d.  d_rows NULL or
 * capacity (rows) below the total: counts only.  Returns the total row count (< 0: error).
 * Synchronizes the handle's stream. */
int64_t dbscan_route_slabs_device(dbscan_handle* h, const double* d_x, const double* d_y,
                                  int64_t m, int64_t start, const double* cuts, int32_t n_cuts,
                                  double eps, int64_t* d_rows, int64_t capacity,
                                  int64_t* counts_out);

/* NodeJob.from_global's slab selection (dbscan_amd/node.py; the slab plan of dbscan_train_node):
 * of the n points (device arrays, global visit order), the ones in zone 0/1/2 of slab `rank`
 * of the x-cuts (node.py zones()), in input order: x, y, zone and input index each, and the
 * slab indices of its shared points (zone 0/1 of two slabs).  Returns the slab's point count m
 * (< 0: error) and *n_shared_out; the outputs are written when d_sx is not NULL and capacity
 * >= m (the shared array must hold *n_shared_out <= m entries).  Synchronizes the handle's
 * stream. */
int64_t dbscan_slab_select_device(dbscan_handle* h, const double* d_x, const double* d_y,
                                  int64_t n, const double* cuts, int32_t n_cuts, int32_t rank,
                                  double eps, double* d_sx, double* d_sy, uint8_t* d_szone,
                                  int64_t* d_sgid, int64_t* d_sshared, int64_t capacity,
                                  int64_t* n_shared_out);
/* NodeJob.from_chunk's received rows (dbscan_route_slabs_device's layout) into the slab's
 * columns: x, y, zone and gid of each of the k rows, and the row indices of the shared ones
 * (d_sshared: capacity k), in row order.  Returns the shared count (< 0: error).
 * Synchronizes the handle's stream. */
int64_t dbscan_rows_unpack_device(dbscan_handle* h, const int64_t* d_rows, int64_t k,
                                  double* d_sx, double* d_sy, uint8_t* d_szone, int64_t* d_sgid,
                                  int64_t* d_sshared);
/* NodeJob.chunk_labels' rows: the zone-0 points of a slab's m points in slab order (ascending
 * gid) as int64 pairs (gid, cluster << 8 | flag).  Returns the row count (< 0: error); writes
 * when d_rows is not NULL and capacity (pairs) suffices.  Synchronizes the handle's stream for
 * the count; the rows are written asynchronously on it. */
int64_t dbscan_owned_rows_device(dbscan_handle* h, const uint8_t* d_zone, const int64_t* d_gid,
                                 const int32_t* d_cluster, const uint8_t* d_flag, int64_t m,
                                 int64_t* d_rows, int64_t capacity);
/* ... and the chunk owner's scatter of the k received pairs into its chunk [start, start + m):
 * d_cluster[gid - start], d_flag[gid - start] (asynchronous on the handle's stream). */
int32_t dbscan_label_scatter_device(dbscan_handle* h, const int64_t* d_rows, int64_t k,
                                    int64_t start, int64_t m, int32_t* d_cluster,
                                    uint8_t* d_flag);

/* Device-side synthetic generator G(n, noise, dense, seed) of SURVEY.md §8d (32 isotropic
 * Gaussian blobs, splitmix64 + Box-Muller, uniform noise), then a seeded shuffle of the
 * visit order.  Writes d_x, d_y (device).  Used by bench.py so 10^7..10^9 points need no PCIe. */
int32_t dbscan_generate_blobs_device(dbscan_handle* h, double* d_x, double* d_y, int64_t n,
                                     double noise_frac, double dense, uint64_t seed);

#ifdef __cplusplus
}
#endif

#endif /* DBSCAN_HIP_H */
