/*
 * reference_pipeline.c -- CPU restatement of the reference's driver around the hot path.
 * TEST INFRASTRUCTURE ONLY (see dbscan_oracle.c header): used by tests/ for end-to-end
 * fixtures and by bench.py's cpu_baseline leg ("reference algorithm, C restatement").
 *
 * Restated (paths relative to src/main/scala/org/apache/spark/mllib/clustering/dbscan/):
 *   DBSCAN.scala:289,345-356        minimumRectangleSize = 2*eps; toMinimumBoundingRectangle,
 *                                   corner(), shiftIfNegative()  (Double.intValue truncation)
 *   EvenSplitPartitioner.scala:44-209  findPartitions / partition / split / complement /
 *                                   findPossibleSplits / canBeSplit / pointsInRectangle
 *   DBSCANRectangle.scala:28-52     contains (inclusive), shrink, almostContains (strict)
 *   DBSCAN.scala:116-137            margins (inner=shrink(eps), main, outer=shrink(-eps)) and
 *                                   duplication of every point into each outer it falls in
 *   DBSCAN.scala:150-155            LocalDBSCANNaive.fit per partition (oracle_fit_sequential)
 *   DBSCAN.scala:158-270            band points, findAdjacencies, DBSCANGraph connectivity,
 *                                   global ids, inner relabel, "last non-Noise wins" dedup
 *
 * Deviations (documented in DESIGN.md, "parity unpinned" where noted):
 *   - pointsInRectangle is answered with a summed-area table; the contained cell-index
 *     range is found by binary search with the reference's exact fp comparisons, so the
 *     answer equals the linear scan (:175-181), including the split-line/cell-corner defect.
 *   - Ties in split cost: `splits.toSet.reduceLeft` (:111-119, :161) keeps the first
 *     minimum in the Set's iteration order -- candidate order (x splits, then y splits) for at
 *     most 4 candidates (Set1..Set4), else the HashTrieSet order of the candidates' hashes,
 *     which the Python side of the oracle computes (oracle/jvm.py split_order_key: Scala 2.10
 *     MurmurHash3.productHash + HashSet.improve) and hands in as a callback, like the range
 *     count.  Full 32-bit hash collisions (ListSet order) are not modelled.
 *   - Scala's Double NumericRange (:150-152) is restated as repeated addition from the
 *     start with its length from quotient/remainder in extended precision.
 *   - Spark shuffle order inside groupByKey is taken as map-partition order, then the
 *     fit's output order; DBSCANPoint identity (full Vector equality) is the input index.
 *   - Global id assignment follows localClusterIds in (partition, cluster) order; the
 *     reference's .distinct().collect() order is unspecified: compare up to permutation.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int32_t oracle_fit_sequential(const double* x, const double* y, int64_t n, double eps,
                              int32_t min_points, int32_t mode, int32_t* cluster,
                              uint8_t* flag);


typedef struct { double x, y, x2, y2; } rect_t;

/* Scala Double.intValue: truncation toward zero, NaN -> 0, saturating. */
static int64_t scala_to_int(double v) {
    if (v != v) return 0;
    if (v >= 2147483647.0) return 2147483647;
    if (v <= -2147483648.0) return -2147483648LL;
    return (int64_t)v;
}

/* DBSCAN.scala:352-356 */
static int64_t corner_index(double p, double mrs) {
    double s = p < 0 ? p - mrs : p;
    return scala_to_int(s / mrs);
}

typedef struct {
    double mrs;
    int64_t imin, jmin, W, H; /* dense cell window */
    int64_t* sat;             /* (H+1)*(W+1) */
} grid_t;

static inline double cell_lo(int64_t i, double mrs) { return (double)i * mrs; }
static inline double cell_hi(int64_t i, double mrs) { return (double)i * mrs + mrs; }

/* first index i in [lo, hi) with pred(i) true, for a monotone false..true predicate */
static int64_t first_lo_ge(double bound, int64_t lo, int64_t hi, double mrs) {
    while (lo < hi) {
        int64_t mid = lo + ((hi - lo) >> 1);
        if (bound <= cell_lo(mid, mrs)) hi = mid; else lo = mid + 1;
    }
    return lo;
}
/* last index i in [lo, hi) with cell_hi(i) <= bound, or lo-1 */
static int64_t last_hi_le(double bound, int64_t lo, int64_t hi, double mrs) {
    int64_t a = lo, b = hi;
    while (a < b) {
        int64_t mid = a + ((b - a) >> 1);
        if (cell_hi(mid, mrs) <= bound) a = mid + 1; else b = mid;
    }
    return a - 1;
}

/* EvenSplitPartitioner.scala:175-181 pointsInRectangle, via SAT; cells contained iff
 * rect.x <= c.x && c.x2 <= rect.x2 && rect.y <= c.y && c.y2 <= rect.y2 (DBSCANRectangle:28-30) */
static int64_t points_in(const grid_t* g, rect_t r) {
    int64_t i0 = first_lo_ge(r.x, g->imin, g->imin + g->W, g->mrs);
    int64_t i1 = last_hi_le(r.x2, g->imin, g->imin + g->W, g->mrs);
    int64_t j0 = first_lo_ge(r.y, g->jmin, g->jmin + g->H, g->mrs);
    int64_t j1 = last_hi_le(r.y2, g->jmin, g->jmin + g->H, g->mrs);
    if (i0 > i1 || j0 > j1) return 0;
    int64_t a0 = i0 - g->imin, a1 = i1 - g->imin + 1, b0 = j0 - g->jmin, b1 = j1 - g->jmin + 1;
    const int64_t w = g->W + 1;
    return g->sat[b1 * w + a1] - g->sat[b0 * w + a1] - g->sat[b1 * w + a0] + g->sat[b0 * w + a0];
}

/* Scala 2.10 `(start until end by step)` over Doubles (EvenSplitPartitioner.scala:150-152):
 * NumericRange.count with Numeric.DoubleAsIfIntegral -- BigDecimal(Double.toString(_)) quot
 * and rem at DECIMAL128.  Decimal arithmetic is done on the Python side of the oracle (the
 * `decimal` module: oracle.py scala_range_count) and handed in as a callback, so this
 * restatement shares no code with the product's (csrc/javanum.hip). */
typedef int64_t (*range_count_fn)(double start, double end, double step);
static range_count_fn g_range_count = NULL;
void oracle_set_range_count(range_count_fn fn) { g_range_count = fn; }

static int64_t range_count(double start, double end, double step) {
    return g_range_count ? g_range_count(start, end, step) : -1;
}

typedef struct { rect_t r; int64_t c; } rc_t;

/* HashTrieSet iteration rank of a candidate rectangle (smaller first): oracle/jvm.py */
typedef uint32_t (*split_key_fn)(double x, double y, double x2, double y2);
static split_key_fn g_split_key = NULL;
void oracle_set_split_key(split_key_fn fn) { g_split_key = fn; }

/* EvenSplitPartitioner.scala:105-123 split + :128-143 complement. Returns 0 on error. */
static int split_rect(const grid_t* g, rect_t box, double mrs, rect_t* s1, rect_t* s2) {
    int64_t total = points_in(g, box);
    int64_t half = total / 2; /* Int division, :81 */
    int have = 0;
    rect_t best = box;
    int64_t best_cost = 0;
    int64_t cnts[2];
    for (int axis = 0; axis < 2; ++axis)
        cnts[axis] = range_count((axis == 0 ? box.x : box.y) + mrs, axis == 0 ? box.x2 : box.y2,
                                 mrs);
    /* more than 4 distinct candidates (a step below ulp(v) repeats a value; the x and y
     * candidates never coincide): a HashTrieSet, ties go to the smaller trie rank */
    int64_t dist[2] = {0, 0};
    for (int axis = 0; axis < 2 && cnts[0] + cnts[1] > 4; ++axis) {
        double v = (axis == 0 ? box.x : box.y) + mrs, prev = 0.0;
        for (int64_t k = 0; k < cnts[axis] && dist[axis] < 5; ++k, v += mrs) {
            if (k == 0 || v != prev) ++dist[axis];
            prev = v;
        }
    }
    const int hashed = dist[0] + dist[1] > 4;
    int have_key = 0;
    uint32_t best_key = 0;
    for (int axis = 0; axis < 2; ++axis) {
        double start = (axis == 0 ? box.x : box.y) + mrs;
        double v = start;
        for (int64_t k = 0; k < cnts[axis]; ++k, v += mrs) {
            rect_t cand = axis == 0 ? (rect_t){box.x, box.y, v, box.y2}
                                    : (rect_t){box.x, box.y, box.x2, v};
            int64_t cost = llabs(half - points_in(g, cand));
            if (!have || cost < best_cost) {
                best = cand;
                best_cost = cost;
                have = 1;
                have_key = 0;
            } else if (cost == best_cost && hashed) {
                if (!g_split_key) return 0;
                if (!have_key) {
                    best_key = g_split_key(best.x, best.y, best.x2, best.y2);
                    have_key = 1;
                }
                uint32_t key = g_split_key(cand.x, cand.y, cand.x2, cand.y2);
                if (key < best_key) {
                    best = cand;
                    best_key = key;
                }
            }
        }
    }
    if (!have) return 0;
    *s1 = best;
    if (best.y2 == box.y2) *s2 = (rect_t){best.x2, best.y, box.x2, box.y2};
    else if (best.x2 == box.x2) *s2 = (rect_t){best.x, best.y2, box.x2, box.y2};
    else return 0; /* "rectangle is not a proper sub-rectangle" */
    return 1;
}

static int build_grid(const double* x, const double* y, int64_t n, double mrs, grid_t* g,
                      int64_t* ci, int64_t* cj) {
    memset(g, 0, sizeof(*g));
    g->mrs = mrs;
    int64_t imin = INT64_MAX, imax = INT64_MIN, jmin = INT64_MAX, jmax = INT64_MIN;
    for (int64_t p = 0; p < n; ++p) {
        ci[p] = corner_index(x[p], mrs);
        cj[p] = corner_index(y[p], mrs);
        if (ci[p] < imin) imin = ci[p];
        if (ci[p] > imax) imax = ci[p];
        if (cj[p] < jmin) jmin = cj[p];
        if (cj[p] > jmax) jmax = cj[p];
    }
    if (n == 0) return 1;
    g->imin = imin;
    g->jmin = jmin;
    g->W = imax - imin + 1;
    g->H = jmax - jmin + 1;
    if ((double)(g->W + 1) * (double)(g->H + 1) > 4e8) return 0;
    const int64_t w = g->W + 1;
    g->sat = (int64_t*)calloc((size_t)((g->H + 1) * w), sizeof(int64_t));
    for (int64_t p = 0; p < n; ++p) g->sat[(cj[p] - jmin + 1) * w + (ci[p] - imin + 1)]++;
    for (int64_t b = 1; b <= g->H; ++b)
        for (int64_t a = 1; a <= g->W; ++a)
            g->sat[b * w + a] += g->sat[(b - 1) * w + a] + g->sat[b * w + a - 1] -
                                 g->sat[(b - 1) * w + a - 1];
    return 1;
}

/* EvenSplitPartitioner.findPartitions (:44-64) over the cell histogram of DBSCAN.scala:91-97.
 * Writes up to max_parts partitions (x,y,x2,y2 quadruples + counts) in the reference's list
 * order; returns the partition count, or -1 on error. */
int64_t ref_partition(const double* x, const double* y, int64_t n, double eps,
                      int64_t max_points_per_partition, double* rects_out, int64_t* counts_out,
                      int64_t max_parts) {
    const double mrs = 2 * eps; /* DBSCAN.scala:289 */
    int64_t* ci = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* cj = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    grid_t g;
    if (!build_grid(x, y, n, mrs, &g, ci, cj)) {
        free(ci);
        free(cj);
        return -1;
    }
    free(ci);
    free(cj);
    if (n == 0) return 0;
    /* findBoundingRectangle (:183-209): min/max over the occupied cells' corners */
    rect_t bound = {INFINITY, INFINITY, -INFINITY, -INFINITY};
    {
        const int64_t w = g.W + 1;
        for (int64_t b = 0; b < g.H; ++b)
            for (int64_t a = 0; a < g.W; ++a) {
                int64_t c = g.sat[(b + 1) * w + a + 1] - g.sat[b * w + a + 1] -
                            g.sat[(b + 1) * w + a] + g.sat[b * w + a];
                if (!c) continue;
                double cx = cell_lo(g.imin + a, mrs), cy = cell_lo(g.jmin + b, mrs);
                double cx2 = cx + mrs, cy2 = cy + mrs;
                if (cx < bound.x) bound.x = cx;
                if (cy < bound.y) bound.y = cy;
                if (cx2 > bound.x2) bound.x2 = cx2;
                if (cy2 > bound.y2) bound.y2 = cy2;
            }
    }
    int64_t cap = 1024, top = 0, nout = 0, outcap = 1024;
    rc_t* stack = (rc_t*)malloc(sizeof(rc_t) * (size_t)cap);
    rc_t* out = (rc_t*)malloc(sizeof(rc_t) * (size_t)outcap);
    stack[top++] = (rc_t){bound, points_in(&g, bound)};
    int err = 0;
    while (top > 0) { /* tail-recursive partition(), :66-103 */
        rc_t cur = stack[--top];
        int keep = 1;
        if (cur.c > max_points_per_partition) {
            rect_t b = cur.r;
            if (b.x2 - b.x > mrs * 2 || b.y2 - b.y > mrs * 2) { /* canBeSplit, :168-171 */
                rect_t s1, s2;
                if (!split_rect(&g, b, mrs, &s1, &s2)) {
                    err = 1;
                    break;
                }
                if (top + 2 > cap) {
                    cap *= 2;
                    stack = (rc_t*)realloc(stack, sizeof(rc_t) * (size_t)cap);
                }
                stack[top++] = (rc_t){s2, points_in(&g, s2)};
                stack[top++] = (rc_t){s1, points_in(&g, s1)}; /* s1 :: s2 :: rest */
                keep = 0;
            }
            /* else logWarning("Can't split") and keep, :89-91 */
        }
        if (keep) {
            if (nout == outcap) {
                outcap *= 2;
                out = (rc_t*)realloc(out, sizeof(rc_t) * (size_t)outcap);
            }
            out[nout++] = cur;
        }
    }
    int64_t np = 0;
    if (!err) {
        /* `partitioned` is built by prepending (:91,:96): reverse; then drop empty (:63) */
        for (int64_t k = nout - 1; k >= 0; --k) {
            if (out[k].c <= 0) continue;
            if (np < max_parts) {
                rects_out[4 * np + 0] = out[k].r.x;
                rects_out[4 * np + 1] = out[k].r.y;
                rects_out[4 * np + 2] = out[k].r.x2;
                rects_out[4 * np + 3] = out[k].r.y2;
                counts_out[np] = out[k].c;
            }
            ++np;
        }
    }
    free(stack);
    free(out);
    free(g.sat);
    return err ? -1 : np;
}

/* EvenSplitPartitioner.partition over an explicit (rectangle, count) set, as the reference's
 * EvenSplitPartitionerSuite calls it (:23-60).  Cells must be unit-aligned grid cells of
 * side `mrs`; they are given by their lower corners and counts. */
int64_t ref_partition_cells(const double* cell_x, const double* cell_y, const int64_t* cell_c,
                            int64_t ncells, int64_t max_points_per_partition, double mrs,
                            double* rects_out, int64_t* counts_out, int64_t max_parts) {
    /* expand into pseudo-points at cell centres so corner_index lands in the same cell */
    int64_t total = 0;
    for (int64_t k = 0; k < ncells; ++k) total += cell_c[k];
    double* px = (double*)malloc(sizeof(double) * (size_t)(total > 0 ? total : 1));
    double* py = (double*)malloc(sizeof(double) * (size_t)(total > 0 ? total : 1));
    int64_t t = 0;
    for (int64_t k = 0; k < ncells; ++k)
        for (int64_t c = 0; c < cell_c[k]; ++c) {
            px[t] = cell_x[k] + 0.5 * mrs;
            py[t] = cell_y[k] + 0.5 * mrs;
            ++t;
        }
    int64_t r = ref_partition(px, py, total, mrs / 2, max_points_per_partition, rects_out,
                              counts_out, max_parts);
    free(px);
    free(py);
    return r;
}

/* ---------------------------- local fits over partitions ---------------------------------- */

static inline int rect_contains_pt(const double* r, double x, double y) { /* :34-37 */
    return r[0] <= x && x <= r[2] && r[1] <= y && y <= r[3];
}
static inline int rect_almost_contains_pt(const double* r, double x, double y) { /* :50-52 */
    return r[0] < x && x < r[2] && r[1] < y && y < r[3];
}
static inline void shrink(const double* r, double a, double* o) { /* :42-44 */
    o[0] = r[0] + a;
    o[1] = r[1] + a;
    o[2] = r[2] - a;
    o[3] = r[3] - a;
}

typedef struct {
    const double* x;
    const double* y;
    int64_t n;
    double eps;
    int32_t min_points;
    const double* rects;
    int64_t nparts;
    /* per partition outputs */
    int64_t** members; /* input indices of the partition's outer points, input order */
    int64_t* msize;
    int32_t** cl;
    uint8_t** fl;
    /* work queue */
    int64_t next;
    int64_t limit;
    pthread_mutex_t mu;
    double deadline; /* CLOCK_MONOTONIC seconds; <= 0: none */
    int64_t done_parts;
    int64_t done_points; /* outer points fitted */
} fit_ctx;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void* fit_worker(void* arg) {
    fit_ctx* f = (fit_ctx*)arg;
    for (;;) {
        pthread_mutex_lock(&f->mu);
        int64_t p = f->next;
        int stop = p >= f->limit || (f->deadline > 0 && now_s() > f->deadline);
        if (!stop) f->next++;
        pthread_mutex_unlock(&f->mu);
        if (stop) break;
        int64_t m = f->msize[p];
        double* px = (double*)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1));
        double* py = (double*)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1));
        for (int64_t k = 0; k < m; ++k) {
            px[k] = f->x[f->members[p][k]];
            py[k] = f->y[f->members[p][k]];
        }
        /* DBSCAN.scala:153-154: new LocalDBSCANNaive(eps, minPoints).fit(points) */
        oracle_fit_sequential(px, py, m, f->eps, f->min_points, 0, f->cl[p], f->fl[p]);
        free(px);
        free(py);
        pthread_mutex_lock(&f->mu);
        f->done_parts++;
        f->done_points += m;
        pthread_mutex_unlock(&f->mu);
    }
    return NULL;
}

static int cmp_i64(const void* a, const void* b) {
    int64_t u = *(const int64_t*)a, v = *(const int64_t*)b;
    return (u > v) - (u < v);
}

static void collect_members(fit_ctx* f) {
    /* DBSCAN.scala:132-137: (id, point) for every margin whose outer contains the point.
     * Points are bucketed on the 2*eps cell grid (DBSCAN.scala:345-356) so each outer
     * rectangle only tests points of the cells it overlaps (+1 cell of slack); membership is
     * still decided by the exact inclusive contains (DBSCANRectangle.scala:34-37). */
    const int64_t np = f->nparts > 0 ? f->nparts : 1;
    f->members = (int64_t**)calloc((size_t)np, sizeof(int64_t*));
    f->msize = (int64_t*)calloc((size_t)np, sizeof(int64_t));
    f->cl = (int32_t**)calloc((size_t)np, sizeof(int32_t*));
    f->fl = (uint8_t**)calloc((size_t)np, sizeof(uint8_t*));
    const double mrs = 2 * f->eps;
    int64_t n = f->n;
    int64_t* ci = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* cj = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t imin = INT64_MAX, imax = INT64_MIN, jmin = INT64_MAX, jmax = INT64_MIN;
    for (int64_t p = 0; p < n; ++p) {
        ci[p] = corner_index(f->x[p], mrs);
        cj[p] = corner_index(f->y[p], mrs);
        if (ci[p] < imin) imin = ci[p];
        if (ci[p] > imax) imax = ci[p];
        if (cj[p] < jmin) jmin = cj[p];
        if (cj[p] > jmax) jmax = cj[p];
    }
    int64_t W = n ? imax - imin + 1 : 1, H = n ? jmax - jmin + 1 : 1;
    int dense = (double)W * (double)H <= 4e8;
    int64_t* start = NULL;
    int64_t* order = NULL;
    if (dense && n) { /* counting sort of points by cell, stable (input order inside a cell) */
        start = (int64_t*)calloc((size_t)(W * H + 1), sizeof(int64_t));
        order = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
        for (int64_t p = 0; p < n; ++p) start[(cj[p] - jmin) * W + (ci[p] - imin) + 1]++;
        for (int64_t c = 0; c < W * H; ++c) start[c + 1] += start[c];
        int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(W * H));
        memcpy(cur, start, sizeof(int64_t) * (size_t)(W * H));
        for (int64_t p = 0; p < n; ++p) order[cur[(cj[p] - jmin) * W + (ci[p] - imin)]++] = p;
        free(cur);
    }
    for (int64_t q = 0; q < f->nparts; ++q) {
        double outer[4];
        shrink(&f->rects[4 * q], -f->eps, outer);
        int64_t cap = 0, m = 0;
        int64_t* mem = NULL;
        if (dense) {
            int64_t i0 = corner_index(outer[0], mrs) - 1, i1 = corner_index(outer[2], mrs) + 1;
            int64_t j0 = corner_index(outer[1], mrs) - 1, j1 = corner_index(outer[3], mrs) + 1;
            if (i0 < imin) i0 = imin;
            if (j0 < jmin) j0 = jmin;
            if (i1 > imax) i1 = imax;
            if (j1 > jmax) j1 = jmax;
            for (int64_t j = j0; j <= j1; ++j)
                for (int64_t i = i0; i <= i1; ++i) {
                    int64_t c = (j - jmin) * W + (i - imin);
                    for (int64_t t = start[c]; t < start[c + 1]; ++t) {
                        int64_t p = order[t];
                        if (!rect_contains_pt(outer, f->x[p], f->y[p])) continue;
                        if (m == cap) {
                            cap = cap ? 2 * cap : 64;
                            mem = (int64_t*)realloc(mem, sizeof(int64_t) * (size_t)cap);
                        }
                        mem[m++] = p;
                    }
                }
            qsort(mem, (size_t)m, sizeof(int64_t), cmp_i64); /* groupByKey order = input order */
        } else {
            for (int64_t p = 0; p < n; ++p) {
                if (!rect_contains_pt(outer, f->x[p], f->y[p])) continue;
                if (m == cap) {
                    cap = cap ? 2 * cap : 64;
                    mem = (int64_t*)realloc(mem, sizeof(int64_t) * (size_t)cap);
                }
                mem[m++] = p;
            }
        }
        f->members[q] = mem;
        f->msize[q] = m;
        f->cl[q] = (int32_t*)malloc(sizeof(int32_t) * (size_t)(m + 1));
        f->fl[q] = (uint8_t*)malloc((size_t)(m + 1));
    }
    free(start);
    free(order);
    free(ci);
    free(cj);
}

static void free_fit(fit_ctx* f) {
    for (int64_t p = 0; p < f->nparts; ++p) {
        free(f->members[p]);
        free(f->cl[p]);
        free(f->fl[p]);
    }
    free(f->members);
    free(f->msize);
    free(f->cl);
    free(f->fl);
}

static void run_fits(fit_ctx* f, int nthreads) {
    pthread_mutex_init(&f->mu, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 512) nthreads = 512;
    pthread_t th[512];
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fit_worker, f);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&f->mu);
}

/* CPU baseline: LocalDBSCANNaive.fit (restated) on the reference's partitions, N threads,
 * stopping at `time_budget_s` (the partition in flight completes).  Returns elapsed seconds;
 * *points_done = outer points fitted, *main_points_done = sum of partition main counts. */
double ref_fit_partitions_timed(const double* x, const double* y, int64_t n, double eps,
                                int32_t min_points, const double* rects,
                                const int64_t* counts, int64_t nparts, int32_t nthreads,
                                double time_budget_s, int64_t* parts_done,
                                int64_t* points_done, int64_t* main_points_done) {
    fit_ctx f;
    memset(&f, 0, sizeof(f));
    f.x = x;
    f.y = y;
    f.n = n;
    f.eps = eps;
    f.min_points = min_points;
    f.rects = rects;
    f.nparts = nparts;
    f.limit = nparts;
    collect_members(&f);
    double t0 = now_s();
    f.deadline = time_budget_s > 0 ? t0 + time_budget_s : 0;
    run_fits(&f, nthreads);
    double el = now_s() - t0;
    /* partitions are taken in list order, so the first done_parts are the finished ones */
    int64_t mp = 0;
    for (int64_t p = 0; p < f.done_parts && p < nparts; ++p) mp += counts[p];
    *parts_done = f.done_parts;
    *points_done = f.done_points;
    *main_points_done = mp;
    free_fit(&f);
    return el;
}

/* ---------------------------------- merge (DBSCAN.scala:158-270) ------------------------ */

typedef struct { int64_t a, b; } edge_t;

static int64_t uf_find64(int64_t* par, int64_t a) {
    while (par[a] != a) {
        par[a] = par[par[a]];
        a = par[a];
    }
    return a;
}

/* Full DBSCAN.train restatement.  Output per input point: final global cluster and flag
 * as the reference's labeledPoints would hold them after collectAsMap (last record for a
 * point wins), out_count[i] = number of records for point i in labeledPoints (0 = lost,
 * >1 = duplicated).  Returns the number of global clusters or -1 on error. */
int64_t ref_train(const double* x, const double* y, int64_t n, double eps, int32_t min_points,
                  int64_t max_points_per_partition, int32_t nthreads, int32_t* cluster_out,
                  uint8_t* flag_out, int32_t* out_count, int64_t* nparts_out,
                  double* rects_out, int64_t max_parts) {
    int64_t cap = 4096;
    double* rects = (double*)malloc(sizeof(double) * 4 * (size_t)cap);
    int64_t* counts = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    int64_t np = ref_partition(x, y, n, eps, max_points_per_partition, rects, counts, cap);
    if (np > cap) {
        cap = np;
        rects = (double*)realloc(rects, sizeof(double) * 4 * (size_t)cap);
        counts = (int64_t*)realloc(counts, sizeof(int64_t) * (size_t)cap);
        np = ref_partition(x, y, n, eps, max_points_per_partition, rects, counts, cap);
    }
    if (np < 0) {
        free(rects);
        free(counts);
        return -1;
    }
    *nparts_out = np;
    for (int64_t p = 0; p < np && p < max_parts; ++p)
        memcpy(&rects_out[4 * p], &rects[4 * p], 4 * sizeof(double));
    fit_ctx f;
    memset(&f, 0, sizeof(f));
    f.x = x;
    f.y = y;
    f.n = n;
    f.eps = eps;
    f.min_points = min_points;
    f.rects = rects;
    f.nparts = np;
    f.limit = np;
    collect_members(&f);
    run_fits(&f, nthreads);

    /* local cluster ids -> node ids: node(p, c) = base[p] + c - 1 */
    int64_t* base = (int64_t*)calloc((size_t)(np + 1), sizeof(int64_t));
    for (int64_t p = 0; p < np; ++p) {
        int32_t mx = 0;
        for (int64_t k = 0; k < f.msize[p]; ++k)
            if (f.cl[p][k] > mx) mx = f.cl[p][k];
        base[p + 1] = base[p] + mx;
    }
    int64_t nnodes = base[np];
    int64_t* par = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nnodes > 0 ? nnodes : 1));
    for (int64_t v = 0; v < nnodes; ++v) par[v] = v;

    /* mergePoints (:161-173): for each clustered (partition, point) and each margin whose
     * main contains the point but whose inner does not almostContain it -> group newPartition.
     * findAdjacencies (:317-342): first non-Noise (partition, cluster) seen for a point, then
     * an edge to each later non-Noise copy.  The edges feed DBSCANGraph (connectivity). */
    int64_t* seen_node = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int32_t* seen_grp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) seen_grp[i] = -1;
    /* labeledOuter dedup: per group, first record of a point inserted; later non-Noise
     * records override flag/cluster (:248-270). */
    int64_t* out_node = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    uint8_t* out_flag = (uint8_t*)malloc((size_t)(n > 0 ? n : 1));
    int32_t* out_grp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        out_count[i] = 0;
        cluster_out[i] = 0;
        flag_out[i] = 3;
        out_grp[i] = -1;
    }
    /* final assignment is done after global ids exist; record (point, node, flag) tuples */
    int64_t rec_cap = 1024, nrec = 0;
    int64_t* rec_pt = (int64_t*)malloc(sizeof(int64_t) * (size_t)rec_cap);
    int64_t* rec_node = (int64_t*)malloc(sizeof(int64_t) * (size_t)rec_cap);
    uint8_t* rec_flag = (uint8_t*)malloc((size_t)rec_cap);

    /* The reference tests every margin for every clustered point (a Spark flatMap over the
     * margins list, O(points x partitions)).  Same decisions here, indexed: the mains are
     * bucketed on the 2*eps cell grid (corner_index is monotone, so a main containing a point
     * is listed in that point's cell), each point tests only its cell's mains with the exact
     * predicates, and the (group, partition, point) records are put back in the reference's
     * iteration order -- groups in id order, partitions in id order, points in partition
     * order -- by a stable counting sort on the group. */
    int64_t nmrec = 0;
    int64_t* mr_g = NULL;
    int64_t* mr_p = NULL;
    int64_t* mr_k = NULL;
    {
        const double mrs = 2 * eps;
        int64_t imin = INT64_MAX, imax = INT64_MIN, jmin = INT64_MAX, jmax = INT64_MIN;
        for (int64_t p = 0; p < np; ++p)
            for (int64_t k = 0; k < f.msize[p]; ++k) {
                int64_t i = f.members[p][k];
                int64_t ci = corner_index(x[i], mrs), cj = corner_index(y[i], mrs);
                if (ci < imin) imin = ci;
                if (ci > imax) imax = ci;
                if (cj < jmin) jmin = cj;
                if (cj > jmax) jmax = cj;
            }
        int64_t W = imin <= imax ? imax - imin + 1 : 1, H = jmin <= jmax ? jmax - jmin + 1 : 1;
        if (imin > imax) imin = imax = jmin = jmax = 0;
        int64_t* bstart = (int64_t*)calloc((size_t)(W * H + 1), sizeof(int64_t));
        for (int pass = 0; pass < 2; ++pass) { /* count, then fill */
            int64_t* bl = pass ? (int64_t*)malloc(sizeof(int64_t) * (size_t)(bstart[W * H] + 1)) : NULL;
            int64_t* cur = NULL;
            if (pass) {
                cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(W * H));
                memcpy(cur, bstart, sizeof(int64_t) * (size_t)(W * H));
            }
            for (int64_t g = 0; g < np; ++g) {
                const double* mg = &rects[4 * g];
                int64_t i0 = corner_index(mg[0], mrs) - 1, i1 = corner_index(mg[2], mrs) + 1;
                int64_t j0 = corner_index(mg[1], mrs) - 1, j1 = corner_index(mg[3], mrs) + 1;
                if (i0 < imin) i0 = imin;
                if (j0 < jmin) j0 = jmin;
                if (i1 > imax) i1 = imax;
                if (j1 > jmax) j1 = jmax;
                for (int64_t j = j0; j <= j1; ++j)
                    for (int64_t i = i0; i <= i1; ++i) {
                        int64_t c = (j - jmin) * W + (i - imin);
                        if (pass) bl[cur[c]++] = g;
                        else bstart[c + 1]++;
                    }
            }
            if (!pass) {
                for (int64_t c = 0; c < W * H; ++c) bstart[c + 1] += bstart[c];
                continue;
            }
            free(cur);
            /* records, partition-major; gcount for the stable sort by group */
            int64_t* gcount = (int64_t*)calloc((size_t)(np + 1), sizeof(int64_t));
            int64_t cap2 = 1024, m2 = 0;
            int64_t* tg = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap2);
            int64_t* tp = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap2);
            int64_t* tk = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap2);
            for (int64_t p = 0; p < np; ++p)
                for (int64_t k = 0; k < f.msize[p]; ++k) {
                    int64_t i = f.members[p][k];
                    int64_t c = (corner_index(y[i], mrs) - jmin) * W + (corner_index(x[i], mrs) - imin);
                    for (int64_t t = bstart[c]; t < bstart[c + 1]; ++t) {
                        int64_t g = bl[t];
                        double inner_g[4];
                        shrink(&rects[4 * g], eps, inner_g);
                        if (!(rect_contains_pt(&rects[4 * g], x[i], y[i]) &&
                              !rect_almost_contains_pt(inner_g, x[i], y[i])))
                            continue;
                        if (m2 == cap2) {
                            cap2 *= 2;
                            tg = (int64_t*)realloc(tg, sizeof(int64_t) * (size_t)cap2);
                            tp = (int64_t*)realloc(tp, sizeof(int64_t) * (size_t)cap2);
                            tk = (int64_t*)realloc(tk, sizeof(int64_t) * (size_t)cap2);
                        }
                        tg[m2] = g;
                        tp[m2] = p;
                        tk[m2] = k;
                        ++m2;
                        gcount[g + 1]++;
                    }
                }
            for (int64_t g = 0; g < np; ++g) gcount[g + 1] += gcount[g];
            mr_g = (int64_t*)malloc(sizeof(int64_t) * (size_t)(m2 + 1));
            mr_p = (int64_t*)malloc(sizeof(int64_t) * (size_t)(m2 + 1));
            mr_k = (int64_t*)malloc(sizeof(int64_t) * (size_t)(m2 + 1));
            for (int64_t r = 0; r < m2; ++r) {
                int64_t o = gcount[tg[r]]++;
                mr_g[o] = tg[r];
                mr_p[o] = tp[r];
                mr_k[o] = tk[r];
            }
            nmrec = m2;
            free(tg);
            free(tp);
            free(tk);
            free(gcount);
            free(bl);
        }
        free(bstart);
    }
    for (int64_t r = 0; r < nmrec; ++r) { /* each merge group (newPartition), in id order */
        const int64_t g = mr_g[r], p = mr_p[r], k = mr_k[r];
        {
            {
                int64_t i = f.members[p][k];
                uint8_t fl = f.fl[p][k];
                int64_t node = fl != 2 ? base[p] + f.cl[p][k] - 1 : -1;
                if (fl != 2) { /* findAdjacencies */
                    if (seen_grp[i] != (int32_t)g) {
                        seen_grp[i] = (int32_t)g;
                        seen_node[i] = node;
                    } else {
                        int64_t ra = uf_find64(par, seen_node[i]), rb = uf_find64(par, node);
                        if (ra != rb) par[ra < rb ? rb : ra] = ra < rb ? ra : rb;
                    }
                }
                if (out_grp[i] != (int32_t)g) { /* first record of this point in group g */
                    if (out_grp[i] >= 0) { /* flush the previous group's record */
                        if (nrec == rec_cap) {
                            rec_cap *= 2;
                            rec_pt = (int64_t*)realloc(rec_pt, sizeof(int64_t) * (size_t)rec_cap);
                            rec_node = (int64_t*)realloc(rec_node, sizeof(int64_t) * (size_t)rec_cap);
                            rec_flag = (uint8_t*)realloc(rec_flag, (size_t)rec_cap);
                        }
                        rec_pt[nrec] = i;
                        rec_node[nrec] = out_node[i];
                        rec_flag[nrec] = out_flag[i];
                        ++nrec;
                    }
                    out_grp[i] = (int32_t)g;
                    out_node[i] = node;
                    out_flag[i] = fl;
                } else if (fl != 2) { /* override unless the new entry is noise */
                    out_node[i] = node;
                    out_flag[i] = fl;
                }
            }
        }
    }
    free(mr_g);
    free(mr_p);
    free(mr_k);
    for (int64_t i = 0; i < n; ++i) { /* flush the last group records */
        if (out_grp[i] < 0) continue;
        if (nrec == rec_cap) {
            rec_cap *= 2;
            rec_pt = (int64_t*)realloc(rec_pt, sizeof(int64_t) * (size_t)rec_cap);
            rec_node = (int64_t*)realloc(rec_node, sizeof(int64_t) * (size_t)rec_cap);
            rec_flag = (uint8_t*)realloc(rec_flag, (size_t)rec_cap);
        }
        rec_pt[nrec] = i;
        rec_node[nrec] = out_node[i];
        rec_flag[nrec] = out_flag[i];
        ++nrec;
    }
    /* global ids (:194-222): over local cluster ids that carry a non-Noise point */
    int64_t* gid = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nnodes > 0 ? nnodes : 1));
    for (int64_t v = 0; v < nnodes; ++v) gid[v] = 0;
    int64_t total = 0;
    for (int64_t v = 0; v < nnodes; ++v) {
        int64_t r = uf_find64(par, v);
        if (gid[r] == 0) gid[r] = ++total;
    }
    /* labeledInner (:232-244): clustered points that their own inner almostContains */
    for (int64_t p = 0; p < np; ++p) {
        double inner_p[4];
        shrink(&rects[4 * p], eps, inner_p);
        for (int64_t k = 0; k < f.msize[p]; ++k) {
            int64_t i = f.members[p][k];
            if (!rect_almost_contains_pt(inner_p, x[i], y[i])) continue;
            uint8_t fl = f.fl[p][k];
            cluster_out[i] = fl != 2 ? (int32_t)gid[uf_find64(par, base[p] + f.cl[p][k] - 1)] : 0;
            flag_out[i] = fl;
            out_count[i]++;
        }
    }
    for (int64_t r = 0; r < nrec; ++r) { /* labeledOuter */
        int64_t i = rec_pt[r];
        cluster_out[i] = rec_flag[r] != 2 ? (int32_t)gid[uf_find64(par, rec_node[r])] : 0;
        flag_out[i] = rec_flag[r];
        out_count[i]++;
    }
    free(rec_pt);
    free(rec_node);
    free(rec_flag);
    free(gid);
    free(seen_node);
    free(seen_grp);
    free(out_node);
    free(out_flag);
    free(out_grp);
    free(par);
    free(base);
    free_fit(&f);
    free(rects);
    free(counts);
    return total;
}
