/*
 * dbscan_oracle.c -- CPU ORACLE for the local DBSCAN fit.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (dbscan-on-spark_amd/csrc, libdbscan_hip.so) never links or calls it.
 *
 * The reference (Scala 2.10 + Spark 2.1.0 + archery 0.3.0) cannot be built here: no JVM,
 * no scalac/sbt/mvn, no jars, no network.  This file is a CPU restatement
 * of its hot path, pinned by the reference's own golden fixture
 * src/test/resources/labeled_data.csv (see tests/test_oracle.py).
 *
 * Reference files restated (paths relative to
 * /root/reference/src/main/scala/org/apache/spark/mllib/clustering/dbscan/):
 *   DBSCANPoint.scala:26-30          distanceSquared: dx=o.x-x; dy=o.y-y; dx*dx+dy*dy (fp64, no FMA)
 *   LocalDBSCANNaive.scala:33        minDistanceSquared = eps * eps
 *   LocalDBSCANNaive.scala:37-70     fit: visit points in array order, Noise / new cluster
 *   LocalDBSCANNaive.scala:72-78     findNeighbors: all.view.filter(d2 <= eps2) (includes self)
 *   LocalDBSCANNaive.scala:80-118    expandCluster: BFS; visited Noise never re-claimed
 *   LocalDBSCANArchery.scala:36-124  same BFS but Noise re-claimed as Border (:103-106 / file
 *                                    lines 223-226), float32 search box (:118-124)
 *   DBSCANLabeledPoint.scala:26,30   Unknown = 0; Flag {Border=0, Core=1, Noise=2, NotFlagged=3}
 *
 * Three independent formulations are provided:
 *   oracle_fit_sequential   literal sequential BFS restatement, O(n^2) (small n)
 *   oracle_fit_bruteforce   order-parametrised closed form with all-pairs counts
 *   oracle_fit_grid         the same closed form on an eps grid, pthreads (large n; also the
 *                           "strong CPU comparator" of BASELINE.md)
 *   oracle_fit_bfs_grid     the literal sequential BFS of (1) with its neighbour queries on the
 *                           eps grid (large n, every mode: the reference for archery's float32
 *                           search box, whose directed neighbour relation the closed form
 *                           does not cover)
 * tests/ fuzz all three against each other and against the golden fixture.
 *
 * MUST be compiled with -ffp-contract=off (see oracle/Makefile): the JVM never fuses
 * dx*dx+dy*dy into an FMA, so neither may we.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define FLAG_BORDER 0
#define FLAG_CORE 1
#define FLAG_NOISE 2
#define FLAG_NOTFLAGGED 3

#define MODE_NAIVE 0
#define MODE_ARCHERY 1
#define MODE_ARCHERY_F32BOX 2 /* sequential oracle only: archery's float32 search box */


/* DBSCANPoint.scala:26-30 used as `d2 <= minDistanceSquared` (LocalDBSCANNaive.scala:77). */
static inline int within(double px, double py, double ox, double oy, double eps2) {
    double dx = ox - px;
    double dy = oy - py;
    double a = dx * dx;
    double b = dy * dy;
    double d2 = a + b;
    return d2 <= eps2;
}

/* LocalDBSCANArchery.scala:118-124 toBoundingBox: Box((x-eps).toFloat, (y-eps).toFloat,
 * (x+eps).toFloat, (y+eps).toFloat); the tree stores Point(p.x.toFloat, p.y.toFloat)
 * (:38-41).  Containment taken inclusive (archery 0.3.0 source absent: parity unpinned). */
static inline int in_f32_box(double px, double py, double ox, double oy, double eps) {
    float x1 = (float)(px - eps), y1 = (float)(py - eps);
    float x2 = (float)(px + eps), y2 = (float)(py + eps);
    float fx = (float)ox, fy = (float)oy;
    return x1 <= fx && fx <= x2 && y1 <= fy && fy <= y2;
}

static inline int is_neighbor(const double* x, const double* y, int64_t p, int64_t o,
                              double eps, double eps2, int mode) {
    if (!within(x[p], y[p], x[o], y[o], eps2)) return 0;
    if (mode == MODE_ARCHERY_F32BOX && !in_f32_box(x[p], y[p], x[o], y[o], eps)) return 0;
    return 1;
}

static int64_t count_all(const double* x, const double* y, int64_t n, int64_t p, double eps,
                         double eps2, int mode) {
    int64_t c = 0;
    for (int64_t o = 0; o < n; ++o) c += is_neighbor(x, y, p, o, eps, eps2, mode);
    return c;
}

/* ------------------------------------------------------------------------------------------
 * 1. Literal sequential restatement.  LocalDBSCANNaive.scala:37-118 (mode 0) and
 *    LocalDBSCANArchery.scala:36-112 (modes 1,2) with the visit order pi = array order.
 *    The reference's queue holds neighbour *views* (lazy filters over `all`, :89,:103);
 *    evaluating a view when dequeued yields the same index list as evaluating it when
 *    enqueued (positions never change), so the queue stores the view's centre index.
 * ------------------------------------------------------------------------------------------ */
int32_t oracle_fit_sequential(const double* x, const double* y, int64_t n, double eps,
                              int32_t min_points, int32_t mode, int32_t* cluster,
                              uint8_t* flag) {
    const double eps2 = eps * eps; /* LocalDBSCANNaive.scala:33 */
    uint8_t* visited = (uint8_t*)calloc((size_t)(n > 0 ? n : 1), 1);
    int64_t* queue = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        cluster[i] = 0;           /* DBSCANLabeledPoint.Unknown */
        flag[i] = FLAG_NOTFLAGGED; /* DBSCANLabeledPoint.scala:39 */
    }
    int32_t total = 0;
    for (int64_t i = 0; i < n; ++i) { /* foldLeft over labeledPoints, :45-64 */
        if (visited[i]) continue;
        visited[i] = 1;
        int64_t cnt = count_all(x, y, n, i, eps, eps2, mode); /* neighbors.size, :52-54 */
        if (cnt < (int64_t)min_points) {
            flag[i] = FLAG_NOISE; /* :55 */
            continue;
        }
        const int32_t c = ++total; /* expandCluster(point, neighbors, all, cluster + 1), :58 */
        flag[i] = FLAG_CORE;       /* :86 */
        cluster[i] = c;            /* :87 */
        int64_t qh = 0, qt = 0;
        queue[qt++] = i; /* Queue(neighbors), :89 */
        while (qh < qt) {
            const int64_t centre = queue[qh++];
            for (int64_t j = 0; j < n; ++j) { /* dequeue().foreach, :93 */
                if (!is_neighbor(x, y, centre, j, eps, eps2, mode)) continue;
                if (!visited[j]) { /* :94 */
                    visited[j] = 1;
                    cluster[j] = c;
                    int64_t nn = count_all(x, y, n, j, eps, eps2, mode); /* :99 */
                    if (nn >= (int64_t)min_points) {
                        flag[j] = FLAG_CORE; /* :102 */
                        queue[qt++] = j;     /* enqueue(neighborNeighbors), :103 */
                    } else {
                        flag[j] = FLAG_BORDER; /* :105 */
                    }
                    /* Naive :108-111 (cluster == Unknown) is dead code: cluster was set above. */
                }
                if (mode != MODE_NAIVE && cluster[j] == 0) {
                    /* LocalDBSCANArchery.scala:103-106: outside the !visited test, so an
                     * earlier Noise point is re-claimed as Border. */
                    cluster[j] = c;
                    flag[j] = FLAG_BORDER;
                }
            }
        }
    }
    free(visited);
    free(queue);
    return total;
}

/* ------------------------------------------------------------------------------------------
 * Union-find keyed by point index; hooking the larger root under the smaller makes every
 * root the minimum visit index of its component, i.e. s(K) of SURVEY §8a-4.
 * ------------------------------------------------------------------------------------------ */
static inline int64_t uf_find(int64_t* parent, int64_t a) {
    for (;;) {
        int64_t p = __atomic_load_n(&parent[a], __ATOMIC_RELAXED);
        if (p == a) return a;
        int64_t gp = __atomic_load_n(&parent[p], __ATOMIC_RELAXED);
        if (gp != p) __atomic_store_n(&parent[a], gp, __ATOMIC_RELAXED); /* path halving */
        a = gp;
    }
}

static inline void uf_union(int64_t* parent, int64_t a, int64_t b) {
    for (;;) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a < b) { int64_t t = a; a = b; b = t; } /* a > b: hook a under b */
        int64_t expect = a;
        if (__atomic_compare_exchange_n(&parent[a], &expect, b, 0, __ATOMIC_RELAXED,
                                        __ATOMIC_RELAXED))
            return;
    }
}

/* Closed form, given counts and core-core components:
 *   core(p) <=> |N(p)| >= minPoints; cluster id = rank of s(K) in increasing order;
 *   non-core b, A = clusters with a core neighbour of b, m = min_{K in A} s(K):
 *     naive:   Noise if A empty or pi(b) < m, else Border of the cluster with s = m
 *     archery: Noise if A empty, else Border of the cluster with s = m                   */
static int32_t finish_labels(int64_t n, const uint8_t* core, int64_t* parent,
                             const int64_t* border_min, int32_t mode, int32_t* cluster,
                             uint8_t* flag) {
    int32_t* id = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t k = 0;
    for (int64_t i = 0; i < n; ++i) {
        id[i] = 0;
        if (core[i] && uf_find(parent, i) == i) id[i] = ++k;
    }
    for (int64_t i = 0; i < n; ++i) {
        if (core[i]) {
            flag[i] = FLAG_CORE;
            cluster[i] = id[uf_find(parent, i)];
        } else {
            int64_t m = border_min[i];
            int ok = (m >= 0) && (mode == MODE_NAIVE ? (m < i) : 1);
            flag[i] = ok ? FLAG_BORDER : FLAG_NOISE;
            cluster[i] = ok ? id[m] : 0;
        }
    }
    free(id);
    return k;
}

/* ------------------------------------------------------------------------------------------
 * 2. Closed form with all-pairs neighbour scans (O(n^2), small n).
 * ------------------------------------------------------------------------------------------ */
int32_t oracle_fit_bruteforce(const double* x, const double* y, int64_t n, double eps,
                              int32_t min_points, int32_t mode, int32_t* cluster,
                              uint8_t* flag, int64_t* counts_out) {
    const double eps2 = eps * eps;
    size_t nn = (size_t)(n > 0 ? n : 1);
    uint8_t* core = (uint8_t*)malloc(nn);
    int64_t* parent = (int64_t*)malloc(sizeof(int64_t) * nn);
    int64_t* bmin = (int64_t*)malloc(sizeof(int64_t) * nn);
    for (int64_t i = 0; i < n; ++i) {
        int64_t c = count_all(x, y, n, i, eps, eps2, MODE_NAIVE);
        if (counts_out) counts_out[i] = c;
        core[i] = c >= (int64_t)min_points;
        parent[i] = i;
    }
    for (int64_t i = 0; i < n; ++i) {
        if (!core[i]) continue;
        for (int64_t j = 0; j < i; ++j)
            if (core[j] && within(x[i], y[i], x[j], y[j], eps2)) uf_union(parent, i, j);
    }
    for (int64_t i = 0; i < n; ++i) {
        bmin[i] = -1;
        if (core[i]) continue;
        for (int64_t j = 0; j < n; ++j) {
            if (!core[j] || !within(x[i], y[i], x[j], y[j], eps2)) continue;
            int64_t s = uf_find(parent, j);
            if (bmin[i] < 0 || s < bmin[i]) bmin[i] = s;
        }
    }
    int32_t k = finish_labels(n, core, parent, bmin, mode, cluster, flag);
    free(core);
    free(parent);
    free(bmin);
    return k;
}

/* ------------------------------------------------------------------------------------------
 * 3. Closed form on an eps grid (pthreads).
 *
 * Grid soundness: if fl(dx*dx)+fl(dy*dy) rounds to <= eps2 = fl(eps*eps) then
 * |x'-x| <= R = max(|eps|*(1+2^-40), 2^-500) (the 2^-500 floor covers squares that
 * underflow to 0 when eps is tiny or zero).  With cell side h >= R*(1+2^-20) and cell
 * coordinates computed with a relative error far below 2^-20, true neighbours always
 * sit in the same or an adjacent cell.  Non-finite coordinates never satisfy the
 * predicate while eps2 is finite, so they are kept out of the grid (count 0).
 * eps2 = +inf (|eps| > ~1.3e154) degenerates to one all-pairs cell; eps2 = NaN has no pairs.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    const double* x;
    const double* y;
    int64_t n;
    double eps2;
    int32_t min_points;
    int all_pairs; /* eps2 == +inf */
    int no_pairs;  /* eps2 is NaN */
    /* grid */
    int64_t nx, ny;
    double xmin2, ymin2, invx, invy; /* cell = floor((v/2 - vmin/2) * inv) */
    int64_t* order;                  /* point indices sorted by cell key (finite only) */
    int64_t* okey;                   /* cell key per sorted slot */
    int64_t nfinite;
    int64_t* ckey;   /* unique cell keys */
    int64_t* cstart; /* start slot of each cell, cstart[ncells] = nfinite */
    int64_t ncells;
    int64_t* cell_of; /* cell index per point (or -1) */
    double* sx;       /* coordinates in sorted-slot order (cache locality only) */
    double* sy;
    uint8_t* score;   /* core flag per sorted slot */
    int64_t next;     /* dynamic cell counter of the running phase */
    uint8_t* core;
    int64_t* counts;
    int64_t* parent;
    int64_t* bmin;
} grid_ctx;

static int64_t lower_bound_key(const int64_t* a, int64_t n, int64_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = lo + ((hi - lo) >> 1);
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* The (up to) 3 contiguous slot ranges of the 3x3 stencil of cell c. */
static int stencil_ranges(const grid_ctx* g, int64_t c, int64_t b[3], int64_t e[3]) {
    int64_t key = g->ckey[c];
    int64_t cy = key / g->nx, cx = key % g->nx;
    int nr = 0;
    for (int64_t dy = -1; dy <= 1; ++dy) {
        int64_t ry = cy + dy;
        if (ry < 0 || ry >= g->ny) continue;
        int64_t lox = cx > 0 ? cx - 1 : cx, hix = cx + 1 < g->nx ? cx + 1 : cx;
        int64_t klo = ry * g->nx + lox, khi = ry * g->nx + hix;
        int64_t a = lower_bound_key(g->ckey, g->ncells, klo);
        int64_t z = lower_bound_key(g->ckey, g->ncells, khi + 1);
        if (a < z) {
            b[nr] = g->cstart[a];
            e[nr] = g->cstart[z];
            ++nr;
        }
    }
    return nr;
}

typedef struct {
    grid_ctx* g;
    int64_t lo, hi;
    int phase;
} job;

/* Grid fits, cell-major: a worker takes chunks of cells (dynamic, for the dense cells of
 * skewed data), computes each cell's stencil ranges once and runs the phase for every point of
 * the cell over the sorted-slot coordinates.  Same predicate, same per-point results as the
 * point-major loop below; only the iteration order (and so the cache behaviour) differs. */
static void* grid_cell_worker(void* arg) {
    job* jb = (job*)arg;
    grid_ctx* g = jb->g;
    const int phase = jb->phase;
    const double* sx = g->sx;
    const double* sy = g->sy;
    for (;;) {
        int64_t c0 = __atomic_fetch_add(&g->next, 64, __ATOMIC_RELAXED);
        if (c0 >= g->ncells) break;
        int64_t c1 = c0 + 64 < g->ncells ? c0 + 64 : g->ncells;
        for (int64_t c = c0; c < c1; ++c) {
            int64_t b[3], e[3];
            int nr = stencil_ranges(g, c, b, e);
            for (int64_t s = g->cstart[c]; s < g->cstart[c + 1]; ++s) {
                const int64_t i = g->order[s];
                const double px = sx[s], py = sy[s];
                if (phase == 0) { /* neighbour counts */
                    int64_t cnt = 0;
                    for (int r = 0; r < nr; ++r)
                        for (int64_t t = b[r]; t < e[r]; ++t) cnt += within(px, py, sx[t], sy[t], g->eps2);
                    g->counts[i] = cnt;
                    g->core[i] = g->score[s] = cnt >= (int64_t)g->min_points;
                    continue;
                }
                if ((phase == 1) != (g->score[s] != 0)) continue;
                int64_t best = -1;
                for (int r = 0; r < nr; ++r)
                    for (int64_t t = b[r]; t < e[r]; ++t) {
                        if (t == s || !g->score[t] || !within(px, py, sx[t], sy[t], g->eps2)) continue;
                        const int64_t j = g->order[t];
                        if (phase == 1) {
                            if (j < i) uf_union(g->parent, i, j);
                        } else {
                            int64_t sk = uf_find(g->parent, j);
                            if (best < 0 || sk < best) best = sk;
                        }
                    }
                if (phase == 2) g->bmin[i] = best;
            }
        }
    }
    return NULL;
}

static void* grid_worker(void* arg) {
    job* jb = (job*)arg;
    grid_ctx* g = jb->g;
    const double* x = g->x;
    const double* y = g->y;
    for (int64_t i = jb->lo; i < jb->hi; ++i) {
        if (jb->phase == 0) { /* neighbour counts */
            int64_t c = 0;
            if (g->all_pairs) {
                for (int64_t j = 0; j < g->n; ++j) c += within(x[i], y[i], x[j], y[j], g->eps2);
            } else if (!g->no_pairs && g->cell_of[i] >= 0) {
                int64_t b[3], e[3];
                int nr = stencil_ranges(g, g->cell_of[i], b, e);
                for (int r = 0; r < nr; ++r)
                    for (int64_t s = b[r]; s < e[r]; ++s) {
                        int64_t j = g->order[s];
                        c += within(x[i], y[i], x[j], y[j], g->eps2);
                    }
            }
            g->counts[i] = c;
            g->core[i] = c >= (int64_t)g->min_points;
        } else { /* phase 1: unions (cores), phase 2: border minima (non-cores) */
            if ((jb->phase == 1) != (g->core[i] != 0)) continue;
            int64_t best = -1;
            if (g->all_pairs) {
                for (int64_t j = 0; j < g->n; ++j) {
                    if (j == i || !g->core[j] || !within(x[i], y[i], x[j], y[j], g->eps2)) continue;
                    if (jb->phase == 1) {
                        if (j < i) uf_union(g->parent, i, j);
                    } else {
                        int64_t s = uf_find(g->parent, j);
                        if (best < 0 || s < best) best = s;
                    }
                }
            } else if (!g->no_pairs && g->cell_of[i] >= 0) {
                int64_t b[3], e[3];
                int nr = stencil_ranges(g, g->cell_of[i], b, e);
                for (int r = 0; r < nr; ++r)
                    for (int64_t s = b[r]; s < e[r]; ++s) {
                        int64_t j = g->order[s];
                        if (j == i || !g->core[j] || !within(x[i], y[i], x[j], y[j], g->eps2))
                            continue;
                        if (jb->phase == 1) {
                            if (j < i) uf_union(g->parent, i, j);
                        } else {
                            int64_t sk = uf_find(g->parent, j);
                            if (best < 0 || sk < best) best = sk;
                        }
                    }
            }
            if (jb->phase == 2) g->bmin[i] = best;
        }
    }
    return NULL;
}

static void run_phase(grid_ctx* g, int phase, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job jobs[256];
    int64_t chunk = (g->n + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].g = g;
        jobs[t].lo = t * chunk < g->n ? t * chunk : g->n;
        jobs[t].hi = (t + 1) * chunk < g->n ? (t + 1) * chunk : g->n;
        jobs[t].phase = phase;
    }
    /* grid fits: cell-major over the occupied cells (non-finite points keep count 0) */
    void* (*fn)(void*) = (g->ncells > 0 && !g->all_pairs) ? grid_cell_worker : grid_worker;
    g->next = 0;
    if (fn == grid_cell_worker && phase == 0) /* points outside the grid: count 0 */
        for (int64_t i = 0; i < g->n; ++i)
            if (g->cell_of[i] < 0) {
                g->counts[i] = 0;
                g->core[i] = 0 >= (int64_t)g->min_points;
            }
    if (fn == grid_cell_worker && phase != 0) /* callers may edit core[] between phases */
        for (int64_t t = 0; t < g->nfinite; ++t) g->score[t] = g->core[g->order[t]];
    if (nthreads == 1) {
        fn(&jobs[0]);
        return;
    }
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* LSD radix sort of (key, idx) pairs; keys are non-negative int64 < 2^bits. */
static void radix_sort_pairs(int64_t* key, int64_t* val, int64_t n, int bits) {
    int64_t* k2 = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t* v2 = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int shift = 0; shift < bits; shift += 11) {
        int64_t cnt[2049];
        memset(cnt, 0, sizeof(cnt));
        for (int64_t i = 0; i < n; ++i) cnt[((key[i] >> shift) & 2047) + 1]++;
        for (int d = 0; d < 2048; ++d) cnt[d + 1] += cnt[d];
        for (int64_t i = 0; i < n; ++i) {
            int64_t d = (key[i] >> shift) & 2047;
            int64_t o = cnt[d]++;
            k2[o] = key[i];
            v2[o] = val[i];
        }
        memcpy(key, k2, sizeof(int64_t) * (size_t)n);
        memcpy(val, v2, sizeof(int64_t) * (size_t)n);
    }
    free(k2);
    free(v2);
}

static void grid_build(grid_ctx* gp, const double* x, const double* y, int64_t n, double eps,
                       int32_t min_points) {
    grid_ctx g;
    memset(&g, 0, sizeof(g));
    g.x = x;
    g.y = y;
    g.n = n;
    g.eps2 = eps * eps;
    g.min_points = min_points;
    g.no_pairs = isnan(g.eps2);
    g.all_pairs = isinf(g.eps2);
    size_t nn = (size_t)(n > 0 ? n : 1);
    g.core = (uint8_t*)calloc(nn, 1);
    g.counts = (int64_t*)calloc(nn, sizeof(int64_t));
    g.parent = (int64_t*)malloc(sizeof(int64_t) * nn);
    g.bmin = (int64_t*)malloc(sizeof(int64_t) * nn);
    g.cell_of = (int64_t*)malloc(sizeof(int64_t) * nn);
    for (int64_t i = 0; i < n; ++i) {
        g.parent[i] = i;
        g.cell_of[i] = -1;
        g.bmin[i] = -1;
    }
    if (!g.no_pairs && !g.all_pairs && n > 0) {
        double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
        int64_t nf = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (!isfinite(x[i]) || !isfinite(y[i])) continue;
            ++nf;
            if (x[i] < xmin) xmin = x[i];
            if (x[i] > xmax) xmax = x[i];
            if (y[i] < ymin) ymin = y[i];
            if (y[i] > ymax) ymax = y[i];
        }
        if (nf > 0) {
            double R = fabs(eps) * (1.0 + 0x1p-40);
            if (R < 0x1p-500) R = 0x1p-500;
            double h0 = R * (1.0 + 0x1p-20);
            double ex = xmax * 0.5 - xmin * 0.5, ey = ymax * 0.5 - ymin * 0.5; /* half extents */
            double hx = h0, hy = h0;
            const double cap = 0x1p24; /* cells per axis */
            if (2.0 * (ex / cap) > hx) hx = 2.0 * (ex / cap) * (1.0 + 0x1p-20);
            if (2.0 * (ey / cap) > hy) hy = 2.0 * (ey / cap) * (1.0 + 0x1p-20);
            g.invx = 2.0 / hx;
            g.invy = 2.0 / hy;
            g.xmin2 = xmin * 0.5;
            g.ymin2 = ymin * 0.5;
            g.nx = (int64_t)floor(ex * g.invx) + 1;
            g.ny = (int64_t)floor(ey * g.invy) + 1;
            g.order = (int64_t*)malloc(sizeof(int64_t) * (size_t)nf);
            g.okey = (int64_t*)malloc(sizeof(int64_t) * (size_t)nf);
            int64_t s = 0;
            for (int64_t i = 0; i < n; ++i) {
                if (!isfinite(x[i]) || !isfinite(y[i])) continue;
                int64_t cx = (int64_t)floor((x[i] * 0.5 - g.xmin2) * g.invx);
                int64_t cy = (int64_t)floor((y[i] * 0.5 - g.ymin2) * g.invy);
                if (cx < 0) cx = 0;
                if (cx >= g.nx) cx = g.nx - 1;
                if (cy < 0) cy = 0;
                if (cy >= g.ny) cy = g.ny - 1;
                g.okey[s] = cy * g.nx + cx;
                g.order[s] = i;
                ++s;
            }
            g.nfinite = nf;
            int bits = 1;
            while (bits < 62 && ((int64_t)1 << bits) <= g.nx * g.ny) ++bits;
            radix_sort_pairs(g.okey, g.order, nf, bits);
            g.ckey = (int64_t*)malloc(sizeof(int64_t) * (size_t)nf);
            g.cstart = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nf + 1));
            int64_t nc = 0;
            for (int64_t t = 0; t < nf; ++t) {
                if (t == 0 || g.okey[t] != g.okey[t - 1]) {
                    g.ckey[nc] = g.okey[t];
                    g.cstart[nc] = t;
                    ++nc;
                }
                g.cell_of[g.order[t]] = nc - 1;
            }
            g.cstart[nc] = nf;
            g.ncells = nc;
            g.sx = (double*)malloc(sizeof(double) * (size_t)nf);
            g.sy = (double*)malloc(sizeof(double) * (size_t)nf);
            g.score = (uint8_t*)calloc((size_t)nf, 1);
            for (int64_t t = 0; t < nf; ++t) {
                g.sx[t] = x[g.order[t]];
                g.sy[t] = y[g.order[t]];
            }
        }
    }
    *gp = g;
}

static void grid_free(grid_ctx* g) {
    free(g->core);
    free(g->counts);
    free(g->parent);
    free(g->bmin);
    free(g->cell_of);
    free(g->order);
    free(g->okey);
    free(g->ckey);
    free(g->cstart);
    free(g->sx);
    free(g->sy);
    free(g->score);
}

int32_t oracle_fit_grid(const double* x, const double* y, int64_t n, double eps,
                        int32_t min_points, int32_t mode, int32_t nthreads, int32_t* cluster,
                        uint8_t* flag, int64_t* counts_out) {
    grid_ctx g;
    grid_build(&g, x, y, n, eps, min_points);
    run_phase(&g, 0, nthreads);
    run_phase(&g, 1, nthreads);
    run_phase(&g, 2, nthreads);
    if (counts_out)
        for (int64_t i = 0; i < n; ++i) counts_out[i] = g.counts[i];
    int32_t k = finish_labels(n, g.core, g.parent, g.bmin, mode, cluster, flag);
    grid_free(&g);
    return k;
}

/* ------------------------------------------------------------------------------------------
 * 3b. The literal sequential BFS of section 1 with grid neighbour queries.  Within one
 *     expandCluster the order in which neighbours are taken does not change which points the
 *     expansion claims (every unvisited point reachable through cores, plus, for archery,
 *     every Noise point a claimed core reaches), so enumerating a neighbourhood over the 3x3
 *     stencil instead of array order gives the same labels.  mode 2 (archery's float32 search
 *     box, LocalDBSCANArchery.scala:38-41,114-124) makes the neighbour relation directed:
 *     N(p) = {o : d2 <= eps2 and (float)o in p's float32 box}.
 * ------------------------------------------------------------------------------------------ */
static int64_t grid_neighbors(const grid_ctx* g, int64_t p, double eps, int mode, int64_t* out) {
    int64_t m = 0;
    if (g->cell_of[p] < 0) return 0;
    int64_t b[3], e[3];
    int nr = stencil_ranges(g, g->cell_of[p], b, e);
    for (int r = 0; r < nr; ++r)
        for (int64_t t = b[r]; t < e[r]; ++t) {
            int64_t o = g->order[t];
            if (is_neighbor(g->x, g->y, p, o, eps, g->eps2, mode)) {
                if (out) out[m] = o;
                ++m;
            }
        }
    return m;
}

int32_t oracle_fit_bfs_grid(const double* x, const double* y, int64_t n, double eps,
                            int32_t min_points, int32_t mode, int32_t* cluster, uint8_t* flag) {
    grid_ctx g;
    grid_build(&g, x, y, n, eps, min_points);
    if (g.all_pairs || g.no_pairs) { /* one all-pairs cell or no pairs: the O(n^2) form */
        grid_free(&g);
        return oracle_fit_sequential(x, y, n, eps, min_points, mode, cluster, flag);
    }
    size_t nn = (size_t)(n > 0 ? n : 1);
    uint8_t* visited = (uint8_t*)calloc(nn, 1);
    int64_t* queue = (int64_t*)malloc(sizeof(int64_t) * nn);
    int64_t* cnt = (int64_t*)malloc(sizeof(int64_t) * nn);
    int64_t cap = 1024;
    int64_t* nb = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    for (int64_t i = 0; i < n; ++i) {
        cluster[i] = 0;
        flag[i] = FLAG_NOTFLAGGED;
        cnt[i] = grid_neighbors(&g, i, eps, mode, NULL);
    }
    int32_t total = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (visited[i]) continue;
        visited[i] = 1;
        if (cnt[i] < (int64_t)min_points) {
            flag[i] = FLAG_NOISE;
            continue;
        }
        const int32_t c = ++total;
        flag[i] = FLAG_CORE;
        cluster[i] = c;
        int64_t qh = 0, qt = 0;
        queue[qt++] = i;
        while (qh < qt) {
            const int64_t centre = queue[qh++];
            if (cnt[centre] > cap) {
                cap = cnt[centre];
                nb = (int64_t*)realloc(nb, sizeof(int64_t) * (size_t)cap);
            }
            int64_t m = grid_neighbors(&g, centre, eps, mode, nb);
            for (int64_t k = 0; k < m; ++k) {
                const int64_t j = nb[k];
                if (!visited[j]) {
                    visited[j] = 1;
                    cluster[j] = c;
                    if (cnt[j] >= (int64_t)min_points) {
                        flag[j] = FLAG_CORE;
                        queue[qt++] = j;
                    } else {
                        flag[j] = FLAG_BORDER;
                    }
                }
                if (mode != MODE_NAIVE && cluster[j] == 0) {
                    cluster[j] = c;
                    flag[j] = FLAG_BORDER;
                }
            }
        }
    }
    free(visited);
    free(queue);
    free(cnt);
    free(nb);
    grid_free(&g);
    return total;
}

/* ------------------------------------------------------------------------------------------
 * 4. Slab semantics of the node path (dbscan_slab_fit_device / dbscan_slab_label_device),
 *    restated on the CPU so the multi-rank merge (dbscan_amd/node.py) can be tested with the
 *    gloo backend on machines without a GPU.  Zones: 0 owned, 1 inner halo, 2 outer halo.
 * ------------------------------------------------------------------------------------------ */
int32_t oracle_slab_fit(const double* x, const double* y, const uint8_t* zone, int64_t n,
                        double eps, int32_t min_points, int32_t nthreads, uint8_t* core_out,
                        int32_t* root_out) {
    grid_ctx g;
    grid_build(&g, x, y, n, eps, min_points);
    run_phase(&g, 0, nthreads);
    for (int64_t i = 0; i < n; ++i)
        if (zone[i] == 2) g.core[i] = 0; /* halo-only candidates are never core */
    run_phase(&g, 1, nthreads);
    for (int64_t i = 0; i < n; ++i) {
        core_out[i] = g.core[i];
        root_out[i] = g.core[i] ? (int32_t)uf_find(g.parent, i) : -1;
    }
    grid_free(&g);
    return 0;
}

int32_t oracle_slab_label(const double* x, const double* y, const uint8_t* zone, int64_t n,
                          double eps, const uint8_t* core, const int32_t* root,
                          const int64_t* gid, const int64_t* gs_of_root,
                          const int32_t* label_of_root, int32_t mode, int32_t* cluster_out,
                          uint8_t* flag_out) {
    grid_ctx g;
    grid_build(&g, x, y, n, eps, 1);
    for (int64_t i = 0; i < n; ++i) {
        if (zone[i] != 0) continue;
        if (core[i]) {
            cluster_out[i] = label_of_root[root[i]];
            flag_out[i] = FLAG_CORE;
            continue;
        }
        int64_t m = INT64_MAX;
        int32_t mr = -1;
        int64_t b[3] = {0, 0, 0}, e[3] = {0, 0, 0};
        int nr = 0;
        if (g.all_pairs) {
            e[0] = n;
            nr = 1;
        } else if (!g.no_pairs && g.cell_of[i] >= 0) {
            nr = stencil_ranges(&g, g.cell_of[i], b, e);
        }
        for (int r = 0; r < nr; ++r)
            for (int64_t t = b[r]; t < e[r]; ++t) {
                int64_t j = g.all_pairs ? t : g.order[t];
                if (!core[j] || !within(x[i], y[i], x[j], y[j], g.eps2)) continue;
                int64_t v = gs_of_root[root[j]];
                if (v < m) {
                    m = v;
                    mr = root[j];
                }
            }
        int ok = mr >= 0 && (mode != MODE_NAIVE || m < gid[i]);
        cluster_out[i] = ok ? label_of_root[mr] : 0;
        flag_out[i] = ok ? FLAG_BORDER : FLAG_NOISE;
    }
    grid_free(&g);
    return 0;
}
