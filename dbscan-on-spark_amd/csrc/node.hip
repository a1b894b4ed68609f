// node.hip -- dbscan_train_node: the whole-node entry of SURVEY.md §8b, one process driving
// every GPU of the node.  The C++ twin of dbscan_amd/node.py (which runs one process per GPU
// over RCCL); the same slab plan, the same exact merge:
//   DBSCAN.scala:91-137    partition the plane, grow partitions by eps, duplicate points
//                          -> n_shards x-slabs at count quantiles snapped to the 2*eps grid,
//                             each with its 2-zone halo (node.py: make_cuts, zones)
//   DBSCAN.scala:150-155   LocalDBSCANNaive.fit per partition
//                          -> dbscan_slab_fit_device per shard, shard s on device
//                             s % device_count, one host thread and one handle (HIP stream) per
//                             device; shards sharing a device run one after another on its
//                             handle and are re-fitted before their label (one workspace per
//                             device, so 8 shards of 10^9 points fit one GPU's HBM)
//   DBSCAN.scala:158-222   band points, findAdjacencies, DBSCANGraph, global ids
//                          -> records (gid of a shared core, gid of its local root) merged by a
//                             host union-find (the records are a thin band: O(1e5) at 1e8 pts),
//                             global s(K) per local root, cluster id = rank of s(K)
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

struct Shard {
    HostVec<int64_t> gid;  // slab points, increasing global visit index
    HostVec<double> x, y;
    HostVec<uint8_t> zone;
    HostVec<int32_t> shared;  // slab indices of points in zones 0/1 of another shard too
    HostVec<int32_t> root;    // slab fit output (-1: not core)
    HostVec<int64_t> gs;      // global s(K) per local root (only the roots' entries are read)
    HostVec<int32_t> cluster;
    HostVec<uint8_t> flag;
    std::string err;
    int32_t rc = DBSCAN_OK;
};

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

uint8_t zone_of(double x, int r, int world, const ZoneCut& c, bool* shared) {
    bool own = (!c.has_lo || x >= c.lo) && (!c.has_hi || x < c.hi);
    if (r == 0 && world > 1 && std::isnan(x)) own = true;
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

// Uploads a shard and runs its slab fit on handle h (device buffers returned in *dev, freed by
// the caller).  Phase 1 reads the roots back; phase 2 re-fits on a handle that held other
// shards meanwhile (the fit is deterministic) and then labels.
struct ShardDev {
    double *x = nullptr, *y = nullptr;
    uint8_t *zone = nullptr, *core = nullptr;
    int32_t* root = nullptr;
    void release() {
        for (void* p : {(void*)x, (void*)y, (void*)zone, (void*)core, (void*)root}) (void)hipFree(p);
        *this = ShardDev();
    }
};

bool shard_upload_fit(Shard& s, dbscan_handle* h, int device, double eps, int32_t min_points,
                      ShardDev* d) {
    const int64_t m = (int64_t)s.gid.size();
    auto fail = [&](hipError_t e, const char* what) {
        s.rc = e == hipErrorOutOfMemory ? DBSCAN_EOOM : DBSCAN_EHIP;
        s.err = std::string(what) + ": " + hipGetErrorString(e);
        return false;
    };
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&d->x, m * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&d->y, m * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&d->zone, m);
    if (e == hipSuccess) e = hipMalloc(&d->core, m);
    if (e == hipSuccess) e = hipMalloc(&d->root, m * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemcpy(d->x, s.x.data(), m * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d->y, s.y.data(), m * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d->zone, s.zone.data(), m, hipMemcpyHostToDevice);
    if (e != hipSuccess) return fail(e, "shard upload");
    s.rc = dbscan_slab_fit_device(h, d->x, d->y, d->zone, m, eps, min_points, d->core, d->root);
    if (s.rc != DBSCAN_OK) {
        s.err = dbscan_last_error();
        return false;
    }
    return true;
}

// Phase 1 of one shard: slab fit, roots back to the host.
void shard_fit(Shard& s, dbscan_handle* h, int device, double eps, int32_t min_points) {
    const int64_t m = (int64_t)s.gid.size();
    s.root.resize(m);  // (downloaded whole)
    if (m == 0) return;
    ShardDev d;
    if (shard_upload_fit(s, h, device, eps, min_points, &d)) {
        const hipError_t e =
            hipMemcpy(s.root.data(), d.root, m * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
            s.rc = DBSCAN_EHIP;
            s.err = std::string("shard download: ") + hipGetErrorString(e);
        }
    }
    d.release();
}

// Phase 2: labels of the shard's zone-0 points from the merged component ids.  refit: the
// handle's last slab fit was another shard's (shards sharing a device run one after another on
// one handle, so a device holds one workspace, not one per shard).
void shard_label(Shard& s, dbscan_handle* h, int device, double eps, int32_t min_points,
                 const std::vector<int64_t>& all_roots, int32_t mode, bool refit) {
    const int64_t m = (int64_t)s.gid.size();
    s.cluster.resize(m);  // (downloaded whole; only zone-0 entries are used)
    s.flag.resize(m);
    if (m == 0) return;
    ShardDev fitd;
    if (refit && !shard_upload_fit(s, h, device, eps, min_points, &fitd)) {
        fitd.release();
        return;
    }
    uint8_t *dz = nullptr, *dfl = nullptr;
    int64_t *dgid = nullptr, *dgs = nullptr, *droots = nullptr;
    int32_t* dcl = nullptr;
    const int64_t nr = (int64_t)all_roots.size();
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&dz, m);
    if (e == hipSuccess) e = hipMalloc(&dfl, m);
    if (e == hipSuccess) e = hipMalloc(&dgid, m * sizeof(int64_t));
    if (e == hipSuccess) e = hipMalloc(&dgs, m * sizeof(int64_t));
    if (e == hipSuccess) e = hipMalloc(&droots, std::max<int64_t>(1, nr) * sizeof(int64_t));
    if (e == hipSuccess) e = hipMalloc(&dcl, m * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemcpy(dz, s.zone.data(), m, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgid, s.gid.data(), m * sizeof(int64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dgs, s.gs.data(), m * sizeof(int64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && nr > 0)
        e = hipMemcpy(droots, all_roots.data(), nr * sizeof(int64_t), hipMemcpyHostToDevice);
    // zone 1/2 entries are not labelled here (the output takes zone-0 entries only)
    if (e == hipSuccess) e = hipMemset(dcl, 0, m * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemset(dfl, DBSCAN_FLAG_NOT_FLAGGED, m);
    if (e != hipSuccess) {
        s.rc = e == hipErrorOutOfMemory ? DBSCAN_EOOM : DBSCAN_EHIP;
        s.err = std::string("shard label upload: ") + hipGetErrorString(e);
    } else {
        s.rc = dbscan_slab_label_device(h, dz, dgid, dgs, droots, nr, mode, dcl, dfl);
        if (s.rc != DBSCAN_OK) {
            s.err = dbscan_last_error();
        } else {
            e = hipMemcpy(s.cluster.data(), dcl, m * sizeof(int32_t), hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(s.flag.data(), dfl, m, hipMemcpyDeviceToHost);
            if (e != hipSuccess) {
                s.rc = DBSCAN_EHIP;
                s.err = std::string("shard label download: ") + hipGetErrorString(e);
            }
        }
    }
    for (void* p : {(void*)dz, (void*)dfl, (void*)dgid, (void*)dgs, (void*)droots, (void*)dcl})
        (void)hipFree(p);
    fitd.release();
}

// Min-root union-find over global visit indices (host; the records are few).
struct GidUnion {
    std::unordered_map<int64_t, int64_t> up;
    int64_t find(int64_t v) {
        auto it = up.find(v);
        if (it == up.end()) return v;
        int64_t r = v;
        while (true) {
            auto jt = up.find(r);
            if (jt == up.end() || jt->second == r) break;
            r = jt->second;
        }
        while (v != r) {  // compress
            int64_t& nx = up[v];
            const int64_t t = nx;
            nx = r;
            v = t;
        }
        return r;
    }
    void unite(int64_t a, int64_t b) {
        a = find(a);
        b = find(b);
        if (a == b) return;
        if (a < b) std::swap(a, b);
        up[a] = b;  // the larger index hangs under the smaller: a root is s(K)
        up.emplace(b, b);
    }
};

}  // namespace

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
    const int world = (int)cuts.size() + 1;
    const double R = reach(eps);
    const std::vector<ZoneCut> zc = zone_cuts(world, cuts, R);
    std::vector<Shard> sh(world);
    // slab plan: every shard's points in increasing global visit order, built by host threads
    // over contiguous chunks of the input (count, then fill at the chunk's offsets)
    const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), n / 65536 + 1));
    std::vector<int64_t> cnt((size_t)nth * world * 2, 0);  // [thread][shard]{points, shared}
    const auto chunk = [&](int t) {
        return std::make_pair(n * t / nth, n * (t + 1) / nth);
    };
    // only the owner and shards whose halo can reach x need a look: scan neighbours of the
    // owner until both directions fall out of reach
    const auto visit = [&](int64_t i, auto&& f) {
        const int own = std::isnan(x[i])  // NaN x is owned by shard 0 (node.py zones)
                            ? 0
                            : (int)(std::upper_bound(cuts.begin(), cuts.end(), x[i]) -
                                    cuts.begin());
        for (int dir = -1; dir <= 1; dir += 2) {
            for (int r = (dir < 0 ? own : own + 1); r >= 0 && r < world; r += dir) {
                // a shard past the owner's is reached only through its outer halo margin
                // (zone_of would say kOut; NaN included): most points stop here at once
                if (r != own && (dir < 0 ? !(x[i] <= zc[r].hi + zc[r].m2hi)
                                         : !(x[i] >= zc[r].lo - zc[r].m2lo)))
                    break;
                bool shared = false;
                const uint8_t z = zone_of(x[i], r, world, zc[r], &shared);
                if (z == kOut) {
                    if (r != own) break;
                    continue;
                }
                f(r, z, shared);
            }
        }
    };
    parallel_for(nth, [&](int t) {
        int64_t* c = &cnt[(size_t)t * world * 2];
        const auto [i0, i1] = chunk(t);
        for (int64_t i = i0; i < i1; ++i)
            visit(i, [&](int r, uint8_t, bool shared) {
                ++c[2 * r];
                c[2 * r + 1] += shared ? 1 : 0;
            });
    });
    tr.mark("plan count");
    std::vector<int64_t> at((size_t)nth * world * 2, 0);
    for (int r = 0; r < world; ++r) {
        int64_t np = 0, ns = 0;
        for (int t = 0; t < nth; ++t) {
            at[((size_t)t * world + r) * 2] = np;
            at[((size_t)t * world + r) * 2 + 1] = ns;
            np += cnt[((size_t)t * world + r) * 2];
            ns += cnt[((size_t)t * world + r) * 2 + 1];
        }
        sh[r].gid.resize((size_t)np);
        sh[r].x.resize((size_t)np);
        sh[r].y.resize((size_t)np);
        sh[r].zone.resize((size_t)np);
        sh[r].shared.resize((size_t)ns);
    }
    tr.mark("plan alloc");
    parallel_for(nth, [&](int t) {
        int64_t* a = &at[(size_t)t * world * 2];
        const auto [i0, i1] = chunk(t);
        for (int64_t i = i0; i < i1; ++i)
            visit(i, [&](int r, uint8_t z, bool shared) {
                Shard& s = sh[r];
                const int64_t k = a[2 * r]++;
                if (shared) s.shared[(size_t)a[2 * r + 1]++] = (int32_t)k;
                s.gid[(size_t)k] = i;
                s.x[(size_t)k] = x[i];
                s.y[(size_t)k] = y[i];
                s.zone[(size_t)k] = z;
            });
    });
    tr.mark("plan fill");
    // one host thread and one handle per device; the shards of a device run one after another
    // on its handle (one workspace per device: 8 shards of a 10^9-point job on one GPU)
    const int nworkers = std::min(world, ndev);
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
    const bool shared_dev = world > nworkers;
    auto each_device = [&](auto&& f) {
        std::vector<std::thread> th;
        for (int w = 0; w < nworkers; ++w)
            th.emplace_back([&, w]() {
                for (int r = w; r < world; r += nworkers) f(r, w);
            });
        for (auto& t : th) t.join();
    };
    each_device([&](int r, int w) { shard_fit(sh[r], hs[w], w, eps, min_points); });
    tr.mark("slab fits");
    int32_t rc = DBSCAN_OK;
    for (auto& s : sh)
        if (s.rc != DBSCAN_OK && rc == DBSCAN_OK) {
            rc = s.rc;
            *err = s.err;
        }
    std::vector<int64_t> all_roots;
    if (rc == DBSCAN_OK) {
        GidUnion uf;  // records: shared core point -- its local root
        for (auto& s : sh)
            for (int32_t p : s.shared) {
                const int32_t r = s.root[p];
                if (r >= 0) uf.unite(s.gid[p], s.gid[r]);
            }
        for (auto& s : sh) {
            const int64_t m = (int64_t)s.gid.size();
            s.gs.resize(m);  // (only the local roots' entries are read)
            // the local roots by host threads (per-thread lists in slab order), then their global
            // s(K) on this thread (the union-find compresses paths as it goes)
            std::vector<std::vector<int32_t>> lr(nth);
            parallel_for(nth, [&](int t) {
                for (int64_t p = m * t / nth, p1 = m * (t + 1) / nth; p < p1; ++p)
                    if (s.root[(size_t)p] == (int32_t)p) lr[t].push_back((int32_t)p);
            });
            for (auto& l : lr)
                for (int32_t p : l) {
                    const int64_t g = s.gid[(size_t)p], gs = uf.find(g);
                    s.gs[(size_t)p] = gs;
                    if (s.zone[(size_t)p] == 0 && gs == g) all_roots.push_back(g);
                }
            HostVec<int32_t>().swap(s.root);
        }
        std::sort(all_roots.begin(), all_roots.end());
        tr.mark("merge + numbering");
        each_device([&](int r, int w) {
            shard_label(sh[r], hs[w], w, eps, min_points, all_roots, mode, shared_dev);
        });
        tr.mark("slab labels");
        for (auto& s : sh)
            if (s.rc != DBSCAN_OK && rc == DBSCAN_OK) {
                rc = s.rc;
                *err = s.err;
            }
    }
    if (rc == DBSCAN_OK) {
        // zone-0 points: each input point is owned by exactly one shard (disjoint writes)
        parallel_for(nth, [&](int t) {
            for (auto& s : sh) {
                const int64_t m = (int64_t)s.gid.size(), p0 = m * t / nth, p1 = m * (t + 1) / nth;
                for (int64_t p = p0; p < p1; ++p)
                    if (s.zone[(size_t)p] == 0) {
                        cluster_out[s.gid[(size_t)p]] = s.cluster[(size_t)p];
                        flag_out[s.gid[(size_t)p]] = s.flag[(size_t)p];
                    }
            }
        });
        *n_clusters_out = (int64_t)all_roots.size();
        tr.mark("output scatter");
    }
    for (auto* h : hs) dbscan_destroy(h);
    tr.mark("teardown");
    return rc;
}

}  // namespace dbscan
