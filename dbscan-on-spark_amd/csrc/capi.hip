// capi.hip -- the C-ABI of libdbscan_hip.so (declared in include/dbscan_hip.h): handles,
// error reporting, host<->device staging, profiling and the synthetic generator.
//
// Boundary replaced: `new LocalDBSCANNaive(eps, minPoints).fit(points)` at DBSCAN.scala:153-154
// (LocalDBSCANNaive.scala:31,37; LocalDBSCANArchery.scala:32,36).  Return codes and ownership
// follow SURVEY.md §8b: the caller owns host arrays, the handle owns grow-only device buffers,
// no pointer is retained past a call, errors go to a thread-local dbscan_last_error().
#include "../../include/dbscan_hip.h"
#include "internal.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>

namespace dbscan {

HipError::HipError(hipError_t e, const char* expr, const char* file, int line) : err(e) {
    char buf[512];
    snprintf(buf, sizeof(buf), "HIP error %d (%s) at %s:%d: %s", (int)e, hipGetErrorString(e),
             file, line, expr);
    what = buf;
}

void* DevBuf::ensure(size_t need) {
    if (need == 0) need = 16;
    if (need <= bytes) return p;
    release();
    size_t cap = need + need / 8;  // grow-only with headroom
    hipError_t e = hipMalloc(&p, cap);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        bytes = 0;
        throw HipError(e, "hipMalloc (workspace)", __FILE__, __LINE__);
    }
    bytes = cap;
    return p;
}

void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}

hipEvent_t Profiler::take() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e;
    DBSCAN_HIP_CHECK(hipEventCreate(&e));
    return e;
}

int Profiler::stage_index(const char* name) {
    for (size_t i = 0; i < stages.size(); ++i)
        if (stages[i].name == name) return (int)i;
    stages.push_back(Stage{name, 0.0, 0});
    return (int)stages.size() - 1;
}

void Profiler::flush() {
    for (auto& pe : pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
            stages[pe.stage].ms += ms;
            stages[pe.stage].launches += 1;
        }
        pool.push_back(pe.a);
        pool.push_back(pe.b);
    }
    pending.clear();
}

void Profiler::flush_ready() {
    std::vector<Pending> keep;
    for (auto& pe : pending) {
        if (hipEventQuery(pe.b) != hipSuccess) {
            keep.push_back(pe);
            continue;
        }
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
            stages[pe.stage].ms += ms;
            stages[pe.stage].launches += 1;
        }
        pool.push_back(pe.a);
        pool.push_back(pe.b);
    }
    pending.swap(keep);
}

void Profiler::destroy() {
    for (auto& pe : pending) {
        pool.push_back(pe.a);
        pool.push_back(pe.b);
    }
    pending.clear();
    for (auto e : pool) (void)hipEventDestroy(e);
    pool.clear();
}

StageTimer::StageTimer(Profiler* p, hipStream_t st, const char* name) : prof(p), s(st) {
    if (!prof || !prof->on || prof->mode != 1) {
        prof = nullptr;
        return;
    }
    stage = prof->stage_index(name);
    a = prof->take();
    DBSCAN_HIP_CHECK(hipEventRecord(a, s));
}

StageTimer::~StageTimer() {
    if (!prof) return;
    hipEvent_t b = prof->take();
    if (hipEventRecord(b, s) == hipSuccess) prof->pending.push_back({stage, a, b});
}

// ------------------------------------ generator -----------------------------------------

namespace {

__host__ __device__ inline uint64_t splitmix64(uint64_t& st) {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline double u01_open(uint64_t v) {  // (0, 1]
    return ((double)(v >> 11) + 1.0) * 0x1p-53;
}

constexpr int kBlobs = 32;
struct BlobParams {
    double cx[kBlobs], cy[kBlobs], sigma[kBlobs];
    double noise_half;  // noise over [-noise_half, noise_half]^2
    double noise_frac;
    uint64_t seed;
};

__global__ __launch_bounds__(256) void gen_blobs_kernel(BlobParams bp, int64_t n, double* x,
                                                        double* y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t st = bp.seed ^ ((uint64_t)i * 0xD1B54A32D192ED03ull);
    (void)splitmix64(st);
    const double u0 = u01_open(splitmix64(st));
    const uint64_t r1 = splitmix64(st);
    const double u2 = u01_open(splitmix64(st));
    const double u3 = u01_open(splitmix64(st));
    if (u0 <= bp.noise_frac) {
        x[i] = (2.0 * u2 - 1.0) * bp.noise_half;
        y[i] = (2.0 * u3 - 1.0) * bp.noise_half;
    } else {
        const int b = (int)(r1 % kBlobs);
        const double rad = sqrt(-2.0 * log(u2));
        const double th = 6.283185307179586 * u3;
        x[i] = bp.cx[b] + bp.sigma[b] * rad * cos(th);
        y[i] = bp.cy[b] + bp.sigma[b] * rad * sin(th);
    }
}

}  // namespace
}  // namespace dbscan

// ------------------------------------ handle --------------------------------------------

struct dbscan_handle {
    int device = 0;
    hipStream_t stream = nullptr;      // where the handle's work runs
    hipStream_t own_stream = nullptr;  // the stream the handle created (and destroys)
    dbscan::Workspace ws;
    dbscan::Profiler prof;
    dbscan::FitStats stats;
    dbscan::SlabState slab;
    dbscan::DevBuf hx, hy, hcl, hfl;  // staging for the host-array entry points
    dbscan::DevBuf boffs, hnk;        // batch fits: offsets + small-partition list; counts
    void* bpinned = nullptr;          // pinned staging of the batch tables (grow-only)
    size_t bpinned_bytes = 0;
    hipEvent_t bcopied = nullptr;     // the last batch tables' upload (pinned buffer reusable)
    int64_t small_max = DBSCAN_SMALL_DEFAULT_POINTS;  // one-workgroup fits up to this many points
    int64_t spread_min = DBSCAN_SPREAD_DEFAULT_POINTS;  // LDS fits from here: several workgroups
    int64_t band_max = DBSCAN_BAND_DEFAULT_POINTS;      // band fits above the LDS capacity
    int64_t band_min = DBSCAN_BAND_MIN_DEFAULT_POINTS;  // ... and inside it from this many points
    bool pending = false;             // an asynchronous fit whose stats are not read yet
    bool prepared = false;            // dbscan_slab_roots_prepare_device ran since the slab fit
    void* pinned = nullptr;           // small pinned host block (stats, root count)
    void* fpinned = nullptr;          // partition-sized dbscan_fit_h: pinned x|y and cluster|flag
    char* fpinned_dev = nullptr;      // ... its device address (the LDS forms write labels there)
    size_t fpinned_bytes = 0;
    dbscan::DevBuf hxy, hclfl;        // ... and their device twins (one copy each way)
    hipEvent_t ready = nullptr;       // marks the root count inside a prepare call
    std::mutex mu;                    // one fit at a time per handle
};

namespace {

thread_local std::string g_err;
thread_local std::unique_ptr<dbscan_handle, void (*)(dbscan_handle*)> g_tls_handle(
    nullptr, dbscan_destroy);

void set_err(const std::string& s) { g_err = s; }

}  // namespace

void dbscan::set_last_error(const std::string& s) { set_err(s); }

namespace {

// dbscan_fit_h fits of at most this many points stage through one pinned block (21 B/point)
constexpr int64_t kPinnedFitMax = 65536;  // (250 / 2000 / 8192 points: 101 / 151 / 240 ->
                                          // 65 / 119 / 207 us per call, one thread)
// ... of which fits of at most this many points taking an LDS form get their labels written into
// that block by the kernel itself
constexpr int64_t kDirectOutMax = 16384;

template <class F>
int32_t guarded(dbscan_handle* h, F&& f) {
    g_err.clear();
    try {
        if (h) {
            hipError_t e = hipSetDevice(h->device);
            if (e != hipSuccess) throw dbscan::HipError(e, "hipSetDevice", __FILE__, __LINE__);
        }
        return f();
    } catch (const dbscan::ArgError& e) {
        set_err(e.what);
        return DBSCAN_EARG;
    } catch (const dbscan::HipError& e) {
        set_err(e.what);
        return (e.err == hipErrorOutOfMemory || e.err == hipErrorMemoryAllocation) ? DBSCAN_EOOM
                                                                                    : DBSCAN_EHIP;
    } catch (const std::bad_alloc&) {
        set_err("host allocation failed");
        return DBSCAN_EOOM;
    } catch (...) {
        set_err("unknown error");
        return DBSCAN_EHIP;
    }
}

// One lock per device over large host<->device copies (>= 2^20 points): see dbscan_fit_h.
// (One lock per direction, so that one handle's D2H runs beside another's H2D, measured slower:
// two executor threads 4.0 -> 4.65 ms per 10^7-point fit, round 3.)
class XferLock {
  public:
    XferLock(int device, int64_t n) {
        static std::mutex mu[64];
        if (n >= (int64_t(1) << 20)) {
            m_ = &mu[device & 63];
            m_->lock();
        }
    }
    ~XferLock() {
        if (m_) m_->unlock();
    }
    bool held() const { return m_ != nullptr; }

  private:
    std::mutex* m_ = nullptr;
};

// local = the local-fit entry points, which also take DBSCAN_MODE_ARCHERY_F32BOX (its
// directed neighbour relation has no slab/merge form)
void check_fit_args(int64_t n, double eps, int32_t mode, const void* a, const void* b,
                    const void* c, const void* d, bool local = false) {
    (void)eps;
    if (n < 0) throw dbscan::ArgError{"n < 0"};
    if (n > DBSCAN_MAX_POINTS) throw dbscan::ArgError{"n exceeds DBSCAN_MAX_POINTS"};
    if (mode == DBSCAN_MODE_ARCHERY_F32BOX && !local)
        throw dbscan::ArgError{"DBSCAN_MODE_ARCHERY_F32BOX is for the local fit entry points only"};
    if (mode != DBSCAN_MODE_NAIVE && mode != DBSCAN_MODE_ARCHERY &&
        mode != DBSCAN_MODE_ARCHERY_F32BOX)
        throw dbscan::ArgError{"mode must be DBSCAN_MODE_NAIVE, _ARCHERY or _ARCHERY_F32BOX"};
    if (n > 0 && (!a || !b || !c || !d)) throw dbscan::ArgError{"NULL array pointer"};
}

}  // namespace

extern "C" {

const char* dbscan_last_error(void) { return g_err.c_str(); }

int32_t dbscan_version(void) { return 100; }

int32_t dbscan_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return c;
}

dbscan_handle* dbscan_create(int32_t device) {
    g_err.clear();
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_err("no HIP device visible");
        return nullptr;
    }
    if (device < 0 || device >= count) {
        set_err("device index out of range");
        return nullptr;
    }
    dbscan_handle* h = new (std::nothrow) dbscan_handle();
    if (!h) {
        set_err("host allocation failed");
        return nullptr;
    }
    h->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    h->stream = h->own_stream;
    if (e != hipSuccess) {
        set_err(std::string("hipStreamCreate failed: ") + hipGetErrorString(e));
        delete h;
        return nullptr;
    }
    return h;
}

void dbscan_destroy(dbscan_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    // The bound stream may be the null stream (dbscan_set_stream(h, NULL, 0), e.g. torch's
    // default stream): synchronizing it is valid and waits for the handle's kernels there.
    (void)hipStreamSynchronize(h->stream);
    if (h->own_stream && h->own_stream != h->stream) (void)hipStreamSynchronize(h->own_stream);
    if (!h->ws.recalls.empty()) {  // queued fits never synced: their re-runs still owed
        try {
            dbscan::drain_recalls(h->stream, &h->prof, h->ws);
        } catch (...) {
        }
    }
    h->prof.destroy();
    h->ws.release();
    h->hx.release();
    h->hy.release();
    h->hcl.release();
    h->hfl.release();
    h->boffs.release();
    h->hnk.release();
    if (h->bpinned) (void)hipHostFree(h->bpinned);
    if (h->bcopied) (void)hipEventDestroy(h->bcopied);
    if (h->pinned) (void)hipHostFree(h->pinned);
    if (h->fpinned) (void)hipHostFree(h->fpinned);
    if (h->ready) (void)hipEventDestroy(h->ready);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
}

void* dbscan_stream(dbscan_handle* h) { return h ? (void*)h->stream : nullptr; }


namespace {
// Completes an asynchronous fit on the host side: waits for the stream, reads its stats
// (raising a device-side error such as an unsizable grid) and accumulates the stage timers.
// Every queued spread / band fit is checked (and re-run when a barrier gave up or a band
// overflowed), not only the last one: each has its own stats block and recall record.
void settle(dbscan_handle* h) {
    if (!h->pending) {
        if (!h->ws.recalls.empty()) {  // (fits queued before a call that consumed the stats)
            DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
            dbscan::drain_recalls(h->stream, &h->prof, h->ws);
        }
        return;
    }
    h->pending = false;
    h->stats = dbscan::read_fit_stats(h->stream, h->ws, &h->prof);
    h->prof.flush();
}
}  // namespace

int32_t dbscan_set_stream(dbscan_handle* h, void* stream, int32_t own) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        settle(h);
        DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
        h->prof.flush();
        h->stream = own ? h->own_stream : static_cast<hipStream_t>(stream);
        return DBSCAN_OK;
    });
}

int32_t dbscan_fit_device_async(dbscan_handle* h, const double* d_x, const double* d_y,
                                int64_t n, double eps, int32_t min_points, int32_t mode,
                                int32_t* d_cluster, uint8_t* d_flag, int32_t* d_n_clusters) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        check_fit_args(n, eps, mode, d_x, d_y, d_cluster, d_flag, true);
        if (h->pending && h->prof.pending.size() > 4096) settle(h);  // bound the event backlog
        // a newer fit replaces the unread stats of an older one; the older one's outcome stays
        // in its own stats block and recall record (checked by dbscan_sync)
        h->pending = false;
        dbscan::FitArgs a{d_x, d_y, nullptr, n, eps, min_points, mode, d_cluster, d_flag,
                          nullptr, nullptr};
        a.small_max = h->small_max;
        a.spread_min = h->spread_min;
        a.band_max = h->band_max;
        a.band_min = h->band_min;
        a.n_clusters_dev = d_n_clusters;
        h->prepared = false;
        dbscan::enqueue_fit(h->stream, h->ws, &h->prof, a, &h->slab);
        if (d_n_clusters) dbscan::write_nclusters(h->stream, h->ws, d_n_clusters);
        h->pending = true;
        return DBSCAN_OK;
    });
}

int32_t dbscan_sync(dbscan_handle* h) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
        settle(h);
        return DBSCAN_OK;
    });
}

int32_t dbscan_fit_device(dbscan_handle* h, const double* d_x, const double* d_y, int64_t n,
                          double eps, int32_t min_points, int32_t mode, int32_t* d_cluster,
                          uint8_t* d_flag, int32_t* n_clusters_out) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        settle(h);
        check_fit_args(n, eps, mode, d_x, d_y, d_cluster, d_flag, true);
        dbscan::FitArgs a{d_x, d_y, nullptr, n, eps, min_points, mode, d_cluster, d_flag,
                          nullptr, nullptr};
        a.small_max = h->small_max;
        a.spread_min = h->spread_min;
        a.band_max = h->band_max;
        a.band_min = h->band_min;
        h->prepared = false;
        int64_t k = dbscan::run_fit(h->stream, h->ws, &h->prof, a, &h->stats, &h->slab);
        h->prof.flush();
        if (n_clusters_out) *n_clusters_out = (int32_t)k;
        return DBSCAN_OK;
    });
}

int32_t dbscan_fit_h(dbscan_handle* h, const double* x, const double* y, int64_t n, double eps,
                     int32_t min_points, int32_t mode, int32_t* cluster_out, uint8_t* flag_out,
                     int32_t* n_clusters_out) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        settle(h);
        check_fit_args(n, eps, mode, x, y, cluster_out, flag_out, true);
        if (n == 0) {
            if (n_clusters_out) *n_clusters_out = 0;
            h->stats = dbscan::FitStats();
            return DBSCAN_OK;
        }
        if (n <= kPinnedFitMax) {
            // partition-sized fits (the seam's call): x|y through one pinned block and ONE DMA,
            // cluster|flag back the same way, one synchronization for the whole call
            const size_t in_b = 16 * (size_t)n, out_b = 5 * (size_t)n;
            if (h->fpinned_bytes < in_b + out_b) {
                if (h->fpinned) (void)hipHostFree(h->fpinned);
                h->fpinned = nullptr;
                h->fpinned_bytes = 0;
                const size_t cap = 21 * (size_t)kPinnedFitMax;
                DBSCAN_HIP_CHECK(hipHostMalloc(&h->fpinned, cap, hipHostMallocDefault));
                h->fpinned_bytes = cap;
                void* dev = nullptr;
                DBSCAN_HIP_CHECK(hipHostGetDevicePointer(&dev, h->fpinned, 0));
                h->fpinned_dev = static_cast<char*>(dev);
            }
            char* pin = static_cast<char*>(h->fpinned);
            memcpy(pin, x, 8 * (size_t)n);
            memcpy(pin + 8 * (size_t)n, y, 8 * (size_t)n);
            double* dxy = static_cast<double*>(h->hxy.ensure(in_b));
            char* dout = static_cast<char*>(h->hclfl.ensure(out_b));
            DBSCAN_HIP_CHECK(hipMemcpyAsync(dxy, pin, in_b, hipMemcpyHostToDevice, h->stream));
            dbscan::FitArgs a{dxy, dxy + n, nullptr, n, eps, min_points, mode,
                              reinterpret_cast<int32_t*>(dout),
                              reinterpret_cast<uint8_t*>(dout + 4 * (size_t)n), nullptr, nullptr};
            a.small_max = h->small_max;
            a.spread_min = h->spread_min;
            a.band_max = h->band_max;
            a.band_min = h->band_min;
            // the LDS forms write cluster|flag straight into the pinned block (no copy back) up
            // to kDirectOutMax points (250 / 2000 / 8192 points 2 us less per call; 4 executor
            // threads over the 1597 G(10^7) partitions 80 -> 74 us per partition); above it
            // their scattered label writes over PCIe cost more than the copy (65536 points: 277
            // -> 343 us per call)
            if (n <= kDirectOutMax) {
                a.cluster_host = reinterpret_cast<int32_t*>(h->fpinned_dev + in_b);
                a.flag_host = reinterpret_cast<uint8_t*>(h->fpinned_dev + in_b + 4 * (size_t)n);
            }
            h->prepared = false;
            dbscan::enqueue_fit(h->stream, h->ws, &h->prof, a, &h->slab);
            const bool direct = h->ws.out_direct;
            if (!direct)
                DBSCAN_HIP_CHECK(
                    hipMemcpyAsync(pin + in_b, dout, out_b, hipMemcpyDeviceToHost, h->stream));
            h->stats = dbscan::read_fit_stats(h->stream, h->ws, &h->prof);  // (synchronizes)
            if (h->ws.spread_recovered && !direct) {  // re-run fit: its labels copied back again
                DBSCAN_HIP_CHECK(
                    hipMemcpyAsync(pin + in_b, dout, out_b, hipMemcpyDeviceToHost, h->stream));
                DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
            }
            h->slab.nf = h->stats.nf;
            memcpy(cluster_out, pin + in_b, 4 * (size_t)n);
            memcpy(flag_out, pin + in_b + 4 * (size_t)n, (size_t)n);
            h->prof.flush();
            if (n_clusters_out) *n_clusters_out = (int32_t)h->stats.nclusters;
            return DBSCAN_OK;
        }
        double* dx = static_cast<double*>(h->hx.ensure(n * sizeof(double)));
        double* dy = static_cast<double*>(h->hy.ensure(n * sizeof(double)));
        int32_t* dcl = static_cast<int32_t*>(h->hcl.ensure(n * sizeof(int32_t)));
        uint8_t* dfl = static_cast<uint8_t*>(h->hfl.ensure(n));
        {
            // Concurrent handles (Spark local[N] executor threads) take turns on the device's
            // PCIe link for large copies, so one fit's kernels overlap another's copies instead
            // of two pageable copies contending (the lock is not held while kernels run)
            XferLock xl(h->device, n);
            DBSCAN_HIP_CHECK(
                hipMemcpyAsync(dx, x, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
            DBSCAN_HIP_CHECK(
                hipMemcpyAsync(dy, y, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
            if (xl.held()) DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
        }
        dbscan::FitArgs a{dx, dy, nullptr, n, eps, min_points, mode, dcl, dfl, nullptr, nullptr};
        a.small_max = h->small_max;
        a.spread_min = h->spread_min;
        a.band_max = h->band_max;
        a.band_min = h->band_min;
        h->prepared = false;
        int64_t k = dbscan::run_fit(h->stream, h->ws, &h->prof, a, &h->stats, &h->slab);
        {
            XferLock xl(h->device, n);  // (run_fit has waited for the fit)
            DBSCAN_HIP_CHECK(hipMemcpyAsync(cluster_out, dcl, n * sizeof(int32_t),
                                            hipMemcpyDeviceToHost, h->stream));
            DBSCAN_HIP_CHECK(hipMemcpyAsync(flag_out, dfl, n, hipMemcpyDeviceToHost, h->stream));
            DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
        }
        h->prof.flush();
        if (n_clusters_out) *n_clusters_out = (int32_t)k;
        return DBSCAN_OK;
    });
}

int32_t dbscan_fit(const double* x, const double* y, int64_t n, double eps, int32_t min_points,
                   int32_t mode, int32_t* cluster_out, uint8_t* flag_out,
                   int32_t* n_clusters_out) {
    if (!g_tls_handle) {
        dbscan_handle* h = dbscan_create(0);
        if (!h) return DBSCAN_EHIP;
        g_tls_handle.reset(h);
    }
    return dbscan_fit_h(g_tls_handle.get(), x, y, n, eps, min_points, mode, cluster_out,
                        flag_out, n_clusters_out);
}

int32_t dbscan_train_node(const double* x, const double* y, int64_t n, double eps,
                          int32_t min_points, int32_t mode, int32_t n_shards,
                          int32_t* cluster_out, uint8_t* flag_out, int64_t* n_clusters_out) {
    return guarded(nullptr, [&]() -> int32_t {
        check_fit_args(n, eps, mode, x, y, cluster_out, flag_out);
        if (!n_clusters_out) throw dbscan::ArgError{"NULL n_clusters_out"};
        *n_clusters_out = 0;
        if (n == 0) return DBSCAN_OK;
        std::string err;
        const int32_t rc = dbscan::train_node(x, y, n, eps, min_points, mode, n_shards,
                                              cluster_out, flag_out, n_clusters_out, &err);
        if (rc != DBSCAN_OK) set_err(err);
        return rc;
    });
}

int32_t dbscan_train_node_shards(int32_t* device_out, int64_t* points_out, int64_t* shared_out,
                                 int32_t max) {
    return guarded(nullptr, [&]() -> int32_t {
        if (max < 0) throw dbscan::ArgError{"max < 0"};
        return dbscan::node_record(device_out, points_out, shared_out, max);
    });
}

int32_t dbscan_selftest_node_plan(int32_t n_shards, int32_t ndev, int32_t fail_device,
                                  int32_t* ran_on, int32_t* rc_of_device) {
    return guarded(nullptr, [&]() -> int32_t {
        if (n_shards < 1 || n_shards > 4096 || ndev < 1 || ndev > 64 || !ran_on || !rc_of_device)
            throw dbscan::ArgError{"selftest: bad arguments"};
        return dbscan::node_plan_selftest(n_shards, ndev, fail_device, ran_on, rc_of_device);
    });
}

int32_t dbscan_selftest_worker_errors(int32_t* rcs, int32_t n) {
    return guarded(nullptr, [&]() -> int32_t {
        if (n < 0 || (n > 0 && !rcs)) throw dbscan::ArgError{"selftest: bad arguments"};
        return dbscan::worker_selftest(rcs, n);
    });
}

int64_t dbscan_route_slabs_device(dbscan_handle* h, const double* d_x, const double* d_y,
                                  int64_t m, int64_t start, const double* cuts, int32_t n_cuts,
                                  double eps, int64_t* d_rows, int64_t capacity,
                                  int64_t* counts_out) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    int64_t total = 0;
    const int32_t rc = guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        if (m < 0 || start < 0 || n_cuts < 0 || !counts_out || (n_cuts > 0 && !cuts) ||
            (m > 0 && (!d_x || !d_y)) || capacity < 0)
            throw dbscan::ArgError{"bad routing arguments"};
        if (!std::isfinite(eps * eps)) throw dbscan::ArgError{"eps*eps must be finite to shard"};
        settle(h);
        total = dbscan::route_slabs(h->stream, h->ws.route, h->ws.route_tab, d_x, d_y, m, start,
                                    cuts, n_cuts, eps, d_rows, capacity, counts_out);
        return DBSCAN_OK;
    });
    return rc == DBSCAN_OK ? total : rc;
}

int64_t dbscan_slab_select_device(dbscan_handle* h, const double* d_x, const double* d_y,
                                  int64_t n, const double* cuts, int32_t n_cuts, int32_t rank,
                                  double eps, double* d_sx, double* d_sy, uint8_t* d_szone,
                                  int64_t* d_sgid, int64_t* d_sshared, int64_t capacity,
                                  int64_t* n_shared_out) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    int64_t m = 0;
    const int32_t rc = guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        if (n < 0 || n_cuts < 0 || n_cuts >= 64 || !n_shared_out || (n_cuts > 0 && !cuts) ||
            (n > 0 && (!d_x || !d_y)) || capacity < 0 ||
            (d_sx && (!d_sy || !d_szone || !d_sgid || !d_sshared)))
            throw dbscan::ArgError{"bad slab selection arguments"};
        if (!std::isfinite(eps * eps)) throw dbscan::ArgError{"eps*eps must be finite to shard"};
        settle(h);
        m = dbscan::select_slab(h->stream, h->ws.route, h->ws.scan, d_x, d_y, n, cuts, n_cuts,
                                rank, eps, d_sx, d_sy, d_szone, d_sgid, d_sshared, capacity,
                                n_shared_out);
        return DBSCAN_OK;
    });
    return rc == DBSCAN_OK ? m : rc;
}

int64_t dbscan_owned_rows_device(dbscan_handle* h, const uint8_t* d_zone, const int64_t* d_gid,
                                 const int32_t* d_cluster, const uint8_t* d_flag, int64_t m,
                                 int64_t* d_rows, int64_t capacity) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    int64_t k = 0;
    const int32_t rc = guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        if (m < 0 || capacity < 0 || (m > 0 && (!d_zone || !d_gid || !d_cluster || !d_flag)))
            throw dbscan::ArgError{"bad owned-rows arguments"};
        settle(h);
        k = dbscan::owned_rows(h->stream, h->ws.route, h->ws.scan, d_zone, d_gid, d_cluster,
                               d_flag, m, d_rows, capacity);
        return DBSCAN_OK;
    });
    return rc == DBSCAN_OK ? k : rc;
}

int64_t dbscan_rows_unpack_device(dbscan_handle* h, const int64_t* d_rows, int64_t k,
                                  double* d_sx, double* d_sy, uint8_t* d_szone, int64_t* d_sgid,
                                  int64_t* d_sshared) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    int64_t ns = 0;
    const int32_t rc = guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        if (k < 0 || (k > 0 && (!d_rows || !d_sx || !d_sy || !d_szone || !d_sgid || !d_sshared)))
            throw dbscan::ArgError{"bad unpack arguments"};
        settle(h);
        ns = dbscan::unpack_rows(h->stream, h->ws.route, h->ws.scan, d_rows, k, d_sx, d_sy,
                                 d_szone, d_sgid, d_sshared);
        return DBSCAN_OK;
    });
    return rc == DBSCAN_OK ? ns : rc;
}

int32_t dbscan_label_scatter_device(dbscan_handle* h, const int64_t* d_rows, int64_t k,
                                    int64_t start, int64_t m, int32_t* d_cluster,
                                    uint8_t* d_flag) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        if (k < 0 || m < 0 || (k > 0 && (!d_rows || !d_cluster || !d_flag)))
            throw dbscan::ArgError{"bad label scatter arguments"};
        dbscan::label_scatter(h->stream, d_rows, k, start, m, d_cluster, d_flag);
        return DBSCAN_OK;
    });
}

}  // extern "C"

namespace {
// Partitions to the caller's buffers: (x, y, x2, y2) quadruples + counts, at most max_parts;
// returns the full count.
int64_t emit_partitions(const std::vector<dbscan::Partition>& parts, double* rects_out,
                        int64_t* counts_out, int64_t max_parts) {
    const int64_t k = (int64_t)parts.size();
    for (int64_t i = 0; i < k && i < max_parts; ++i) {
        rects_out[4 * i + 0] = parts[i].x;
        rects_out[4 * i + 1] = parts[i].y;
        rects_out[4 * i + 2] = parts[i].x2;
        rects_out[4 * i + 3] = parts[i].y2;
        counts_out[i] = parts[i].count;
    }
    return k;
}

template <class F>
int64_t guarded64(dbscan_handle* h, F&& f) {
    int64_t r = 0;
    const int32_t rc = guarded(h, [&]() -> int32_t {
        r = f();
        return DBSCAN_OK;
    });
    return rc == DBSCAN_OK ? r : (int64_t)rc;
}
}  // namespace

extern "C" {

int64_t dbscan_partition_device(dbscan_handle* h, const double* d_x, const double* d_y, int64_t n,
                                double eps, int64_t max_points_per_partition, double* rects_out,
                                int64_t* counts_out, int64_t max_parts) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded64(h, [&]() -> int64_t {
        std::lock_guard<std::mutex> lk(h->mu);
        settle(h);
        if (n < 0 || max_parts < 0 || (n > 0 && (!d_x || !d_y)) ||
            (max_parts > 0 && (!rects_out || !counts_out)))
            throw dbscan::ArgError{"bad partition arguments"};
        std::vector<dbscan::Partition> parts;
        dbscan::run_partition(h->stream, h->ws, d_x, d_y, n, eps, max_points_per_partition,
                              &parts);
        return emit_partitions(parts, rects_out, counts_out, max_parts);
    });
}

int64_t dbscan_partition(dbscan_handle* h, const double* x, const double* y, int64_t n,
                         double eps, int64_t max_points_per_partition, double* rects_out,
                         int64_t* counts_out, int64_t max_parts) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded64(h, [&]() -> int64_t {
        std::lock_guard<std::mutex> lk(h->mu);
        settle(h);
        if (n < 0 || max_parts < 0 || (n > 0 && (!x || !y)) ||
            (max_parts > 0 && (!rects_out || !counts_out)))
            throw dbscan::ArgError{"bad partition arguments"};
        std::vector<dbscan::Partition> parts;
        if (n > 0) {
            double* dx = static_cast<double*>(h->hx.ensure(n * sizeof(double)));
            double* dy = static_cast<double*>(h->hy.ensure(n * sizeof(double)));
            DBSCAN_HIP_CHECK(
                hipMemcpyAsync(dx, x, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
            DBSCAN_HIP_CHECK(
                hipMemcpyAsync(dy, y, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
            dbscan::run_partition(h->stream, h->ws, dx, dy, n, eps, max_points_per_partition,
                                  &parts);
        }
        return emit_partitions(parts, rects_out, counts_out, max_parts);
    });
}

int64_t dbscan_partition_cells(const double* cell_x, const double* cell_y,
                               const int64_t* cell_counts, int64_t ncells,
                               int64_t max_points_per_partition, double min_rect_size,
                               double* rects_out, int64_t* counts_out, int64_t max_parts) {
    return guarded64(nullptr, [&]() -> int64_t {
        if (ncells < 0 || max_parts < 0 || (ncells > 0 && (!cell_x || !cell_y || !cell_counts)) ||
            (max_parts > 0 && (!rects_out || !counts_out)) || !(min_rect_size > 0))
            throw dbscan::ArgError{"bad partition arguments"};
        std::vector<dbscan::Partition> parts;
        dbscan::partition_cells(cell_x, cell_y, cell_counts, ncells, max_points_per_partition,
                                min_rect_size, &parts);
        return emit_partitions(parts, rects_out, counts_out, max_parts);
    });
}

int64_t dbscan_csv_read(const char* path, double* x_out, double* y_out, int64_t capacity) {
    return guarded64(nullptr, [&]() -> int64_t {
        if (!path || capacity < 0 || ((x_out == nullptr) != (y_out == nullptr)))
            throw dbscan::ArgError{"bad csv arguments"};
        return dbscan::csv_read(path, x_out, y_out, capacity);
    });
}

int32_t dbscan_csv_write(const char* path, const double* x, const double* y,
                         const int32_t* cluster, int64_t n) {
    return guarded(nullptr, [&]() -> int32_t {
        if (!path || n < 0 || (n > 0 && (!x || !y || !cluster)))
            throw dbscan::ArgError{"bad csv arguments"};
        dbscan::csv_write(path, x, y, cluster, n);
        return DBSCAN_OK;
    });
}

int32_t dbscan_format_double(double v, char* buf) {
    if (!buf) return DBSCAN_EARG;
    return dbscan::jdk8_double_string(v, buf);
}

int64_t dbscan_scala_range_count(double start, double end, double step, int32_t inclusive) {
    int64_t r = DBSCAN_EARG;
    const int32_t rc = guarded(nullptr, [&]() -> int32_t {
        r = dbscan::scala_range_count(start, end, step, inclusive != 0);
        return DBSCAN_OK;
    });
    return rc == DBSCAN_OK ? r : rc;
}

int32_t dbscan_slab_fit_device(dbscan_handle* h, const double* d_x, const double* d_y,
                               const uint8_t* d_zone, int64_t n, double eps,
                               int32_t min_points, uint8_t* d_core, int32_t* d_root) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        settle(h);
        check_fit_args(n, eps, DBSCAN_MODE_NAIVE, d_x, d_y, d_core, d_root);
        if (n > 0 && !d_zone) throw dbscan::ArgError{"NULL zone pointer"};
        dbscan::FitArgs a{d_x, d_y, d_zone, n, eps, min_points, DBSCAN_MODE_NAIVE, nullptr,
                          nullptr, d_core, d_root};
        h->prepared = false;
        dbscan::run_fit(h->stream, h->ws, &h->prof, a, &h->stats, &h->slab);
        h->prof.flush();
        return DBSCAN_OK;
    });
}

int32_t dbscan_slab_fit_device_async(dbscan_handle* h, const double* d_x, const double* d_y,
                                     const uint8_t* d_zone, int64_t n, double eps,
                                     int32_t min_points, uint8_t* d_core, int32_t* d_root) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        check_fit_args(n, eps, DBSCAN_MODE_NAIVE, d_x, d_y, d_core, d_root);
        if (n > 0 && !d_zone) throw dbscan::ArgError{"NULL zone pointer"};
        if (h->pending && h->prof.pending.size() > 4096) settle(h);
        h->pending = false;
        dbscan::FitArgs a{d_x, d_y, d_zone, n, eps, min_points, DBSCAN_MODE_NAIVE, nullptr,
                          nullptr, d_core, d_root};
        h->prepared = false;
        dbscan::enqueue_fit(h->stream, h->ws, &h->prof, a, &h->slab);
        h->pending = true;
        return DBSCAN_OK;
    });
}

int32_t dbscan_slab_fit_shared_device_async(dbscan_handle* h, const double* d_x,
                                            const double* d_y, const uint8_t* d_zone, int64_t n,
                                            double eps, int32_t min_points,
                                            const int64_t* d_shared, int64_t n_shared,
                                            uint8_t* d_core, int32_t* d_root) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        check_fit_args(n, eps, DBSCAN_MODE_NAIVE, d_x, d_y, d_core, d_root);
        if (n > 0 && !d_zone) throw dbscan::ArgError{"NULL zone pointer"};
        if (n_shared < 0 || n_shared > n || (n_shared > 0 && !d_shared))
            throw dbscan::ArgError{"bad shared point list"};
        if (h->pending && h->prof.pending.size() > 4096) settle(h);
        h->pending = false;
        dbscan::FitArgs a{d_x, d_y, d_zone, n, eps, min_points, DBSCAN_MODE_NAIVE, nullptr,
                          nullptr, d_core, d_root};
        static const int64_t kNone = 0;
        a.shared_idx = n_shared > 0 ? d_shared : &kNone;  // non-null: the lean output
        a.n_shared = n_shared;
        h->prepared = false;
        dbscan::enqueue_fit(h->stream, h->ws, &h->prof, a, &h->slab);
        h->pending = true;
        return DBSCAN_OK;
    });
}

int32_t dbscan_slab_merge_roots_device(dbscan_handle* h, int64_t n, const uint8_t* d_zone,
                                       const int64_t* d_gid, const int32_t* d_root,
                                       const int32_t* d_parent, int64_t* d_gs_of_root,
                                       int64_t* d_own_roots, int64_t* n_own_out) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        settle(h);
        if (n < 0 || !n_own_out) throw dbscan::ArgError{"bad merge-roots arguments"};
        if (n > 0 && (!d_zone || !d_gid || !d_root || !d_parent || !d_gs_of_root || !d_own_roots))
            throw dbscan::ArgError{"NULL array pointer"};
        *n_own_out = dbscan::run_slab_merge_roots(h->stream, h->ws, n, d_zone, d_gid, d_root,
                                                  d_parent, d_gs_of_root, d_own_roots);
        return DBSCAN_OK;
    });
}

int32_t dbscan_slab_roots_prepare_device(dbscan_handle* h, int64_t n, const uint8_t* d_zone,
                                         const int64_t* d_gid, const int32_t* d_root,
                                         const int32_t* d_parent, int64_t* d_gs_of_root,
                                         int32_t mode, int64_t* d_own_roots,
                                         int64_t* n_own_out) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        if (n < 0 || !n_own_out) throw dbscan::ArgError{"bad merge-roots arguments"};
        if (mode != DBSCAN_MODE_NAIVE && mode != DBSCAN_MODE_ARCHERY)
            throw dbscan::ArgError{"bad mode"};
        if (!h->slab.valid) throw dbscan::ArgError{"no slab fit on this handle"};
        if (n != h->slab.n) throw dbscan::ArgError{"n differs from the slab fit's point count"};
        if (n > 0 && (!d_zone || !d_gid || !d_root || !d_parent || !d_gs_of_root || !d_own_roots))
            throw dbscan::ArgError{"NULL array pointer"};
        if (!h->pinned)
            DBSCAN_HIP_CHECK(hipHostMalloc(&h->pinned, 512, hipHostMallocDefault));
        if (!h->ready) DBSCAN_HIP_CHECK(hipEventCreateWithFlags(&h->ready, hipEventDisableTiming));
        double* stats_buf = static_cast<double*>(h->pinned);
        int32_t* total = reinterpret_cast<int32_t*>(stats_buf + dbscan::kFitStatsDoubles);
        const bool fit_pending = h->pending;
        if (fit_pending) dbscan::enqueue_fit_stats_copy(h->stream, h->ws, stats_buf);
        int32_t* lroots = static_cast<int32_t*>(h->ws.lroots.ensure(std::max<int64_t>(1, n) * sizeof(int32_t)));
        dbscan::enqueue_slab_merge_roots(h->stream, h->ws, n, d_zone, d_gid, d_root, d_parent,
                                         d_gs_of_root, d_own_roots, total, lroots);
        DBSCAN_HIP_CHECK(hipEventRecord(h->ready, h->stream));
        // Enqueued behind the count: the GPU labels while the host waits, gathers and numbers.
        dbscan::enqueue_slab_label_prepare(h->stream, h->ws, &h->prof, h->slab, d_zone, d_gid,
                                           d_gs_of_root, mode);
        DBSCAN_HIP_CHECK(hipEventSynchronize(h->ready));
        if (fit_pending) {
            h->pending = false;
            h->stats = dbscan::parse_fit_stats(h->ws, stats_buf);
            h->slab.nf = h->stats.nf;
        }
        h->prof.flush_ready();
        h->prepared = true;
        h->slab.nlroots = total[1] - total[0];
        *n_own_out = total[0];
        return DBSCAN_OK;
    });
}

int32_t dbscan_slab_label_finish_device_async(dbscan_handle* h, const uint8_t* d_zone,
                                              const int64_t* d_gs_of_root,
                                              const int64_t* d_all_roots, int64_t n_all_roots,
                                              int32_t* d_cluster, uint8_t* d_flag) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        if (!h->prepared) throw dbscan::ArgError{"no dbscan_slab_roots_prepare_device since the slab fit"};
        if (n_all_roots < 0) throw dbscan::ArgError{"n_all_roots < 0"};
        if (h->slab.n > 0 && (!d_zone || !d_gs_of_root || !d_cluster || !d_flag ||
                              (n_all_roots > 0 && !d_all_roots)))
            throw dbscan::ArgError{"NULL array pointer"};
        dbscan::run_slab_label_finish(h->stream, h->ws, &h->prof, h->slab, d_zone, d_gs_of_root,
                                      d_all_roots, n_all_roots, d_cluster, d_flag);
        return DBSCAN_OK;
    });
}

namespace {
int32_t slab_label(dbscan_handle* h, const uint8_t* d_zone, const int64_t* d_gid,
                   const int64_t* d_gs_of_root, const int64_t* d_all_roots, int64_t n_all_roots,
                   int32_t mode, int32_t* d_cluster, uint8_t* d_flag, bool sync) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        if (mode != DBSCAN_MODE_NAIVE && mode != DBSCAN_MODE_ARCHERY)
            throw dbscan::ArgError{"bad mode"};
        if (n_all_roots < 0) throw dbscan::ArgError{"n_all_roots < 0"};
        if (h->slab.n > 0 && (!d_zone || !d_gid || !d_gs_of_root || !d_cluster || !d_flag ||
                              (n_all_roots > 0 && !d_all_roots)))
            throw dbscan::ArgError{"NULL array pointer"};
        dbscan::run_slab_label(h->stream, h->ws, &h->prof, h->slab, d_zone, d_gid, d_gs_of_root,
                               d_all_roots, n_all_roots, mode, d_cluster, d_flag);
        if (sync) {
            DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
            settle(h);
            h->prof.flush();
        }
        return DBSCAN_OK;
    });
}
}  // namespace

int32_t dbscan_slab_label_device(dbscan_handle* h, const uint8_t* d_zone, const int64_t* d_gid,
                                 const int64_t* d_gs_of_root, const int64_t* d_all_roots,
                                 int64_t n_all_roots, int32_t mode, int32_t* d_cluster,
                                 uint8_t* d_flag) {
    return slab_label(h, d_zone, d_gid, d_gs_of_root, d_all_roots, n_all_roots, mode, d_cluster,
                      d_flag, true);
}

int32_t dbscan_slab_label_device_async(dbscan_handle* h, const uint8_t* d_zone,
                                       const int64_t* d_gid, const int64_t* d_gs_of_root,
                                       const int64_t* d_all_roots, int64_t n_all_roots,
                                       int32_t mode, int32_t* d_cluster, uint8_t* d_flag) {
    return slab_label(h, d_zone, d_gid, d_gs_of_root, d_all_roots, n_all_roots, mode, d_cluster,
                      d_flag, false);
}

int32_t dbscan_last_stats(dbscan_handle* h, int64_t* out, int32_t max) {
    if (!h || !out) return DBSCAN_EARG;
    if (h->pending && dbscan_sync(h) != DBSCAN_OK) return DBSCAN_EHIP;
    const int64_t v[14] = {h->stats.n,         h->stats.nf,         h->stats.ncells,
                           h->stats.ncore,     h->stats.nclusters,  h->stats.nx,
                           h->stats.ny,        h->stats.bits,       h->stats.grid_mode,
                           h->stats.ntiles,    h->stats.clique,     h->stats.pts_small,
                           h->stats.pts_medium, h->stats.pts_big};
    int k = 0;
    for (; k < max && k < 14; ++k) out[k] = v[k];
    return k;
}

int32_t dbscan_profile_enable(dbscan_handle* h, int32_t on) {
    if (!h || on < 0 || on > 2) return DBSCAN_EARG;
    h->prof.on = on != 0;
    h->prof.mode = on;
    return DBSCAN_OK;
}

int32_t dbscan_profile_only(dbscan_handle* h, const char* kernel) {
    if (!h) return DBSCAN_EARG;
    h->prof.only = kernel ? kernel : "";
    return DBSCAN_OK;
}

int32_t dbscan_profile_reset(dbscan_handle* h) {
    if (!h) return DBSCAN_EARG;
    h->prof.stages.clear();
    return DBSCAN_OK;
}

int32_t dbscan_profile_read(dbscan_handle* h, char* names, int32_t names_cap, double* total_ms,
                            int64_t* launches, int32_t max) {
    if (!h) return DBSCAN_EARG;
    int32_t k = 0, off = 0;
    for (auto& st : h->prof.stages) {
        if (k >= max) break;
        const int len = (int)st.name.size() + 1;
        if (names) {
            if (off + len > names_cap) break;
            memcpy(names + off, st.name.c_str(), (size_t)len);
        }
        off += len;
        if (total_ms) total_ms[k] = st.ms;
        if (launches) launches[k] = st.launches;
        ++k;
    }
    return k;
}

int64_t dbscan_set_small_max(dbscan_handle* h, int64_t max_points) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    std::lock_guard<std::mutex> lk(h->mu);
    const int64_t prev = h->small_max;
    h->small_max = std::min<int64_t>(std::max<int64_t>(max_points, 0), dbscan::kSmallMaxPoints);
    return prev;
}

int64_t dbscan_set_spread_min(dbscan_handle* h, int64_t min_points) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    std::lock_guard<std::mutex> lk(h->mu);
    const int64_t prev = h->spread_min;
    h->spread_min = std::max<int64_t>(min_points, 0);
    return prev;
}

int64_t dbscan_set_band_max(dbscan_handle* h, int64_t max_points) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    std::lock_guard<std::mutex> lk(h->mu);
    const int64_t prev = h->band_max;
    h->band_max = std::max<int64_t>(0, std::min<int64_t>(max_points, DBSCAN_BAND_MAX_POINTS));
    return prev;
}

int64_t dbscan_set_band_min(dbscan_handle* h, int64_t min_points) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    std::lock_guard<std::mutex> lk(h->mu);
    const int64_t prev = h->band_min;
    h->band_min = std::max<int64_t>(min_points, 0);
    return prev;
}

int64_t dbscan_set_spread_spin_limit(dbscan_handle* h, int64_t polls) {
    if (!h || polls < 0 || polls > (int64_t)UINT32_MAX) {
        set_err(h ? "polls out of range" : "NULL handle");
        return DBSCAN_EARG;
    }
    std::lock_guard<std::mutex> lk(h->mu);
    const int64_t prev = h->ws.spread_spin_limit;
    h->ws.spread_spin_limit = (uint32_t)polls;
    return prev;
}

int64_t dbscan_spread_fallbacks(dbscan_handle* h) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    std::lock_guard<std::mutex> lk(h->mu);
    return h->ws.spread_fallbacks;
}

}  // extern "C"

namespace {

// Validates a batch's offsets (n_parts + 1 non-decreasing, >= 0) and returns the total span.
int64_t batch_span(const int64_t* offsets, int32_t n_parts) {
    if (n_parts < 0) throw dbscan::ArgError{"n_parts < 0"};
    if (!offsets) throw dbscan::ArgError{"NULL offsets"};
    if (offsets[0] < 0) throw dbscan::ArgError{"offsets[0] < 0"};
    for (int32_t p = 0; p < n_parts; ++p)
        if (offsets[p + 1] < offsets[p]) throw dbscan::ArgError{"offsets must not decrease"};
    if (offsets[n_parts] > DBSCAN_MAX_POINTS) throw dbscan::ArgError{"too many points"};
    return offsets[n_parts];
}

// Batches that span at least this many points (or hold a partition over the one-workgroup
// capacity) run as ONE tiled fit over per-partition grids (batch.hip); smaller ones as one
// launch of the one-workgroup kernel (small.hip).
constexpr int64_t kBatchTiledSpan = 65536;

// Pinned staging of the batch tables (grow-only), free once the last upload from it is done.
char* batch_pinned(dbscan_handle* h, size_t need) {
    if (!h->bcopied) DBSCAN_HIP_CHECK(hipEventCreateWithFlags(&h->bcopied, hipEventDisableTiming));
    else DBSCAN_HIP_CHECK(hipEventSynchronize(h->bcopied));
    if (h->bpinned_bytes < need) {
        if (h->bpinned) (void)hipHostFree(h->bpinned);
        h->bpinned = nullptr;
        h->bpinned_bytes = 0;
        DBSCAN_HIP_CHECK(hipHostMalloc(&h->bpinned, need + need / 2, hipHostMallocDefault));
        h->bpinned_bytes = need + need / 2;
    }
    return static_cast<char*>(h->bpinned);
}

// Enqueues one batch on the handle's stream (device arrays indexed like the offsets, host
// offsets).  Large batches: one tiled fit over the partitions' own grids (batch.hip; one host
// synchronization, for the partitions' boxes), the partitions it cannot place fitted one after
// another.  Small batches: the partitions the one-workgroup kernel serves in ONE launch, the
// others through the tiled pipeline one after another (stream-ordered on the handle's workspace).
void batch_enqueue(dbscan_handle* h, const double* dx, const double* dy, const int64_t* offs,
                   int32_t n_parts, double eps, int32_t min_points, int32_t mode, int32_t* dcl,
                   uint8_t* dfl, int32_t* dnk) {
    const int64_t cap = std::min<int64_t>(h->small_max, dbscan::kSmallMaxPoints);
    const int64_t o0 = n_parts > 0 ? offs[0] : 0, span = n_parts > 0 ? offs[n_parts] - o0 : 0;
    bool over = false;
    for (int32_t p = 0; p < n_parts && !over; ++p) over = offs[p + 1] - offs[p] > cap;
    const bool tiled = n_parts > 1 && (mode == DBSCAN_MODE_NAIVE || mode == DBSCAN_MODE_ARCHERY) &&
                       std::isfinite(eps * eps) && (over || span >= kBatchTiledSpan);
    std::vector<int32_t> alone;
    h->pending = false;
    if (tiled) {
        const size_t offs_b = (size_t)(n_parts + 1) * sizeof(int64_t);
        const size_t box_b = (size_t)n_parts * 5 * sizeof(double);
        const size_t tab_b = (size_t)n_parts * sizeof(dbscan::PartGrid);
        char* pin = batch_pinned(h, offs_b + box_b + tab_b);
        int64_t* rel = reinterpret_cast<int64_t*>(pin);
        double* box = reinterpret_cast<double*>(pin + offs_b);
        auto* tab = reinterpret_cast<dbscan::PartGrid*>(pin + offs_b + box_b);
        for (int32_t p = 0; p <= n_parts; ++p) rel[p] = offs[p] - o0;
        char* dev = static_cast<char*>(h->boffs.ensure(offs_b + tab_b));
        auto* d_offs = reinterpret_cast<int64_t*>(dev);
        auto* d_tab = reinterpret_cast<dbscan::PartGrid*>(dev + offs_b);
        double* d_box = static_cast<double*>(h->ws.pbox.ensure(box_b));
        DBSCAN_HIP_CHECK(hipMemcpyAsync(d_offs, rel, offs_b, hipMemcpyHostToDevice, h->stream));
        dbscan::enqueue_batch_bbox(h->stream, dx + o0, dy + o0, d_offs, n_parts, d_box);
        DBSCAN_HIP_CHECK(hipMemcpyAsync(box, d_box, box_b, hipMemcpyDeviceToHost, h->stream));
        DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
        dbscan::BatchFit bf;
        if (dbscan::plan_batch_grid(box, rel, n_parts, eps, tab, &bf, &alone)) {
            DBSCAN_HIP_CHECK(hipMemcpyAsync(d_tab, tab, tab_b, hipMemcpyHostToDevice, h->stream));
            bf.g.parts = d_tab;
            bf.g.poffs = d_offs;
            bf.nclusters = dnk;
            dbscan::FitArgs a{dx + o0, dy + o0, nullptr, span, eps, min_points, mode,
                              dcl + o0, dfl + o0, nullptr, nullptr};
            a.small_max = 0;
            a.batch = &bf;
            dbscan::enqueue_fit(h->stream, h->ws, &h->prof, a, &h->slab);
            h->pending = true;
        }
        DBSCAN_HIP_CHECK(hipEventRecord(h->bcopied, h->stream));
    } else {
        std::vector<int32_t> small;
        for (int32_t p = 0; p < n_parts; ++p) {
            const int64_t m = offs[p + 1] - offs[p];
            if (m <= cap && dbscan::small_fit_eligible(m, eps, mode)) small.push_back(p);
            else alone.push_back(p);
        }
        if (!small.empty()) {
            const size_t need =
                (size_t)(n_parts + 1) * sizeof(int64_t) + small.size() * sizeof(int32_t);
            char* pin = batch_pinned(h, need);
            memcpy(pin, offs, (size_t)(n_parts + 1) * sizeof(int64_t));
            memcpy(pin + (size_t)(n_parts + 1) * sizeof(int64_t), small.data(),
                   small.size() * sizeof(int32_t));
            char* dev = static_cast<char*>(h->boffs.ensure(need));
            DBSCAN_HIP_CHECK(hipMemcpyAsync(dev, pin, need, hipMemcpyHostToDevice, h->stream));
            DBSCAN_HIP_CHECK(hipEventRecord(h->bcopied, h->stream));
            dbscan::enqueue_small_fits(
                h->stream, &h->prof, dx, dy, reinterpret_cast<const int64_t*>(dev),
                reinterpret_cast<const int32_t*>(dev + (size_t)(n_parts + 1) * sizeof(int64_t)),
                (int32_t)small.size(), 0, eps, min_points, mode, dcl, dfl, dnk, nullptr, nullptr);
        }
    }
    for (int32_t p : alone) {
        const int64_t o = offs[p], m = offs[p + 1] - o;
        dbscan::FitArgs a{dx + o, dy + o, nullptr, m, eps, min_points, mode, dcl + o, dfl + o,
                          nullptr, nullptr};
        a.small_max = 0;
        a.n_clusters_dev = dnk + p;
        dbscan::enqueue_fit(h->stream, h->ws, &h->prof, a, &h->slab);
        dbscan::write_nclusters(h->stream, h->ws, dnk + p);
        h->pending = true;
    }
    if (!h->pending) {
        h->stats = dbscan::FitStats();
        h->stats.n = span;
    }
    h->prepared = false;
}

}  // namespace

extern "C" {

int32_t dbscan_fit_batch_device_async(dbscan_handle* h, const double* d_x, const double* d_y,
                                      const int64_t* offsets, int32_t n_parts, double eps,
                                      int32_t min_points, int32_t mode, int32_t* d_cluster,
                                      uint8_t* d_flag, int32_t* d_n_clusters) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        const int64_t span = batch_span(offsets, n_parts);
        check_fit_args(span, eps, mode, d_x, d_y, d_cluster, d_flag, true);
        if (n_parts > 0 && !d_n_clusters) throw dbscan::ArgError{"NULL n_clusters array"};
        if (h->pending && h->prof.pending.size() > 4096) settle(h);
        batch_enqueue(h, d_x, d_y, offsets, n_parts, eps, min_points, mode, d_cluster, d_flag,
                      d_n_clusters);
        return DBSCAN_OK;
    });
}

int32_t dbscan_fit_batch(dbscan_handle* h, const double* x, const double* y,
                         const int64_t* offsets, int32_t n_parts, double eps, int32_t min_points,
                         int32_t mode, int32_t* cluster_out, uint8_t* flag_out,
                         int32_t* n_clusters_out) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        std::lock_guard<std::mutex> lk(h->mu);
        settle(h);
        const int64_t span = batch_span(offsets, n_parts);
        check_fit_args(span, eps, mode, x, y, cluster_out, flag_out, true);
        if (n_parts > 0 && !n_clusters_out) throw dbscan::ArgError{"NULL n_clusters_out"};
        if (n_parts == 0) return DBSCAN_OK;
        const int64_t o0 = offsets[0], n = span - o0;
        std::vector<int64_t> rel((size_t)n_parts + 1);
        for (int32_t p = 0; p <= n_parts; ++p) rel[(size_t)p] = offsets[p] - o0;
        const size_t nn = (size_t)std::max<int64_t>(n, 1);
        double* dx = static_cast<double*>(h->hx.ensure(nn * sizeof(double)));
        double* dy = static_cast<double*>(h->hy.ensure(nn * sizeof(double)));
        int32_t* dcl = static_cast<int32_t*>(h->hcl.ensure(nn * sizeof(int32_t)));
        uint8_t* dfl = static_cast<uint8_t*>(h->hfl.ensure(nn));
        int32_t* dnk = static_cast<int32_t*>(h->hnk.ensure((size_t)n_parts * sizeof(int32_t)));
        if (n > 0) {
            DBSCAN_HIP_CHECK(hipMemcpyAsync(dx, x + o0, n * sizeof(double), hipMemcpyHostToDevice,
                                            h->stream));
            DBSCAN_HIP_CHECK(hipMemcpyAsync(dy, y + o0, n * sizeof(double), hipMemcpyHostToDevice,
                                            h->stream));
        }
        batch_enqueue(h, dx, dy, rel.data(), n_parts, eps, min_points, mode, dcl, dfl, dnk);
        if (n > 0) {
            DBSCAN_HIP_CHECK(hipMemcpyAsync(cluster_out + o0, dcl, n * sizeof(int32_t),
                                            hipMemcpyDeviceToHost, h->stream));
            DBSCAN_HIP_CHECK(hipMemcpyAsync(flag_out + o0, dfl, n, hipMemcpyDeviceToHost,
                                            h->stream));
        }
        DBSCAN_HIP_CHECK(hipMemcpyAsync(n_clusters_out, dnk, (size_t)n_parts * sizeof(int32_t),
                                        hipMemcpyDeviceToHost, h->stream));
        DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
        settle(h);
        h->prof.flush();
        return DBSCAN_OK;
    });
}

int64_t dbscan_duplicate(const double* x, const double* y, int64_t n, const double* rects,
                         int64_t n_parts, double eps, int64_t* offsets_out, int64_t* index_out,
                         int64_t capacity) {
    return guarded64(nullptr, [&]() -> int64_t {
        if (n < 0 || n_parts < 0 || capacity < 0 || !offsets_out || (n > 0 && (!x || !y)) ||
            (n_parts > 0 && !rects))
            throw dbscan::ArgError{"bad duplicate arguments"};
        return dbscan::duplicate_points(x, y, n, rects, n_parts, eps, offsets_out, index_out,
                                        capacity);
    });
}

int32_t dbscan_generate_blobs_device(dbscan_handle* h, double* d_x, double* d_y, int64_t n,
                                     double noise_frac, double dense, uint64_t seed) {
    if (!h) {
        set_err("NULL handle");
        return DBSCAN_EARG;
    }
    return guarded(h, [&]() -> int32_t {
        if (n < 0 || (n > 0 && (!d_x || !d_y))) throw dbscan::ArgError{"bad generator args"};
        if (n == 0) return DBSCAN_OK;
        dbscan::BlobParams bp;
        const double s = std::sqrt((double)n / 1e6);  // SURVEY §8d scale-invariant generator
        uint64_t st = seed * 0x2545F4914F6CDD1Dull + 0x1234567ull;
        for (int b = 0; b < dbscan::kBlobs; ++b) {
            bp.cx[b] = (2.0 * dbscan::u01_open(dbscan::splitmix64(st)) - 1.0) * 1000.0 * s;
            bp.cy[b] = (2.0 * dbscan::u01_open(dbscan::splitmix64(st)) - 1.0) * 1000.0 * s;
            bp.sigma[b] = (20.0 + 40.0 * dbscan::u01_open(dbscan::splitmix64(st))) * s;
            if (b < 4 && dense > 0) bp.sigma[b] /= dense;
        }
        bp.noise_half = 1100.0 * s;
        bp.noise_frac = noise_frac;
        bp.seed = seed;
        hipLaunchKernelGGL(dbscan::gen_blobs_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256),
                           0, h->stream, bp, n, d_x, d_y);
        DBSCAN_HIP_CHECK(hipGetLastError());
        DBSCAN_HIP_CHECK(hipStreamSynchronize(h->stream));
        return DBSCAN_OK;
    });
}

}  // extern "C"
