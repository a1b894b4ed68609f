// calib.hip -- measurement tooling only (not the product): kernels with a KNOWN byte count in
// the access patterns of the fit's gathers, to calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a wide coalesced streaming read; other
// widths uncalibrated).  Built by tools/pmc_calibrate.py into tools/libcalib.so.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
constexpr int kB = 256;

// coalesced 16 B per lane (the guide's calibrated case)
__global__ __launch_bounds__(kB) void stream16(const double2* __restrict__ a, int64_t n,
                                               double* __restrict__ sink) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const double2 v = a[i];
    if (v.x == 1234.5 && v.y == -1.0) sink[0] = v.x;  // (never: keeps the load)
}

// gather_bucket's pattern: one random 32-B record per lane (idx: a random permutation inside
// bands of `band` records), idx read coalesced
__global__ __launch_bounds__(kB) void gather32(const double4* __restrict__ rec,
                                               const int32_t* __restrict__ idx, int64_t n,
                                               double* __restrict__ sink) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const double4 v = rec[idx[i]];
    if (v.x == 1234.5 && v.w == -1.0) sink[0] = v.y;
}

// permute_out's pattern: one random 4-B word per lane over the whole array
__global__ __launch_bounds__(kB) void gather4(const uint32_t* __restrict__ w,
                                              const int32_t* __restrict__ idx, int64_t n,
                                              uint32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    out[i] = w[idx[i]];
}
}  // namespace

extern "C" int calib_run(int which, void* a, void* idx, int64_t n, void* out) {
    const unsigned g = (unsigned)((n + kB - 1) / kB);
    if (which == 0) hipLaunchKernelGGL(stream16, dim3(g), dim3(kB), 0, 0, (const double2*)a, n, (double*)out);
    if (which == 1)
        hipLaunchKernelGGL(gather32, dim3(g), dim3(kB), 0, 0, (const double4*)a, (const int32_t*)idx, n,
                           (double*)out);
    if (which == 2)
        hipLaunchKernelGGL(gather4, dim3(g), dim3(kB), 0, 0, (const uint32_t*)a, (const int32_t*)idx, n,
                           (uint32_t*)out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
