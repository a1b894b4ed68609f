// primitives.hip -- hand-written device-wide primitives for the fit pipeline (gfx950).
//
//   exclusive_scan     one launch: 4096-element tiles held in registers (LDS transpose to
//                      16 consecutive elements per thread), tiles chained by decoupled look-back
//   radix_sort_pairs   stable LSD radix sort, 8-bit digits, 4096-key tiles:
//                      upsweep (per-wave LDS histograms) -> scan -> downsweep that ranks keys
//                      with 64-bit wave ballots (match-any over the 8 digit bits) against
//                      per-wave running digit counters, sorts the tile in LDS and writes
//                      each digit run contiguously (coalesced) to its global offset
//   bbox_partials      per-block min/max of finite coordinates + finite counts (grid sizing;
//                      the final reduction is fit.hip bbox_grid_kernel)
#include "internal.h"

#include <cmath>
#include <cstdio>
#include <type_traits>
#include <utility>

namespace dbscan {

namespace {

#ifndef RADIX_ITEMS
#define RADIX_ITEMS 8
#endif
constexpr int kItems = 16;                  // rounds per scan tile
constexpr int kTile = kBlock * kItems;      // 4096
constexpr int kWaves = kBlock / 64;         // 4

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// The radix tile a downsweep block sorts, XCD-contiguous: blocks are dealt round-robin over
// the 8 XCDs, so block b sorts tile (b % 8) * q + b / 8 and each XCD walks one contiguous run
// of tiles: the digit runs of consecutive tiles land next to each other in ONE L2 (bucket_lsd
// 0.140 -> 0.106 ms per fit at 10^7 points, 2.28 -> 1.78 at 1.25*10^8; round 5 A/B).
__device__ __forceinline__ int64_t sort_tile() {
    const int64_t G = gridDim.x, b = blockIdx.x;
    const int64_t x = b & 7, j = b >> 3, q = G >> 3, r = G & 7;
    return x * q + (x < r ? x : r) + j;
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Scan inputs: MODE 0 int32 values, MODE 1 uint8 flags (nonzero -> 1), MODE 2 the popcounts of
// uint64 bit words.
template <int MODE>
__device__ __forceinline__ int scan_value(const void* in, int64_t i, int64_t n) {
    if (i >= n) return 0;
    if constexpr (MODE == 0) {
        return static_cast<const int32_t*>(in)[i];
    } else if constexpr (MODE == 1) {
        return static_cast<const uint8_t*>(in)[i] ? 1 : 0;
    } else {
        return __popcll(static_cast<const uint64_t*>(in)[i]);
    }
}

// Single-pass exclusive scan: one 4096-element tile per block, chained by decoupled look-back.
// Tile = blockIdx.x: workgroups are dispatched in index order (per XCD), so the lowest
// unfinished tile only ever waits on finished ones and the chain always drains.  (A tile
// counter taken with a device-scope atomic would guarantee that on any dispatcher, but it
// serialises at ~20 ns a block across the XCDs: 50 us for 2442 tiles.)  A bounded spin keeps
// the kernel finite even if that assumption broke: it then flags state[0] and the results
// are wrong, never hung.  A block loads its tile with 16 coalesced rounds issued back to back,
// transposes it through LDS so each thread owns 16 consecutive elements (one 17-word padded
// row: conflict-free), scans in registers, publishes the tile aggregate, sums its predecessors'
// published values 64 tiles at a time -- aggregates until the nearest inclusive prefix --
// publishes its own inclusive prefix and stores the tile back through LDS, coalesced.  A status
// word packs (epoch, flag, value) in 64 bits, stored and polled with agent-scope atomics; the
// epoch (one per scan call) makes words of earlier scans unreadable, so the status array is
// never cleared.  In place (out == in) is fine: a block reads its whole tile before writing.
constexpr uint64_t kStAgg = 1, kStIncl = 2;
constexpr int kSpinLimit = 1 << 22;
constexpr int kRow = kItems + 1;  // padded LDS row per thread

__device__ __forceinline__ uint64_t scan_status(uint32_t epoch, uint64_t flag, int32_t v) {
    return ((uint64_t)epoch << 34) | (flag << 32) | (uint32_t)v;
}

__device__ __forceinline__ int lds_slot(int e) { return e + (e >> 4); }  // e = r*256 + tid

template <int MODE>
__device__ __forceinline__ void scan_body(int t, const void* in, int64_t n, int32_t* out,
                                          int32_t* total, uint64_t* state, uint32_t epoch,
                                          int64_t ntiles) {
    __shared__ int wtot[kWaves], wstop[kWaves], wsum[kWaves];
    __shared__ int buf[kBlock * kRow];
    const int tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const int64_t base = (int64_t)t * kTile;
    int v[kItems];
#pragma unroll
    for (int r = 0; r < kItems; ++r) v[r] = scan_value<MODE>(in, base + r * kBlock + tid, n);
#pragma unroll
    for (int r = 0; r < kItems; ++r) buf[lds_slot(r * kBlock + tid)] = v[r];
    __syncthreads();
    int sum = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {  // thread-local exclusive scan of its 16 elements
        const int x = buf[tid * kRow + k];
        v[k] = sum;
        sum += x;
    }
    const int incl = wave_incl_scan(sum);
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    int agg = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) agg += wtot[k];
    int prefix = 0;
    if (ntiles > 1) {
        uint64_t* status = state + 1;
        if (tid == 0) {
            __hip_atomic_store(status + t, scan_status(epoch, t == 0 ? kStIncl : kStAgg, agg),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // all 256 threads look back, one predecessor each per round: when every block is
        // resident at once the inclusive prefixes advance a whole window per L2 round trip
        for (int j = t - 1; j >= 0; j -= kBlock) {
            const int idx = j - tid;
            uint64_t st = 0;
            if (idx >= 0) {
                for (int spin = 0;; ++spin) {
                    st = __hip_atomic_load(status + idx, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    if ((uint32_t)(st >> 34) == epoch && ((st >> 32) & 3u) != 0) break;
                    if (spin == kSpinLimit) {  // watchdog: never reached with in-order dispatch
                        __hip_atomic_fetch_or(state, 1ull, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                        st = scan_status(epoch, kStIncl, 0);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            const uint64_t inc = __ballot(idx >= 0 && ((st >> 32) & 3u) == kStIncl);
            if (lane == 0) wstop[w] = inc ? __builtin_ctzll(inc) : 64;
            __syncthreads();
            int first = kWaves;  // nearest wave holding an inclusive prefix
#pragma unroll
            for (int k = kWaves - 1; k >= 0; --k) first = wstop[k] < 64 ? k : first;
            const bool take = idx >= 0 && (w < first || (w == first && lane <= wstop[first]));
            const int part = wave_sum(take ? (int32_t)(uint32_t)st : 0);
            if (lane == 0) wsum[w] = part;
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kWaves; ++k) prefix += wsum[k];
            if (first < kWaves) break;
        }
        if (tid == 0 && t > 0)
            __hip_atomic_store(status + t, scan_status(epoch, kStIncl, prefix + agg),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0 && t == ntiles - 1 && total) *total = prefix + agg;
    int off = prefix + incl - sum;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) off += (k < w) ? wtot[k] : 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) buf[tid * kRow + k] = off + v[k];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const int64_t i = base + r * kBlock + tid;
        if (i < n) out[i] = buf[lds_slot(r * kBlock + tid)];
    }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void scan_kernel(const void* in, int64_t n, int32_t* out,
                                                      int32_t* total, uint64_t* state,
                                                      uint32_t epoch, int64_t ntiles) {
    scan_body<MODE>(blockIdx.x, in, n, out, total, state, epoch, ntiles);
}

// Three independent int32 scans of <= kTile elements each in ONE launch, one workgroup each:
// array b is in[b * stride, b * stride + n), its total to totals[b].
struct Totals3 {
    int32_t* t[3];
};
__global__ __launch_bounds__(kBlock) void scan3_kernel(const int32_t* in, int64_t n,
                                                       int64_t stride, int32_t* out, Totals3 tt) {
    const int b = blockIdx.x;
    scan_body<0>(0, in + b * stride, n, out + b * stride, tt.t[b], nullptr, 0, 1);
}

template <int MODE>
void scan_impl(hipStream_t s, const void* in, int32_t* out, int64_t n, int32_t* total_dev,
               ScanState& ss) {
    const int64_t nb = (n + kTile - 1) / kTile;
    uint64_t* state = nb > 1 ? ss.prepare(s, nb) : nullptr;
    hipLaunchKernelGGL(scan_kernel<MODE>, dim3((unsigned)nb), dim3(kBlock), 0, s, in, n, out,
                       total_dev, state, ss.epoch, nb);
    DBSCAN_HIP_CHECK(hipGetLastError());
}

// ------------------------------------ radix sort ------------------------------------------

// Radix tiles: 2048 keys (8 rounds of 256).  Half the scan tiles' size keeps the downsweep at
// 22 KB of LDS and ~70 VGPRs: 6+ workgroups per CU instead of 4 (measured in r05 against
// 4096-key tiles: see DESIGN.md §3).
constexpr int kRItems = RADIX_ITEMS;
constexpr int kRTile = kBlock * kRItems;

// Digits of W bits (RB = 2^W buckets, W = 7..9): the passes are 8 + 8 + 9 + 7 bits, so keys
// of up to 25 bits (an eps grid of up to 2^23 cells x 4 quarters: 10^7 points of the bench)
// sort in three passes; passes at or beyond the device-side key width return at once.
template <int W>
__global__ __launch_bounds__(kBlock) void radix_upsweep_kernel(const uint32_t* __restrict__ key,
                                                               int64_t n, int shift,
                                                               const int32_t* __restrict__ bits_p,
                                                               int64_t nblocks,
                                                               int32_t* __restrict__ hist) {
    constexpr int RB = 1 << W;
    if (shift < 0) {  // the bucketed sort's MSD pass: the top 8 bits of the device-side width
        const int b = *bits_p;
        shift = b > 8 ? b - 8 : 0;
    } else if (shift >= *bits_p) {
        return;  // digit beyond the key width: nothing left to sort
    }
    __shared__ uint32_t h[kWaves][RB];
    const int w = threadIdx.x >> 6;
    for (int d = threadIdx.x; d < kWaves * RB; d += kBlock) (&h[0][0])[d] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kRTile;
    if (base + kRTile <= n) {  // a full tile: 16-B key loads, all in flight together
        static_assert(kRItems % 4 == 0, "whole uint4s per thread");
        const uint4* k4 = reinterpret_cast<const uint4*>(key + base);
        uint4 v[kRItems / 4];
#pragma unroll
        for (int r = 0; r < kRItems / 4; ++r) v[r] = k4[r * kBlock + threadIdx.x];
#pragma unroll
        for (int r = 0; r < kRItems / 4; ++r) {
            atomicAdd(&h[w][(v[r].x >> shift) & (RB - 1u)], 1u);
            atomicAdd(&h[w][(v[r].y >> shift) & (RB - 1u)], 1u);
            atomicAdd(&h[w][(v[r].z >> shift) & (RB - 1u)], 1u);
            atomicAdd(&h[w][(v[r].w >> shift) & (RB - 1u)], 1u);
        }
    } else {
#pragma unroll 4
        for (int r = 0; r < kRItems; ++r) {
            const int64_t i = base + r * kBlock + threadIdx.x;
            if (i < n) atomicAdd(&h[w][(key[i] >> shift) & (RB - 1u)], 1u);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < RB; d += kBlock) {
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) c += h[k][d];
        hist[(int64_t)blockIdx.x * RB + d] = (int32_t)c;  // block-major: one coalesced row
    }
}

// The bucketed sort's MSD histogram (top 8 bits of the device-side key width) binning x, y on
// the fly (grid_key): the MSD pass never reads a key array, so bin_kernel's pass is skipped.
__global__ __launch_bounds__(kBlock) void msd_upsweep_xy_kernel(const double* __restrict__ x,
                                                                const double* __restrict__ y,
                                                                int64_t n,
                                                                const GridParams* __restrict__ gp,
                                                                const int32_t* __restrict__ bits_p,
                                                                int32_t* __restrict__ hist) {
    constexpr int RB = 256;
    const int b = *bits_p;
    const int shift = b > 8 ? b - 8 : 0;
    const GridParams g = *gp;
    __shared__ uint32_t h[kWaves][RB];
    const int w = threadIdx.x >> 6;
    for (int d = threadIdx.x; d < kWaves * RB; d += kBlock) (&h[0][0])[d] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kRTile;
    double a[kRItems], c[kRItems];
#pragma unroll
    for (int r = 0; r < kRItems; ++r) {  // every load in flight together
        const int64_t i = base + r * kBlock + threadIdx.x;
        a[r] = i < n ? x[i] : 0.0;
        c[r] = i < n ? y[i] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < kRItems; ++r) {
        const int64_t i = base + r * kBlock + threadIdx.x;
        if (i < n)
            atomicAdd(&h[w][(grid_key(a[r], c[r], g.xmin2, g.ymin2, g.invx, g.invy, g.nx, g.ny,
                                      g.ntx) >> shift) & (RB - 1u)], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < RB; d += kBlock) {
        uint32_t t = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) t += h[k][d];
        hist[(int64_t)blockIdx.x * RB + d] = (int32_t)t;  // block-major: one coalesced row
    }
}

// Global offset of every (radix tile, digit) from the block-major count table, in one launch:
// off[b][d] = sum over digits d' < d of all tiles' counts + sum over tiles b' < b of digit d.
// kOffBlocks workgroups of 1024 threads, RB digits x (1024 / RB) row groups: each sums its
// rows of the table (coalesced rows) and publishes the per-digit aggregates; every workgroup
// then reads all aggregates (the grid is far smaller than the GPU, so every workgroup is
// resident and the wait always ends; a bounded spin flags state[0] instead of hanging),
// derives the digit bases and its rows' running offsets, and writes them row by row.  A
// digit-major table instead scattered each tile's counts over RB lines on the upsweep's
// writes and the downsweep's reads (8x amplification).
constexpr int kOffBlocks = 64;  // workgroups
constexpr int kOffThreads = 1024;
constexpr int kOffRows = 24;    // rows per thread held in registers (more: a second round)

template <int W>
__global__ __launch_bounds__(kOffThreads) void radix_offsets_kernel(
    const int32_t* __restrict__ cnt, int64_t nb, int32_t* __restrict__ off,
    uint64_t* __restrict__ state, uint32_t epoch, const int32_t* __restrict__ bits_p,
    int shift) {
    constexpr int RB = 1 << W, G = kOffThreads / RB;
    if (shift >= 0 && shift >= *bits_p) return;  // (shift < 0: the bucketed sort's MSD pass)
    __shared__ int gsum[G][RB], gtot[G][RB], gbef[G][RB];
    __shared__ int wsum[RB / 64];
    const int d = threadIdx.x % RB, g = threadIdx.x / RB;
    const int64_t per = (nb + kOffBlocks - 1) / kOffBlocks;
    const int64_t b0 = blockIdx.x * per, b1 = b0 + per < nb ? b0 + per : nb;
    const int64_t gper = (per + G - 1) / G;
    const int64_t r0 = b0 + g * gper, r1 = r0 + gper < b1 ? r0 + gper : b1;
    // phase 1: this group's rows of digit d (all loads in flight together)
    int agg = 0;
    for (int64_t rb = r0; rb < r1; rb += kOffRows) {
        int v[kOffRows];
#pragma unroll
        for (int k = 0; k < kOffRows; ++k) v[k] = rb + k < r1 ? cnt[(rb + k) * RB + d] : 0;
#pragma unroll
        for (int k = 0; k < kOffRows; ++k) agg += v[k];
    }
    gsum[g][d] = agg;
    __syncthreads();
    uint64_t* status = state + 1;
    if (g == 0) {
        int a = 0;
#pragma unroll
        for (int q = 0; q < G; ++q) a += gsum[q][d];
        __hip_atomic_store(status + blockIdx.x * RB + d, scan_status(epoch, kStIncl, a),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // phase 2: every workgroup's aggregate of digit d (group g reads its share of them)
    int total = 0, before = 0;
    constexpr int kPerG = kOffBlocks / G;
    const auto ready = [&](uint64_t v) {
        return (uint32_t)(v >> 34) == epoch && ((v >> 32) & 3u) != 0;
    };
    uint64_t sv[kPerG];
#pragma unroll
    for (int q = 0; q < kPerG; ++q)  // all in flight at once; re-polled only if not yet set
        sv[q] = __hip_atomic_load(status + (g * kPerG + q) * RB + d, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int q = 0; q < kPerG; ++q) {
        const int k = g * kPerG + q;
        uint64_t v = sv[q];
        for (int spin = 0; !ready(v); ++spin) {
            if (spin == (1 << 22)) {  // watchdog: never reached while the grid is resident
                __hip_atomic_fetch_or(state, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v = scan_status(epoch, kStIncl, 0);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            v = __hip_atomic_load(status + k * RB + d, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        }
        total += (int32_t)(uint32_t)v;
        before += k < (int)blockIdx.x ? (int32_t)(uint32_t)v : 0;
    }
    gtot[g][d] = total;
    gbef[g][d] = before;
    __syncthreads();
    if (g == 0) {  // digit base: exclusive scan of the digit totals over the RB digits
        int t = 0, b = 0;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            t += gtot[q][d];
            b += gbef[q][d];
        }
        const int incl = wave_incl_scan(t);
        if ((d & 63) == 63) wsum[d >> 6] = incl;
        gtot[0][d] = incl - t + b;  // (reused: this workgroup's offset of digit d, partial)
    }
    __syncthreads();
    if (g == 0) {
        int r = gtot[0][d];
        for (int q = 0; q < (d >> 6); ++q) r += wsum[q];
        gtot[0][d] = r;
    }
    __syncthreads();
    // phase 3: this group's rows, after the earlier groups' rows of this workgroup
    int run = gtot[0][d];
    for (int q = 0; q < g; ++q) run += gsum[q][d];
    for (int64_t rb = r0; rb < r1; rb += kOffRows) {
        int v[kOffRows];
#pragma unroll
        for (int k = 0; k < kOffRows; ++k) v[k] = rb + k < r1 ? cnt[(rb + k) * RB + d] : 0;
#pragma unroll
        for (int k = 0; k < kOffRows; ++k) {
            if (rb + k < r1) off[(rb + k) * RB + d] = run;
            run += v[k];
        }
    }
}

// Downsweep: wave w ranks the contiguous quarter [w*512, (w+1)*512) of the 2048-key tile in
// 8 rounds of 64 keys (coalesced), so (wave, round, lane) order IS tile order and per-wave
// running digit counters give stable ranks: per round, lanes with equal digits are matched by W
// ballots, the lowest such lane (the leader) bumps the wave's counter for that digit, and each
// lane's rank = counter before the bump (read from its leader) + its rank among the matches.
// Then per digit a 4-wave prefix and a block scan of the digit totals place every key in LDS
// (tile sorted by digit), and each digit run is written coalesced to its global offset.
// The last sorting pass (shift + W >= the key width) writes the final buffers (key_fin,
// val_fin) and the inverse permutation; passes after it return at once.
template <int W>
struct DownsweepSmem {
    static constexpr int RB = 1 << W;
    uint16_t cnt[kWaves][RB];  // per-wave digit counters -> wave offsets within a digit
    uint32_t keys[kRTile];
    int32_t vals[kRTile];
    int32_t tile_start[RB + 1];
    int32_t gofs[RB];
    int32_t wsum[kWaves];
};

template <int W>
__global__ __launch_bounds__(kBlock) void radix_downsweep_kernel(
    const uint32_t* __restrict__ key, const int32_t* __restrict__ val,
    uint32_t* __restrict__ key_next, int32_t* __restrict__ val_next,
    uint32_t* __restrict__ key_fin, int32_t* __restrict__ val_fin, int64_t n, int shift,
    const int32_t* __restrict__ bits_p, int64_t nblocks,
    const int32_t* __restrict__ hist_off, int32_t* __restrict__ inv) {
    constexpr int RB = 1 << W;
    constexpr int DPT = RB > kBlock ? RB / kBlock : 1;  // digits per thread in the block scan
    __shared__ DownsweepSmem<W> sm;
    const int t = threadIdx.x, w = t >> 6, lane = lane_id();
    const int64_t tb = sort_tile();
    const int64_t base = tb * kRTile;
    const int tile_n = (int)((n - base) < kRTile ? (n - base) : kRTile);
    const int bits = *bits_p;
    if (bits == 0 && shift == 0) {  // nothing to sort (no grid key bits): the final copy
        for (int j = t; j < tile_n; j += kBlock) {
            const int32_t v = val ? val[base + j] : (int32_t)(base + j);
            key_fin[base + j] = key[base + j];
            val_fin[base + j] = v;
            if (inv) inv[v] = (int32_t)(base + j);
        }
        return;
    }
    if (shift >= bits) return;  // an earlier pass was the last
    const bool last = shift + W >= bits;
    uint32_t* __restrict__ key_out = last ? key_fin : key_next;
    int32_t* __restrict__ val_out = last ? val_fin : val_next;
    for (int k = t; k < kWaves * RB; k += kBlock) (&sm.cnt[0][0])[k] = 0;
    __syncthreads();

    uint32_t k_r[kRItems];
    int32_t v_r[kRItems];
    uint32_t dr[kRItems];  // digit | (rank within the wave's digit run << 10); ~0u invalid
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int64_t wbase = base + (int64_t)w * (kRTile / kWaves);
#pragma unroll
    for (int r = 0; r < kRItems; ++r) {
        const int64_t i = wbase + r * 64 + lane;
        const bool valid = i < base + tile_n;
        const uint32_t k = valid ? key[i] : kSentinelKey;
        const int32_t v = valid ? (val ? val[i] : (int32_t)i) : 0;  // val null: the identity
        const uint32_t d = (k >> shift) & (RB - 1u);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < W; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const int leader = peers ? __builtin_ctzll(peers) : 0;
        int old = 0;
        if (valid && lane == leader) {
            old = sm.cnt[w][d];
            sm.cnt[w][d] = old + __popcll(peers);
        }
        old = __shfl(old, leader, 64);
        k_r[r] = k;
        v_r[r] = v;
        dr[r] = valid ? (d | ((uint32_t)(old + __popcll(peers & lt_mask)) << 10)) : 0xFFFFFFFFu;
    }
    __syncthreads();
    {  // digits t*DPT .. t*DPT+DPT-1: wave offsets (prefix over the 4 waves), tile totals
        int tot[DPT];
        int mine = 0;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const int dd = t * DPT + j;
            int running = 0;
            if (dd < RB) {
#pragma unroll
                for (int k = 0; k < kWaves; ++k) {
                    const int c = sm.cnt[k][dd];
                    sm.cnt[k][dd] = running;
                    running += c;
                }
            }
            tot[j] = running;
            mine += running;
        }
        const int incl = wave_incl_scan(mine);  // block exclusive scan of the threads' totals
        if (lane == 63) sm.wsum[w] = incl;
        __syncthreads();
        int woff = 0;
        for (int q = 0; q < w; ++q) woff += sm.wsum[q];
        int at = woff + incl - mine;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const int dd = t * DPT + j;
            if (dd < RB) {
                sm.tile_start[dd] = at;
                sm.gofs[dd] = hist_off[tb * RB + dd];  // block-major row
            }
            at += tot[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRItems; ++r) {
        if (dr[r] != 0xFFFFFFFFu) {
            const uint32_t d = dr[r] & 1023u;
            const int lpos = sm.tile_start[d] + sm.cnt[w][d] + (int)(dr[r] >> 10);
            sm.keys[lpos] = k_r[r];
            sm.vals[lpos] = v_r[r];
        }
    }
    __syncthreads();
    for (int j = t; j < tile_n; j += kBlock) {
        const uint32_t k = sm.keys[j];
        const uint32_t d = (k >> shift) & (RB - 1u);
        const int64_t g = (int64_t)sm.gofs[d] + (j - sm.tile_start[d]);
        const int32_t v = sm.vals[j];
        key_out[g] = k;
        val_out[g] = v;
        if (last && inv) inv[v] = (int32_t)g;
    }
}

// ------------------------------- bucketed radix sort -------------------------------------
// For fits whose arrays outgrow the Infinity Cache (DESIGN.md §3 "bucketed sort"): the plain LSD
// sort's last pass and the coordinate scatter write to random places over the whole n-sized
// targets, and out of the 256 MB MALL every such partial-line write costs a line read and a line
// write of HBM.  Here the sort starts with ONE MSD pass on the top 8 key bits (tile-row bands):
// every point is moved, with its coordinates, into its band's segment of a padded array (each
// segment starts on a 2048-key tile, pads hold the sentinel key), and then the low bits are
// sorted by LSD passes that stay inside each segment (per-segment digit offsets).  So every
// later random write or read (the last pass's inverse, the coordinate scatter, the label
// gather) lands inside one band's segment: a few MB to ~100 MB, cache-resident while the
// launch sweeps the segments in order.

// Segment tables after the MSD pass (one workgroup of 256 threads = the 256 top digits):
// from the dense digit offsets of tile 0 (= the digit bases) the bucket sizes, their padded
// bases, the per-digit shift padded - dense, the segment tile ranges and the low key width.
//   seg layout (int32): [0..257] first padded tile of segment d (256: the all-pad tail; 257:
//   the end), [258..514] padded base, [515..771] dense base, [772..1028] count, [1029] low bits
constexpr int kSegTile = 0, kSegPBase = 258, kSegDBase = 515, kSegCnt = 772, kSegLBits = 1029;
constexpr int kSegInts = 1032;

__global__ __launch_bounds__(256) void bucket_table_kernel(const int32_t* __restrict__ hist_off,
                                                           int64_t n, int64_t np_max,
                                                           const int32_t* __restrict__ bits_p,
                                                           int32_t* __restrict__ seg,
                                                           int32_t* __restrict__ pshift) {
    __shared__ int ws[4];
    const int d = threadIdx.x, lane = lane_id(), w = d >> 6;
    const int bits = *bits_p;
    const int32_t db = hist_off[d];  // tile 0's offsets are the digit bases
    __shared__ int32_t dbs[257];
    dbs[d] = db;
    if (d == 0) dbs[256] = (int32_t)n;
    __syncthreads();
    const int32_t cnt = dbs[d + 1] - db;
    const int32_t pc = (cnt + kRTile - 1) / kRTile * kRTile;
    const int incl = wave_incl_scan(pc);
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    int before = 0;
    for (int k = 0; k < w; ++k) before += ws[k];
    const int32_t pb = before + incl - pc;
    seg[kSegTile + d] = pb / kRTile;
    seg[kSegPBase + d] = pb;
    seg[kSegDBase + d] = db;
    seg[kSegCnt + d] = cnt;
    pshift[d] = pb - db;
    if (d == 255) {  // the all-pad tail up to np_max: a segment of no real keys
        const int32_t used = pb + pc;
        seg[kSegTile + 256] = used / kRTile;
        seg[kSegPBase + 256] = used;
        seg[kSegDBase + 256] = (int32_t)n;
        seg[kSegCnt + 256] = 0;
        seg[kSegTile + 257] = (int32_t)(np_max / kRTile);
        seg[kSegLBits] = bits > 8 ? bits - 8 : 0;
    }
}

// The pads: every padded slot no real key lands on gets the sentinel key.
// Blocks 0..255: the pads after segment d's keys (< 2048 each); blocks 256.. share the tail after
// the last segment (up to 256 tiles of 2048 keys: one block alone took ~29 us of every fit).
constexpr int kPadTailBlocks = 64;
__device__ __forceinline__ void bucket_pad_body(const int32_t* __restrict__ seg, int64_t np_max,
                                                uint32_t* __restrict__ key) {
    const int d = blockIdx.x < 256 ? (int)blockIdx.x : 256;
    const int64_t a = (int64_t)seg[kSegPBase + d] + seg[kSegCnt + d];
    const int64_t b = d < 256 ? (int64_t)seg[kSegPBase + d + 1] : np_max;
    const int part = (int)blockIdx.x - d, parts = d < 256 ? 1 : kPadTailBlocks;
    for (int64_t j = a + (int64_t)part * kBlock + threadIdx.x; j < b; j += (int64_t)parts * kBlock)
        key[j] = kSentinelKey;
}

// Per padded tile: (padded base - dense base of its segment, end of its real keys).
__device__ __forceinline__ void bucket_tseg_body(const int32_t* __restrict__ seg, int64_t t,
                                                 int64_t ntiles, int2* __restrict__ tseg) {
    if (t >= ntiles) return;
    int lo = 0, hi = 257;  // segment s with seg[s] <= t < seg[s + 1] (tail: s = 256)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (seg[kSegTile + mid] <= t) lo = mid; else hi = mid;
    }
    tseg[t] = make_int2(seg[kSegPBase + lo] - seg[kSegDBase + lo],
                        seg[kSegPBase + lo] + seg[kSegCnt + lo]);
}

// bucket_pad's blocks, then the tile table's (one launch: both read the segment table only)
__global__ __launch_bounds__(kBlock) void bucket_pad_tseg_kernel(const int32_t* __restrict__ seg,
                                                                 int64_t np_max,
                                                                 uint32_t* __restrict__ key,
                                                                 int64_t ntiles,
                                                                 int2* __restrict__ tseg) {
    if (blockIdx.x < 256 + kPadTailBlocks) {
        bucket_pad_body(seg, np_max, key);
        return;
    }
    bucket_tseg_body(seg, (int64_t)(blockIdx.x - 256 - kPadTailBlocks) * kBlock + threadIdx.x,
                     ntiles, tseg);
}

// Per-segment digit offsets for an LSD pass over the padded array: one workgroup per segment
// (257: the tail's pads too), RB digits x G row groups; off[t][d] = padded base of t's segment
// + the segment's keys of smaller digits + digit d's keys in the segment's earlier tiles.
template <int W>
__global__ __launch_bounds__(1024) void bucket_offsets_kernel(const int32_t* __restrict__ cnt,
                                                              int32_t* __restrict__ off,
                                                              const int32_t* __restrict__ seg,
                                                              int shift) {
    constexpr int RB = 1 << W, G = 1024 / RB;
    if (shift >= seg[kSegLBits]) return;
    __shared__ int gsum[G][RB];
    __shared__ int dex[RB];
    __shared__ int wsum[(RB + 63) / 64];
    const int s = blockIdx.x;
    const int64_t t0 = seg[kSegTile + s], t1 = seg[kSegTile + s + 1];
    const int d = threadIdx.x % RB, g = threadIdx.x / RB;
    const int64_t per = (t1 - t0 + G - 1) / G;
    const int64_t r0 = t0 + g * per < t1 ? t0 + g * per : t1;
    const int64_t r1 = r0 + per < t1 ? r0 + per : t1;
    // the counts kOffBatch tiles at a time (their loads in flight together: a segment of
    // config 5's share spans ~240 tiles, the tail segment up to 256)
    constexpr int kOffBatch = 8;
    int agg = 0;
    int64_t r = r0;
    for (; r + kOffBatch <= r1; r += kOffBatch) {
        int v[kOffBatch];
#pragma unroll
        for (int u = 0; u < kOffBatch; ++u) v[u] = cnt[(r + u) * RB + d];
#pragma unroll
        for (int u = 0; u < kOffBatch; ++u) agg += v[u];
    }
    for (; r < r1; ++r) agg += cnt[r * RB + d];
    gsum[g][d] = agg;
    __syncthreads();
    if (g == 0) {  // the segment's digit totals, exclusive scan over the digits
        int tot = 0;
#pragma unroll
        for (int q = 0; q < G; ++q) tot += gsum[q][d];
        const int incl = wave_incl_scan(tot);
        if ((d & 63) == 63) wsum[d >> 6] = incl;
        dex[d] = incl - tot;
    }
    __syncthreads();
    int run = seg[kSegPBase + s] + dex[d];
    for (int q = 0; q < (d >> 6); ++q) run += wsum[q];
    for (int q = 0; q < g; ++q) run += gsum[q][d];
    for (r = r0; r + kOffBatch <= r1; r += kOffBatch) {
        int v[kOffBatch];
#pragma unroll
        for (int u = 0; u < kOffBatch; ++u) v[u] = cnt[(r + u) * RB + d];
#pragma unroll
        for (int u = 0; u < kOffBatch; ++u) {
            off[(r + u) * RB + d] = run;
            run += v[u];
        }
    }
    for (; r < r1; ++r) {
        const int c = cnt[r * RB + d];
        off[r * RB + d] = run;
        run += c;
    }
}

// The MSD pass: radix_downsweep_kernel's ranking (one 2048-key tile per workgroup, per-wave
// match-any ballots, the tile sorted in LDS) on the top 8 bits (shift = bits - 8 from the
// device); keys and records (x, y, input index, zone) written by digit run to the digit's
// padded segment (pshift[d]), pos[i] = the padded place.  The records are staged in LDS a
// quarter of the tile at a time (kMsdParts): each wave store then covers a few digit runs
// instead of 64 scattered 32-B records (0.186 -> 0.136 ms per 10^7 points; the whole tile
// staged at once: 0.183, its 64 KB of LDS leaving 2 workgroups per CU; eighths 0.147).
struct BucketExtra {
    const double* x;
    const double* y;
    double4* rec_out;  // (x, y, input index bits, zone | shared << 8) per padded place
    int32_t* pos;
    const uint8_t* zone;  // slab fits: zone per input point (else nullptr)
    const uint8_t* shm;   // lean slab fits: 1 for the listed shared points (or nullptr)
    const int32_t* pshift;
    const GridParams* gp;  // key == nullptr: bin x, y here (grid_key)
};

constexpr int kMsdParts = 4;
// 25.6 KB (the input index held as its offset in the tile: 29.7 KB with 32-bit indices, 0.135
// -> 0.129 ms per 10^7 points)
template <int W>
struct MsdSmem {
    static constexpr int RB = 1 << W;
    uint16_t cnt[kWaves][RB];  // per-wave digit counters -> wave offsets within a digit
    uint32_t keys[kRTile];
    uint16_t vals[kRTile];  // the input index - the tile's base
    int32_t tile_start[RB + 1];
    int32_t gofs[RB];
    int32_t wsum[kWaves];
    double2 xy[kRTile / kMsdParts];  // one part's coordinates in sorted order
    uint16_t zn[kRTile / kMsdParts];  // and zones
};
template <int W>
__global__ __launch_bounds__(kBlock) void bucket_msd_kernel(const uint32_t* __restrict__ key,
                                                            uint32_t* __restrict__ key_out,
                                                            int64_t n,
                                                            const int32_t* __restrict__ bits_p,
                                                            const int32_t* __restrict__ hist_off,
                                                            BucketExtra ex) {
    constexpr int RB = 1 << W;
    constexpr int DPT = RB > kBlock ? RB / kBlock : 1;
    __shared__ MsdSmem<W> sm;
    const int t = threadIdx.x, w = t >> 6, lane = lane_id();
    const int64_t tb = sort_tile();
    const int64_t base = tb * kRTile;
    const int tile_n = (int)((n - base) < kRTile ? (n - base) : kRTile);
    const int bits = *bits_p;
    const int shift = bits > 8 ? bits - 8 : 0;
    for (int k = t; k < kWaves * RB; k += kBlock) (&sm.cnt[0][0])[k] = 0;
    __syncthreads();

    // per item: the key, its coordinates, (digit | rank in the wave's digit << 10); the input
    // index is rematerialised, not held in registers (96 VGPRs: 5 waves per SIMD)
    uint32_t k_r[kRItems];
    uint32_t dr[kRItems];
    double2 c_r[kRItems];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int64_t wbase = base + (int64_t)w * (kRTile / kWaves);
#pragma unroll
    for (int r = 0; r < kRItems; ++r) {
        const int64_t i = wbase + r * 64 + lane;
        const bool valid = i < base + tile_n;
        uint32_t k = kSentinelKey;
        c_r[r] = valid ? make_double2(ex.x[i], ex.y[i]) : make_double2(0.0, 0.0);
        if (valid)
            k = key ? key[i]
                    : grid_key(c_r[r].x, c_r[r].y, ex.gp->xmin2, ex.gp->ymin2, ex.gp->invx,
                               ex.gp->invy, ex.gp->nx, ex.gp->ny, ex.gp->ntx);
        const uint32_t d = (k >> shift) & (RB - 1u);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < W; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const int leader = peers ? __builtin_ctzll(peers) : 0;
        int old = 0;
        if (valid && lane == leader) {
            old = sm.cnt[w][d];
            sm.cnt[w][d] = old + __popcll(peers);
        }
        old = __shfl(old, leader, 64);
        k_r[r] = k;
        dr[r] = valid ? (d | ((uint32_t)(old + __popcll(peers & lt_mask)) << 10)) : 0xFFFFFFFFu;
    }
    __syncthreads();
    {
        int tot[DPT];
        int mine = 0;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const int dd = t * DPT + j;
            int running = 0;
            if (dd < RB) {
#pragma unroll
                for (int k = 0; k < kWaves; ++k) {
                    const int c = sm.cnt[k][dd];
                    sm.cnt[k][dd] = running;
                    running += c;
                }
            }
            tot[j] = running;
            mine += running;
        }
        const int incl = wave_incl_scan(mine);
        if (lane == 63) sm.wsum[w] = incl;
        __syncthreads();
        int woff = 0;
        for (int q = 0; q < w; ++q) woff += sm.wsum[q];
        int at = woff + incl - mine;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const int dd = t * DPT + j;
            if (dd < RB) {
                sm.tile_start[dd] = at;
                sm.gofs[dd] = hist_off[tb * RB + dd] + ex.pshift[dd];
            }
            at += tot[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRItems; ++r) {
        if (dr[r] != 0xFFFFFFFFu) {
            const uint32_t d = dr[r] & 1023u;
            const int within = sm.cnt[w][d] + (int)(dr[r] >> 10);
            const int lpos = sm.tile_start[d] + within;
            const int32_t i = (int32_t)(wbase + r * 64 + lane);
            sm.keys[lpos] = k_r[r];
            sm.vals[lpos] = (uint16_t)(i - base);
            ex.pos[i] = sm.gofs[d] + within;  // the place
        }
    }
    __syncthreads();
    // keys and records by digit run, a part of the tile at a time
    constexpr int PS = kRTile / kMsdParts;
    for (int p = 0; p < kMsdParts; ++p) {
        if (p) __syncthreads();
#pragma unroll
        for (int r = 0; r < kRItems; ++r) {
            if (dr[r] == 0xFFFFFFFFu) continue;
            const uint32_t d = dr[r] & 1023u;
            const int lpos = sm.tile_start[d] + sm.cnt[w][d] + (int)(dr[r] >> 10) - p * PS;
            if (lpos >= 0 && lpos < PS) {
                const int64_t i = wbase + r * 64 + lane;
                sm.xy[lpos] = c_r[r];
                sm.zn[lpos] =
                    ex.zone ? (uint16_t)(ex.zone[i] | ((ex.shm && ex.shm[i]) ? 256u : 0u)) : 0;
            }
        }
        __syncthreads();
        const int je = tile_n < (p + 1) * PS ? tile_n : (p + 1) * PS;
        for (int j = p * PS + t; j < je; j += kBlock) {
            const uint32_t k = sm.keys[j];
            const uint32_t d = (k >> shift) & (RB - 1u);
            const int64_t g = (int64_t)sm.gofs[d] + (j - sm.tile_start[d]);
            key_out[g] = k;
            const double2 c = sm.xy[j - p * PS];
            const long long vi = base + sm.vals[j];
            ex.rec_out[g] = make_double4(c.x, c.y, __longlong_as_double(vi),
                                         __longlong_as_double((long long)sm.zn[j - p * PS]));
        }
    }
}

// The LSD passes inside the segments (bits = the low width, seg[kSegLBits]): the same ranking,
// payload = padded place (identity on the first pass); the last pass writes the dense order,
// key_fin and val_fin (slot -> padded place), pads dropped.  16-bit digit counters, and the
// tile's digit offsets written over them once the tile is ranked into LDS: 22.5 KB for 9-bit
// digits instead of 28.7, and at most 72 VGPRs, so 7 workgroups per CU instead of 5 (0.104 ->
// 0.090 ms per 10^7 points for the two 9-bit passes, 1.77 -> 1.55 at config 5's share).
// Not kept: two tiles per workgroup ranked together (digit runs twice as long): 0.104 -> 0.144.
template <int W>
struct LsdSmem {
    static constexpr int RB = 1 << W;
    union {
        uint16_t cnt[kWaves][RB];  // per-wave digit counters -> wave offsets within a digit
        int32_t gofs[RB];          // then the tile's digit offsets in the output
    } u;
    uint32_t keys[kRTile];
    int32_t vals[kRTile];
    int32_t tile_start[RB + 1];
    int32_t wsum[kWaves];
};

template <int W>
__global__ __launch_bounds__(kBlock, 7) void bucket_lsd_kernel(
    const uint32_t* __restrict__ key, const int32_t* __restrict__ val,
    uint32_t* __restrict__ key_out, int32_t* __restrict__ val_out, uint32_t* __restrict__ key_fin,
    int32_t* __restrict__ val_fin, int64_t n, int shift, const int32_t* __restrict__ bits_p,
    const int32_t* __restrict__ hist_off, const int2* __restrict__ tseg) {
    constexpr int RB = 1 << W;
    constexpr int DPT = RB > kBlock ? RB / kBlock : 1;
    __shared__ LsdSmem<W> sm;
    const int t = threadIdx.x, w = t >> 6, lane = lane_id();
    const int64_t tb = sort_tile();
    const int64_t base = tb * kRTile;
    const int tile_n = (int)((n - base) < kRTile ? (n - base) : kRTile);
    const int bits = *bits_p;
    if (bits == 0) {  // the MSD pass sorted everything: the dense copy (first pass only)
        if (shift != 0) return;
        const int2 ts = tseg[tb];
        for (int j = t; j < tile_n; j += kBlock) {
            const int64_t gp = base + j;
            if (gp >= ts.y) continue;
            key_fin[gp - ts.x] = key[gp];
            val_fin[gp - ts.x] = val ? val[gp] : (int32_t)gp;
        }
        return;
    }
    if (shift >= bits) return;
    const bool last = shift + W >= bits;
    for (int k = t; k < kWaves * RB; k += kBlock) (&sm.u.cnt[0][0])[k] = 0;
    __syncthreads();

    uint32_t k_r[kRItems];
    int32_t v_r[kRItems];
    uint32_t dr[kRItems];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int64_t wbase = base + (int64_t)w * (kRTile / kWaves);
#pragma unroll
    for (int r = 0; r < kRItems; ++r) {
        const int64_t i = wbase + r * 64 + lane;
        const bool valid = i < base + tile_n;
        const uint32_t k = valid ? key[i] : kSentinelKey;
        const int32_t v = valid ? (val ? val[i] : (int32_t)i) : 0;
        const uint32_t d = (k >> shift) & (RB - 1u);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < W; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const int leader = peers ? __builtin_ctzll(peers) : 0;
        int old = 0;
        if (valid && lane == leader) {
            old = sm.u.cnt[w][d];
            sm.u.cnt[w][d] = (uint16_t)(old + __popcll(peers));
        }
        old = __shfl(old, leader, 64);
        k_r[r] = k;
        v_r[r] = v;
        dr[r] = valid ? (d | ((uint32_t)(old + __popcll(peers & lt_mask)) << 10)) : 0xFFFFFFFFu;
    }
    __syncthreads();
    int32_t go[DPT];
    {
        int tot[DPT];
        int mine = 0;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const int dd = t * DPT + j;
            int running = 0;
            if (dd < RB) {
                go[j] = hist_off[tb * RB + dd];
#pragma unroll
                for (int k = 0; k < kWaves; ++k) {
                    const int c = sm.u.cnt[k][dd];
                    sm.u.cnt[k][dd] = (uint16_t)running;
                    running += c;
                }
            }
            tot[j] = running;
            mine += running;
        }
        const int incl = wave_incl_scan(mine);
        if (lane == 63) sm.wsum[w] = incl;
        __syncthreads();
        int woff = 0;
        for (int q = 0; q < w; ++q) woff += sm.wsum[q];
        int at = woff + incl - mine;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const int dd = t * DPT + j;
            if (dd < RB) sm.tile_start[dd] = at;
            at += tot[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRItems; ++r) {
        if (dr[r] != 0xFFFFFFFFu) {
            const uint32_t d = dr[r] & 1023u;
            const int lpos = sm.tile_start[d] + sm.u.cnt[w][d] + (int)(dr[r] >> 10);
            sm.keys[lpos] = k_r[r];
            sm.vals[lpos] = v_r[r];
        }
    }
    __syncthreads();  // the counters are done with: the digit offsets over them
#pragma unroll
    for (int j = 0; j < DPT; ++j)
        if (t * DPT + j < RB) sm.u.gofs[t * DPT + j] = go[j];
    __syncthreads();
    const int2 ts = last ? tseg[tb] : make_int2(0, 0);
    for (int j = t; j < tile_n; j += kBlock) {
        const uint32_t k = sm.keys[j];
        const uint32_t d = (k >> shift) & (RB - 1u);
        const int64_t g = (int64_t)sm.u.gofs[d] + (j - sm.tile_start[d]);
        const int32_t v = sm.vals[j];
        if (last) {
            if (g >= ts.y) continue;  // a pad (pads sort after the segment's keys)
            key_fin[g - ts.x] = k;
            val_fin[g - ts.x] = v;
        } else {
            key_out[g] = k;
            val_out[g] = v;
        }
    }
}

// ------------------------------------ bbox -----------------------------------------------

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ __launch_bounds__(kBlock) void bbox_partial_kernel(const double* __restrict__ x,
                                                              const double* __restrict__ y,
                                                              int64_t n, double* partial) {
    __shared__ double sm[kWaves][5];
    double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY, cnt = 0;
    const auto take = [&](double a, double b) {
        if (__builtin_isfinite(a) && __builtin_isfinite(b)) {
            xmin = fmin(xmin, a);
            xmax = fmax(xmax, a);
            ymin = fmin(ymin, b);
            ymax = fmax(ymax, b);
            cnt += 1.0;
        }
    };
    const int64_t gt = (int64_t)blockIdx.x * kBlock + threadIdx.x, stride = (int64_t)gridDim.x * kBlock;
    if ((((uintptr_t)x | (uintptr_t)y) & 15u) == 0) {
        // 16-B loads, two pairs in flight per thread and trip (the plain form read 4.7 TB/s)
        const double2* x2 = reinterpret_cast<const double2*>(x);
        const double2* y2 = reinterpret_cast<const double2*>(y);
        const int64_t n2 = n >> 1;
        int64_t i = gt;
        for (; i + stride < n2; i += 2 * stride) {
            const double2 a0 = x2[i], b0 = y2[i], a1 = x2[i + stride], b1 = y2[i + stride];
            take(a0.x, b0.x);
            take(a0.y, b0.y);
            take(a1.x, b1.x);
            take(a1.y, b1.y);
        }
        if (i < n2) {
            const double2 a0 = x2[i], b0 = y2[i];
            take(a0.x, b0.x);
            take(a0.y, b0.y);
        }
        if ((n & 1) && gt == 0) take(x[n - 1], y[n - 1]);
    } else {
        for (int64_t i = gt; i < n; i += stride) take(x[i], y[i]);
    }
    xmin = wave_min(xmin);
    xmax = wave_max(xmax);
    ymin = wave_min(ymin);
    ymax = wave_max(ymax);
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) {
        sm[w][0] = xmin;
        sm[w][1] = xmax;
        sm[w][2] = ymin;
        sm[w][3] = ymax;
        sm[w][4] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kWaves; ++k) {
            sm[0][0] = fmin(sm[0][0], sm[k][0]);
            sm[0][1] = fmax(sm[0][1], sm[k][1]);
            sm[0][2] = fmin(sm[0][2], sm[k][2]);
            sm[0][3] = fmax(sm[0][3], sm[k][3]);
            sm[0][4] += sm[k][4];
        }
        for (int c = 0; c < 5; ++c) partial[blockIdx.x * 5 + c] = sm[0][c];
    }
}

}  // namespace

uint64_t* ScanState::prepare(hipStream_t s, int64_t ntiles) {
    void* old = buf.p;
    uint64_t* p = static_cast<uint64_t*>(buf.ensure((size_t)(ntiles + 1) * sizeof(uint64_t)));
    if (p != old || epoch == 0x3FFFFFFFu) {  // fresh memory or epoch wrap: clear, restart at 1
        DBSCAN_HIP_CHECK(hipMemsetAsync(p, 0, buf.bytes, s));
        epoch = 0;
    }
    ++epoch;
    return p;
}

void exclusive_scan(hipStream_t s, int mode, const void* in, int32_t* out, int64_t n,
                    int32_t* total_dev, ScanState& ss) {
    if (n <= 0) {
        if (total_dev) DBSCAN_HIP_CHECK(hipMemsetAsync(total_dev, 0, sizeof(int32_t), s));
        return;
    }
    if (mode == 0)
        scan_impl<0>(s, in, out, n, total_dev, ss);
    else if (mode == 1)
        scan_impl<1>(s, in, out, n, total_dev, ss);
    else
        scan_impl<2>(s, in, out, n, total_dev, ss);
}

void radix_sort_pairs(hipStream_t s, uint32_t*& key, int32_t*& val, uint32_t*& key2,
                      int32_t*& val2, uint32_t*& key3, int32_t*& val3, int64_t n,
                      const int32_t* bits_dev, DevBuf& hist, ScanState& scan, Profiler* prof,
                      int32_t* inv, bool iota) {
    if (n <= 0) return;
    bool first = true;
    const int64_t nb = (n + kRTile - 1) / kRTile;
    // per-tile digit counts (block-major) and the tiles' global digit offsets, for RB <= 512
    int32_t* h = static_cast<int32_t*>(hist.ensure((size_t)2 * nb * 512 * sizeof(int32_t)));
    int32_t* ho = h + nb * 512;
    // ping-pong A = (key, val) -> B = (key2, val2) -> A ...; the last sorting pass writes C
    uint32_t* kin = key;
    int32_t* vin = val;
    uint32_t* kpp = key2;
    int32_t* vpp = val2;
    const auto pass = [&](auto wtag, int shift) {
        constexpr int W = decltype(wtag)::value;
        // profile names per template instance (the digit widths run differently)
        const char* up = W == 8 ? "radix_upsweep<8>" : W == 9 ? "radix_upsweep<9>" : "radix_upsweep<7>";
        const char* of = W == 8 ? "radix_offsets<8>" : W == 9 ? "radix_offsets<9>" : "radix_offsets<7>";
        const char* dn = W == 8   ? "radix_downsweep<8>"
                         : W == 9 ? "radix_downsweep<9>"
                                  : "radix_downsweep<7>";
        {
            StageTimer st(prof, s, "sort_upsweep");
            klaunch(prof, up, radix_upsweep_kernel<W>, dim3((unsigned)nb),
                    dim3(kBlock), 0, s, kin, n, shift, bits_dev, nb, h);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        {
            StageTimer st(prof, s, "sort_scan");
            uint64_t* state = scan.prepare(s, (int64_t)kOffBlocks * 512);
            klaunch(prof, of, radix_offsets_kernel<W>, dim3(kOffBlocks),
                    dim3(kOffThreads), 0, s, (const int32_t*)h, nb, ho, state, scan.epoch,
                    bits_dev, shift);
        }
        {
            StageTimer st(prof, s, "sort_downsweep");
            klaunch(prof, dn, radix_downsweep_kernel<W>, dim3((unsigned)nb),
                    dim3(kBlock), 0, s, kin, (first && iota) ? (const int32_t*)nullptr : vin, kpp,
                    vpp, key3, val3, n, shift, bits_dev, nb, ho, inv);
            DBSCAN_HIP_CHECK(hipGetLastError());
        }
        first = false;
        std::swap(kin, kpp);
        std::swap(vin, vpp);
    };
    // the 9-bit digit last: the high key bits (tile rows) are the most concentrated digits,
    // so its 512 digit runs per tile stay long enough to write coalesced
    pass(std::integral_constant<int, 8>{}, 0);
    pass(std::integral_constant<int, 8>{}, 8);
    pass(std::integral_constant<int, 9>{}, 16);
    pass(std::integral_constant<int, 7>{}, 25);
    // the sorted pairs are in C whatever the key width
    std::swap(key, key3);
    std::swap(val, val3);
}

int64_t bucket_padded(int64_t n) { return ((n + kRTile - 1) / kRTile + 256) * kRTile; }

void bucket_sort(hipStream_t s, const double* x, const double* y, const uint32_t* key, int64_t n,
                 const int32_t* bits_dev, BucketSort& b, DevBuf& hist, ScanState& scan,
                 Profiler* prof, const uint8_t* zone, const uint8_t* shm, const GridParams* gp) {
    if (!key && !gp) throw ArgError{"bucket_sort: no keys and no grid"};
    if (n <= 0) return;
    const int64_t np = bucket_padded(n), ntp = np / kRTile, nb = (n + kRTile - 1) / kRTile;
    int32_t* h = static_cast<int32_t*>(hist.ensure((size_t)2 * ntp * 512 * sizeof(int32_t)));
    int32_t* ho = h + ntp * 512;
    uint32_t* ka = static_cast<uint32_t*>(b.ka.ensure(np * sizeof(uint32_t)));
    uint32_t* kb = static_cast<uint32_t*>(b.kb.ensure(np * sizeof(uint32_t)));
    int32_t* jb = static_cast<int32_t*>(b.jb.ensure(np * sizeof(int32_t)));
    uint32_t* kc = static_cast<uint32_t*>(b.kc.ensure(np * sizeof(uint32_t)));
    int32_t* jc = static_cast<int32_t*>(b.jc.ensure(np * sizeof(int32_t)));
    b.rec = static_cast<double4*>(b.recb.ensure(np * sizeof(double4)));
    b.pos = static_cast<int32_t*>(b.posb.ensure(n * sizeof(int32_t)));
    b.key_fin = static_cast<uint32_t*>(b.kf.ensure(n * sizeof(uint32_t)));
    b.slot_place = static_cast<int32_t*>(b.jf.ensure(n * sizeof(int32_t)));
    int32_t* tab = static_cast<int32_t*>(
        b.tab.ensure((kSegInts + 256) * sizeof(int32_t) + ntp * sizeof(int2)));
    int32_t* seg = tab;
    int32_t* pshift = tab + kSegInts;
    int2* tseg = reinterpret_cast<int2*>(tab + kSegInts + 256);
    b.np = np;
    {  // the MSD pass: top 8 bits, into padded segments, coordinates moved along
        StageTimer st(prof, s, "sort_msd");
        if (key)
            klaunch(prof, "radix_upsweep<8>", radix_upsweep_kernel<8>, dim3((unsigned)nb),
                    dim3(kBlock), 0, s, key, n, -1, bits_dev, nb, h);
        else  // (bins x, y itself: no bin_kernel pass)
            klaunch(prof, "msd_upsweep", msd_upsweep_xy_kernel, dim3((unsigned)nb), dim3(kBlock),
                    0, s, x, y, n, gp, bits_dev, h);
        uint64_t* state = scan.prepare(s, (int64_t)kOffBlocks * 512);
        klaunch(prof, "radix_offsets<8>", radix_offsets_kernel<8>, dim3(kOffBlocks),
                dim3(kOffThreads), 0, s, (const int32_t*)h, nb, ho, state, scan.epoch, bits_dev,
                -1);
        klaunch(prof, "bucket_table", bucket_table_kernel, dim3(1), dim3(256), 0, s,
                (const int32_t*)ho, n, np, bits_dev, seg, pshift);
        klaunch(prof, "bucket_pad", bucket_pad_tseg_kernel,
                dim3((unsigned)(256 + kPadTailBlocks + (ntp + kBlock - 1) / kBlock)), dim3(kBlock),
                0, s, (const int32_t*)seg, np, ka, ntp, tseg);

        const BucketExtra ex{x, y, b.rec, b.pos, zone, shm, pshift, gp};
        klaunch(prof, "bucket_msd", bucket_msd_kernel<8>, dim3((unsigned)nb), dim3(kBlock), 0, s,
                key, ka, n, bits_dev, (const int32_t*)ho, ex);

        DBSCAN_HIP_CHECK(hipGetLastError());
    }
    // LSD passes over the low bits inside the segments (payload: padded place)
    const int32_t* lbits = seg + kSegLBits;
    const uint32_t* kin = ka;
    const int32_t* vin = nullptr;  // the first pass generates the identity
    uint32_t* kout = kb;
    int32_t* vout = jb;
    const auto pass = [&](auto wtag, int shift) {
        constexpr int W = decltype(wtag)::value;
        StageTimer st(prof, s, "sort_bucket");
        const char* dn = W == 8 ? "bucket_lsd<8>" : "bucket_lsd<9>";
        klaunch(prof, W == 8 ? "radix_upsweep<8>" : "radix_upsweep<9>", radix_upsweep_kernel<W>,
                dim3((unsigned)ntp), dim3(kBlock), 0, s, (const uint32_t*)kin, np, shift, lbits,
                ntp, h);
        klaunch(prof, W == 8 ? "bucket_offsets<8>" : "bucket_offsets<9>",
                bucket_offsets_kernel<W>, dim3(257), dim3(1024), 0, s, (const int32_t*)h, ho,
                (const int32_t*)seg, shift);
        klaunch(prof, dn, bucket_lsd_kernel<W>, dim3((unsigned)ntp), dim3(kBlock), 0, s, kin, vin,
                kout, vout, b.key_fin, b.slot_place, np, shift, lbits, (const int32_t*)ho,
                (const int2*)tseg);
        DBSCAN_HIP_CHECK(hipGetLastError());
        kin = kout;
        vin = vout;
        kout = kout == kb ? kc : kb;
        vout = vout == jb ? jc : jb;
    };
    // 9 + 9 + 8 bits: the low width is <= 24 (32-bit keys minus the MSD pass's 8); keys of
    // <= 26 bits (low width <= 18) sort in two passes
    pass(std::integral_constant<int, 9>{}, 0);
    pass(std::integral_constant<int, 9>{}, 9);
    pass(std::integral_constant<int, 8>{}, 18);
}

int bbox_partials(hipStream_t s, const double* x, const double* y, int64_t n, DevBuf& tmp,
                  double** partial_out) {
    int nb = (int)((n + kBlock - 1) / kBlock);
    if (nb > 1024) nb = 1024;
    if (nb < 1) nb = 1;
    double* partial = static_cast<double*>(tmp.ensure((size_t)nb * 5 * sizeof(double)));
    hipLaunchKernelGGL(bbox_partial_kernel, dim3(nb), dim3(kBlock), 0, s, x, y, n, partial);
    DBSCAN_HIP_CHECK(hipGetLastError());
    *partial_out = partial;
    return nb;
}

void scan3(hipStream_t s, const int32_t* in, int64_t n, int64_t stride, int32_t* out,
           int32_t* t0, int32_t* t1, int32_t* t2) {
    if (n <= 0 || n > kTile) throw ArgError{"scan3: each array must hold 1..4096 values"};
    hipLaunchKernelGGL(scan3_kernel, dim3(3), dim3(kBlock), 0, s, in, n, stride, out,
                       Totals3{{t0, t1, t2}});
    DBSCAN_HIP_CHECK(hipGetLastError());
}


}  // namespace dbscan
