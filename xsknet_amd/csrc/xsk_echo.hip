// xsk_echo.hip — the product entry points of the gfx950 ICMP-echo transform: xsk_gpu_echo_dev() and
// xsk_gpu_echo_dev_opts() (one launch of the round kernel echo_kernel6, reference or wire mode), the
// workspace query, the kernel timer the bench reads, and the error plumbing of the C ABI
// (include/xsk_gpu.h).  Device code: xsk_echo_device.h.  Tuning variants live in the separate
// libxsknet_amd_tune.so (tune/), never in this library.
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

#include "xsk_echo_device.h"
#include "xsk_gpu_internal.h"
#include "xsk_hip_util.h"

using namespace xskgpu;

namespace {

// Fold the per-workgroup partials into the caller's stats_record-compatible counters: 1024 threads,
// thread t sums counter t % 4 over rows t/4, t/4 + 256, ... with 4 independent chains, then a tree.
// Only for counters in mapped host memory (device atomics are not an option there).
__global__ __launch_bounds__(1024) void fold_counters_kernel(const unsigned long long* partials, uint32_t nwg,
                                                            xsk_gpu_stats* st) {
    __shared__ unsigned long long s[1024];
    const uint32_t c = threadIdx.x & 3u;
    unsigned long long acc[4] = {0ull, 0ull, 0ull, 0ull};
    uint32_t w = threadIdx.x >> 2;
    for (; w + 768u < nwg; w += 1024u) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] += partials[(w + 256u * i) * 4u + c];
    }
    for (; w < nwg; w += 256u) acc[0] += partials[w * 4u + c];
    s[threadIdx.x] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    __syncthreads();
    for (uint32_t o = 512; o >= 4; o >>= 1) {
        if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x < 4) {
        unsigned long long* ctr = (unsigned long long*)&st->rx_packets;
        ctr[threadIdx.x] += s[threadIdx.x];
    }
}

thread_local const char* g_last_error = "ok";

constexpr uint32_t kSmallWG = 16;  // workgroups a small batch's sub-tiles may spread over

// ---- kernel timing (bench instrumentation) -------------------------------------------------------
// Events are created per device, lazily, on the device of the launch they bracket; a slot is claimed
// only once its start event has been recorded.
constexpr int kTimerCap = 4096;
constexpr int kMaxDev = 64;
struct TimerPool {
    hipEvent_t ev[kTimerCap][2];
};
struct Timer {
    bool on = false;
    int count = 0;              // claimed slots since enable
    int dev[kTimerCap];         // device of slot i; -1 when its end event failed to record
    TimerPool* pool[kMaxDev] = {};
};
Timer g_timer;
std::mutex g_timer_mu;

int timer_begin(int device, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_timer_mu);
    if (!g_timer.on || g_timer.count >= kTimerCap || device < 0 || device >= kMaxDev) return -1;
    TimerPool*& p = g_timer.pool[device];
    if (!p) {  // the current device is `device`: create its events here
        TimerPool* np = new (std::nothrow) TimerPool;
        if (!np) return -1;
        for (int i = 0; i < kTimerCap; ++i) {
            if (hipEventCreate(&np->ev[i][0]) != hipSuccess || hipEventCreate(&np->ev[i][1]) != hipSuccess) {
                delete np;  // (events leak on this rare path; timing is bench instrumentation)
                return -1;
            }
        }
        p = np;
    }
    const int slot = g_timer.count;
    if (hipEventRecord(p->ev[slot][0], s) != hipSuccess) return -1;
    g_timer.dev[slot] = device;
    g_timer.count++;
    return slot;
}

void timer_end(int slot, hipStream_t s) {
    if (slot < 0) return;
    std::lock_guard<std::mutex> lk(g_timer_mu);
    const int d = g_timer.dev[slot];
    if (d < 0 || hipEventRecord(g_timer.pool[d]->ev[slot][1], s) != hipSuccess) g_timer.dev[slot] = -1;
}

// Compute units per device, looked up once (the round kernel launches one workgroup per CU).
std::atomic<int> g_num_cu[kMaxDev];

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

int xsk_gpu__hip_fail(hipError_t e) {
    g_last_error = hipGetErrorName(e);
    return e == hipErrorOutOfMemory ? -ENOMEM : -EIO;
}

int xsk_gpu_abi_version(void) { return XSK_GPU_ABI_VERSION; }
#ifndef XSK_GPU_BUILD_ID
#error "XSK_GPU_BUILD_ID is set by the Makefile (hash of the kernel sources and flags)"
#endif
const char* xsk_gpu_build_id(void) { return XSK_GPU_BUILD_ID; }
const char* xsk_gpu_last_error(void) { return g_last_error; }

size_t xsk_gpu_workspace_size(int device, uint32_t n) {
    if (device < 0) return 0;
    // room for the partial rows of the round kernel's grid (<= one workgroup per CU), or of a small batch's
    // sub-tiles (<= kSmallWG workgroups)
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    uint32_t g = ntiles < kMaxCuBound ? ntiles : kMaxCuBound;
    if (g < kSmallWG) g = kSmallWG;
    return (size_t)g * 4 * sizeof(unsigned long long);
}

// Compute units of `device` (cached, race-free: concurrent first lookups store the same value).
uint32_t xsk_gpu__num_cu(int device) {
    if (device < 0 || device >= kMaxDev) return 0;
    int v = g_num_cu[device].load(std::memory_order_relaxed);
    if (v <= 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0) return 0;
        if (v > (int)kMaxCuBound) v = (int)kMaxCuBound;
        g_num_cu[device].store(v, std::memory_order_relaxed);
    }
    return (uint32_t)v;
}

// One transform launch (reference mode for opts == 0, wire mode otherwise).  Counters: device memory
// (hoststats == 0) -> every workgroup adds its four counters with device-scope atomics, one launch;
// mapped host memory (hoststats == 1, the zerocopy host context: d_stats is a slot the host zeroed for
// this call) -> a one-workgroup launch stores them itself, a larger grid writes per-workgroup partials
// that a one-workgroup fold launch adds.
static int echo_launch(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n, uint32_t opts,
                       uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, struct xsk_gpu_stats* d_stats,
                       void* d_workspace, void* stream, int hoststats, uint32_t tile, uint32_t grid_force = 0) {
    if (opts & ~XSK_GPU_OPT_ALL) return -EINVAL;
    if (n == 0) return 0;
    if (n > XSK_GPU_MAX_BATCH) return -EINVAL;
    if (!d_umem || !d_descs || ((uintptr_t)d_umem & 15u) || (umem_size & 15u) || ((uintptr_t)d_descs & 15u) ||
        ((uintptr_t)d_recs & 15u))
        return -EINVAL;
    if (d_stats && !d_workspace) return -EINVAL;
    if (umem_size >> 48) return -EINVAL;  // FrameMeta6 carries 48-bit UMEM offsets (both modes)
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    const uint32_t ncu = xsk_gpu__num_cu(device);
    if (!ncu) return xsk_gpu__hip_fail(hipErrorInvalidDevice);
    uint32_t grid = 0, tiles_per_wg = 0;
    // a small batch (the RX loop's) runs as sub-tiles, one per wave, instead of 64-frame tiles: over PCIe
    // (zerocopy host UMEM) one wave alone would stream its 64 frames with only its own loads in flight, and in
    // HBM a 64-frame tile per CU leaves the batch's latency to one wave
    const bool small = n <= (uint32_t)XSK_GPU_LOWLAT_MAX;
    uint32_t tl = kTile;
    if (small) {
        // sub-tiles of tl frames, one per wave, over up to kSmallWG workgroups of 16 waves: a device-resident
        // batch on every one of them (tl = ceil(n / 256), >= 4: tools/smallbatch.py measured 1024 x 1500 B in
        // 14.6 us over 16 workgroups against 44.1 us on one); a zerocopy batch with the caller's tile (about
        // 8 KiB of PCIe reads per wave, xsk_gpu__small_tile_w), 16 waves per workgroup
        tl = tile ? ((tile + 3u) & ~3u)
                  : ((n + kWaves6 * (grid_force ? grid_force : kSmallWG) - 1) /
                         (kWaves6 * (grid_force ? grid_force : kSmallWG)) + 3u) & ~3u;
        tl = tl < 4u ? 4u : (tl > (uint32_t)kTile ? (uint32_t)kTile : tl);
        const uint32_t nt = (n + tl - 1) / tl;
        tiles_per_wg = grid_force ? (nt + grid_force - 1) / grid_force : (uint32_t)kWaves6;
        grid = (nt + tiles_per_wg - 1) / tiles_per_wg;
    } else {
        echo6_geometry(n, grid_force ? grid_force : ncu, &grid, &tiles_per_wg);
    }
    const hipStream_t s = (hipStream_t)stream;
    EchoArgs args;
    args.umem = (uint8_t*)d_umem;
    args.umem_size = umem_size;
    args.descs = d_descs;
    args.n = n;
    args.verdicts = d_verdicts;
    args.recs = d_recs;
    args.partials = nullptr;
    args.opts = opts;
    args.tile_live = tl;
    bool fold = false;
    if (d_stats) {
        if (!hoststats) {
            args.stats_direct = (unsigned long long*)&d_stats->rx_packets;
        } else if (grid == 1) {
            args.stats_direct = (unsigned long long*)&d_stats->rx_packets;
            args.stats_plain = 1;
        } else {
            args.partials = (unsigned long long*)d_workspace;
            fold = true;
        }
    }
    // A batch of more than kMaxRounds rounds per workgroup runs as consecutive launches of about kPieceRounds rounds
    // each, over consecutive slices of its descriptors: every launch's last round scatters its windows while no
    // workgroup of that launch still reads, where a long share writes every round's windows into other
    // workgroups' reads (tools/split_bench.py, profiles/r04/split/: 8 M x 1500 B at 4 KiB, one launch 300.5 us per
    // M frames, launches of 1 M 264.3; c5's 64 M at 2 KiB 19.50 -> 18.66 ms).
    constexpr uint32_t kRound = (uint32_t)kWaves6 * kRefTPW, kMaxRounds = 4, kPieceRounds = 2;
    const uint32_t ntiles = (n + tl - 1) / tl;
    uint32_t pieces = 1;
    if (!small && !args.stats_plain && (tiles_per_wg + kRound - 1) / kRound > kMaxRounds)  // (plain: one writer)
        pieces = ((tiles_per_wg + kRound - 1) / kRound + kPieceRounds - 1) / kPieceRounds;
    const uint32_t piece_tiles = (ntiles + pieces - 1) / pieces;
    const int slot = timer_begin(device, s);
    for (uint32_t t0 = 0; t0 < ntiles; t0 += piece_tiles) {
        EchoArgs pa = args;
        const uint64_t i0 = (uint64_t)t0 * tl;
        pa.n = (uint32_t)(n - i0 < (uint64_t)piece_tiles * tl ? n - i0 : (uint64_t)piece_tiles * tl);
        pa.descs = d_descs + i0;
        pa.verdicts = d_verdicts ? d_verdicts + i0 : nullptr;
        pa.recs = d_recs ? d_recs + i0 : nullptr;
        uint32_t pg = grid, ptw = tiles_per_wg;
        if (pieces > 1) echo6_geometry(pa.n, grid_force ? grid_force : ncu, &pg, &ptw);
        if (opts == 0 && !small)
            echo_round_kernel<false, false><<<dim3(pg), dim3(kThreads6), 0, s>>>(pa, ptw);
        else if (opts == 0)  // rounds of sub-tiles, writes as soon as a wave has read
            echo_round_kernel<false, true><<<dim3(pg), dim3(kThreads6), 0, s>>>(pa, ptw);
        else if (!small)  // wire mode: the reference mode's 64-B windows and rounds, wire_header_phase64
            echo_round_kernel<true, false><<<dim3(pg), dim3(kThreads6), 0, s>>>(pa, ptw);
        else
            echo_round_kernel<true, true><<<dim3(pg), dim3(kThreads6), 0, s>>>(pa, ptw);
        const hipError_t le = hipGetLastError();
        if (le != hipSuccess) {
            timer_end(slot, s);
            return xsk_gpu__hip_fail(le);
        }
        if (fold) {  // (the partial rows are reused by the next piece's launch, after this fold on the same stream)
            hipLaunchKernelGGL(fold_counters_kernel, dim3(1), dim3(1024), 0, s, (const unsigned long long*)d_workspace,
                               pg, d_stats);
            const hipError_t fe = hipGetLastError();
            if (fe != hipSuccess) {
                timer_end(slot, s);
                return xsk_gpu__hip_fail(fe);
            }
        }
    }
    timer_end(slot, s);
    return 0;
}

int xsk_gpu_echo_dev(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                     uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, struct xsk_gpu_stats* d_stats,
                     void* d_workspace, void* stream) {
    return echo_launch(d_umem, umem_size, d_descs, n, 0, d_verdicts, d_recs, d_stats, d_workspace, stream, 0, 0);
}

int xsk_gpu_echo_dev_opts(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                          uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs,
                          struct xsk_gpu_stats* d_stats, void* d_workspace, void* stream) {
    return echo_launch(d_umem, umem_size, d_descs, n, opts, d_verdicts, d_recs, d_stats, d_workspace, stream, 0, 0);
}

// Internal (xsk_gpu_host.c, zerocopy mode): d_stats is mapped pinned host memory -> no device atomics.
int xsk_gpu__echo_dev_opts_hoststats(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                                     uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs,
                                     struct xsk_gpu_stats* d_stats, void* d_workspace, void* stream, uint32_t tile) {
    return echo_launch(d_umem, umem_size, d_descs, n, opts, d_verdicts, d_recs, d_stats, d_workspace, stream, 1,
                       tile);
}

// Internal (tests / tools, not in include/xsk_gpu.h): xsk_gpu_echo_dev_opts with the workgroup count forced to
// `grid` (0 = the default: one per CU for a large batch, one for a small one), so that shares of several rounds --
// paired short tiles, uniform and ranked streams in every round of a share -- run on small batches too, and small
// batches' sub-tiles can be spread over several workgroups (tools/smallbatch.py).
int xsk_gpu__echo_dev_grid(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                           uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, struct xsk_gpu_stats* d_stats,
                           void* d_workspace, void* stream, uint32_t grid) {
    return echo_launch(d_umem, umem_size, d_descs, n, opts, d_verdicts, d_recs, d_stats, d_workspace, stream, 0, 0,
                       grid);
}

int xsk_gpu_timing_enable(int enable) {
    std::lock_guard<std::mutex> lk(g_timer_mu);
    g_timer.on = enable != 0;
    g_timer.count = 0;
    return 0;
}

int xsk_gpu_timing_read(double* total_ms, uint64_t* launches) {
    std::lock_guard<std::mutex> lk(g_timer_mu);
    double tot = 0.0;
    uint64_t cnt = 0;
    for (int i = 0; i < g_timer.count; ++i) {
        const int d = g_timer.dev[i];
        if (d < 0) continue;
        HIP_TRY(hipEventSynchronize(g_timer.pool[d]->ev[i][1]));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, g_timer.pool[d]->ev[i][0], g_timer.pool[d]->ev[i][1]));
        tot += ms;
        cnt++;
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = cnt;
    g_timer.count = 0;
    return 0;
}

}  // extern "C"
