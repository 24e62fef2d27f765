// xsk_echo.hip — the product entry point of the gfx950 ICMP-echo transform: xsk_gpu_echo_dev() (one
// launch of the round kernel echo_kernel6 + the counter fold), the workspace query, the kernel timer the bench reads,
// and the error plumbing of the C ABI (include/xsk_gpu.h).  Device code: xsk_echo_device.h.
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "xsk_echo_device.h"
#include "xsk_hip_util.h"

using namespace xskgpu;

namespace {

// Fold the per-workgroup partials into the caller's stats_record-compatible counters: 1024 threads,
// thread t sums counter t % 4 over rows t/4, t/4 + 256, ... with 4 independent chains, then a tree.
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

// Counter delivery of xsk_gpu_echo_dev(_opts): 1 = every workgroup adds its four counters to d_stats with
// device-scope atomics (shipped: 1.5-2.5 % less time per call than the fold launch, profiles/r01/stats_delivery.log);
// 0 = per-workgroup partials + the fold launch.  Tuning switch: xsk_gpu__set_stats_atomic.
int g_stats_atomic = 1;

// ---- kernel timing (bench instrumentation) -------------------------------------------------------
constexpr int kTimerCap = 8192;
struct Timer {
    bool on = false;
    int count = 0;  // recorded pairs since enable
    hipEvent_t ev[kTimerCap][2];
    bool created = false;
    int dev[kTimerCap];
};
Timer g_timer;
std::mutex g_timer_mu;

// Timer slot for the next transform launch (-1 when timing is off or full).
int timer_slot(int device) {
    std::lock_guard<std::mutex> lk(g_timer_mu);
    if (!g_timer.on || g_timer.count >= kTimerCap) return -1;
    const int slot = g_timer.count++;
    g_timer.dev[slot] = device;
    return slot;
}

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
const char* xsk_gpu_last_error(void) { return g_last_error; }

size_t xsk_gpu_workspace_size(int device, uint32_t n) {
    if (device < 0) return 0;
    // room for the partial rows of either launch geometry (round kernel: <= one workgroup per CU)
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    uint32_t g = echo_grid(n);
    const uint32_t g6 = ntiles < kMaxCuBound ? ntiles : kMaxCuBound;
    if (g6 > g) g = g6;
    return (size_t)g * 4 * sizeof(unsigned long long);
}

// Compute units of `device` (cached): the round kernel launches one workgroup per CU.
uint32_t xsk_gpu__num_cu(int device) {
    static int cache[64];
    if (device < 0 || device >= 64) return 0;
    if (cache[device] <= 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || v <= 0) return 0;
        cache[device] = v > (int)kMaxCuBound ? (int)kMaxCuBound : v;
    }
    return (uint32_t)cache[device];
}


// fold = 1: per-workgroup partials in the workspace + the one-workgroup fold launch (the stats may live in
// mapped host memory, where device-scope atomics are not an option); 0: every workgroup adds its counters to
// d_stats (device memory) with device-scope atomics, no second launch.
static int echo_dev_impl(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                         uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, struct xsk_gpu_stats* d_stats,
                         void* d_workspace, void* stream, int fold) {
    if (n == 0) return 0;
    if (n > XSK_GPU_MAX_BATCH) return -EINVAL;
    if (!d_umem || !d_descs || ((uintptr_t)d_umem & 15u) || (umem_size & 15u) || ((uintptr_t)d_descs & 15u) ||
        ((uintptr_t)d_recs & 15u))
        return -EINVAL;
    if (d_stats && !d_workspace) return -EINVAL;
    if (umem_size >> 48) return -EINVAL;  // FrameMeta6 carries 48-bit UMEM offsets
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    const uint32_t ncu = xsk_gpu__num_cu(device);
    if (!ncu) return xsk_gpu__hip_fail(hipErrorInvalidDevice);
    uint32_t grid = 0, tiles_per_wg = 0;
    echo6_geometry(n, ncu, &grid, &tiles_per_wg);
    hipStream_t s = (hipStream_t)stream;
    EchoArgs args;
    args.umem = (uint8_t*)d_umem;
    args.umem_size = umem_size;
    args.descs = d_descs;
    args.n = n;
    args.verdicts = d_verdicts;
    args.recs = d_recs;
    args.partials = d_stats ? (unsigned long long*)d_workspace : nullptr;
    if (d_stats && (grid == 1 || !fold)) {  // the workgroups add their counters themselves
        args.partials = nullptr;
        args.stats_direct = (unsigned long long*)&d_stats->rx_packets;
    }

    const int slot = timer_slot(device);
    if (slot >= 0) HIP_TRY(hipEventRecord(g_timer.ev[slot][0], s));
    echo_kernel6<kShip6U, kShip6TPW, kShip6Sync, kShip6Stream, false, false, false, false, false, kShip6Mid, kShip6D2,
                 kShip6Skm>
        <<<dim3(grid), dim3(kThreads6), 0, s>>>(args, tiles_per_wg);
    HIP_TRY(hipGetLastError());
    if (slot >= 0) HIP_TRY(hipEventRecord(g_timer.ev[slot][1], s));
    if (d_stats && grid > 1 && fold) {
        hipLaunchKernelGGL(fold_counters_kernel, dim3(1), dim3(1024), 0, s, (const unsigned long long*)d_workspace, grid,
                           d_stats);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}

int xsk_gpu_echo_dev(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                     uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, struct xsk_gpu_stats* d_stats,
                     void* d_workspace, void* stream) {
    return echo_dev_impl(d_umem, umem_size, d_descs, n, d_verdicts, d_recs, d_stats, d_workspace, stream,
                         !g_stats_atomic);
}

int xsk_gpu__echo_wire_dev(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                           uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, void* d_partials,
                           struct xsk_gpu_stats* d_stats, int fold, uint32_t* grid_out, void* stream);  // xsk_wire.hip

static int echo_dev_opts_impl(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                              uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs,
                              struct xsk_gpu_stats* d_stats, void* d_workspace, void* stream, int fold) {
    if (opts & ~XSK_GPU_OPT_ALL) return -EINVAL;
    if (opts == 0)
        return echo_dev_impl(d_umem, umem_size, d_descs, n, d_verdicts, d_recs, d_stats, d_workspace, stream, fold);
    if (n == 0) return 0;
    if (n > XSK_GPU_MAX_BATCH) return -EINVAL;
    if (!d_umem || !d_descs || ((uintptr_t)d_umem & 15u) || (umem_size & 15u) || ((uintptr_t)d_descs & 15u) ||
        ((uintptr_t)d_recs & 15u))
        return -EINVAL;
    if (d_stats && !d_workspace) return -EINVAL;
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    uint32_t grid = 0;
    const int slot = timer_slot(device);
    if (slot >= 0) HIP_TRY(hipEventRecord(g_timer.ev[slot][0], (hipStream_t)stream));
    const int rc = xsk_gpu__echo_wire_dev(d_umem, umem_size, d_descs, n, opts, d_verdicts, d_recs,
                                          d_stats ? d_workspace : nullptr, d_stats, fold, &grid, stream);
    if (rc) return rc;
    if (slot >= 0) HIP_TRY(hipEventRecord(g_timer.ev[slot][1], (hipStream_t)stream));
    if (d_stats && grid > 1 && fold) {  // otherwise the workgroups added their counters themselves
        hipLaunchKernelGGL(fold_counters_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream,
                           (const unsigned long long*)d_workspace, grid, d_stats);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}

int xsk_gpu_echo_dev_opts(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                          uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs,
                          struct xsk_gpu_stats* d_stats, void* d_workspace, void* stream) {
    return echo_dev_opts_impl(d_umem, umem_size, d_descs, n, opts, d_verdicts, d_recs, d_stats, d_workspace, stream,
                              !g_stats_atomic);
}

// Internal (xsk_gpu_host.c, zerocopy mode): d_stats is mapped pinned host memory -> always the fold.
int xsk_gpu__echo_dev_opts_hoststats(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                                     uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs,
                                     struct xsk_gpu_stats* d_stats, void* d_workspace, void* stream) {
    return echo_dev_opts_impl(d_umem, umem_size, d_descs, n, opts, d_verdicts, d_recs, d_stats, d_workspace, stream, 1);
}

int xsk_gpu__set_stats_atomic(int on) {
    if (on < 0 || on > 1) return -EINVAL;
    g_stats_atomic = on;
    return 0;
}

int xsk_gpu_timing_enable(int enable) {
    std::lock_guard<std::mutex> lk(g_timer_mu);
    if (enable && !g_timer.created) {
        for (int i = 0; i < kTimerCap; ++i) {
            HIP_TRY(hipEventCreate(&g_timer.ev[i][0]));
            HIP_TRY(hipEventCreate(&g_timer.ev[i][1]));
        }
        g_timer.created = true;
    }
    g_timer.on = enable != 0;
    g_timer.count = 0;
    return 0;
}

int xsk_gpu_timing_read(double* total_ms, uint64_t* launches) {
    std::lock_guard<std::mutex> lk(g_timer_mu);
    double tot = 0.0;
    for (int i = 0; i < g_timer.count; ++i) {
        HIP_TRY(hipEventSynchronize(g_timer.ev[i][1]));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, g_timer.ev[i][0], g_timer.ev[i][1]));
        tot += ms;
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = (uint64_t)g_timer.count;
    g_timer.count = 0;
    return 0;
}

}  // extern "C"
