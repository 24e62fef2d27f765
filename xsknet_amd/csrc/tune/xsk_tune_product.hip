// xsk_tune_product.hip — the PRODUCT round kernel (../xsk_echo_device.h, the same source libxsknet_amd.so
// compiles) at alternative values of its remaining template switches, for in-process A/B against the shipped
// instance (tools/abbench.py variants >= 1000, bench.py --variant).  Tuning library only.
//   0  as shipped (reference mode)            2  wire mode as shipped (every option)
// (round 3 also measured RMETA -- ranked streams reading their step's metadata rows in rank order, one LDS read
// per step instead of two dependent ones: c4 195.5 vs 187.2 us, profiles/r03/ab_rank_ordered_meta_*.log -- and
// ROLL, the tiles of a round in a rolled loop so the kernel's code shrinks from 78 to 46 KB: c4 185.9 vs 185.9 us,
// c3 275.8 vs 276.0, profiles/r03/ab_rolled_tile_loop_*.log; neither shipped.  New candidates get the free slots.)
// (round 3 measured RAGGED 2 here -- ragged tiles with their ICMP masks computed once per frame -- against the
// shipped ranked streams: c4 193.0 vs 185.7 us, profiles/r03/ab_ragged_masks_once_*.log; not shipped)
#include <errno.h>

#include "../xsk_echo_device.h"
#include "../xsk_gpu_internal.h"
#include "../xsk_hip_util.h"

using namespace xskgpu;

extern "C" uint32_t xsk_gpu__num_cu(int device);

// Workgroup timing probes (diagnostics, variants 10-12): the shipped body, each workgroup stamping its start, its
// end (after its last store), its XCC and HW_ID into wgt[4 g .. 4 g + 3].  PERM 0: share g (as shipped); 1: share
// g ^ 1 (does a slow XCD stay slow when it reads its neighbour's addresses?); 2: round-interleaved shares -- round
// k of workgroup g is tiles [(k * grid + g) * 32, + 32) (counters are not meaningful: one partial row per round).
template <int PERM>
__global__ __launch_bounds__(kThreads6, 1) void timed_round_kernel(EchoArgs a, uint32_t per, unsigned long long* wgt) {
    __shared__ Echo6Smem<kRefTPW, false> sm;
    const uint64_t t0 = wall_clock64();
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    constexpr uint32_t kRound = (uint32_t)kWaves6 * kRefTPW;
    if (PERM == 2) {
        for (uint32_t k = 0;; ++k) {
            const uint32_t tb = (k * gridDim.x + blockIdx.x) * kRound;
            if (tb >= ntiles) break;
            echo6_body<kRefTPW, 2, false, false, false, false, true, kRefHeavy>(a, tb, min(ntiles, tb + kRound), sm);
        }
    } else {
        const uint32_t g = (PERM == 1 && (blockIdx.x ^ 1u) < gridDim.x) ? blockIdx.x ^ 1u : blockIdx.x;
        const uint32_t t_begin = g * per, t_end = min(ntiles, t_begin + per);
        echo6_body<kRefTPW, 2, false, false, false, false, true, kRefHeavy>(a, t_begin, t_end, sm);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t xcc, hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        wgt[4 * blockIdx.x] = t0;
        wgt[4 * blockIdx.x + 1] = wall_clock64();
        wgt[4 * blockIdx.x + 2] = xcc;
        wgt[4 * blockIdx.x + 3] = hwid;
    }
}

// BAL (candidate): static shares for frames [0, f0), then a pool the workgroups drain with claims on a device
// counter (queue[0]; queue[1] counts the workgroups out, the last one zeroes both): stage 1 frames [f0, f1) in units
// of 16 sub-tiles of tl1 frames, stage 2 [f1, n) in units of 16 sub-tiles of tl2 (shrinking units: the tail ends
// within about one small sub-tile's time).  The next claim is issued when a unit starts, so its latency hides under
// the unit; the claim travels through LDS with a bare s_barrier (no release fence: the write-through stores of the
// previous unit need not drain first).  Counters: summed over the bodies, stored once.
union BalSmem {
    Echo6Smem<kRefTPW, false> s2;
    Echo6Smem<1, false> s1;
};
__global__ __launch_bounds__(kThreads6, 1) void echo_bal_kernel(EchoArgs a, uint32_t per, uint32_t f0, uint32_t f1,
                                                                uint32_t tl1, uint32_t tl2, uint32_t* queue,
                                                                unsigned long long* wgt) {
    __shared__ BalSmem sm;
    const uint64_t t0 = wall_clock64();
    __shared__ uint32_t s_claim[2];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    Counters cnt;
    const uint32_t nt_s = (f0 + kTile - 1) / kTile;  // f0: a multiple of 64, or n
    const uint32_t t_begin = min(nt_s, blockIdx.x * per), t_end = min(nt_s, t_begin + per);
    if (t_begin < t_end)
        echo6_body<kRefTPW, 2, false, false, false, false, true, kRefHeavy, true>(a, t_begin, t_end, sm.s2, &cnt);
    const uint32_t u1 = (f1 - f0 + 16u * tl1 - 1u) / (16u * tl1);
    const uint32_t units = u1 + (a.n - f1 + 16u * tl2 - 1u) / (16u * tl2);
    uint32_t claim = 0;
    const uint64_t t_static = wall_clock64();
    if (threadIdx.x == 0) claim = __hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t k = 0;
    for (;; ++k) {
        if (threadIdx.x == 0) s_claim[k & 1u] = claim;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const uint32_t u = uniform(s_claim[k & 1u]);
        if (u >= units) break;
        if (threadIdx.x == 0) claim = __hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool st1 = u < u1;
        const uint32_t tl = st1 ? tl1 : tl2;
        const uint32_t fb = st1 ? f0 + u * 16u * tl1 : f1 + (u - u1) * 16u * tl2;
        const uint32_t fe = min(st1 ? f1 : a.n, fb + 16u * tl);
        EchoArgs b = a;
        b.descs = a.descs + fb;
        b.verdicts = a.verdicts ? a.verdicts + fb : nullptr;
        b.recs = a.recs ? a.recs + fb : nullptr;
        b.n = fe - fb;
        b.tile_live = tl;
        echo6_body<1, 0, false, true, false, false, true, kRefHeavy, true>(b, 0u, (b.n + tl - 1u) / tl, sm.s1, &cnt);
    }
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(queue + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u) {
        __hip_atomic_store(queue, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(queue + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    store_counters(a, cnt, sm.s2.cnt, wave, lane);
    if (wgt) {  // timing stamps (diagnostics): start, end, XCC, static part's end (wave 0), pool units run
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            wgt[4 * blockIdx.x] = t0;
            wgt[4 * blockIdx.x + 1] = wall_clock64();
            wgt[4 * blockIdx.x + 2] = xcc | ((uint64_t)k << 32);
            wgt[4 * blockIdx.x + 3] = t_static;
        }
    }
}

// BAL geometry: pool = 1/pool_div of the tiles (at least 0), stage 2 = the last 1/4 of the pool.
static void bal_geometry(uint32_t n, uint32_t grid, uint32_t pool_div, uint32_t* per, uint32_t* f0, uint32_t* f1) {
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    const uint32_t nt_pool = pool_div ? ntiles / pool_div : 0u;
    const uint32_t nt_s = ntiles - nt_pool;
    *per = (nt_s + grid - 1) / grid;
    *f0 = min(n, nt_s * (uint32_t)kTile);
    *f1 = *f0 + (n - *f0) * 3u / 4u;
}

extern "C" int xsk_gpu__product_variant(int variant, uint32_t grid_force, void* d_umem, uint64_t umem_size,
                                        const struct xsk_gpu_desc* d_descs, uint32_t n, uint8_t* d_verdicts,
                                        struct xsk_gpu_rec* d_recs, void* d_workspace, void* stream) {
    if (n == 0) return 0;
    if (n <= XSK_GPU_LOWLAT_MAX || !d_workspace) return -EINVAL;  // large batches: the round kernel's geometry
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    uint32_t grid = 0, per = 0;
    echo6_geometry(n, grid_force ? grid_force : xsk_gpu__num_cu(device), &grid, &per);
    EchoArgs args;
    args.umem = (uint8_t*)d_umem;
    args.umem_size = umem_size;
    args.descs = d_descs;
    args.n = n;
    args.verdicts = d_verdicts;
    args.recs = d_recs;
    args.partials = (unsigned long long*)d_workspace;  // counters as per-workgroup partial rows
    const hipStream_t s = (hipStream_t)stream;
    const dim3 gg(grid), bb(kThreads6);
    switch (variant) {
        case 0: echo_round_kernel<false, false><<<gg, bb, 0, s>>>(args, per); break;
        case 2: args.opts = XSK_GPU_OPT_ALL; echo_round_kernel<true, false><<<gg, bb, 0, s>>>(args, per); break;
        // timing probes: workgroup stamps at workspace u64 offset 8192 (grid <= 1024: 4096 u64)
        case 10: timed_round_kernel<0><<<gg, bb, 0, s>>>(args, per, args.partials + 8192); break;
        case 11: timed_round_kernel<1><<<gg, bb, 0, s>>>(args, per, args.partials + 8192); break;
        case 12: timed_round_kernel<2><<<gg, bb, 0, s>>>(args, per, args.partials + 8192); break;
        // BAL: pool of 1/8, 1/16, 1/4 of the tiles in sub-tiles of 16 then 8 frames; 23: 1/8 in 32 then 8; the queue
        // counters at workspace byte 512 KiB (zero on entry, left zero)
        // 24: no pool (the BAL kernel's structure alone); 25: 1/16 in whole tiles; 26: 1/16 in 16-frame sub-tiles
        // only; 27: 1/32 in 16 then 8
        case 20: case 21: case 22: case 23: case 24: case 25: case 26: case 27: {
            static const uint32_t kDiv[8] = {8, 16, 4, 8, 0, 16, 16, 32}, kTl1[8] = {16, 16, 16, 32, 16, 64, 16, 16},
                                  kTl2[8] = {8, 8, 8, 8, 8, 64, 16, 8};
            const int i = variant - 20;
            uint32_t bper = 0, f0 = 0, f1 = 0;
            bal_geometry(n, grid, kDiv[i], &bper, &f0, &f1);
            echo_bal_kernel<<<gg, bb, 0, s>>>(args, bper, f0, f1, kTl1[i], kTl2[i],
                                              (uint32_t*)((uint8_t*)d_workspace + (1u << 19)), args.partials + 8192);
            break;
        }
        default: return -EINVAL;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}
