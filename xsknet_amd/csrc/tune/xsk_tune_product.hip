// xsk_tune_product.hip — the PRODUCT round kernel (../xsk_echo_device.h, the same source libxsknet_amd.so
// compiles) at alternative values of its remaining template switches, for in-process A/B against the shipped
// instance (tools/abbench.py variants >= 1000, bench.py --variant).  Tuning library only.
//   0  as shipped (reference mode)            2  wire mode as shipped (every option)
// (round 4 removed the round-1/2 laboratory -- tune/xsk_echo_lab.h, xsk_echo_variants.h, xsk_tune.hip, xsk_wire_v1.hip,
// the variants of tools/kbench.py and bench.py --variant < 1000 -- and the SLACK patch unit: every variant there lost
// by more than 2 % in a committed A/B log or was shipped; the logs under profiles/r01-r03 and DESIGN.md stay the record,
// and the sources are in git history before commit "Prune the tuning laboratory".)
// (round 3 also measured RMETA -- ranked streams reading their step's metadata rows in rank order, one LDS read
// per step instead of two dependent ones: c4 195.5 vs 187.2 us, profiles/r03/ab_rank_ordered_meta_*.log -- and
// ROLL, the tiles of a round in a rolled loop so the kernel's code shrinks from 78 to 46 KB: c4 185.9 vs 185.9 us,
// c3 275.8 vs 276.0, profiles/r03/ab_rolled_tile_loop_*.log; neither shipped.  New candidates get the free slots.)
// (round 3 measured RAGGED 2 here -- ragged tiles with their ICMP masks computed once per frame -- against the
// shipped ranked streams: c4 193.0 vs 185.7 us, profiles/r03/ab_ragged_masks_once_*.log; not shipped)
// (round 3 measured SWZ -- the header-window rows in LDS swizzled by 16-B chunk (chunk c of frame f at (c + f/4)
// mod 4), against the 16-way bank conflicts of the per-lane header-phase reads (6.7 M conflict cycles per launch,
// profiles/r03/lds/): c2 34.7 vs 35.2 us, c3 274.2 vs 275.1, c4 183.4 vs 182.8 against the same kernel without it,
// profiles/r03/ab_lds_swizzle_stdout.jsonl; within noise, removed)
// (round 3 measured RH2 again in the sustained regime, tools/abbench.py --burst: c4 179.6 vs 179.8 us shipped, 181.9
// without PRIO, profiles/r03/ab_burst_prio_rh2_c4.log)
// (round 3 measured RH2 -- the ranked streams summing 16-bit halves with v_dot2 in 32 bits -- and PRIO2 -- also the
// descriptor, paired-short and short / ping-size loads at s_setprio 2: c4 182.5 / 182.0 vs 182.9 us, c3 274.7 / 275.2
// vs 274.7, p98 64.0 / 64.6 vs 64.1, within noise, profiles/r03/ab_rh2_prio2_*.log; removed)
// (round 3 measured RLANE -- the uniform stream taking its rows' frame offsets from the owner lanes by readlane
// instead of one LDS read of the step's metadata: c3 274.2 vs 274.8 and 281.8 vs 281.5 us, within noise,
// profiles/r03/ab_uniform_rlane*_c3.log; removed)
// (round 3 measured BAL -- static shares for 15/16 .. 3/4 of the tiles, the rest a pool drained with claims on a
// device counter in shrinking sub-tile units -- as variants 20-27 of commit a9c3d74: c3 +19 to +60 us, c4 +8 to +48,
// c2 +11 to +30; profiles/r03/balance/.  Removed: it needed a counter-output switch in the product body.)
// (round 4 measured DEFER -- rounds in pairs, the first parking its patched windows in a contiguous workspace scratch for
// ONE scatter at the end of a two-round share: c3 286.4 vs 281.8 us, c4 191.8 vs 180.3, c2 46.6 vs 36.7; and the first
// round's records and verdicts held in VGPRs until the second's write phase: c3 280.1 vs 278.8, c4 179.5 vs 179.3, c2
// 34.9 vs 34.9, wire c3 286.1 vs 286.5; profiles/r04/defer/; removed)
// (round 4 measured GBAR -- a non-final round's write phase held until every workgroup of the grid has read its round, a
// grid arrival counter with a 20-us bound: c3 275.5 vs 274.8 us, c4 190.1 vs 180.6, c2 47.2 vs 35.6, wire c3 284.5 vs
// 285.9; profiles/r04/writes/; removed)
// (round 4 measured PDSC -- the descriptors a failed pairing attempt loaded reused by the tiles' own streams instead of
// reloaded, 119 VGPRs: c3 273.5 vs 273.5 us, c4 181.5 vs 180.3, c2 34.6 vs 34.5, p98 63.4 vs 64.4, wire c3 276.4 vs
// 276.9; profiles/r04/pdsc/; removed)
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
    __shared__ Echo6Smem<kRefTPW> sm;
    const uint64_t t0 = wall_clock64();
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    constexpr uint32_t kRound = (uint32_t)kWaves6 * kRefTPW;
    if (PERM == 2) {
        for (uint32_t k = 0;; ++k) {
            const uint32_t tb = (k * gridDim.x + blockIdx.x) * kRound;
            if (tb >= ntiles) break;
            echo6_body<kRefTPW, 2, false, false, false, false, true, kRefHeavy, kUR, true, true, kRefSlack, true>(a, tb, min(ntiles, tb + kRound), sm);
        }
    } else {
        const uint32_t g = (PERM == 1 && (blockIdx.x ^ 1u) < gridDim.x) ? blockIdx.x ^ 1u : blockIdx.x;
        const uint32_t t_begin = g * per, t_end = min(ntiles, t_begin + per);
        echo6_body<kRefTPW, 2, false, false, false, false, true, kRefHeavy, kUR, true, true, kRefSlack, true>(a, t_begin, t_end, sm);
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
        // (3 / 4, ranked streams with 4 / 8 row-loads per batch: measured against kUR = 6 in rounds 3-4 and removed)
        // 5 / 6: the uniform stream's row-loads in batches of 4 and a remainder (round 2's, no SPLIT), reference / wire
        case 5: echo_round_kernel<false, false, kUR, false><<<gg, bb, 0, s>>>(args, per); break;
        case 6: args.opts = XSK_GPU_OPT_ALL; echo_round_kernel<true, false, kUR, false><<<gg, bb, 0, s>>>(args, per); break;
        // 7 / 8: without PRIO (a stream batch's address work and loads at the default priority), reference / wire mode
        case 7: echo_round_kernel<false, false, kUR, true, false><<<gg, bb, 0, s>>>(args, per); break;
        case 8: args.opts = XSK_GPU_OPT_ALL; echo_round_kernel<true, false, kUR, true, false><<<gg, bb, 0, s>>>(args, per); break;
        // 9: SLACK 0 -- heavy waves wait for every wave of the workgroup (round 3's write-phase wait); 13: SLACK 4
        case 9: echo_round_kernel<false, false, kUR, true, true, 0><<<gg, bb, 0, s>>>(args, per); break;
        case 13: echo_round_kernel<false, false, kUR, true, true, 4><<<gg, bb, 0, s>>>(args, per); break;
        // (14-16, RS 2 -- the lean ranked streams, stream_tile_ranked2 -- with 6 / 8 / 4 row-loads per batch: c4 177.9 /
        // 179.5 / 180.8 vs 177.4 us, profiles/r04/ab/; 17 / 18, LASTW -- no write-phase wait in a share's last round: c3
        // +1.1 us, c4 +3.0; 21, wire mode on 128-B windows, the wire kernel of rounds 1-4: c2 70.7 vs 44.0 us, c3 297.8 vs
        // 279.7, profiles/r04/wire64/; 24, wire mode without paired short tiles: c2 44.5 vs 43.4, c3 284.4 vs 277.8,
        // profiles/r04/wpair/.  Removed from the product header in round 5, with the 128-B wire_header_phase)
        // 22: wire mode as shipped with no option bit but VLAN; 23: wire mode with SLACK 0
        case 22: args.opts = XSK_GPU_OPT_VLAN; echo_round_kernel<true, false><<<gg, bb, 0, s>>>(args, per); break;
        case 23: args.opts = XSK_GPU_OPT_ALL; echo_round_kernel<true, false, kUR, true, true, 0><<<gg, bb, 0, s>>>(args, per); break;
        // (25, one tile per wave per round -- four rounds per 1 M-frame share, a quarter of the windows in the last write
        // phase: c2 35.9 vs 35.3 us, p98 63.5 vs 63.8, c3 287.5 vs 276.4; profiles/r04/tpw1/, removed)
        // (26, REREAD -- the share's second-to-last round stores records and verdicts but not its windows, which are read
        // again, re-patched and stored after the last round's write phase: c3 284.1 vs 274.9 us, c4 190.3 vs 176.0, c2
        // 39.6 vs 35.0, p98 74.8 vs 63.9, outputs equal; profiles/r04/reread/, removed)
        // (30-41, round 5, VERDICT r04 next #3 -- c2's short tiles on other orchestrations, each lost in-process against the
        // shipped kernel's 37.6-38.1 us: SG, a non-persistent grid of 4- / 8- / 1- / 16-wave workgroups, one tile pair per
        // wave, writing at once (37.9 / 40.1 / 37.7 / 38.3; plain stores 38.0); SGP, the same with a two-deep software
        // pipeline over each wave's pairs (42.1 / 42.5 / 37.5 / 42.6, 147-152 VGPRs); the diagnostics SG without the header
        // phase 32.6 and without LDS 33.3 located the cost in the header phase, whence HB.  profiles/r05/s1/; removed)
        // 42 / 43: without HB (shipped in round 5: the header phase's window read as three ds_read_b128 in aligned waves,
        // an aligned reply's patch stored as two b128 + one b64) -- eleven ds_read_b32, seven ds_write_b32; reference / wire
        case 42: echo_round_kernel<false, false, kUR, true, true, kRefSlack, false><<<gg, bb, 0, s>>>(args, per); break;
        case 43: args.opts = XSK_GPU_OPT_ALL; echo_round_kernel<true, false, kUR, true, true, kRefSlack, false><<<gg, bb, 0, s>>>(args, per); break;
        // timing probes: workgroup stamps at workspace u64 offset 8192 (grid <= 1024: 4096 u64)
        case 10: timed_round_kernel<0><<<gg, bb, 0, s>>>(args, per, args.partials + 8192); break;
        case 11: timed_round_kernel<1><<<gg, bb, 0, s>>>(args, per, args.partials + 8192); break;
        case 12: timed_round_kernel<2><<<gg, bb, 0, s>>>(args, per, args.partials + 8192); break;
        default: return -EINVAL;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

// The tuning library's own copy of the error hook (the product library's is hidden).
extern "C" __attribute__((visibility("hidden"))) int xsk_gpu__hip_fail(hipError_t e) {
    return e == hipErrorOutOfMemory ? -ENOMEM : -EIO;
}
