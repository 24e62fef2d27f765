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

// SGP (round 5): the SG kernel with every wave looping over PPW tile pairs in a two-deep software pipeline -- pair p + 1's
// frame loads and pair p + 2's descriptor loads are issued before pair p's header phase and stores, so no load waits
// behind this wave's earlier stores (vmcnt counts loads and stores in one in-order counter).  The pair's descriptors,
// frame loads and rest are read_round_short2's three parts, restated here (the product header keeps them in one
// function: its instruction stream is pinned, tests/test_kernel_isa.py).  PERSIST: grid = one 16-wave workgroup per CU
// over contiguous shares (wave w takes pairs w, w + 16, ... of its share); else WPB-wave workgroups of PPW pairs each.
struct SgPair {  // (the frames' FrameIn is recomputed from the descriptors where needed: fewer live VGPRs)
    u32x4 d0, d1;
    u32x4 x0[4], x1[4];
    bool in0, in1;
};
__device__ __forceinline__ void sg_desc(const EchoArgs& a, uint32_t t0, uint32_t lane, SgPair& S) {
    const uint32_t fi0 = t0 * kTile + lane, fi1 = (t0 + 1u) * kTile + lane;
    S.in0 = fi0 < a.n;
    S.in1 = fi1 < a.n;
    S.d0 = u32x4{0u, 0u, 0u, 0u};
    S.d1 = u32x4{0u, 0u, 0u, 0u};
    if (S.in0) S.d0 = *(const u32x4*)(a.descs + fi0);
    if (S.in1) S.d1 = *(const u32x4*)(a.descs + fi1);
}
template <bool WIRE>
__device__ __forceinline__ bool sg_frames(const EchoArgs& a, uint32_t lane, SgPair& S) {
    const FrameIn F0 = frame_in<WIRE>(a, S.d0, S.in0), F1 = frame_in<WIRE>(a, S.d1, S.in1);
    if ((__ballot(F0.lim > (uint32_t)kWin) | __ballot(F1.lim > (uint32_t)kWin)) != 0ull) return false;
    const uint32_t ro = 16u * (lane & 3u);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int src = r * 16 + (int)(lane >> 2);
        const uint64_t b0 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(F0.a16 >> 32), src, 64) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)F0.a16, src, 64);
        const uint64_t b1 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(F1.a16 >> 32), src, 64) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)F1.a16, src, 64);
        const uint32_t m0 = (uint32_t)__shfl((int)F0.lim, src, 64), m1 = (uint32_t)__shfl((int)F1.lim, src, 64);
        S.x0[r] = u32x4{0u, 0u, 0u, 0u};
        S.x1[r] = u32x4{0u, 0u, 0u, 0u};
        if (ro < m0) S.x0[r] = __builtin_nontemporal_load((const u32x4*)(a.umem + b0 + ro));
        if (ro < m1) S.x1[r] = __builtin_nontemporal_load((const u32x4*)(a.umem + b1 + ro));
    }
    return true;
}
template <bool WIRE>
__device__ __forceinline__ void sg_finish_store(const EchoArgs& a, const SgPair& S, uint32_t t0, uint8_t* rows0,
                                                uint8_t* rows1, uint32_t* sums0, uint32_t* sums1, uint32_t lane,
                                                Counters& cnt) {
    const uint32_t kk = lane & 3u, ro = 16u * kk;
    u32x4 rec[2];
    uint32_t verd[2];
    uint64_t wbm[2];
    const FrameIn F0 = frame_in<WIRE>(a, S.d0, S.in0), F1 = frame_in<WIRE>(a, S.d1, S.in1);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const FrameIn& F = tt ? F1 : F0;
        uint8_t* rows = tt ? rows1 : rows0;
        uint32_t* sums = tt ? sums1 : sums0;
        const uint32_t kf = (F.off << 24) ^ F.rowhi;
        const bool uni = __ballot(kf != uniform(kf)) == 0ull;
        const u32x4 mk = range_mask((int)ro, (int)uniform(F.off) + 34, (int)uniform(F.rowhi));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
            const u32x4 v = tt ? S.x1[r] : S.x0[r];
            *(u32x4*)(rows + f * kWin + ro) = v;
            uint32_t ric;
            if (uni) {
                ric = sum_halves(v & mk, 0u);
            } else {
                const int fo = __shfl((int)F.off, (int)f, 64), fh = __shfl((int)F.rowhi, (int)f, 64);
                ric = sum_range_h(v, (int)ro, fo + 34, fh);
            }
            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0xB1, 0xF, 0xF, false);  // xor 1
            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x4E, 0xF, 0xF, false);  // xor 2
            if (kk == 0u) sums[f] = ric;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const FrameIn& F = tt ? F1 : F0;
        uint8_t* rows = tt ? rows1 : rows0;
        uint32_t* sums = tt ? sums1 : sums0;
        const bool in = tt ? S.in1 : S.in0;
        const bool wb = WIRE ? wire_header_phase64(a, rows + lane * kWin, sums[lane], F.addr, F.len, F.ok, in, F.wend, cnt,
                                                   &rec[tt], &verd[tt])
                             : header_phase_ref(a, rows + lane * kWin, sums[lane], F.addr, F.len, in, F.ok, F.parse, cnt,
                                                &rec[tt], &verd[tt]);
        wbm[tt] = __ballot(wb);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const uint32_t t = t0 + (uint32_t)tt;
        const uint8_t* rows = tt ? rows1 : rows0;
        const u32x4 dd = tt ? S.d1 : S.d0;
        if (wbm[tt]) {
            const uint32_t hi_u = rdlane(dd.y, (uint32_t)__builtin_ctzll(wbm[tt]));
            const bool wt_tile = __ballot(((wbm[tt] >> lane) & 1ull) && (dd.y != hi_u || dd.x > 0xFFFFFFC0u)) == 0ull;
            const __amdgpu_buffer_rsrc_t wrs =
                __builtin_amdgcn_make_buffer_rsrc((void*)(a.umem + ((uint64_t)hi_u << 32)), (short)0, -1, kRsrcFlags);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                const uint32_t flo = (uint32_t)__shfl((int)dd.x, (int)f, 64);
                const uint32_t fhi = (uint32_t)__shfl((int)dd.y, (int)f, 64);
                if ((wbm[tt] >> f) & 1ull) {
                    const u32x4 w = *(const u32x4*)(rows + f * kWin + 16u * kk);
                    if (wt_tile) __builtin_amdgcn_raw_buffer_store_b128(w, wrs, (int)(flo + 16u * kk), 0, kAuxSC1);
                    else *(u32x4*)(a.umem + ((uint64_t)flo | ((uint64_t)fhi << 32)) + 16u * kk) = w;
                }
            }
        }
        const uint32_t fi = t * (uint32_t)kTile + lane;
        if (fi < a.n) {
            if (a.recs)
                __builtin_amdgcn_raw_buffer_store_b128(
                    rec[tt], __builtin_amdgcn_make_buffer_rsrc((void*)((u32x4*)a.recs + (uint64_t)t * kTile), (short)0, -1, kRsrcFlags),
                    (int)(lane * 16u), 0, kAuxSC1);
            if (a.verdicts) a.verdicts[fi] = (uint8_t)verd[tt];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // rows / sums are rewritten by the next pair
}

// SG (round 5): c2's all-short batches on a NON-persistent grid of small workgroups -- WPB waves
// each, every wave one pair of short tiles (read_round_short2: both descriptor loads, then all eight frame loads, the
// header phase of each tile), written as soon as the wave has read (no rounds, no arrival counter).  The upper bound of
// the idea: a tile with a longer frame is not processed (its verdicts stay as they were; outputs_equal_shipped flags
// it), so it is only measured on all-short batches.  WT: windows and records stored write-through as in the product.
// DIAG (diagnostics, wrong outputs): 1 = no header phase (windows stored as read, records zero); 2 = no LDS either --
// each quad of lanes stores the 64 bytes it loaded straight back, c2floor mode 3's traffic in this kernel's skeleton.
template <bool WIRE, int WPB, bool WT, int DIAG = 0>
__global__ __launch_bounds__(WPB * 64) void short_grid_kernel(EchoArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t hdr[WPB][2][kTile * kWin];
    __shared__ uint32_t sums[WPB][2][kTile];
    __shared__ unsigned long long cnts[WPB][4];
    const uint32_t wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t t0 = 2u * (blockIdx.x * (uint32_t)WPB + wave);
    Counters cnt;
    if (t0 + 1u < ntiles) {  // wave-uniform (the batch is a whole number of tile pairs in the A/B)
        u32x4 rec[2];
        uint32_t verd[2], alo[2], ahi[2], round_long = 0;
        uint64_t wbm[2];
        if (DIAG) {
            SgPair S;
            sg_desc(a, t0, lane, S);
            const bool ok = sg_frames<WIRE>(a, lane, S);
            if (DIAG == 2 && ok) {  // straight back, 4 lanes per frame
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    const u32x4 dd = tt ? S.d1 : S.d0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                        const uint32_t flo = (uint32_t)__shfl((int)dd.x, (int)f, 64);
                        const uint32_t fhi = (uint32_t)__shfl((int)dd.y, (int)f, 64);
                        *(u32x4*)(a.umem + ((uint64_t)flo | ((uint64_t)fhi << 32)) + 16u * (lane & 3u)) = tt ? S.x1[r] : S.x0[r];
                    }
                    const uint32_t fi = (t0 + (uint32_t)tt) * (uint32_t)kTile + lane;
                    if (fi < a.n) {
                        if (a.recs) ((u32x4*)a.recs)[fi] = dd;
                        if (a.verdicts) a.verdicts[fi] = 0;
                    }
                }
            } else if (ok) {  // through LDS, no header phase
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    uint8_t* rows = hdr[wave][tt];
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        *(u32x4*)(rows + ((uint32_t)r * 16u + (lane >> 2)) * kWin + 16u * (lane & 3u)) = tt ? S.x1[r] : S.x0[r];
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    const u32x4 dd = tt ? S.d1 : S.d0;
                    const uint8_t* rows = hdr[wave][tt];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                        const uint32_t flo = (uint32_t)__shfl((int)dd.x, (int)f, 64);
                        const uint32_t fhi = (uint32_t)__shfl((int)dd.y, (int)f, 64);
                        const u32x4 w = *(const u32x4*)(rows + f * kWin + 16u * (lane & 3u));
                        *(u32x4*)(a.umem + ((uint64_t)flo | ((uint64_t)fhi << 32)) + 16u * (lane & 3u)) = w;
                    }
                    const uint32_t fi = (t0 + (uint32_t)tt) * (uint32_t)kTile + lane;
                    if (fi < a.n) {
                        if (a.recs) ((u32x4*)a.recs)[fi] = dd;
                        if (a.verdicts) a.verdicts[fi] = 0;
                    }
                }
            }
        } else if (read_round_short2<kRefHeavy, WIRE>(a, t0, t0 + 1u, hdr[wave][0], hdr[wave][1], sums[wave][0], sums[wave][1],
                                              lane, cnt, rec, verd, alo, ahi, wbm, round_long)) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t t = t0 + (uint32_t)i;
                const uint8_t* rows = hdr[wave][i];
                if (wbm[i]) {
                    const uint32_t hi_u = WT ? rdlane(ahi[i], (uint32_t)__builtin_ctzll(wbm[i])) : 0u;
                    const bool wt_tile = WT && __ballot(((wbm[i] >> lane) & 1ull) &&
                                                        (ahi[i] != hi_u || alo[i] > 0xFFFFFFC0u)) == 0ull;
                    const __amdgpu_buffer_rsrc_t wrs =
                        __builtin_amdgcn_make_buffer_rsrc((void*)(a.umem + ((uint64_t)hi_u << 32)), (short)0, -1, kRsrcFlags);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                        const uint32_t kk = lane & 3u;
                        const uint32_t flo = (uint32_t)__shfl((int)alo[i], (int)f, 64);
                        const uint32_t fhi = (uint32_t)__shfl((int)ahi[i], (int)f, 64);
                        if ((wbm[i] >> f) & 1ull) {
                            const u32x4 w = *(const u32x4*)(rows + f * kWin + 16u * kk);
                            if (WT && wt_tile) __builtin_amdgcn_raw_buffer_store_b128(w, wrs, (int)(flo + 16u * kk), 0, kAuxSC1);
                            else *(u32x4*)(a.umem + ((uint64_t)flo | ((uint64_t)fhi << 32)) + 16u * kk) = w;
                        }
                    }
                }
                const uint32_t fi = t * (uint32_t)kTile + lane;
                if (fi < a.n) {
                    if (a.recs) {
                        if (WT)
                            __builtin_amdgcn_raw_buffer_store_b128(
                                rec[i], __builtin_amdgcn_make_buffer_rsrc((void*)((u32x4*)a.recs + (uint64_t)t * kTile), (short)0, -1, kRsrcFlags),
                                (int)(lane * 16u), 0, kAuxSC1);
                        else ((u32x4*)a.recs)[fi] = rec[i];
                    }
                    if (a.verdicts) a.verdicts[fi] = (uint8_t)verd[i];
                }
            }
        }
    }
    // counters: one partial row per workgroup (the A/B's workspace holds 32 768 rows)
    cnt.rxp = wave_sum_u64(cnt.rxp);
    cnt.rxb = wave_sum_u64(cnt.rxb);
    cnt.txp = wave_sum_u64(cnt.txp);
    cnt.txb = wave_sum_u64(cnt.txb);
    if (lane == 0) {
        cnts[wave][0] = cnt.rxp;
        cnts[wave][1] = cnt.rxb;
        cnts[wave][2] = cnt.txp;
        cnts[wave][3] = cnt.txb;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (threadIdx.x < 4 && a.partials) {
        unsigned long long s = 0;
#pragma unroll
        for (int w = 0; w < WPB; ++w) s += cnts[w][threadIdx.x];
        a.partials[blockIdx.x * 4 + threadIdx.x] = s;
    }
}

template <bool WIRE, int WPB, int PPW, bool PERSIST>
__global__ __launch_bounds__(WPB * 64) void short_pipe_kernel(EchoArgs a, uint32_t pairs_per_wg) {
    __shared__ __attribute__((aligned(16))) uint8_t hdr[WPB][2][kTile * kWin];
    __shared__ uint32_t sums[WPB][2][kTile];
    __shared__ unsigned long long cnts[WPB][4];
    const uint32_t wave = uniform(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t npairs = (a.n + 2 * kTile - 1) / (2 * kTile);
    // the wave's pairs: PERSIST p_k = g * ppw + w + k * WPB (k < ceil), else (g * WPB + w) * PPW + k
    const uint32_t first = PERSIST ? blockIdx.x * pairs_per_wg + wave : (blockIdx.x * (uint32_t)WPB + wave) * PPW;
    const uint32_t stepp = PERSIST ? (uint32_t)WPB : 1u;
    const uint32_t end = PERSIST ? min(npairs, (blockIdx.x + 1u) * pairs_per_wg) : min(npairs, first + PPW);
    Counters cnt;
    if (first < end) {
        SgPair cur, nxt;
        sg_desc(a, 2u * first, lane, cur);
        bool ok = sg_frames<WIRE>(a, lane, cur);
        if (first + stepp < end) sg_desc(a, 2u * (first + stepp), lane, nxt);
        for (uint32_t p = first; p < end && ok; p += stepp) {  // wave-uniform
            const uint32_t pn = p + stepp;
            bool ok_n = true;
            SgPair nn;
            if (pn < end) {
                ok_n = sg_frames<WIRE>(a, lane, nxt);  // pair p + 1's frame loads, before p's stores
                if (pn + stepp < end) sg_desc(a, 2u * (pn + stepp), lane, nn);
            }
            sg_finish_store<WIRE>(a, cur, 2u * p, hdr[wave][0], hdr[wave][1], sums[wave][0], sums[wave][1], lane, cnt);
            cur = nxt;
            nxt = nn;
            ok = ok_n;
        }
    }
    cnt.rxp = wave_sum_u64(cnt.rxp);
    cnt.rxb = wave_sum_u64(cnt.rxb);
    cnt.txp = wave_sum_u64(cnt.txp);
    cnt.txb = wave_sum_u64(cnt.txb);
    if (lane == 0) {
        cnts[wave][0] = cnt.rxp;
        cnts[wave][1] = cnt.rxb;
        cnts[wave][2] = cnt.txp;
        cnts[wave][3] = cnt.txb;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (threadIdx.x < 4 && a.partials) {
        unsigned long long s = 0;
#pragma unroll
        for (int w = 0; w < WPB; ++w) s += cnts[w][threadIdx.x];
        a.partials[blockIdx.x * 4 + threadIdx.x] = s;
    }
}

template <bool WIRE, int WPB, int PPW, bool PERSIST>
static int short_pipe(const EchoArgs& args, hipStream_t s, uint32_t ncu) {
    const uint32_t pairs = (args.n + 2 * kTile - 1) / (2 * kTile);
    uint32_t grid, ppw = 0;
    if (PERSIST) {
        ppw = (pairs + ncu - 1) / ncu;
        grid = (pairs + ppw - 1) / ppw;
    } else {
        grid = (pairs + WPB * PPW - 1) / (WPB * PPW);
    }
    if (grid > 32768u) return -EINVAL;
    short_pipe_kernel<WIRE, WPB, PPW, PERSIST><<<dim3(grid), dim3(WPB * 64), 0, s>>>(args, ppw);
    return 0;
}

template <bool WIRE, int WPB, bool WT, int DIAG = 0>
static int short_grid(const EchoArgs& args, hipStream_t s) {
    const uint32_t pairs = (args.n + 2 * kTile - 1) / (2 * kTile);
    const uint32_t grid = (pairs + WPB - 1) / WPB;
    if (grid > 32768u) return -EINVAL;  // partial rows in the A/B's 1 MiB workspace
    short_grid_kernel<WIRE, WPB, WT, DIAG><<<dim3(grid), dim3(WPB * 64), 0, s>>>(args);
    return 0;
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
        // 30-35: SG -- all-short batches on a non-persistent grid of WPB-wave workgroups, one tile pair per wave
        case 30: if (short_grid<false, 4, true>(args, s)) return -EINVAL; break;
        case 31: if (short_grid<false, 8, true>(args, s)) return -EINVAL; break;
        case 32: if (short_grid<false, 1, true>(args, s)) return -EINVAL; break;
        case 33: if (short_grid<false, 4, false>(args, s)) return -EINVAL; break;
        case 34: if (short_grid<false, 16, true>(args, s)) return -EINVAL; break;
        case 35: args.opts = XSK_GPU_OPT_ALL; if (short_grid<true, 4, true>(args, s)) return -EINVAL; break;
        // 36-39: SGP -- the same with a two-deep software pipeline over each wave's pairs
        case 36: if (short_pipe<false, 8, 1, true>(args, s, 2u * xsk_gpu__num_cu(device))) return -EINVAL; break;
        case 37: if (short_pipe<false, 4, 2, false>(args, s, 0)) return -EINVAL; break;
        case 38: if (short_pipe<false, 4, 4, false>(args, s, 0)) return -EINVAL; break;
        case 39: if (short_pipe<false, 8, 2, false>(args, s, 0)) return -EINVAL; break;
        // 40 / 41: diagnostics (wrong outputs): SG without the header phase / without LDS and header phase
        case 40: if (short_grid<false, 4, true, 1>(args, s)) return -EINVAL; break;
        case 41: if (short_grid<false, 4, true, 2>(args, s)) return -EINVAL; break;
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
