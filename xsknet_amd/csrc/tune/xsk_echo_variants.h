// xsk_echo_variants.h — kernels kept for the tuning sweep (tools/kbench.py, xsk_tune.hip) and their
// parity tests, not on the product path: echo_kernel5 (the previous shipped kernel: non-persistent grid,
// header sectors written at each tile's end) and echo_kernel7 (rounds + flattened row streams).
// DESIGN.md §3 has their measurements.
#pragma once

#include "xsk_echo_lab.h"

namespace xskgpu {
namespace {

template <int U, int MINW>
__global__ __launch_bounds__(kThreads, MINW) void echo_kernel5(EchoArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[kWaves][kTile * kWin];
    __shared__ __attribute__((aligned(16))) FrameMeta s_meta[kWaves][kTile];
    __shared__ uint32_t s_sum[kWaves][2][kTile];  // [ic, ip] folded row sums per frame
    __shared__ unsigned long long s_cnt[kWaves][4];

    const uint32_t wave = uniform(threadIdx.x >> 6);
    uint8_t* rows = s_hdr[wave];
    FrameMeta* meta = s_meta[wave];
    uint32_t* sums_ic = s_sum[wave][0];
    uint32_t* sums_ip = s_sum[wave][1];
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t nwaves = gridDim.x * kWaves;
    Counters cnt;
    uint32_t lane = threadIdx.x & 63u;

    for (uint32_t t = blockIdx.x * kWaves + wave; t < ntiles; t += nwaves) {
        // A wave normally runs one tile: keep the compiler from hoisting lane-derived values out of
        // this loop into VGPRs that would stay live (and cut occupancy) for the whole kernel.
        asm volatile("" : "+v"(lane));
        const uint32_t q = lane >> 4, k = lane & 15u;
        // ---- 1. descriptors (xsk_receive.c:222-223): lane i <- frame t*64+i -> LDS metadata ----------
        uint32_t nit;
        uint64_t wlo, span;
        bool short_tile;  // every frame of the tile lies within its 64-B window
        {
            const uint32_t fi = t * kTile + lane;
            u32x4 dsc = u32x4{0u, 0u, 0u, 0u};
            if (fi < a.n) dsc = *(const u32x4*)(a.descs + fi);
            const uint64_t addr = (uint64_t)dsc.x | ((uint64_t)dsc.y << 32);
            const uint32_t len = dsc.z;
            // build-added bounds check; the reference reads bytes [0,38) whenever len >= 20
            const uint64_t need = len >= 20 ? (len > 38 ? len : 38) : len;
            const bool ok = fi < a.n && len <= kMaxLen && addr <= a.umem_size && need <= a.umem_size - addr;
            const bool parse = ok && len >= 20;
            const uint64_t a16 = addr & ~15ull;
            const uint32_t off = (uint32_t)addr & 15u;
            const uint32_t rowhi = parse ? off + len : 0u;
            const uint32_t win = parse ? (uint32_t)min(a.umem_size - a16, (uint64_t)kWin) : 0u;
            const uint32_t lim = max(rowhi, win);
            nit = (lim + 255u) >> 8;
            short_tile = __ballot(lim > (uint32_t)kWin) == 0ull;
            if (short_tile) {  // short tiles use per-frame 64-bit loads: no window needed
                wlo = 0;
                span = ~0ull;
            } else {
                wlo = wave_min_u64(nit ? a16 : ~0ull);
                span = wave_max_u64(nit ? a16 + lim : 0ull) - wlo;
            }
            FrameMeta m;
            m.rel = nit && !short_tile ? (uint32_t)(a16 - wlo) : 0u;
            m.rowhi = rowhi;
            m.lim = lim;
            m.packed = off | ((parse ? off + min(len, 34u) : 0u) << 8) | ((ok ? 1u : 0u) << 16) |
                       ((parse ? 2u : 0u) << 16);
            m.nit = nit;
            m.addr_lo = dsc.x;
            m.addr_hi = dsc.y;
            m.len = len;
            meta[lane] = m;
        }

        // ---- 2. stream every row byte once; windows -> LDS rows, row sums -> LDS ---------------------
        if (__ballot(nit != 0u) != 0ull) {
            __builtin_amdgcn_wave_barrier();
            const bool fast = span < 0x80000000ull;  // wave-uniform
            WinLoader ld;
            ld.r = __builtin_amdgcn_make_buffer_rsrc((void*)(a.umem + (fast ? wlo : 0ull)), (short)0,
                                                     fast ? (int)((span + 15u) & ~15ull) : 0, kRsrcFlags);
            if (short_tile) {
                // ---- short tile (every frame within its 64-B window): 4 lanes per frame, 16 frames per
                // wave-load (all four issued before the first is used), quad DPP reduction
                const uint32_t kk = lane & 3u, ro = 16u * kk;
                u32x4 x[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const FrameMeta& fm = meta[(uint32_t)r * 16u + (lane >> 2)];
                    const uint64_t fa = (((uint64_t)fm.addr_hi) << 32) | (uint64_t)fm.addr_lo;
                    const bool in = ro < fm.lim;
                    x[r] = __builtin_nontemporal_load((const u32x4*)(a.umem + (in ? (fa & ~15ull) + ro : 0ull)));
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                    const FrameMeta& fm = meta[f];
                    const uint32_t f_packed = fm.packed;
                    const u32x4 v = ro < fm.lim ? x[r] : u32x4{0u, 0u, 0u, 0u};
                    *(u32x4*)(rows + f * kWin + ro) = v;
                    const int f_off = (int)(f_packed & 0xFFu), f_iphi = (int)((f_packed >> 8) & 0xFFu);
                    uint32_t rip = fold64(sum_range(v, (int)ro, f_off + 14, f_iphi));
                    uint32_t ric = fold64(sum_range(v, (int)ro, f_off + 34, (int)fm.rowhi));
                    rip += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rip, 0xB1, 0xF, 0xF, false);  // quad [1,0,3,2]
                    ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0xB1, 0xF, 0xF, false);
                    rip += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rip, 0x4E, 0xF, 0xF, false);  // quad [2,3,0,1]
                    ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x4E, 0xF, 0xF, false);
                    if (kk == 0u) {
                        sums_ic[f] = ric;
                        sums_ip[f] = rip;
                    }
                }
            } else
            for (uint32_t s = 0; s < 16; ++s) {
                const uint32_t f = 4u * s + q;
                const FrameMeta& fm = meta[f];  // broadcast read: one entry per 16-lane row
                const uint32_t f_nit = fm.nit;
                const uint32_t ns = max(max(rdlane(f_nit, 0), rdlane(f_nit, 16)), max(rdlane(f_nit, 32), rdlane(f_nit, 48)));
                if (ns == 0) continue;
                const uint32_t f_rowhi = fm.rowhi, f_lim = fm.lim, f_packed = fm.packed;
                const uint32_t f_off = f_packed & 0xFFu, f_iphi = (f_packed >> 8) & 0xFFu;
                RowSums rs;
                if (fast) {
                    ld.rel = fm.rel;
                    stream_frame<U>(ld, ns, f_rowhi, f_lim, f_off, f_iphi, k, rows + f * kWin, rs);
                } else {  // frames of one tile more than 2 GiB apart (never in AF_XDP layouts)
                    FarLoader fl;
                    fl.fbase = a.umem + (f_nit ? ((((uint64_t)fm.addr_hi) << 32) | (uint64_t)fm.addr_lo) & ~15ull : 0ull);
                    stream_frame<U>(fl, ns, f_rowhi, f_lim, f_off, f_iphi, k, rows + f * kWin, rs);
                }
                const uint32_t ric = row_sum_dpp(fold64(rs.ic));
                const uint32_t rip = row_sum_dpp(fold64(rs.ip));
                if (k == 15u) {
                    sums_ic[f] = ric;
                    sums_ip[f] = rip;
                }
            }
        }

        // ---- 3. header phase (lane = frame) ----------------------------------------------------------
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const FrameMeta m = meta[lane];
        const uint32_t fi = t * kTile + lane;
        const uint64_t addr = (uint64_t)m.addr_lo | ((uint64_t)m.addr_hi << 32);
        const bool ok = (m.packed >> 16) & 1u, parse = (m.packed >> 17) & 1u;
        const uint32_t ic_raw = m.nit ? sums_ic[lane] : 0u;
        const uint32_t ip_raw = m.nit ? sums_ip[lane] : 0u;
        const bool wb = header_phase5(a, rows + lane * kWin, ip_raw, ic_raw, addr, m.len, fi < a.n, ok, parse, fi, cnt);

        // ---- 4. patched windows -> UMEM: 16 frames x 64 B per wave-store, whole 64-B sectors ---------
        const uint64_t wbm = __ballot(wb);
        if (wbm) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                const uint32_t kk = lane & 3u;
                if ((wbm >> f) & 1ull) {
                    const uint64_t fa = (uint64_t)meta[f].addr_lo | ((uint64_t)meta[f].addr_hi << 32);
                    const u32x4 w = *(const u32x4*)(rows + f * kWin + 16u * kk);
                    *(u32x4*)(a.umem + fa + 16u * kk) = w;
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // LDS rows are rewritten by the next tile
    }
    store_partials(a, cnt, s_cnt, wave, lane);
}



// ================================================================================================
// Round kernel with flattened row streams (echo_kernel7).  Same rounds as echo_kernel6, but a row's 16
// frames are streamed back to back: global step g of row q is row-load j of frame 4m+q where m is the
// last row frame whose exclusive prefix of row-load counts is <= g (a ballot + popcount per step),
// so U row-loads stay in flight per lane across frame boundaries instead of draining at every frame.
// A frame's ICMP sum is reduced (row DPP) at the step that holds its last row-load; the IPv4 header
// sum comes from the LDS window in the header phase.  Descriptors of the round's tiles are loaded up
// front.
// ================================================================================================
template <int U, bool FAST>
__device__ __forceinline__ void stream_tile_flat(const EchoArgs& a, __amdgpu_buffer_rsrc_t rsrc,
                                                 const FrameMeta6* meta, uint8_t* rows, uint32_t* sums_ic,
                                                 uint32_t nit_own, uint32_t lane) {
    const uint32_t q = lane >> 4, k = lane & 15u;
    const uint32_t nitk = (uint32_t)__shfl((int)nit_own, (int)(4u * k + q), 64);  // row frame k = frame 4k+q
    const uint32_t incl = row_sum_dpp(nitk);                                      // inclusive row prefix
    const uint32_t P = incl - nitk;
    const uint32_t total = max(max(rdlane(incl, 15), rdlane(incl, 31)), max(rdlane(incl, 47), rdlane(incl, 63)));
    uint64_t ic = 0;
    for (uint32_t g0 = 0; g0 < total; g0 += U) {
        u32x4 v[U];
        uint32_t sf[U], sj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t g = g0 + (uint32_t)u;
            const uint64_t M = __ballot(P <= g);
            const uint32_t m = (uint32_t)__popc((uint32_t)(M >> (16u * q)) & 0xFFFFu) - 1u;
            const uint32_t Pm = (uint32_t)__shfl((int)P, (int)(16u * q + m), 64);
            const uint32_t f = 4u * m + q, j = g - Pm;
            const FrameMeta6 fm = meta[f];
            const uint32_t ro = 256u * j + 16u * k;
            const bool in = ro < fm.lim;
            if (FAST) {
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(in ? fm.rel + ro : 0x80000000u), 0, kAuxNT);
            } else {
                const u32x4 y = __builtin_nontemporal_load((const u32x4*)(a.umem + (in ? meta6_a16(fm) + ro : 0ull)));
                v[u] = in ? y : u32x4{0u, 0u, 0u, 0u};
            }
            sf[u] = f;
            sj[u] = j;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t f = sf[u], j = sj[u];
            const FrameMeta6 fm = meta[f];
            const uint32_t ro = 256u * j + 16u * k;
            const u32x4 x = v[u];
            const uint32_t f_off = fm.packed & 0xFFu;
            if (j == 0u) {
                if (k < 4u) *(u32x4*)(rows + f * kWin + ro) = x;  // the frame's 64-B header window
                ic += sum_range(x, (int)ro, (int)f_off + 34, (int)fm.rowhi);
            } else {
                const int nb = (int)(fm.rowhi - min(ro, fm.rowhi));  // frame bytes in this block
                u32x4 y = x;
                y.x &= dw_mask(nb);
                y.y &= dw_mask(nb - 4);
                y.z &= dw_mask(nb - 8);
                y.w &= dw_mask(nb - 12);
                ic += sum_dw(y);
            }
            const bool last = 256u * j < fm.lim && 256u * (j + 1u) >= fm.lim;  // row-uniform
            if (__ballot(last) != 0ull) {
                const uint32_t r = row_sum_dpp(fold64(ic));
                if (last && k == 15u) sums_ic[f] = r;
                if (last) ic = 0;
            }
        }
    }
}

template <int U, int TPW>
__global__ __launch_bounds__(kThreads6, 1) void echo_kernel7(EchoArgs a, uint32_t tiles_per_wg) {
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[kWaves6][TPW][kTile * kWin];  // 128 KiB at TPW 2
    __shared__ __attribute__((aligned(16))) FrameMeta6 s_meta[kWaves6][kTile];          // 16 KiB
    __shared__ uint32_t s_sum[kWaves6][kTile];                                           // 4 KiB
    __shared__ unsigned long long s_cnt[kWaves6][4];

    const uint32_t wave = uniform(threadIdx.x >> 6);
    FrameMeta6* meta = s_meta[wave];
    uint32_t* sums_ic = s_sum[wave];
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t t_begin = blockIdx.x * tiles_per_wg;
    const uint32_t t_end = min(ntiles, t_begin + tiles_per_wg);
    constexpr uint32_t kRound = (uint32_t)kWaves6 * TPW;
    Counters cnt;
    uint32_t lane = threadIdx.x & 63u;

    for (uint32_t r0 = t_begin; r0 < t_end; r0 += kRound) {  // workgroup-uniform
        u32x4 rec[TPW], dsc[TPW];
        uint32_t verd[TPW];
        uint64_t wbm[TPW];
#pragma unroll
        for (int i = 0; i < TPW; ++i) {  // descriptors of every tile of the round (xsk_receive.c:222-223)
            const uint32_t fi = (r0 + (uint32_t)i * kWaves6 + wave) * kTile + lane;
            dsc[i] = u32x4{0u, 0u, 0u, 0u};
            if (fi < a.n) dsc[i] = *(const u32x4*)(a.descs + fi);
        }
        // ================= read phase =================
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const uint32_t t = r0 + (uint32_t)i * kWaves6 + wave;
            wbm[i] = 0ull;
            rec[i] = u32x4{0u, 0u, 0u, 0u};
            verd[i] = 0u;
            if (t >= t_end) continue;  // wave-uniform
            asm volatile("" : "+v"(lane));
            uint8_t* rows = s_hdr[wave][i];
            const uint32_t fi = t * kTile + lane;
            const uint64_t addr = (uint64_t)dsc[i].x | ((uint64_t)dsc[i].y << 32);
            const uint32_t len = dsc[i].z;
            const uint64_t need = len >= 20 ? (len > 38 ? len : 38) : len;
            const bool ok = fi < a.n && len <= kMaxLen && addr <= a.umem_size && need <= a.umem_size - addr;
            const bool parse = ok && len >= 20;
            const uint64_t a16 = addr & ~15ull;
            const uint32_t off = (uint32_t)addr & 15u;
            const uint32_t rowhi = parse ? off + len : 0u;
            const uint32_t win = parse ? (uint32_t)min(a.umem_size - a16, (uint64_t)kWin) : 0u;
            const uint32_t lim = max(rowhi, win);
            const uint32_t nit = (lim + 255u) >> 8;
            const bool short_tile = __ballot(lim > (uint32_t)kWin) == 0ull;
            uint64_t wlo = 0, span = ~0ull;
            if (!short_tile) {
                wlo = wave_min_u64(nit ? a16 : ~0ull);
                span = wave_max_u64(nit ? a16 + lim : 0ull) - wlo;
            }
            const bool fast = !short_tile && span < 0x80000000ull;  // wave-uniform
            {
                FrameMeta6 m;
                m.rel = fast ? (nit ? (uint32_t)(a16 - wlo) : 0u) : (uint32_t)(a16 >> 4);
                m.rowhi = rowhi;
                m.lim = lim;
                m.packed = off | ((ok ? 1u : 0u) << 16) | ((parse ? 2u : 0u) << 16) | ((uint32_t)(a16 >> 36) << 20);
                meta[lane] = m;
            }
            if (__ballot(nit != 0u) != 0ull) {
                __builtin_amdgcn_wave_barrier();
                if (short_tile) {
                    // every frame within its 64-B window: 4 lanes per frame, 16 frames per wave-load
                    const uint32_t kk = lane & 3u, ro = 16u * kk;
                    u32x4 x[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const FrameMeta6& fm = meta[(uint32_t)r * 16u + (lane >> 2)];
                        const bool in = ro < fm.lim;
                        x[r] = __builtin_nontemporal_load((const u32x4*)(a.umem + (in ? meta6_a16(fm) + ro : 0ull)));
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                        const FrameMeta6& fm = meta[f];
                        const u32x4 v = ro < fm.lim ? x[r] : u32x4{0u, 0u, 0u, 0u};
                        *(u32x4*)(rows + f * kWin + ro) = v;
                        const int f_off = (int)(fm.packed & 0xFFu);
                        uint32_t ric = fold64(sum_range(v, (int)ro, f_off + 34, (int)fm.rowhi));
                        ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0xB1, 0xF, 0xF, false);
                        ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x4E, 0xF, 0xF, false);
                        if (kk == 0u) sums_ic[f] = ric;
                    }
                } else {
                    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
                        (void*)(a.umem + (fast ? wlo : 0ull)), (short)0, fast ? (int)((span + 15u) & ~15ull) : 0,
                        kRsrcFlags);
                    if (fast) stream_tile_flat<U, true>(a, rsrc, meta, rows, sums_ic, nit, lane);
                    else stream_tile_flat<U, false>(a, rsrc, meta, rows, sums_ic, nit, lane);
                }
            }

            // ---- header phase (lane = frame); the window stays patched in LDS --------------------------
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            const uint32_t ic_raw = nit ? sums_ic[lane] : 0u;
            const bool wb = header_phase5<true, true>(a, rows + lane * kWin, 0u, ic_raw, addr, len, fi < a.n, ok,
                                                      parse, fi, cnt, &rec[i], &verd[i]);
            wbm[i] = __ballot(wb);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();  // meta/sums are rewritten by the next tile
        }

        // ================= write phase: every wave of the workgroup has finished reading =================
        __syncthreads();
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const uint32_t t = r0 + (uint32_t)i * kWaves6 + wave;
            if (t >= t_end) continue;
            const uint8_t* rows = s_hdr[wave][i];
            if (wbm[i]) {  // patched windows: 16 frames x 64 B per wave-store, whole 64-B sectors
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                    const uint32_t kk = lane & 3u;
                    const uint32_t flo = (uint32_t)__shfl((int)dsc[i].x, (int)f, 64);
                    const uint32_t fhi = (uint32_t)__shfl((int)dsc[i].y, (int)f, 64);
                    if ((wbm[i] >> f) & 1ull) {
                        const uint64_t fa = (uint64_t)flo | ((uint64_t)fhi << 32);
                        *(u32x4*)(a.umem + fa + 16u * kk) = *(const u32x4*)(rows + f * kWin + 16u * kk);
                    }
                }
            }
            const uint32_t fi = t * kTile + lane;
            if (fi < a.n) {
                if (a.recs) ((u32x4*)a.recs)[fi] = rec[i];
                if (a.verdicts) a.verdicts[fi] = (uint8_t)verd[i];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // LDS rows are rewritten by the next round
    }
    store_partials<kWaves6>(a, cnt, s_cnt, wave, lane);
}


}  // namespace
}  // namespace xskgpu
