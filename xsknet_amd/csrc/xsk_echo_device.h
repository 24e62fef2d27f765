// xsk_echo_device.h — device code of the gfx950 (MI355X / CDNA4) ICMP-echo transform: the round kernel
// the product launches (xsk_echo.hip) and whose body the low-latency resident kernel runs (xsk_lowlat.hip).
// Only the shipped parameter set and the switches an in-process A/B still needs live here (tune/xsk_tune_product.hip
// instantiates those for tools/abbench.py); the alternatives measured and lost in rounds 1-4 are recorded with their A/B
// logs in DESIGN.md §4 and in git history.
//
// Replaces, for a whole batch of AF_XDP descriptors at once, the per-frame call
//   process_packet()   /root/reference/src/lib/xsk_receive.c:113-190   (gates, field swap, type 8->0,
//   csum_replace2()    /root/reference/src/lib/xsk_receive.c:101-111    RFC 1624 incremental update)
// and the counter updates of the batch loop at xsk_receive.c:171-172,229,233.  No MFMA: the op is
// integer byte arithmetic and HBM bound.
#pragma once

#include "../../include/xsk_gpu.h"
#include "xsk_echo_kernels.h"

namespace xskgpu {
namespace {

constexpr int kTile = XSK_GPU_TILE_FRAMES;  // frames per wave tile (= RX_BATCH_SIZE, xsk_utils.h:8)
constexpr int kWin = 64;                    // header window [a16, a16 + 64), reference and wire mode
constexpr uint32_t kMaxLen = 1u << 30;      // build-added descriptor sanity bound (XSK_GPU_MAX_LEN)
constexpr int kWaves6 = 16;                 // waves per workgroup (one workgroup per CU)
constexpr int kThreads6 = kWaves6 * 64;     // 1024
constexpr int kU = 4;                       // 256-B row-loads in flight per lane in the row streams
constexpr int kUR = 6;                      // the same for the launched kernel's ranked (ragged-tile) streams:
                                            // c4 185.4 -> 182.6 us, c3 / p98 unchanged (profiles/r03/ab_ranked_u6_u8_*)
constexpr int kRefTPW = 2;                  // reference mode: tiles per wave per round (2048 frames per CU)
constexpr int kRefHeavy = 512;              // SYNC 2's heavy-frame threshold (bytes)
constexpr int kRefSlack = 2;                // reference mode: a heavy wave writes once all but 2 waves have read the
                                            // round (SLACK): c4 181.4 -> 176.5 us, c3 274.0 -> 272.9 in-process A/B
                                            // (profiles/r03/ab_slack_confirm_*.log)

struct EchoArgs {
    uint8_t* umem;
    uint64_t umem_size;
    const xsk_gpu_desc* descs;
    uint32_t n;
    uint8_t* verdicts;
    xsk_gpu_rec* recs;
    unsigned long long* partials;  // [gridDim.x][4]: rx_packets, rx_bytes, tx_packets, tx_bytes
    uint32_t opts = 0;             // XSK_GPU_OPT_* (wire-mode kernels only)
    // every workgroup adds its counters straight into the caller's stats (no fold launch): device-scope
    // atomics, or -- stats_plain, a one-workgroup launch on a zeroed per-call slot of mapped host memory --
    // plain stores (no read across PCIe)
    unsigned long long* stats_direct = nullptr;  // &stats->rx_packets (4 consecutive u64)
    uint32_t stats_plain = 0;
    // SUBT kernels only: live frames per 64-lane tile (a multiple of 4, <= 64); tile t holds frames
    // [t * tile_live, t * tile_live + tile_live) in lanes 0 .. tile_live - 1 -- a small batch spreads over
    // more waves (the low-latency kernel: a 64-frame batch is 16 tiles of 4 frames, one per wave)
    uint32_t tile_live = 64;
    // TRACE kernels only: wave 0's wall clock at the body's phase boundaries (diagnostics, 6 x u64)
    unsigned long long* trace = nullptr;
    // DLDS kernels only: nonzero = the batch's descriptors (n <= 64) are already in the LDS (Echo6Smem::desc)
    uint32_t desc_in_lds = 0;
};

// Buffer-resource word 3 for gfx950 raw buffers (cdna_hip_programming.md §5.5 T8).
constexpr int kRsrcFlags = 0x00020000;
constexpr int kAuxNT = 2;    // nontemporal: payload bytes are read exactly once
constexpr int kAuxSC1 = 16;  // sc1 (gfx940+ cache policy): write-through past the XCD's L2

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);  // keep it unsigned: no sign-extension
}

__device__ __forceinline__ uint32_t row_sum_dpp(uint32_t x) {  // lane 15 of each 16-lane row: row total
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    return x;
}

// Mask keeping the low nb bytes of a dword (nb <= 0: none, nb >= 4: all).
__device__ __forceinline__ uint32_t dw_mask(int nb) {
    return nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
}

struct Counters {
    uint64_t rxp = 0, rxb = 0, txp = 0, txb = 0;
};

// Counters: wave -> workgroup -> the caller's stats (device atomics or a plain store) or one partial row
// per workgroup.
__device__ __forceinline__ void store_counters(const EchoArgs& a, Counters c, unsigned long long (*s_cnt)[4],
                                               uint32_t wave, uint32_t lane) {
    if (!a.partials && !a.stats_direct) return;
    c.rxp = wave_sum_u64(c.rxp);
    c.rxb = wave_sum_u64(c.rxb);
    c.txp = wave_sum_u64(c.txp);
    c.txb = wave_sum_u64(c.txb);
    if (lane == 0) {
        s_cnt[wave][0] = c.rxp;
        s_cnt[wave][1] = c.rxb;
        s_cnt[wave][2] = c.txp;
        s_cnt[wave][3] = c.txb;
    }
    // the rows travel through LDS only: wait for the LDS writes, then meet -- not __syncthreads(), whose
    // workgroup-scope release would first wait for every outstanding global store (a PCIe round trip
    // when the frames live in mapped host memory)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (threadIdx.x < 4) {
        unsigned long long s = 0;
#pragma unroll
        for (int w = 0; w < kWaves6; ++w) s += s_cnt[w][threadIdx.x];
        if (a.stats_direct && a.stats_plain) a.stats_direct[threadIdx.x] = s;  // sole writer of a zeroed slot
        else if (a.stats_direct)  // every workgroup adds its own: non-returning device-scope atomics
            __hip_atomic_fetch_add(a.stats_direct + threadIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else a.partials[blockIdx.x * 4 + threadIdx.x] = s;
    }
}

__device__ __forceinline__ uint32_t max_nit_lane(uint32_t x) {  // wave max (every lane gets it)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
    return x;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {  // uniform result (SGPRs)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = __shfl_xor(x, o, 64);
        x = y < x ? y : x;
    }
    return ((uint64_t)uniform((uint32_t)(x >> 32)) << 32) | (uint64_t)uniform((uint32_t)x);
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t y = __shfl_xor(x, o, 64);
        x = y > x ? y : x;
    }
    return ((uint64_t)uniform((uint32_t)(x >> 32)) << 32) | (uint64_t)uniform((uint32_t)x);
}

// Stream loaders: `in` = the block lies (at least partly) inside the lane's frame.
struct WinLoader {  // tile-wide buffer window; out-of-range offsets return zeros, no memory access
    __amdgpu_buffer_rsrc_t r;
    uint32_t rel;  // frame's a16 relative to the window base
    __device__ __forceinline__ u32x4 load(uint32_t ro, bool in) const {
        return __builtin_amdgcn_raw_buffer_load_b128(r, (int)(in ? rel + ro : 0x80000000u), 0, kAuxNT);
    }
};
struct FarLoader {  // 64-bit addresses; lanes past the frame re-read its first block, then select zeros
    const uint8_t* fbase;
    __device__ __forceinline__ u32x4 load(uint32_t ro, bool in) const {
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)(fbase + (in ? ro : 0u)));
        return in ? v : u32x4{0u, 0u, 0u, 0u};
    }
};

// ================================================================================================
// Row streams.  One read of every byte: the payload is streamed by 16-lane DPP rows (row q of step s
// owns frame 4s+q, 256-B row-loads), starting at row byte 0, so the first four (wire: eight) lanes of a
// frame's first row-load carry its header window, which they drop into the frame's LDS row -- no
// separate header read.  Each frame's loads span max(frame end, window end) row bytes; the stream sums
// the ICMP bytes (row [off + 34, rowhi), or [128, rowhi) in wire mode), the header phase the rest.
// ================================================================================================
// One frame's row sums, both in the absolute-alignment domain (64-bit sums of LE dwords):
//   ic: ICMP bytes, row [off + 34, rowhi)      ip: IPv4 header bytes, row [off + 14, ip_hi)
struct RowSums {
    uint64_t ic = 0, ip = 0;
};

__device__ __forceinline__ uint64_t sum_dw(u32x4 x) {
    return (uint64_t)x.x + (uint64_t)x.y + (uint64_t)x.z + (uint64_t)x.w;
}
// acc + the eight 16-bit halves of x: one v_dot2_u32_u16 per dword (against 1,1) instead of a 64-bit add
// pair.  Sum of halves == sum of dwords mod 0xFFFF and both are zero only for all-zero data, so the folded
// RFC 1071 result is the same; callers flush acc into their 64-bit sum every few blocks (no overflow).
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t dot2_halves(uint32_t v, uint32_t acc) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, v), u16x2_t{1, 1}, acc, false);
}
__device__ __forceinline__ uint32_t sum_halves(u32x4 x, uint32_t acc) {
    return dot2_halves(x.w, dot2_halves(x.z, dot2_halves(x.y, dot2_halves(x.x, acc))));
}
// Byte-keep masks of block [ro, ro+16) for the range [lo, hi) (keep_bytes of all-ones per dword).
__device__ __forceinline__ u32x4 range_mask(int ro, int lo, int hi) {
    return u32x4{keep_bytes(~0u, ro, lo, hi), keep_bytes(~0u, ro + 4, lo, hi), keep_bytes(~0u, ro + 8, lo, hi),
                 keep_bytes(~0u, ro + 12, lo, hi)};
}
// sum_range() as a sum of 16-bit halves (< 2^20; no 64-bit adds, no fold needed before a DPP reduction)
__device__ __forceinline__ uint32_t sum_range_h(u32x4 x, int ro, int lo, int hi) {
    uint32_t acc = dot2_halves(keep_bytes(x.x, ro, lo, hi), 0u);
    acc = dot2_halves(keep_bytes(x.y, ro + 4, lo, hi), acc);
    acc = dot2_halves(keep_bytes(x.z, ro + 8, lo, hi), acc);
    return dot2_halves(keep_bytes(x.w, ro + 12, lo, hi), acc);
}
// sum of the bytes of block x (row bytes [ro, ro+16)) that lie in [lo, hi)
__device__ __forceinline__ uint64_t sum_range(u32x4 x, int ro, int lo, int hi) {
    return (uint64_t)keep_bytes(x.x, ro, lo, hi) + (uint64_t)keep_bytes(x.y, ro + 4, lo, hi) +
           (uint64_t)keep_bytes(x.z, ro + 8, lo, hi) + (uint64_t)keep_bytes(x.w, ro + 12, lo, hi);
}

// 16-B per-frame stream metadata of a tile, kept in LDS so that the row streams of step s read frame
// 4s+q's entry by broadcast LDS reads (the header phase keeps addr/len in the owning lane's VGPRs).
struct FrameMeta6 {
    uint32_t rel;     // a16 - window base (fast tiles); a16 >> 4 (short and far tiles)
    uint32_t rowhi;   // frame end, row coordinates (0 unless parsed)
    uint32_t lim;     // row bytes to load: max(rowhi, window bytes in the UMEM)
    uint32_t packed;  // off | iphi << 8 | flags << 16 (1 ok, 2 parse) | (a16 >> 36) << 20
};
__device__ __forceinline__ uint64_t meta6_a16(const FrameMeta6& m) {
    return ((uint64_t)(m.packed >> 20) << 36) | ((uint64_t)m.rel << 4);
}

// One frame's row stream: row-loads j = 0 .. ns-1 (lane k takes row bytes [256 j + 16 k, +16)).  The
// first row-load carries the window: lanes 0-3 drop it into the frame's LDS row and every lane sums its
// bytes by exact range (ICMP [off+34, rowhi), IPv4 header [off+14, iphi)); later blocks only need the
// frame-end mask.
template <int U, class L, bool D2>
__device__ __forceinline__ void stream_frame(const L& ld, uint32_t ns, uint32_t f_rowhi, uint32_t f_lim,
                                             uint32_t f_off, uint32_t f_iphi, uint32_t k, uint8_t* hdr_row,
                                             RowSums& rs) {
    const int ic_lo = (int)f_off + 34;
    if (ns == 1u) {
        const uint32_t ro = 16u * k;
        const u32x4 x = ld.load(ro, ro < f_lim);
        if (k < 4u) *(u32x4*)(hdr_row + ro) = x;
        rs.ip += k < 4u ? sum_range(x, (int)ro, (int)f_off + 14, (int)f_iphi) : 0ull;
        rs.ic += sum_range(x, (int)ro, ic_lo, (int)f_rowhi);
        return;
    }
    for (uint32_t j0 = 0; j0 < ns; j0 += U) {
        u32x4 v[U];
        uint32_t h = 0;  // D2: halves of this batch's blocks
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t ro = 256u * (j0 + (uint32_t)u) + 16u * k;
            v[u] = ld.load(ro, ro < f_lim);  // past the frame: zeros, no memory access
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t ro = 256u * (j0 + (uint32_t)u) + 16u * k;
            const u32x4 x = v[u];
            if (u == 0 && j0 == 0u) {
                if (k < 4u) *(u32x4*)(hdr_row + ro) = x;
                rs.ip += k < 4u ? sum_range(x, (int)ro, (int)f_off + 14, (int)f_iphi) : 0ull;
                rs.ic += sum_range(x, (int)ro, ic_lo, (int)f_rowhi);
            } else {
                const int nb = (int)(f_rowhi - min(ro, f_rowhi));      // frame bytes in this block
                if (__ballot(nb > 0 && nb < 16) != 0ull) {             // a block that ends a frame
                    u32x4 y = x;
                    y.x &= dw_mask(nb);
                    y.y &= dw_mask(nb - 4);
                    y.z &= dw_mask(nb - 8);
                    y.w &= dw_mask(nb - 12);
                    if (D2) h = sum_halves(y, h);
                    else rs.ic += sum_dw(y);
                } else if (D2) {
                    h = sum_halves(x, h);
                } else {
                    rs.ic += sum_dw(x);  // whole block in the frame, or zeros past it
                }
            }
        }
        if (D2) rs.ic += h;
    }
}

// Sorted, step-packed row streams (ragged tiles).  The tile's frames are ranked by their row-load count
// (ascending, ties by index); step s streams ranked frames 4s..4s+3, one per 16-lane row, so the four
// frames of a step need about the same number of row-loads (ragged batches waste fewer lanes), and each
// batch of U row-loads is packed across consecutive steps by a wave-uniform cursor (short frames share
// one round trip instead of paying one per step).  The IPv4 header sum is taken in the header phase from
// the LDS window.  SKM: tiles of frames <= 7 row-loads are ranked by counting (one ballot per value), and
// blocks past row 0 are masked only where one of the slot's frames ends.
template <int U, bool FAST, bool SKM, bool PRIO = false>
__device__ __forceinline__ void stream_tile_sorted(const EchoArgs& a, __amdgpu_buffer_rsrc_t rsrc,
                                                   const FrameMeta6* meta, uint32_t* sort, uint8_t* rows,
                                                   uint32_t* sums_ic, uint32_t nit_own, uint32_t lane) {
    constexpr uint32_t kRowW = (uint32_t)kWin;  // LDS row (window) bytes
    const uint32_t q = lane >> 4, k = lane & 15u;
    uint32_t rank = 0;
    if (SKM && __ballot(nit_own > 7u) == 0ull) {
        // counting rank: per value v one ballot; rank = lanes with fewer row-loads + lanes below with as
        // many (the same order as the compare loop below)
        uint32_t below = 0;
#pragma unroll
        for (uint32_t v = 0; v < 8u; ++v) {
            const uint64_t bv = __ballot(nit_own == v);
            const uint32_t cv = (uint32_t)__popcll(bv);
            const uint32_t mb = __builtin_amdgcn_mbcnt_hi((uint32_t)(bv >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bv, 0u));
            if (nit_own == v) rank = below + mb;
            below += cv;
        }
    } else {
        for (uint32_t j = 0; j < 64u; ++j) {
            const uint32_t nj = rdlane(nit_own, j);
            rank += (nj < nit_own || (nj == nit_own && j < lane)) ? 1u : 0u;
        }
    }
    sort[rank] = lane;                                    // sort[0..63]: frame of rank r
    if ((rank & 3u) == 3u) sort[64u + (rank >> 2)] = nit_own;  // sort[64 + s]: row-loads of step s
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const uint32_t stepns = sort[64u + (lane & 15u)];     // lane s (< 16): row-loads of step s
    uint32_t s = 0, j = 0;
    while (s < 16u && rdlane(stepns, s) == 0u) ++s;
    uint32_t cur = 16u, cur_f = 0u;
    uint64_t ic = 0;
    uint32_t cs = 16u, cf = 0u, crel = 0u, clim = 0u, crowhi = 0u, coff = 0u;  // metadata of step cs (per row)
    uint64_t ca16 = 0;
    while (s < 16u) {
        u32x4 v[U];
        uint32_t us[U], uj[U], uf[U], urowhi[U], ulim[U], uoff[U];
        // PRIO (the launched kernel since round 3): the batch's address work and loads ahead of the other waves' VALU
        // on the SIMD -- c4 185.5 -> 183.5 us, c3 274.7 -> 273.7, c2 35.1 -> 34.8 (profiles/r03/ab_stream_prio_*.log)
        if (PRIO) __builtin_amdgcn_s_setprio(2);
#pragma unroll
        for (int u = 0; u < U; ++u) {  // wave-uniform slot assignment
            us[u] = s;
            uj[u] = j;
            if (s < 16u) {
                if (++j >= rdlane(stepns, s)) {
                    ++s;
                    j = 0;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = u32x4{0u, 0u, 0u, 0u};
            if (us[u] < 16u && us[u] != cs) {  // uniform: this slot starts a new step -> its rows' metadata
                cs = us[u];
                cf = sort[4u * cs + q];
                const FrameMeta6 fm = meta[cf];
                crel = fm.rel;
                clim = fm.lim;
                crowhi = fm.rowhi;
                coff = fm.packed & 0xFFu;
                if (!FAST) ca16 = meta6_a16(fm);
            }
            uf[u] = cf;
            urowhi[u] = crowhi;
            ulim[u] = clim;
            uoff[u] = coff;
            if (us[u] < 16u) {
                const uint32_t ro = 256u * uj[u] + 16u * k;
                const bool in = ro < clim;
                if (FAST) {
                    v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(in ? crel + ro : 0x80000000u), 0, kAuxNT);
                } else {
                    if (in) v[u] = __builtin_nontemporal_load((const u32x4*)(a.umem + ca16 + ro));
                }
            }
        }
        if (PRIO) __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (us[u] >= 16u) continue;  // uniform
            if (us[u] != cur) {          // uniform: a new step begins in this slot
                if (cur < 16u) {
                    const uint32_t r = row_sum_dpp(fold64(ic));
                    if (k == 15u) sums_ic[cur_f] = r;
                }
                cur = us[u];
                cur_f = uf[u];
                ic = 0;
            }
            const uint32_t ro = 256u * uj[u] + 16u * k;
            const u32x4 x = v[u];
            if (uj[u] == 0u) {
                if (k < kRowW / 16u && ulim[u]) *(u32x4*)(rows + uf[u] * kRowW + ro) = x;  // the header window
                ic += sum_range(x, (int)ro, (int)uoff[u] + 34, (int)urowhi[u]);
            } else {
                const int nb = (int)(urowhi[u] - min(ro, urowhi[u]));
                u32x4 y = x;
                // SKM: blocks past row 0 are whole (nb >= 16) or zeros (not loaded) unless one of the slot's
                // frames ends inside it -- mask only then (wave-uniform test, as in stream_frame)
                if (!SKM || __ballot(nb > 0 && nb < 16) != 0ull) {
                    y.x &= dw_mask(nb);
                    y.y &= dw_mask(nb - 4);
                    y.z &= dw_mask(nb - 8);
                    y.w &= dw_mask(nb - 12);
                }
                ic += sum_dw(y);
            }
        }
    }
    if (cur < 16u) {
        const uint32_t r = row_sum_dpp(fold64(ic));
        if (k == 15u) sums_ic[cur_f] = r;
    }
}

// Uniform long tiles: every frame of the tile parsed, at the same 16-B offset and with the same end, so
// the ICMP byte range [lo, hi) = [off + 34, off + len) is the same in every row.  A lane's byte masks are
// then the same for every step: computed once per tile for the first and the last row-load (the only blocks
// the range can cut; the others are whole or, past `lim`, not loaded), and a step costs its loads, one
// v_dot2_u32_u16 per dword, two masks and the row reduction.  The sums are plain 32-bit sums of 16-bit halves
// (< 2^32 for frames <= 64 KiB: 257 blocks x 8 halves x 65535 x 16 lanes); the IPv4 header sum comes from the
// window in the header phase.
template <int U, bool SPLIT = false, bool PRIO = false>
__device__ __forceinline__ void stream_tile_uniform(__amdgpu_buffer_rsrc_t rsrc, const FrameMeta6* meta, uint8_t* rows,
                                                    uint32_t* sums_ic, uint32_t ns, uint32_t lo, uint32_t hi,
                                                    uint32_t lane) {
    constexpr uint32_t kRowW = (uint32_t)kWin;
    const uint32_t q = lane >> 4, k = lane & 15u;
    const u32x4 mf = range_mask((int)(16u * k), (int)lo, (int)hi);                    // row-load 0
    const u32x4 ml = range_mask((int)(256u * (ns - 1u) + 16u * k), (int)lo, (int)hi);  // row-load ns - 1
    // SPLIT (the launched kernel since round 3): a step's ns row-loads in equal batches of at most U (c3: 3 + 3
    // instead of 4 + 2 and two loads past the frame that only cost their issue; 274.4 vs 275.4 us in-process A/B,
    // profiles/r03/ab_uniform_split_*.log)
    const uint32_t ub = SPLIT ? (ns + (ns + U - 1) / U - 1) / ((ns + U - 1) / U) : (uint32_t)U;  // wave-uniform
    for (uint32_t s = 0; s < 16u; ++s) {
        const uint32_t f = 4u * s + q;
        const FrameMeta6& fm = meta[f];  // broadcast read: one entry per 16-lane row
        const uint32_t rel = fm.rel, lim = fm.lim;
        uint32_t h = 0;
        for (uint32_t j0 = 0; j0 < ns; j0 += ub) {
            u32x4 v[U];
            if (PRIO) __builtin_amdgcn_s_setprio(2);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t ro = 256u * (j0 + (uint32_t)u) + 16u * k;
                if (SPLIT && ((uint32_t)u >= ub || j0 + (uint32_t)u >= ns)) break;  // wave-uniform
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(ro < lim ? rel + ro : 0x80000000u), 0, kAuxNT);
            }
            if (PRIO) __builtin_amdgcn_s_setprio(0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = j0 + (uint32_t)u;  // wave-uniform
                if (j >= ns || (SPLIT && (uint32_t)u >= ub)) break;
                u32x4 x = v[u];
                if (j == 0u && k < kRowW / 16u) *(u32x4*)(rows + f * kRowW + 16u * k) = x;  // the header window
                if (j == 0u) x &= mf;
                if (j == ns - 1u) x &= ml;
                h = sum_halves(x, h);
            }
        }
        const uint32_t r = row_sum_dpp(h);
        if (k == 15u) sums_ic[f] = r;
    }
}

// ================================================================================================
// Reference-mode header phase (lane = frame): from its LDS window and the stream's folded ICMP sum, the
// gates of process_packet() in order, the MAC / IPv4 address swap and type = 0 as dword shuffles, and the
// checksum patch in closed form.  The verdict and record are returned in *verd_out / *rec_out (the round
// kernel stores them in its write phase); a 16-B aligned reply whose 64-B window lies in the UMEM is
// patched in LDS and returns true (the caller stores the whole window), any other reply is written here,
// byte-exact.
// ================================================================================================
// HB (round 5, shipped): a wave whose frames all start 16-B aligned reads its window's first 48 bytes with three
// ds_read_b128 instead of eleven ds_read_b32 -- the rows are 64 B apart, so a b32 read of one dword in every row meets
// 16 lanes on each of two banks (16-way), a b128 read 4-way -- and an aligned reply's patch goes back as two b128 and one
// b64 store instead of seven b32 ones (the unchanged dwords 3-5 rewritten with the values read).  c2 LDS bank-conflict
// cycles 6.72 M -> 1.87 M per launch; in-process A/B over two sessions, µs: c2 34.94 / 35.00 -> 34.20 / 34.36, c3 274.3 /
// 274.7 -> 272.8 / 273.3, c4 179.6 / 180.3 -> 178.5 / 179.2, p98 63.8 / 63.9 -> 62.6 / 62.7; wire mode (every option)
// c2 36.5 -> 35.0, c3 275.2 -> 274.5, c4 183.0 -> 182.1 (profiles/r05/hb/).
template <bool HB = false>
__device__ __forceinline__ bool header_phase_ref(const EchoArgs& a, uint8_t* row, uint32_t ic_raw, uint64_t addr,
                                                 uint32_t len, bool live, bool ok, bool parse, Counters& cnt,
                                                 u32x4* rec_out, uint32_t* verd_out) {
    const uint32_t off = (uint32_t)addr & 15u;
    uint32_t h[10];  // frame-relative dwords: h[k] = bytes [4k, 4k+4) of the frame
    const bool hb = HB && __ballot(off != 0u) == 0ull;  // wave-uniform
    if (hb) {
        const u32x4 q0 = *(const u32x4*)row, q1 = *(const u32x4*)(row + 16), q2 = *(const u32x4*)(row + 32);
        h[0] = q0.x, h[1] = q0.y, h[2] = q0.z, h[3] = q0.w, h[4] = q1.x, h[5] = q1.y, h[6] = q1.z, h[7] = q1.w;
        h[8] = q2.x, h[9] = q2.y;
    } else {
        const uint32_t* rw = (const uint32_t*)(row + (off & ~3u));
#pragma unroll
        for (int k = 0; k < 10; ++k) h[k] = __builtin_amdgcn_alignbyte(rw[k + 1], rw[k], off & 3u);
    }

    // parsed fields (xsk_receive.c:135,140,144,157)
    const uint32_t eth_proto = parse ? (((h[3] & 0xFFu) << 8) | ((h[3] >> 8) & 0xFFu)) : 0u;
    const uint32_t vihl = parse ? (h[3] >> 16) & 0xFFu : 0u;
    const uint32_t proto = parse ? h[5] >> 24 : 0u;
    const uint32_t itype = parse ? (h[8] >> 16) & 0xFFu : 0u;
    const uint32_t icode = parse ? h[8] >> 24 : 0u;
    const uint32_t csum_le = parse ? h[9] & 0xFFFFu : 0u;  // the reference's uint16_t load (:157)

    uint32_t verdict;
    if (!ok) verdict = XSK_GPU_DROP_BAD_DESC;
    else if (len < 20) verdict = XSK_GPU_DROP_SHORT;                 // :123-133
    else if (eth_proto != 0x0800u) verdict = XSK_GPU_DROP_NOT_IPV4;  // :135
    else if (proto != 1u) verdict = XSK_GPU_DROP_NOT_ICMP;           // :140
    else if (itype != 8u) verdict = XSK_GPU_DROP_NOT_ECHO;           // :144
    else verdict = XSK_GPU_TX_REPLY;
    const bool tx = verdict == XSK_GPU_TX_REPLY;

    // csum_replace2(&icmp->checksum, ICMP_ECHO, ICMP_ECHOREPLY), xsk_receive.c:101-111,157
    uint32_t c16 = (~csum_le) & 0xFFFFu;
    c16 = (c16 + 0xFFF7u) & 0xFFFFu;  // csum += ~old  (old = 8)
    c16 += c16 < 0xFFF7u ? 1u : 0u;   // end-around carry; csum += new (0) is a no-op
    const uint32_t csum_new_le = tx ? (~c16) & 0xFFFFu : csum_le;

    // RFC 1071 sums of the input frame (build-added verification fields): the ICMP message from the stream,
    // the IPv4 header bytes [14, min(len, 34)) from the frame-relative dwords (LE halves of frame-even-aligned
    // words are byte-swapped network words, RFC 1071 §2(B))
    uint32_t ic_sum = fold32(ic_raw);
    if (!((uint32_t)addr & 1u)) ic_sum = bswap16(ic_sum);
    uint32_t ip_sum;
    {
        const int e = (int)min(len, 34u);
        uint32_t acc = 0;
        if (__ballot(e < 34) == 0ull) {  // every frame has the whole 20-B header: fixed masks
            acc = dot2_halves(h[3] >> 16, dot2_halves(h[4], dot2_halves(h[5], 0u)));
            acc = dot2_halves(h[8] & 0xFFFFu, dot2_halves(h[7], dot2_halves(h[6], acc)));
        } else {
#pragma unroll
            for (int kk = 3; kk <= 8; ++kk) acc += halves(keep_bytes(h[kk], 4 * kk, 14, e));
        }
        ip_sum = bswap16(fold32(acc));
    }
    uint32_t flags = 0;
    if (parse && len >= 34 && ip_sum == 0xFFFFu) flags |= XSK_GPU_F_IP_CSUM_OK;
    if (parse && len >= 42 && ic_sum == 0xFFFFu) flags |= XSK_GPU_F_ICMP_CSUM_OK;

    // echo-reply rewrite, xsk_receive.c:148-157 (bytes 0-11, 26-34, 36-37)
    bool wb = false;
    if (tx) {
        const uint32_t n0 = (h[1] >> 16) | (h[2] << 16);              // s0 s1 s2 s3
        const uint32_t n1 = (h[2] >> 16) | (h[0] << 16);              // s4 s5 d0 d1
        const uint32_t n2 = (h[0] >> 16) | (h[1] << 16);              // d2 d3 d4 d5
        const uint32_t n6 = (h[6] & 0xFFFFu) | (h[7] & 0xFFFF0000u);  // csum(ip) | daddr[0:2]
        const uint32_t n7 = (h[8] & 0xFFFFu) | (h[6] & 0xFFFF0000u);  // daddr[2:4] | saddr[0:2]
        const uint32_t n8 = (h[7] & 0xFFFFu) | (h[8] & 0xFF000000u);  // saddr[2:4] | type=0 | code
        if (off == 0 && a.umem_size - addr >= (uint64_t)kWin) {
            uint32_t* r32 = (uint32_t*)row;  // patched in LDS, stored as a whole window by the caller
            if (HB) {
                *(u32x4*)row = u32x4{n0, n1, n2, h[3]};
                *(u32x4*)(row + 16) = u32x4{h[4], h[5], n6, n7};
                r32[8] = n8;
                r32[9] = (h[9] & 0xFFFF0000u) | csum_new_le;
            } else {
                r32[0] = n0;
                r32[1] = n1;
                r32[2] = n2;
                r32[6] = n6;
                r32[7] = n7;
                r32[8] = n8;
                r32[9] = (h[9] & 0xFFFF0000u) | csum_new_le;
            }
            wb = true;
        } else {
            uint8_t* pkt = a.umem + addr;
            if ((off & 3u) == 0) {
                uint32_t* p32 = (uint32_t*)pkt;
                p32[0] = n0;
                p32[1] = n1;
                p32[2] = n2;
                p32[6] = n6;
                p32[7] = n7;
                p32[8] = n8;
                *(uint16_t*)(pkt + 36) = (uint16_t)csum_new_le;
            } else {
                const uint32_t w[6] = {n0, n1, n2, n6, n7, n8};
#pragma unroll
                for (int b = 0; b < 12; ++b) pkt[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
#pragma unroll
                for (int b = 0; b < 12; ++b) pkt[24 + b] = (uint8_t)(w[3 + (b >> 2)] >> (8 * (b & 3)));
                pkt[36] = (uint8_t)csum_new_le;
                pkt[37] = (uint8_t)(csum_new_le >> 8);
            }
        }
    }
    u32x4 r;
    r.x = verdict | (flags << 8) | (proto << 16) | (itype << 24);
    r.y = icode | (vihl << 8) | (eth_proto << 16);
    r.z = (parse ? bswap16(csum_le) : 0u) | ((parse ? bswap16(csum_new_le) : 0u) << 16);
    r.w = (parse ? ip_sum : 0u) | ((parse ? ic_sum : 0u) << 16);
    *rec_out = r;
    *verd_out = verdict;
    if (live) {
        cnt.rxp += 1;
        cnt.rxb += len;
        if (tx) {
            cnt.txp += 1;
            cnt.txb += len;
        }
    }
    return wb;
}

// ================================================================================================
// Wire-format header phase (xsk_gpu_echo_dev_opts; spec: include/xsk_gpu.h).
// ================================================================================================
// Tag types for the two instantiations of the IPv4 gates of the wire header phase (untagged frame: every field at a
// constant offset).
struct WireAt14 {
    static constexpr bool kPlain = true;
};
struct WireAtL3 {
    static constexpr bool kPlain = false;
};

// Lane = frame.  The frame's 16-B aligned 64-B window in LDS (`row`, frame byte i at row[off + i] while off + i < 64;
// bytes past it -- an ICMP header behind two VLAN tags and IPv4 options -- are read from the UMEM) and the stream's
// ICMP sum of row bytes [off + 34, off + len), i.e. of the message of a PLAIN frame (no tag, IHL 5, no Ethernet
// padding under STRICT).  Parses VLAN tags / IHL / tot_len / fragments, decides, patches the reply in LDS; a plain
// frame's sums come from the window and the stream exactly as in reference mode, any other frame's from a re-read of
// its header and message bytes (rare traffic, per lane).  Returns true when the patched 64-B window should leave as a
// whole sector (aligned, rewrite inside the first 64 B).
__device__ __forceinline__ uint64_t sum_row_range(const uint8_t* rb, uint32_t lo, uint32_t hi) {
    uint64_t acc = 0;  // LE dwords of the 16-B aligned row at rb, bytes [lo, hi) (absolute-alignment domain)
    for (uint32_t o = lo & ~3u; o < hi; o += 4u) acc += keep_bytes(*(const uint32_t*)(rb + o), (int)o, (int)lo, (int)hi);
    return acc;
}

template <bool HB = false>
__device__ __forceinline__ bool wire_header_phase64(const EchoArgs& a, uint8_t* row, uint32_t ic_raw, uint64_t addr,
                                                    uint32_t len, bool ok, bool live, uint32_t wend, Counters& cnt,
                                                    u32x4* rec_out, uint32_t* verd_out) {
    const bool strict = (a.opts & XSK_GPU_OPT_STRICT_IPV4) != 0u;
    const bool vlan = (a.opts & XSK_GPU_OPT_VLAN) != 0u;
    const bool verify = (a.opts & XSK_GPU_OPT_VERIFY_CSUM) != 0u;
    const uint32_t off = (uint32_t)addr & 15u;
    uint8_t* p = row + off;
    const uint8_t* g = a.umem + addr;
    // frame byte i (i < len, so inside the UMEM): the window, or memory behind it
    auto fb = [&](uint32_t i) -> uint32_t { return off + i < (uint32_t)kWin ? (uint32_t)p[i] : (uint32_t)g[i]; };
    auto be16 = [&](uint32_t i) -> uint32_t { return (fb(i) << 8) | fb(i + 1); };
    // the frame's first 40 bytes as frame-relative LE dwords (window bytes off .. off + 43 < 64): an untagged frame's
    // fields at constant offsets come from registers instead of one LDS byte read each
    uint32_t h[10];
    if (HB && __ballot(off != 0u) == 0ull) {  // as header_phase_ref<HB>: three ds_read_b128 for an aligned wave
        const u32x4 q0 = *(const u32x4*)row, q1 = *(const u32x4*)(row + 16), q2 = *(const u32x4*)(row + 32);
        h[0] = q0.x, h[1] = q0.y, h[2] = q0.z, h[3] = q0.w, h[4] = q1.x, h[5] = q1.y, h[6] = q1.z, h[7] = q1.w;
        h[8] = q2.x, h[9] = q2.y;
    } else {
        const uint32_t* rw = (const uint32_t*)(row + (off & ~3u));
#pragma unroll
        for (int k = 0; k < 10; ++k) h[k] = __builtin_amdgcn_alignbyte(rw[k + 1], rw[k], off & 3u);
    }
    auto hb = [&](uint32_t i) -> uint32_t { return (h[i >> 2] >> (8u * (i & 3u))) & 0xFFu; };  // i < 40, constant
    auto hbe16 = [&](uint32_t i) -> uint32_t { return (hb(i) << 8) | hb(i + 1u); };
    uint32_t verdict = XSK_GPU_TX_REPLY;
    uint32_t l3 = 14, hl = 20, end = len, et = 0, tags = 0;
    bool hdrs = false;
    // the IPv4 / ICMP gates after the tags (untagged: l3 = 14, every byte from h[])
    auto ipv4_gates = [&](auto at) {
        constexpr bool PL = decltype(at)::kPlain;
        auto B = [&](uint32_t k) -> uint32_t { return PL ? hb(14u + k) : fb(l3 + k); };
        auto BE = [&](uint32_t k) -> uint32_t { return PL ? hbe16(14u + k) : be16(l3 + k); };
        bool bad = false;
        if (strict) {
            const uint32_t vihl = B(0);
            if ((vihl >> 4) != 4u || (vihl & 15u) < 5u) bad = true;
            else {
                hl = 4u * (vihl & 15u);
                const uint32_t tot = BE(2);
                if (tot < hl + 8 || l3 + tot > len) bad = true;
                else if (BE(6) & 0x3FFFu) bad = true;
                else end = l3 + tot;
            }
        }
        if (bad) verdict = XSK_GPU_DROP_BAD_IP;
        else if (B(9) != 1u) verdict = XSK_GPU_DROP_NOT_ICMP;
        else if (len < l3 + hl + 8) verdict = XSK_GPU_DROP_SHORT;
        else hdrs = true;
    };
    if (!ok) verdict = XSK_GPU_DROP_BAD_DESC;
    else if (len < 14) verdict = XSK_GPU_DROP_SHORT;
    else {
        et = hbe16(12);
        bool cut = false;
        if (vlan) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                if (!cut && (et == 0x8100u || et == 0x88A8u) && tags == (uint32_t)t) {
                    if (len < l3 + 4) cut = true;
                    else {
                        et = be16(l3 + 2);
                        l3 += 4;
                        tags++;
                    }
                }
            }
        }
        if (cut) verdict = XSK_GPU_DROP_SHORT;
        else if (et != 0x0800u) verdict = XSK_GPU_DROP_NOT_IPV4;
        else if (len < l3 + 20) verdict = XSK_GPU_DROP_SHORT;
        else if (tags == 0u) ipv4_gates(WireAt14{});
        else ipv4_gates(WireAtL3{});
    }
    const uint32_t l4 = l3 + hl;
    const bool std34 = tags == 0u && hl == 20u;  // l3 = 14, l4 = 34: the reference's offsets
    uint32_t ip_sum = 0, ic_sum = 0, itype = 0, icode = 0, csum_in = 0, flags = 0;
    if (hdrs) {
        if (std34 && end == len) {
            // plain: the IPv4 header [14, 34) from the frame-relative dwords (as header_phase_ref) and the
            // message [34, len) from the stream
            uint32_t acc = dot2_halves(h[3] >> 16, dot2_halves(h[4], dot2_halves(h[5], 0u)));
            acc = dot2_halves(h[8] & 0xFFFFu, dot2_halves(h[7], dot2_halves(h[6], acc)));
            ip_sum = bswap16(fold32(acc));
            ic_sum = fold32(ic_raw);
            if (!((uint32_t)addr & 1u)) ic_sum = bswap16(ic_sum);
        } else {  // tags, options or padding: re-read the header and the message (absolute-alignment domain)
            const uint8_t* rb = a.umem + (addr & ~15ull);
            ip_sum = fold64(sum_row_range(rb, off + l3, off + l4));
            ic_sum = fold64(sum_row_range(rb, off + l4, off + end));
            if (!((uint32_t)addr & 1u)) {
                ip_sum = bswap16(ip_sum);
                ic_sum = bswap16(ic_sum);
            }
        }
        itype = std34 ? hb(34) : fb(l4);
        icode = std34 ? hb(35) : fb(l4 + 1);
        csum_in = std34 ? hbe16(36) : be16(l4 + 2);
        if (ip_sum == 0xFFFFu) flags |= XSK_GPU_F_IP_CSUM_OK;
        if (ic_sum == 0xFFFFu) flags |= XSK_GPU_F_ICMP_CSUM_OK;
        if (tags) flags |= XSK_GPU_F_VLAN;
        if (hl > 20u) flags |= XSK_GPU_F_IP_OPTIONS;
        if (itype != 8u || (strict && icode != 0u)) verdict = XSK_GPU_DROP_NOT_ECHO;
        else if (verify && (ip_sum != 0xFFFFu || ic_sum != 0xFFFFu)) verdict = XSK_GPU_DROP_BAD_CSUM;
    }
    const bool tx = hdrs && verdict == XSK_GPU_TX_REPLY;
    const uint32_t vihl = hdrs ? (tags == 0u ? hb(14) : fb(l3)) : 0u, proto = hdrs ? 1u : 0u;
    uint32_t csum_out = csum_in;
    bool wb = false;
    if (tx) {
        // csum_replace2(&icmp->checksum, ICMP_ECHO, ICMP_ECHOREPLY) on the LE-loaded field (xsk_receive.c:101-111)
        const uint32_t csum_le = ((csum_in & 0xFFu) << 8) | (csum_in >> 8);
        uint32_t c16 = (~csum_le) & 0xFFFFu;
        c16 = (c16 + 0xFFF7u) & 0xFFFFu;
        c16 += c16 < 0xFFF7u ? 1u : 0u;
        const uint32_t csum_new_le = (~c16) & 0xFFFFu;
        csum_out = bswap16(csum_new_le);
        if (std34) {
            // the reference's offsets: the rewrite of xsk_receive.c:148-157 as header_phase_ref's dword shuffles
            const uint32_t n0 = (h[1] >> 16) | (h[2] << 16);              // s0 s1 s2 s3
            const uint32_t n1 = (h[2] >> 16) | (h[0] << 16);              // s4 s5 d0 d1
            const uint32_t n2 = (h[0] >> 16) | (h[1] << 16);              // d2 d3 d4 d5
            const uint32_t n6 = (h[6] & 0xFFFFu) | (h[7] & 0xFFFF0000u);  // csum(ip) | daddr[0:2]
            const uint32_t n7 = (h[8] & 0xFFFFu) | (h[6] & 0xFFFF0000u);  // daddr[2:4] | saddr[0:2]
            const uint32_t n8 = (h[7] & 0xFFFFu) | (h[8] & 0xFF000000u);  // saddr[2:4] | type=0 | code
            if (off == 0u && wend >= (uint32_t)kWin) {
                uint32_t* r32 = (uint32_t*)row;  // patched in LDS, stored as a whole window in the write phase
                if (HB) {
                    *(u32x4*)row = u32x4{n0, n1, n2, h[3]};
                    *(u32x4*)(row + 16) = u32x4{h[4], h[5], n6, n7};
                    r32[8] = n8;
                    r32[9] = (h[9] & 0xFFFF0000u) | csum_new_le;
                } else {
                    r32[0] = n0;
                    r32[1] = n1;
                    r32[2] = n2;
                    r32[6] = n6;
                    r32[7] = n7;
                    r32[8] = n8;
                    r32[9] = (h[9] & 0xFFFF0000u) | csum_new_le;
                }
                wb = true;
            } else {  // byte-exact: only the rewritten bytes
                uint8_t* pkt = a.umem + addr;
                const uint32_t w[6] = {n0, n1, n2, n6, n7, n8};
#pragma unroll
                for (int b = 0; b < 12; ++b) pkt[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
#pragma unroll
                for (int b = 26; b < 35; ++b) pkt[b] = (uint8_t)(w[3 + ((b - 24) >> 2)] >> (8 * (b & 3)));
                pkt[36] = (uint8_t)csum_new_le;
                pkt[37] = (uint8_t)(csum_new_le >> 8);
            }
        } else {
            // xsk_receive.c:148-157 at the parsed offsets: MACs and addresses lie in the window (off + l3 + 20 <= 57)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const uint8_t x = p[i];
                p[i] = p[6 + i];
                p[6 + i] = x;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint8_t x = p[l3 + 12 + i];
                p[l3 + 12 + i] = p[l3 + 16 + i];
                p[l3 + 16 + i] = x;
            }
            if (off == 0u && l4 + 4u <= (uint32_t)kWin && wend >= (uint32_t)kWin) {
                p[l4] = 0;  // whole 64-B sector, stored in the write phase
                p[l4 + 2] = (uint8_t)csum_new_le;
                p[l4 + 3] = (uint8_t)(csum_new_le >> 8);
                wb = true;
            } else {  // byte-exact: only the rewritten bytes
                uint8_t* pkt = a.umem + addr;
#pragma unroll
                for (int i = 0; i < 12; ++i) pkt[i] = p[i];
#pragma unroll
                for (int i = 0; i < 8; ++i) pkt[l3 + 12 + i] = p[l3 + 12 + i];
                pkt[l4] = 0;
                pkt[l4 + 2] = (uint8_t)csum_new_le;
                pkt[l4 + 3] = (uint8_t)(csum_new_le >> 8);
            }
        }
    }
    u32x4 r;
    r.x = verdict | (flags << 8) | (proto << 16) | (itype << 24);
    r.y = icode | (vihl << 8) | ((hdrs ? et : 0u) << 16);
    r.z = csum_in | (csum_out << 16);
    r.w = ip_sum | (ic_sum << 16);
    *rec_out = r;
    *verd_out = verdict;
    if (live) {
        cnt.rxp += 1;
        cnt.rxb += len;
        if (tx) {
            cnt.txp += 1;
            cnt.txb += len;
        }
    }
    return wb;
}

// LDS of one round-kernel workgroup (152.5 KiB of the CU's 160 KiB): TPW header-window tiles per wave, the
// per-frame metadata and sums, the ranked streams' sort rows, the counter rows.
template <int TPW>
struct Echo6Smem {
    __attribute__((aligned(16))) uint8_t hdr[kWaves6][TPW][kTile * kWin];  // 128 KiB: header windows
    __attribute__((aligned(16))) FrameMeta6 meta[kWaves6][kTile];          // 16 KiB
    uint32_t sum[kWaves6][2][kTile];                                        // 8 KiB
    uint32_t sort[kWaves6][80];                                             // 5 KiB
    unsigned long long cnt[kWaves6][4];
    uint32_t arrive;
    u32x4 desc[kTile];  // DLDS: the descriptors of a batch of <= 64 frames, delivered with its doorbell
};

// One frame's descriptor checks and stream geometry on 64-B windows, as the round body computes them (WIRE: the
// wire mode's -- it reads only [addr, addr + len) plus the window, and parses from 14 bytes on).
struct FrameIn {
    uint64_t addr, a16;
    uint32_t len, off, rowhi, lim, wend;
    bool ok, parse;
};
template <bool WIRE>
__device__ __forceinline__ FrameIn frame_in(const EchoArgs& a, u32x4 dsc, bool in_n) {
    FrameIn F;
    F.addr = (uint64_t)dsc.x | ((uint64_t)dsc.y << 32);
    F.len = dsc.z;
    const uint64_t need = WIRE ? F.len : (F.len >= 20 ? (F.len > 38 ? F.len : 38) : F.len);  // xsk_receive.c:120-157
    F.ok = in_n && F.len <= kMaxLen && F.addr <= a.umem_size && need <= a.umem_size - F.addr;
    F.parse = F.ok && F.len >= (WIRE ? 14u : 20u);
    F.a16 = F.addr & ~15ull;
    F.off = (uint32_t)F.addr & 15u;
    F.rowhi = F.parse ? F.off + F.len : 0u;
    F.wend = F.ok ? (uint32_t)min(a.umem_size - F.a16, (uint64_t)kWin) : 0u;
    F.lim = max(F.rowhi, F.parse ? F.wend : 0u);
    return F;
}

// Paired short tiles: both tiles of a wave's round read at once when every frame of both fits its 64-B
// window (c2: minimum-size frames).  The two descriptor loads go out together, then all eight 16-B frame
// loads of the two tiles (4 lanes per frame, 16 frames per wave-load; a frame's address and limit come from
// its owner lane by bpermute, so neither tile needs the LDS metadata), and only then are they summed -- the
// round pays two memory round trips instead of four, with twice the bytes in flight.  The windows go to the
// two LDS slots, the ICMP sums to the two sum rows, then the header phase of each tile.  Returns false
// (nothing written) when either tile has a longer frame.
template <int HEAVY, bool WIRE, bool HB = false>
__device__ __forceinline__ bool read_round_short2(const EchoArgs& a, uint32_t t0, uint32_t t1, uint8_t* rows0,
                                                  uint8_t* rows1, uint32_t* sums0, uint32_t* sums1, uint32_t lane,
                                                  Counters& cnt, u32x4* rec, uint32_t* verd, uint32_t* alo,
                                                  uint32_t* ahi, uint64_t* wbm, uint32_t& round_long) {
    const uint32_t fi0 = t0 * kTile + lane, fi1 = t1 * kTile + lane;
    const bool in0 = fi0 < a.n, in1 = fi1 < a.n;
    u32x4 d0 = u32x4{0u, 0u, 0u, 0u}, d1 = u32x4{0u, 0u, 0u, 0u};
    if (in0) d0 = *(const u32x4*)(a.descs + fi0);
    if (in1) d1 = *(const u32x4*)(a.descs + fi1);
    const FrameIn F0 = frame_in<WIRE>(a, d0, in0), F1 = frame_in<WIRE>(a, d1, in1);
    if ((__ballot(F0.lim > (uint32_t)kWin) | __ballot(F1.lim > (uint32_t)kWin)) != 0ull) return false;
    const uint32_t kk = lane & 3u, ro = 16u * kk;
    u32x4 x0[4], x1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int src = r * 16 + (int)(lane >> 2);
        const uint64_t b0 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(F0.a16 >> 32), src, 64) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)F0.a16, src, 64);
        const uint64_t b1 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(F1.a16 >> 32), src, 64) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)F1.a16, src, 64);
        const uint32_t m0 = (uint32_t)__shfl((int)F0.lim, src, 64), m1 = (uint32_t)__shfl((int)F1.lim, src, 64);
        x0[r] = u32x4{0u, 0u, 0u, 0u};
        x1[r] = u32x4{0u, 0u, 0u, 0u};
        if (ro < m0) x0[r] = __builtin_nontemporal_load((const u32x4*)(a.umem + b0 + ro));
        if (ro < m1) x1[r] = __builtin_nontemporal_load((const u32x4*)(a.umem + b1 + ro));
    }
    // the ICMP bytes [off + 34, rowhi): masks once per tile when every frame has the same offset and end
    const uint32_t k0 = (F0.off << 24) ^ F0.rowhi, k1 = (F1.off << 24) ^ F1.rowhi;
    const bool u0 = __ballot(k0 != uniform(k0)) == 0ull, u1 = __ballot(k1 != uniform(k1)) == 0ull;
    const u32x4 mk0 = range_mask((int)ro, (int)uniform(F0.off) + 34, (int)uniform(F0.rowhi));
    const u32x4 mk1 = range_mask((int)ro, (int)uniform(F1.off) + 34, (int)uniform(F1.rowhi));
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const FrameIn& F = tt ? F1 : F0;
        uint8_t* rows = tt ? rows1 : rows0;
        uint32_t* sums = tt ? sums1 : sums0;
        const bool uni = tt ? u1 : u0;
        const u32x4 mk = tt ? mk1 : mk0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
            const u32x4 v = tt ? x1[r] : x0[r];
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
    bool wb = WIRE ? wire_header_phase64<HB>(a, rows0 + lane * kWin, sums0[lane], F0.addr, F0.len, F0.ok, in0, F0.wend, cnt,
                                         &rec[0], &verd[0])
                   : header_phase_ref<HB>(a, rows0 + lane * kWin, sums0[lane], F0.addr, F0.len, in0, F0.ok, F0.parse, cnt,
                                      &rec[0], &verd[0]);
    wbm[0] = __ballot(wb);
    wb = WIRE ? wire_header_phase64<HB>(a, rows1 + lane * kWin, sums1[lane], F1.addr, F1.len, F1.ok, in1, F1.wend, cnt, &rec[1],
                                    &verd[1])
              : header_phase_ref<HB>(a, rows1 + lane * kWin, sums1[lane], F1.addr, F1.len, in1, F1.ok, F1.parse, cnt, &rec[1],
                                 &verd[1]);
    wbm[1] = __ballot(wb);
    alo[0] = d0.x;
    ahi[0] = d0.y;
    alo[1] = d1.x;
    ahi[1] = d1.y;
    round_long += (uint32_t)__popcll(__ballot(in0 && F0.len >= (uint32_t)HEAVY)) +
                  (uint32_t)__popcll(__ballot(in1 && F1.len >= (uint32_t)HEAVY));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // the sums / windows are rewritten by the next round
    return true;
}

// ================================================================================================
// The round kernel.  Measured on cold 4 GiB slabs (tools/wexp.hip): a read stream that meets scattered
// 64-B writes pays for them at DRAM read/write turnarounds while the same writes issued as a burst with
// no reads around them cost far less.  So the grid is persistent -- one 16-wave workgroup per CU, every
// workgroup the same contiguous share of tiles -- and works in ROUNDS: each wave streams TPW tiles (the
// read phase: descriptors, payload, header phase, patched windows into LDS, records into VGPRs), and
// then stores its patched 64-B windows, records and verdicts (the write phase), write-through (WT) so
// the bytes leave the XCD's L2 during the write phase.
//
// echo6_body: the work over the tiles [t_begin, t_end) of one workgroup (every wave of the workgroup calls
// it with the same range); echo_round_kernel runs it once per workgroup on its static share, the
// low-latency resident kernel (xsk_lowlat.hip) once per doorbell.
//   TPW   tiles per wave per round (2; sub-tiles 1)
//   SYNC  how a wave enters its write phase.  0: at once (one-round small batches); 2: a wave at least half
//         of whose frames this round have >= HEAVY bytes waits until every wave of the workgroup but SLACK has
//         read the round (LDS arrival counter), lighter waves go ahead -- the phase separation pays where reads
//         dominate, and costs latency hiding where frames are short
//   WIRE  the wire-format mode (a.opts != 0): the reference mode's streams and rounds with wire_header_phase64
//   SUBT  tiles of a.tile_live frames (small batches: the batch spreads over every wave)
//   TRACE wave 0 stamps the body's phase boundaries into a.trace (the low-latency kernel's diagnostics)
//   DLDS  the descriptors may already be in the LDS (a.desc_in_lds, the low-latency kernel's first poll)
//   WT    write-phase windows and records stored write-through (sc1 raw buffer stores)
// The per-tile stream choices: tiles whose frames all fit their 64-B windows (c2)
// skip the row stream (and two such tiles of a round are read together, PAIR), ping-size tiles (every frame
// within 128 B) are read by 8-lane groups, uniform long tiles (c3, c5) take masks computed once per tile,
// ragged tiles (c4) the ranked step-packed streams.
// ================================================================================================
template <int TPW, int SYNC, bool WIRE, bool SUBT, bool TRACE, bool DLDS, bool WT, int HEAVY, int UR = kU,
          bool USPLIT = false, bool PRIO = false, int SLACK = 0, bool HB = false>
__device__ __forceinline__ void echo6_body(const EchoArgs& a, uint32_t t_begin, uint32_t t_end, Echo6Smem<TPW>& sm) {
    static_assert(SYNC == 0 || SYNC == 2, "write phases: at once (0) or heavy waves wait for the round (2)");
    static_assert(SLACK >= 0 && SLACK < kWaves6, "SLACK: waves a heavy wave does not wait for");
    constexpr int U = kU;
    constexpr bool PAIR = TPW == 2 && !SUBT;  // paired short tiles (header_phase_ref / wire_header_phase64)
    constexpr uint32_t kRowW = (uint32_t)kWin;  // LDS row (header window) bytes
    auto& s_hdr = sm.hdr;
    uint32_t& s_arrive = sm.arrive;
    if (SYNC == 2) {
        if (threadIdx.x == 0) s_arrive = 0u;
        __syncthreads();
    }
    uint32_t rounds_done = 0;

    const uint32_t wave = uniform(threadIdx.x >> 6);
    FrameMeta6* meta = sm.meta[wave];
    uint32_t* sums_ic = sm.sum[wave][0];
    constexpr uint32_t kRound = (uint32_t)kWaves6 * TPW;
    Counters cnt;
    uint32_t lane = threadIdx.x & 63u;
    for (uint32_t r0 = t_begin; r0 < t_end; r0 += kRound) {  // rounds, workgroup-uniform
        // slot i of this round: wave w streams tile r0 + i * 16 + w when it is below t_end
        u32x4 rec[TPW];
        uint32_t verd[TPW], alo[TPW], ahi[TPW];
        uint64_t wbm[TPW];
        uint32_t round_long = 0;  // SYNC 2: frames of >= HEAVY bytes this wave read this round (uniform)
        // ================= read phase =================
        bool paired = false;
        if (PAIR && r0 + wave < t_end && r0 + (uint32_t)kWaves6 + wave < t_end)  // wave-uniform
            paired = read_round_short2<HEAVY, WIRE, HB>(a, r0 + wave, r0 + (uint32_t)kWaves6 + wave, s_hdr[wave][0],
                                              s_hdr[wave][TPW > 1 ? 1 : 0], sm.sum[wave][0], sm.sum[wave][1], lane,
                                              cnt, rec, verd, alo, ahi, wbm, round_long);
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            if (PAIR && paired) continue;  // wave-uniform: both tiles are done
            u32x4 rec_o;
            uint32_t verd_o, alo_o, ahi_o;
            uint64_t wbm_o;
            do {  // one tile; `break` = the slot has no tile for this wave
                const uint32_t t = r0 + (uint32_t)i * kWaves6 + wave;
                wbm_o = 0ull;
                rec_o = u32x4{0u, 0u, 0u, 0u};
                verd_o = 0u;
                alo_o = 0u;
                ahi_o = 0u;
                if (t >= t_end) break;  // wave-uniform
                asm volatile("" : "+v"(lane));
                uint8_t* rows = s_hdr[wave][i];
                const uint32_t q = lane >> 4, k = lane & 15u;
                const uint32_t fi = t * (SUBT ? a.tile_live : (uint32_t)kTile) + lane;
                const bool in_n = (!SUBT || lane < a.tile_live) && fi < a.n;  // a live frame of the batch
                // ---- 1. descriptors (xsk_receive.c:222-223): lane i <- frame t*64+i ----------------------
                u32x4 dsc = u32x4{0u, 0u, 0u, 0u};
                if (DLDS && a.desc_in_lds) {
                    if (in_n) dsc = sm.desc[fi];  // n <= 64: fi < 64
                } else if (in_n) {
                    dsc = *(const u32x4*)(a.descs + fi);
                }
                const uint64_t addr = (uint64_t)dsc.x | ((uint64_t)dsc.y << 32);
                const uint32_t len = dsc.z;
                // reference mode reads bytes [0, 38) whenever len >= 20 (xsk_receive.c:120-157); wire mode
                // reads only [addr, addr + len) plus the window
                const uint64_t need = WIRE ? len : (len >= 20 ? (len > 38 ? len : 38) : len);
                const bool ok = in_n && len <= kMaxLen && addr <= a.umem_size && need <= a.umem_size - addr;
                const bool parse = ok && len >= (WIRE ? 14u : 20u);
                const uint64_t a16 = addr & ~15ull;
                const uint32_t off = (uint32_t)addr & 15u;
                const uint32_t rowhi = parse ? off + len : 0u;
                const uint32_t wend = ok ? (uint32_t)min(a.umem_size - a16, (uint64_t)kRowW) : 0u;
                const uint32_t win = parse ? wend : 0u;
                const uint32_t lim = max(rowhi, win);
                const uint32_t nit = (lim + 255u) >> 8;
                const bool short_tile = __ballot(lim > kRowW) == 0ull;
                const bool mid_tile = !short_tile && __ballot(lim > 128u) == 0ull;
                // every frame of the tile at the same 16-B offset with the same end (c2, pings): the ICMP
                // byte masks of a lane's block are the same for all its frames -> computed once per tile
                const uint32_t ukey = (off << 24) ^ rowhi;
                const bool uni_tile = (short_tile || mid_tile) && __ballot(ukey != uniform(ukey)) == 0ull;
                uint64_t wlo = 0, span = ~0ull;
                if (!short_tile) {
                    wlo = wave_min_u64(nit ? a16 : ~0ull);
                    span = wave_max_u64(nit ? a16 + lim : 0ull) - wlo;
                }
                const bool fast = !short_tile && !mid_tile && span < 0x80000000ull;  // wave-uniform
                {
                    FrameMeta6 m;
                    m.rel = fast ? (nit ? (uint32_t)(a16 - wlo) : 0u) : (uint32_t)(a16 >> 4);
                    m.rowhi = rowhi;
                    m.lim = lim;
                    m.packed = off | ((parse ? off + min(len, 34u) : 0u) << 8) | ((ok ? 1u : 0u) << 16) |
                               ((parse ? 2u : 0u) << 16) | ((uint32_t)(a16 >> 36) << 20);
                    meta[lane] = m;
                }
                alo_o = dsc.x;
                ahi_o = dsc.y;
                if (SYNC == 2) round_long += (uint32_t)__popcll(__ballot(in_n && len >= (uint32_t)HEAVY));
                if (TRACE && threadIdx.x == 0 && i == 0) a.trace[0] = wall_clock64();  // descriptors parsed
                // ---- 2. stream every row byte once; windows -> LDS rows, row sums -> LDS -----------------
                if (__ballot(nit != 0u) != 0ull) {
                    __builtin_amdgcn_wave_barrier();
                    WinLoader ld;
                    ld.r = __builtin_amdgcn_make_buffer_rsrc((void*)(a.umem + (fast ? wlo : 0ull)), (short)0,
                                                             fast ? (int)((span + 15u) & ~15ull) : 0, kRsrcFlags);
                    if (short_tile) {
                        // every frame within its 64-B window: 4 lanes per frame, 16 frames per wave-load
                        const uint32_t kk = lane & 3u, ro = 16u * kk;
                        const u32x4 umk = uni_tile ? range_mask((int)ro, (int)off + 34, (int)rowhi) : u32x4{0u, 0u, 0u, 0u};
                        u32x4 x[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const FrameMeta6& fm = meta[(uint32_t)r * 16u + (lane >> 2)];
                            const bool in = ro < fm.lim;
                            x[r] = u32x4{0u, 0u, 0u, 0u};  // lanes past their frame: no memory access at all
                            if (in) x[r] = __builtin_nontemporal_load((const u32x4*)(a.umem + meta6_a16(fm) + ro));
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                            const FrameMeta6& fm = meta[f];
                            const u32x4 v = ro < fm.lim ? x[r] : u32x4{0u, 0u, 0u, 0u};
                            *(u32x4*)(rows + f * kRowW + ro) = v;
                            const int f_off = (int)(fm.packed & 0xFFu);
                            uint32_t ric = uni_tile ? sum_halves(v & umk, 0u) : sum_range_h(v, (int)ro, f_off + 34, (int)fm.rowhi);
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0xB1, 0xF, 0xF, false);  // xor 1
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x4E, 0xF, 0xF, false);  // xor 2
                            if (kk == 0u) sums_ic[f] = ric;
                        }
                    } else if (mid_tile) {
                        // every frame within 128 B of its 16-B aligned start (pings): 8 lanes per frame, 8 frames
                        // per wave-load, all 8 loads in flight at once; the ICMP sum by exact byte range, reduced
                        // over the 8 lanes (the IPv4 header sum comes from the window in the header phase)
                        const uint32_t kk = lane & 7u, ro = 16u * kk;
                        const u32x4 umk = uni_tile ? range_mask((int)ro, (int)off + 34, (int)rowhi) : u32x4{0u, 0u, 0u, 0u};
                        u32x4 x[8];
#pragma unroll
                        for (int r = 0; r < 8; ++r) {
                            const FrameMeta6& fm = meta[(uint32_t)r * 8u + (lane >> 3)];
                            const bool in = ro < fm.lim;
                            x[r] = u32x4{0u, 0u, 0u, 0u};  // lanes past their frame: no memory access at all
                            if (in) x[r] = __builtin_nontemporal_load((const u32x4*)(a.umem + meta6_a16(fm) + ro));
                        }
#pragma unroll
                        for (int r = 0; r < 8; ++r) {
                            const uint32_t f = (uint32_t)r * 8u + (lane >> 3);
                            const FrameMeta6& fm = meta[f];
                            const u32x4 v = ro < fm.lim ? x[r] : u32x4{0u, 0u, 0u, 0u};
                            if (kk < 4u) *(u32x4*)(rows + f * kRowW + ro) = v;
                            uint32_t ric = uni_tile ? sum_halves(v & umk, 0u)
                                                    : sum_range_h(v, (int)ro, (int)(fm.packed & 0xFFu) + 34, (int)fm.rowhi);
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0xB1, 0xF, 0xF, false);   // xor 1
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x4E, 0xF, 0xF, false);   // xor 2
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x141, 0xF, 0xF, false);  // half-row mirror
                            if (kk == 0u) sums_ic[f] = ric;
                        }
                    } else if (__ballot(nit != 0u && nit != uniform(max_nit_lane(nit))) != 0ull ||
                               uniform(max_nit_lane(nit)) < (uint32_t)U) {
                        // ragged tile (or one too short to fill a batch of U row-loads): ranked streams
                        if (fast) stream_tile_sorted<UR, true, true, PRIO>(a, ld.r, meta, sm.sort[wave], rows, sums_ic, nit, lane);
                        else stream_tile_sorted<UR, false, true, PRIO>(a, ld.r, meta, sm.sort[wave], rows, sums_ic, nit, lane);
                    } else if (fast && __ballot(!parse) == 0ull && __ballot(ukey != uniform(ukey)) == 0ull) {
                        stream_tile_uniform<U, USPLIT, PRIO>(ld.r, meta, rows, sums_ic, uniform(nit), uniform(off) + 34u,
                                                             uniform(rowhi), lane);
                    } else {
                        // every frame the same number of row-loads, but different offsets or ends: per-step streams
                        for (uint32_t s = 0; s < 16; ++s) {
                            const uint32_t f = 4u * s + q;
                            const FrameMeta6& fm = meta[f];  // broadcast read: one entry per 16-lane row
                            const uint32_t f_lim = fm.lim;
                            const uint32_t f_nit = (f_lim + 255u) >> 8;
                            const uint32_t ns = max(max(rdlane(f_nit, 0), rdlane(f_nit, 16)),
                                                    max(rdlane(f_nit, 32), rdlane(f_nit, 48)));
                            if (ns == 0) continue;
                            const uint32_t f_rowhi = fm.rowhi, f_packed = fm.packed;
                            const uint32_t f_off = f_packed & 0xFFu, f_iphi = (f_packed >> 8) & 0xFFu;
                            RowSums rs;
                            if (fast) {
                                ld.rel = fm.rel;
                                stream_frame<U, WinLoader, true>(ld, ns, f_rowhi, f_lim, f_off, f_iphi, k, rows + f * kRowW, rs);
                            } else {  // frames of one tile more than 2 GiB apart (never in AF_XDP layouts)
                                FarLoader fl;
                                fl.fbase = a.umem + (f_nit ? meta6_a16(fm) : 0ull);
                                stream_frame<U, FarLoader, true>(fl, ns, f_rowhi, f_lim, f_off, f_iphi, k, rows + f * kRowW, rs);
                            }
                            const uint32_t ric = row_sum_dpp(fold64(rs.ic));
                            if (k == 15u) sums_ic[f] = ric;
                        }
                    }
                }

                // ---- 3. header phase (lane = frame); the window stays patched in LDS ---------------------
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (TRACE && threadIdx.x == 0 && i == 0) a.trace[1] = wall_clock64();  // frames streamed
                __builtin_amdgcn_wave_barrier();
                const uint32_t ic_raw = nit ? sums_ic[lane] : 0u;
                bool wb;
                if (WIRE)
                    wb = wire_header_phase64<HB>(a, rows + lane * kRowW, ic_raw, addr, len, ok, in_n, wend, cnt, &rec_o,
                                             &verd_o);
                else
                    wb = header_phase_ref<HB>(a, rows + lane * kWin, ic_raw, addr, len, in_n, ok, parse, cnt, &rec_o,
                                          &verd_o);
                wbm_o = __ballot(wb);
            } while (0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();  // meta/sums are rewritten by the next tile
            rec[i] = rec_o;
            verd[i] = verd_o;
            alo[i] = alo_o;
            ahi[i] = ahi_o;
            wbm[i] = wbm_o;
        }

        if (TRACE && threadIdx.x == 0) a.trace[2] = wall_clock64();  // header phase done
        // ================= write phase =================
        if (SYNC == 2) {
            ++rounds_done;
            if (lane == 0) atomicAdd(&s_arrive, 1u);
            if (uniform(round_long) * 2u >= (uint32_t)(kTile * TPW)) {  // at least half its frames long
                // (every wave but SLACK: the last waves of a round are usually ragged ones still streaming)
                while (__hip_atomic_load(&s_arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
                       rounds_done * (uint32_t)kWaves6 - (uint32_t)SLACK)
                    __builtin_amdgcn_s_sleep(2);
            }
        }
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const uint32_t t = r0 + (uint32_t)i * kWaves6 + wave;
            if (t >= t_end) continue;
            const uint8_t* rows = s_hdr[wave][i];
            if (wbm[i]) {  // patched windows: 16 frames x 64 B per wave-store, whole 64-B sectors
                // WT: the 4 GiB region of the tile's first written window; every written window inside it?
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
                        const uint64_t fa = (uint64_t)flo | ((uint64_t)fhi << 32);
                        const u32x4 w = *(const u32x4*)(rows + f * kRowW + 16u * kk);
                        if (WT && wt_tile) __builtin_amdgcn_raw_buffer_store_b128(w, wrs, (int)(flo + 16u * kk), 0, kAuxSC1);
                        else *(u32x4*)(a.umem + fa + 16u * kk) = w;
                    }
                }
            }
            const uint32_t fi = t * (SUBT ? a.tile_live : (uint32_t)kTile) + lane;
            if ((!SUBT || lane < a.tile_live) && fi < a.n) {
                if (a.recs) {
                    if (WT)
                        __builtin_amdgcn_raw_buffer_store_b128(
                            rec[i],
                            __builtin_amdgcn_make_buffer_rsrc((void*)((u32x4*)a.recs + (uint64_t)uniform(t) * (SUBT ? a.tile_live : (uint32_t)kTile)),
                                                              (short)0, -1, kRsrcFlags),
                            (int)(lane * 16u), 0, kAuxSC1);
                    else ((u32x4*)a.recs)[fi] = rec[i];
                }
                if (a.verdicts) a.verdicts[fi] = (uint8_t)verd[i];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // LDS rows are rewritten by the next round
    }
    if (TRACE && threadIdx.x == 0) a.trace[3] = wall_clock64();  // write phase issued
    store_counters(a, cnt, sm.cnt, wave, lane);
    if (TRACE && threadIdx.x == 0) a.trace[4] = wall_clock64();  // counters added
}

// The launched transform: one 16-wave workgroup per CU, each the same contiguous share of tiles_per_wg
// tiles (echo6_geometry); reference or wire mode (WIRE), large batches or one workgroup of sub-tiles of
// a.tile_live frames (SUBT: writes as soon as a wave has read, plain stores).  Wire batches run on the same 64-B
// windows (44 / 280 / 185 us for c2 / c3 / c4 against 71 / 298 / 215 on the 128-B windows of rounds 1-4, in-process
// A/B, profiles/r04/wire64/).
template <bool WIRE, bool SUBT, int UR = SUBT ? kU : kUR, bool USPLIT = !SUBT, bool PRIO = !SUBT,
          int SLACK = SUBT ? 0 : kRefSlack, bool HB = true>
__global__ __launch_bounds__(kThreads6, 1) void echo_round_kernel(EchoArgs a, uint32_t tiles_per_wg) {
    constexpr int TPW = SUBT ? 1 : kRefTPW;
    __shared__ Echo6Smem<TPW> sm;
    const uint32_t tl = SUBT ? a.tile_live : (uint32_t)kTile;
    const uint32_t ntiles = (a.n + tl - 1) / tl;
    const uint32_t t_begin = blockIdx.x * tiles_per_wg;
    const uint32_t t_end = min(ntiles, t_begin + tiles_per_wg);
    echo6_body<TPW, SUBT ? 0 : 2, WIRE, SUBT, false, false, !SUBT, kRefHeavy, UR, USPLIT, PRIO, SLACK, HB>(a, t_begin,
                                                                                                        t_end, sm);
}

// Round kernel geometry: one workgroup per CU (fewer for small batches), equal contiguous tile shares.
constexpr uint32_t kMaxCuBound = 1024;  // workspace bound for the round kernel's one-workgroup-per-CU grid
inline void echo6_geometry(uint32_t n, uint32_t num_cu, uint32_t* grid, uint32_t* tiles_per_wg) {
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    uint32_t g = num_cu < 1 ? 1 : num_cu;
    if (g > ntiles) g = ntiles < 1 ? 1 : ntiles;
    const uint32_t per = (ntiles + g - 1) / g;
    *tiles_per_wg = per < 1 ? 1 : per;
    *grid = (ntiles + *tiles_per_wg - 1) / *tiles_per_wg;
    if (*grid < 1) *grid = 1;
}

}  // namespace
}  // namespace xskgpu
