// xsk_echo_lab.h — the tuning laboratory of the gfx950 ICMP-echo round kernel: echo_kernel6 / echo6_body with
// every switch measured in rounds 1-2 (descriptor prefetches, dynamic and tail-pool schedules, chip-wide
// barriers, carried / deferred windows, wave-front and rotated tile orders, pipelined streams, the
// one-round 8-wave kernel, diagnostics with wrong results).  Only the tuning library (tune/xsk_tune.hip,
// tools/kbench.py, tools/abbench.py, bench.py --variant) compiles it; the product kernel lives in
// ../xsk_echo_device.h with the shipped parameter set only.  DESIGN.md §4 records what each switch measured.
//
// Replaces, for a whole batch of AF_XDP descriptors at once, the per-frame call
//   process_packet()   /root/reference/src/lib/xsk_receive.c:113-190   (gates, field swap, type 8->0,
//   csum_replace2()    /root/reference/src/lib/xsk_receive.c:101-111    RFC 1624 incremental update)
// and the counter updates of the batch loop at xsk_receive.c:171-172,229,233.  No MFMA: the op is
// integer byte arithmetic and HBM bound.
#pragma once

#include "../../../include/xsk_gpu.h"
#include "../xsk_echo_kernels.h"

namespace xskgpu {
namespace {

constexpr int kTile = XSK_GPU_TILE_FRAMES;  // frames per wave tile
constexpr int kWaves = 4;                   // waves per workgroup
constexpr int kThreads = kTile * kWaves;    // 256
constexpr int kWin = 64;                    // header window [a16, a16 + 64)
constexpr int kShipU = 4;                   // shipped kernel: row-loads in flight per lane
constexpr int kShipMinW = 6;                // shipped kernel: waves per SIMD it is register-bounded for
constexpr uint32_t kMaxLen = 1u << 30;      // build-added descriptor sanity bound (XSK_GPU_MAX_LEN)

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
    // DYN kernels only: 9 u32 queue counters (per-region heads, exit count), zero on entry and left zero
    uint32_t* queue = nullptr;
    // TRACE kernels only: wave 0's wall clock at the body's phase boundaries (diagnostics, 6 x u64)
    unsigned long long* trace = nullptr;
    // DLDS kernels only: nonzero = the batch's descriptors (n <= 64) are already in the LDS (Echo6Smem::desc)
    uint32_t desc_in_lds = 0;
    // round kernel, static shares only: nonzero = the WAVE-FRONT tile order.  The grid's front = 16 * grid
    // waves sweep the batch in passes of `front` consecutive tiles (pass p: tiles [p * front, p * front +
    // front)), every wave one tile per pass, so at any moment the whole chip reads one compact region
    // instead of one separate region per workgroup.  front_mode 1: wave w of workgroup g takes tile
    // 16 g + w of a pass; 2: tile w * grid + g.  Each workgroup then runs logical tiles [0, 16 * passes).
    uint32_t front = 0;
    uint32_t front_mode = 1;
    // round kernel, static shares only (tuning): nonzero = ROTATED shares.  Workgroup g starts its share of
    // L tiles at logical tile (g * rot) mod L and wraps, so the workgroups that run in step are not all at
    // the same offset of their (power-of-two aligned) shares at the same time.
    uint32_t rot = 0;
    // uniform long-tile stream only (tuning): nonzero = the 16 steps of a tile start at step
    // (wave * srot + blockIdx.x) mod 16 instead of 0, so the waves of the chip do not stream the same
    // frame slots of their tiles at the same time
    uint32_t srot = 0;
};

// Physical tile of logical tile lt (lt & 15 = the wave, lt >> 4 = the pass) in the wave-front order.
__device__ __forceinline__ uint32_t front_tile(const EchoArgs& a, uint32_t lt) {
    const uint32_t pass = lt >> 4, w = lt & 15u;
    return pass * a.front + (a.front_mode == 2 ? w * gridDim.x + blockIdx.x : blockIdx.x * 16u + w);
}

// Physical tile of logical tile t of the share [tb, te) in the rotated order (a.rot != 0).
__device__ __forceinline__ uint32_t rot_tile(const EchoArgs& a, uint32_t t, uint32_t tb, uint32_t te) {
    const uint32_t L = te - tb;
    uint32_t x = t - tb + (blockIdx.x * a.rot) % L;
    x = x >= L ? x - L : x;
    return tb + x;
}

// Buffer-resource word 3 for gfx950 raw buffers (cdna_hip_programming.md §5.5 T8).
constexpr int kRsrcFlags = 0x00020000;
constexpr int kAuxNT = 2;  // nontemporal: payload bytes are read exactly once
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

// Counters: wave -> workgroup -> one partial row per workgroup (no atomics).
template <int NW = kWaves>
__device__ __forceinline__ void store_partials(const EchoArgs& a, Counters c, unsigned long long (*s_cnt)[4],
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
        for (int w = 0; w < NW; ++w) s += s_cnt[w][threadIdx.x];
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
    static constexpr bool kZeroFill = true;
    __amdgpu_buffer_rsrc_t r;
    uint32_t rel;  // frame's a16 relative to the window base
    __device__ __forceinline__ u32x4 load(uint32_t ro, bool in) const {
        return __builtin_amdgcn_raw_buffer_load_b128(r, (int)(in ? rel + ro : 0x80000000u), 0, kAuxNT);
    }
};
struct FarLoader {  // 64-bit addresses; lanes past the frame re-read its first block, then select zeros
    static constexpr bool kZeroFill = true;
    const uint8_t* fbase;
    __device__ __forceinline__ u32x4 load(uint32_t ro, bool in) const {
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)(fbase + (in ? ro : 0u)));
        return in ? v : u32x4{0u, 0u, 0u, 0u};
    }
};

// ================================================================================================
// Row streams and the header phase shared by every transform kernel (the previous shipped kernel,
// echo_kernel5, now lives with the other tuning variants in xsk_echo_variants.h).  One read of every byte.  The payload is streamed by 16-lane DPP rows (row q of step s
// owns frame 4s+q, 256-B row-loads), but the stream starts at row byte 0: the first four lanes of a
// frame's first row-load carry its 64-B header window, which they drop into the frame's LDS row, so
// no separate header read is issued.  Each frame's loads span max(frame end, window end) row bytes;
// the payload sum takes row bytes [64, rowhi) and the header phase the window part.  Patched windows
// of 16-B aligned replies leave as whole 64-B sectors, 16 frames per wave-store, after the tile.
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

// Per-frame metadata of a tile, kept in LDS so that the row streams of step s read frame 4s+q's
// entry by broadcast LDS reads instead of holding it in VGPRs across the stream loop.
struct FrameMeta {
    uint32_t rel;     // a16 relative to the tile's buffer window (fast path)
    uint32_t rowhi;   // frame end, row coordinates (0 unless parsed)
    uint32_t lim;     // row bytes to load: max(rowhi, window bytes in the UMEM)
    uint32_t packed;  // off | iphi << 8 | flags << 16 (1 ok, 2 parse)
    uint32_t nit;     // 256-B row-loads: ceil(lim / 256)
    uint32_t addr_lo, addr_hi, len;
};

// One frame's row stream: row-loads j = 0 .. ns-1 (lane k takes row bytes [256 j + 16 k, +16)).  The
// first row-load carries the 64-B window: lanes 0-3 drop it into the frame's LDS row and every lane
// sums its bytes by exact range (ICMP [off+34, rowhi), IPv4 header [off+14, iphi)); later blocks only
// need the frame-end mask.
// WIRE (wire-format mode): the window is 128 B (lanes 0-7) and the stream sums only row bytes
// [128, rowhi) -- the parse, and so the ICMP start and end, are known only in the header phase, which
// sums the in-window part from LDS (wire_header_phase).
template <int U, class L, bool WIRE = false, bool D2 = false>
__device__ __forceinline__ void stream_frame(const L& ld, uint32_t ns, uint32_t f_rowhi, uint32_t f_lim,
                                             uint32_t f_off, uint32_t f_iphi, uint32_t k, uint8_t* hdr_row,
                                             RowSums& rs) {
    const int ic_lo = WIRE ? 128 : (int)f_off + 34;
    if (ns == 1u) {
        const uint32_t ro = 16u * k;
        const u32x4 x = ld.load(ro, ro < f_lim);
        if (k < (WIRE ? 8u : 4u)) *(u32x4*)(hdr_row + ro) = x;
        if (!WIRE) rs.ip += k < 4u ? sum_range(x, (int)ro, (int)f_off + 14, (int)f_iphi) : 0ull;
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
                if (k < (WIRE ? 8u : 4u)) *(u32x4*)(hdr_row + ro) = x;
                if (!WIRE) rs.ip += k < 4u ? sum_range(x, (int)ro, (int)f_off + 14, (int)f_iphi) : 0ull;
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

// Header work of one frame (lane = frame) from its LDS row and its two folded row sums.  DEFER: the
// verdict and record are returned in *verd_out / *rec_out instead of being stored (the round kernel
// stores them in its write phase).
template <bool DEFER = false, bool IPH = false, bool FASTIP = false>
__device__ __forceinline__ bool header_phase5(const EchoArgs& a, uint8_t* row, uint32_t ip_raw, uint32_t ic_raw,
                                              uint64_t addr, uint32_t len, bool live, bool ok, bool parse,
                                              uint32_t fi, Counters& cnt, u32x4* rec_out = nullptr,
                                              uint32_t* verd_out = nullptr) {
    const uint32_t off = (uint32_t)addr & 15u;
    const uint32_t* rw = (const uint32_t*)(row + (off & ~3u));
    uint32_t h[10];  // frame-relative dwords: h[k] = bytes [4k, 4k+4) of the frame
#pragma unroll
    for (int k = 0; k < 10; ++k) h[k] = __builtin_amdgcn_alignbyte(rw[k + 1], rw[k], off & 3u);

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

    // RFC 1071 sums of the input frame (build-added verification fields)
    uint32_t ip_sum = fold32(ip_raw);
    uint32_t ic_sum = fold32(ic_raw);
    if (!((uint32_t)addr & 1u)) {
        ip_sum = bswap16(ip_sum);
        ic_sum = bswap16(ic_sum);
    }
    if (IPH) {  // IPv4 header bytes [14, min(len, 34)) from the frame-relative dwords: LE halves of
                // frame-even-aligned words are byte-swapped network words (RFC 1071 §2(B))
        const int e = (int)min(len, 34u);
        uint32_t acc = 0;
        if (FASTIP && __ballot(e < 34) == 0ull) {  // every frame has the whole 20-B header: fixed masks
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
            r32[0] = n0;
            r32[1] = n1;
            r32[2] = n2;
            r32[6] = n6;
            r32[7] = n7;
            r32[8] = n8;
            r32[9] = (h[9] & 0xFFFF0000u) | csum_new_le;
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
    if (DEFER) {
        u32x4 r;
        r.x = verdict | (flags << 8) | (proto << 16) | (itype << 24);
        r.y = icode | (vihl << 8) | (eth_proto << 16);
        r.z = (parse ? bswap16(csum_le) : 0u) | ((parse ? bswap16(csum_new_le) : 0u) << 16);
        r.w = (parse ? ip_sum : 0u) | ((parse ? ic_sum : 0u) << 16);
        *rec_out = r;
        *verd_out = verdict;
    }
    if (live) {
        if (!DEFER && a.verdicts) a.verdicts[fi] = (uint8_t)verdict;
        if (!DEFER && a.recs) {
            u32x4 r;
            r.x = verdict | (flags << 8) | (proto << 16) | (itype << 24);
            r.y = icode | (vihl << 8) | (eth_proto << 16);
            r.z = (parse ? bswap16(csum_le) : 0u) | ((parse ? bswap16(csum_new_le) : 0u) << 16);
            r.w = (parse ? ip_sum : 0u) | ((parse ? ic_sum : 0u) << 16);
            ((u32x4*)a.recs)[fi] = r;
        }
        cnt.rxp += 1;
        cnt.rxb += len;
        if (tx) {
            cnt.txp += 1;
            cnt.txb += len;
        }
    }
    return wb;
}

// The echo-reply rewrite of a 16-B aligned frame's 64-B window in place (header_phase5's `wb` branch, from the
// window's own bytes): for a frame already known to be a TX_REPLY whose window is written back whole.
__device__ __forceinline__ void repatch_window(uint8_t* row) {
    uint32_t* r32 = (uint32_t*)row;
    uint32_t h[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) h[k] = r32[k];
    const uint32_t csum_le = h[9] & 0xFFFFu;
    uint32_t c16 = (~csum_le) & 0xFFFFu;
    c16 = (c16 + 0xFFF7u) & 0xFFFFu;
    c16 += c16 < 0xFFF7u ? 1u : 0u;
    r32[0] = (h[1] >> 16) | (h[2] << 16);
    r32[1] = (h[2] >> 16) | (h[0] << 16);
    r32[2] = (h[0] >> 16) | (h[1] << 16);
    r32[6] = (h[6] & 0xFFFFu) | (h[7] & 0xFFFF0000u);
    r32[7] = (h[8] & 0xFFFFu) | (h[6] & 0xFFFF0000u);
    r32[8] = (h[7] & 0xFFFFu) | (h[8] & 0xFF000000u);
    r32[9] = (h[9] & 0xFFFF0000u) | ((~c16) & 0xFFFFu);
}

// ================================================================================================
// The round kernel (shipped).  Measured on cold 4 GiB slabs (tools/wexp.hip): a read stream that
// meets scattered 64-B writes pays for them at DRAM read/write turnarounds (+61 us for 1 M header
// sectors deferred to each tile's end, +69 us for the same bytes written to a contiguous side buffer)
// while the same writes issued as a burst with no reads around them cost +20 us.  So the grid is
// persistent -- one 16-wave workgroup per CU, every workgroup the same contiguous share of tiles --
// and works in ROUNDS: each wave streams TPW tiles (the read phase: descriptors, payload, header
// phase, patched windows into LDS, records into VGPRs), the workgroup meets at a barrier, and every
// wave then stores its patched 64-B windows, records and verdicts (the write phase).  Equal shares
// keep the workgroups' rounds in step, so the chip alternates between pure read and pure write
// traffic instead of mixing them.
// ================================================================================================
constexpr int kWaves6 = 16;                 // waves per workgroup (one workgroup per CU)
constexpr int kThreads6 = kWaves6 * 64;     // 1024
constexpr int kShip6U = 4;                  // row-loads in flight per lane
constexpr int kShip6TPW = 2;                // tiles per wave per round: 2048 frames per CU per round
constexpr int kShip6Sync = 2;               // heavy waves wait for the round, light ones go ahead
constexpr int kShip6Stream = 2;             // per-step streams for uniform long tiles, sorted step-packed otherwise
constexpr bool kShip6Mid = true;            // ping-size tiles (every frame within 128 B): 8 loads at once
constexpr bool kShip6D2 = true;             // v_dot2_u32_u16 sums of halves (short, ping and per-step paths)
constexpr bool kShip6Skm = true;            // ranked streams mask only slots where a frame ends
constexpr int kShip6Ulong = 1;              // uniform long tiles: byte masks once per tile (stream_tile_uniform)
constexpr bool kShip6Pair = true;           // both tiles of a round read at once when all frames fit their windows
constexpr int kShip6Wt = 2;                 // write-phase windows and records stored write-through (sc1)
constexpr int kShip6Heavy = 512;            // SYNC 2: a wave most of whose frames have >= 512 B waits for the round

// 16-B per-frame stream metadata (the header phase keeps addr/len in the owning lane's VGPRs).
struct FrameMeta6 {
    uint32_t rel;     // a16 - window base (fast tiles); a16 >> 4 (short and far tiles)
    uint32_t rowhi;   // frame end, row coordinates (0 unless parsed)
    uint32_t lim;     // row bytes to load: max(rowhi, window bytes in the UMEM)
    uint32_t packed;  // off | iphi << 8 | flags << 16 (1 ok, 2 parse) | (a16 >> 36) << 20
};
__device__ __forceinline__ uint64_t meta6_a16(const FrameMeta6& m) {
    return ((uint64_t)(m.packed >> 20) << 36) | ((uint64_t)m.rel << 4);
}


// Sorted, step-packed row streams (echo_kernel6 with STREAM 1).  The tile's frames are ranked by their
// row-load count (ascending, ties by index; 64 readlane compares per lane); step s streams ranked frames
// 4s..4s+3, one per 16-lane row, so the four frames of a step need about the same number of row-loads
// (ragged batches waste fewer lanes), and each batch of U row-loads is packed across consecutive steps
// by a wave-uniform cursor (short frames share one round trip instead of paying one per step).  The
// IPv4 header sum is taken in the header phase from the LDS window (header_phase5<.., IPH = true>).
template <int U, bool FAST, bool WIRE = false, bool D2 = false, bool SKM = false>
__device__ __forceinline__ void stream_tile_sorted(const EchoArgs& a, __amdgpu_buffer_rsrc_t rsrc,
                                                   const FrameMeta6* meta, uint32_t* sort, uint8_t* rows,
                                                   uint32_t* sums_ic, uint32_t nit_own, uint32_t lane) {
    constexpr uint32_t kRowW = WIRE ? 128u : (uint32_t)kWin;  // LDS row (window) bytes
    const uint32_t q = lane >> 4, k = lane & 15u;
    uint32_t rank = 0;
    if (SKM && __ballot(nit_own > 7u) == 0ull) {
        // counting rank (every frame <= 7 row-loads, i.e. up to ~1.8 KB): per value v one ballot; rank =
        // lanes with fewer row-loads + lanes below with as many (same order as the compare loop below)
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
        uint32_t h = 0;  // D2: halves of this batch's blocks of step `cur`
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (us[u] >= 16u) continue;  // uniform
            if (us[u] != cur) {          // uniform: a new step begins in this slot
                if (cur < 16u) {
                    const uint32_t r = row_sum_dpp(fold64(ic + h));
                    if (k == 15u) sums_ic[cur_f] = r;
                }
                cur = us[u];
                cur_f = uf[u];
                ic = 0;
                h = 0;
            }
            const uint32_t ro = 256u * uj[u] + 16u * k;
            const u32x4 x = v[u];
            if (uj[u] == 0u) {
                if (k < kRowW / 16u && ulim[u]) *(u32x4*)(rows + uf[u] * kRowW + ro) = x;  // the header window
                if (D2) h += sum_range_h(x, (int)ro, WIRE ? 128 : (int)uoff[u] + 34, (int)urowhi[u]);
                else ic += sum_range(x, (int)ro, WIRE ? 128 : (int)uoff[u] + 34, (int)urowhi[u]);
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
                if (D2) h = sum_halves(y, h);
                else ic += sum_dw(y);
            }
        }
        if (D2) ic += h;
    }
    if (cur < 16u) {
        const uint32_t r = row_sum_dpp(fold64(ic));
        if (k == 15u) sums_ic[cur_f] = r;
    }
}


// Uniform long tiles (ULONG): every frame of the tile parsed, at the same 16-B offset and with the same end,
// so the ICMP byte range [lo, hi) = [off + 34, off + len) is the same in every row.  A lane's byte masks are
// then the same for every step: computed once per tile for the first and the last row-load (the only blocks
// the range can cut; the others are whole or, past `lim`, not loaded), and a step costs its loads, one
// v_dot2_u32_u16 per dword, two masks and the row reduction.  The sums are plain 32-bit sums of 16-bit halves
// (< 2^32 for frames <= 64 KiB: 257 blocks x 8 halves x 65535 x 16 lanes); the IPv4 header sum comes from the
// window in the header phase (IPH).
// WIRE (wire-format mode): 128-B windows, and the stream sums row bytes [128, rowhi) (lo = 128): the header
// phase completes the message sum from the window once it has parsed the headers.
template <int U, bool WIRE = false>
__device__ __forceinline__ void stream_tile_uniform(__amdgpu_buffer_rsrc_t rsrc, const FrameMeta6* meta, uint8_t* rows,
                                                    uint32_t* sums_ic, uint32_t ns, uint32_t lo, uint32_t hi,
                                                    uint32_t lane, uint32_t s0 = 0) {
    constexpr uint32_t kRowW = WIRE ? 128u : (uint32_t)kWin;
    const uint32_t q = lane >> 4, k = lane & 15u;
    const u32x4 mf = range_mask((int)(16u * k), (int)lo, (int)hi);                    // row-load 0
    const u32x4 ml = range_mask((int)(256u * (ns - 1u) + 16u * k), (int)lo, (int)hi);  // row-load ns - 1
    for (uint32_t s = 0; s < 16u; ++s) {
        const uint32_t f = 4u * ((s + s0) & 15u) + q;
        const FrameMeta6& fm = meta[f];  // broadcast read: one entry per 16-lane row
        const uint32_t rel = fm.rel, lim = fm.lim;
        uint32_t h = 0;
        for (uint32_t j0 = 0; j0 < ns; j0 += U) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t ro = 256u * (j0 + (uint32_t)u) + 16u * k;
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(ro < lim ? rel + ro : 0x80000000u), 0, kAuxNT);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = j0 + (uint32_t)u;  // wave-uniform
                if (j >= ns) break;
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

// stream_tile_uniform with the row-loads software-pipelined (ULONG 2): the tile's 16 x ns row-loads per lane
// form one sequence, issued in batches of U that may straddle steps, batch b + 1 issued before batch b is
// summed, so a lane always has loads in flight while it sums (the per-step form drains to zero twice per
// 1500-B step).  A step's frame (rel, lim) is read from the LDS metadata when its first row-load is issued;
// its row sum is reduced and stored when its last row-load has been summed.
struct UniCursor {
    uint32_t s, j;     // next row-load to issue: step s, row-load j (wave-uniform)
    uint32_t rel, lim; // the issuing step's frame (per 16-lane row)
};
template <int U>
__device__ __forceinline__ void uni_issue(u32x4 (&v)[U], uint32_t (&tag)[U], UniCursor& c, uint32_t ns,
                                          __amdgpu_buffer_rsrc_t rsrc, const FrameMeta6* meta, uint32_t q, uint32_t k) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        tag[u] = 0xFFFFFFFFu;
        v[u] = u32x4{0u, 0u, 0u, 0u};
        if (c.s < 16u) {  // uniform
            if (c.j == 0u) {
                const FrameMeta6& fm = meta[4u * c.s + q];
                c.rel = fm.rel;
                c.lim = fm.lim;
            }
            const uint32_t ro = 256u * c.j + 16u * k;
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(ro < c.lim ? c.rel + ro : 0x80000000u), 0, kAuxNT);
            tag[u] = (c.s << 16) | c.j;
            if (++c.j == ns) {
                c.j = 0;
                ++c.s;
            }
        }
    }
}
template <int U>
__device__ __forceinline__ void uni_consume(const u32x4 (&v)[U], const uint32_t (&tag)[U], uint32_t& h, uint32_t ns,
                                            u32x4 mf, u32x4 ml, uint8_t* rows, uint32_t* sums_ic, uint32_t q,
                                            uint32_t k) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (tag[u] == 0xFFFFFFFFu) continue;  // uniform
        const uint32_t s = tag[u] >> 16, j = tag[u] & 0xFFFFu, f = 4u * s + q;
        u32x4 x = v[u];
        if (j == 0u && k < 4u) *(u32x4*)(rows + f * kWin + 16u * k) = x;  // the 64-B header window
        if (j == 0u) x &= mf;
        if (j == ns - 1u) x &= ml;
        h = sum_halves(x, h);
        if (j == ns - 1u) {  // the step's frames are summed: reduce each row
            const uint32_t r = row_sum_dpp(h);
            if (k == 15u) sums_ic[f] = r;
            h = 0;
        }
    }
}
template <int U>
__device__ __forceinline__ void stream_tile_uniform_pl(__amdgpu_buffer_rsrc_t rsrc, const FrameMeta6* meta, uint8_t* rows,
                                                       uint32_t* sums_ic, uint32_t ns, uint32_t lo, uint32_t hi,
                                                       uint32_t lane) {
    const uint32_t q = lane >> 4, k = lane & 15u;
    const u32x4 mf = range_mask((int)(16u * k), (int)lo, (int)hi);
    const u32x4 ml = range_mask((int)(256u * (ns - 1u) + 16u * k), (int)lo, (int)hi);
    UniCursor c{0u, 0u, 0u, 0u};
    u32x4 A[U], B[U];
    uint32_t ta[U], tb[U];
    uint32_t h = 0;
    uni_issue<U>(A, ta, c, ns, rsrc, meta, q, k);
    for (;;) {  // ping-pong: issue the next batch, then sum the older one
        if (c.s >= 16u) {
            uni_consume<U>(A, ta, h, ns, mf, ml, rows, sums_ic, q, k);
            break;
        }
        uni_issue<U>(B, tb, c, ns, rsrc, meta, q, k);
        uni_consume<U>(A, ta, h, ns, mf, ml, rows, sums_ic, q, k);
        if (c.s >= 16u) {
            uni_consume<U>(B, tb, h, ns, mf, ml, rows, sums_ic, q, k);
            break;
        }
        uni_issue<U>(A, ta, c, ns, rsrc, meta, q, k);
        uni_consume<U>(B, tb, h, ns, mf, ml, rows, sums_ic, q, k);
    }
}

// stream_tile_sorted with the batches software-pipelined: batch b+1's U row-loads are issued before
// batch b is consumed, so 1-2 batches stay in flight per lane instead of draining to zero at every
// batch end.  The consume side re-reads each slot's frame metadata from LDS (issued under the loads).
template <int U>
struct SortedBatch {
    u32x4 v[U];
    uint32_t s[U], j[U], f[U];  // s, j wave-uniform; f per 16-lane row
};

template <int U, bool FAST>
__device__ __forceinline__ void sp_issue(SortedBatch<U>& B, uint32_t& s, uint32_t& j, uint32_t stepns,
                                         uint32_t& cs, uint32_t& cf, uint32_t& crel, uint32_t& clim, uint64_t& ca16,
                                         const uint32_t* sort, const FrameMeta6* meta, __amdgpu_buffer_rsrc_t rsrc,
                                         const EchoArgs& a, uint32_t q, uint32_t k) {
#pragma unroll
    for (int u = 0; u < U; ++u) {  // wave-uniform slot assignment
        B.s[u] = s;
        B.j[u] = j;
        if (s < 16u) {
            if (++j >= rdlane(stepns, s)) {
                ++s;
                j = 0;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        B.v[u] = u32x4{0u, 0u, 0u, 0u};
        if (B.s[u] < 16u) {
            if (B.s[u] != cs) {  // uniform: the slot starts a new step
                cs = B.s[u];
                cf = sort[4u * cs + q];
                const FrameMeta6 fm = meta[cf];
                crel = fm.rel;
                clim = fm.lim;
                if (!FAST) ca16 = meta6_a16(fm);
            }
            const uint32_t ro = 256u * B.j[u] + 16u * k;
            const bool in = ro < clim;
            if (FAST) {
                B.v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(in ? crel + ro : 0x80000000u), 0, kAuxNT);
            } else {
                const u32x4 y = __builtin_nontemporal_load((const u32x4*)(a.umem + (in ? ca16 + ro : 0ull)));
                B.v[u] = in ? y : u32x4{0u, 0u, 0u, 0u};
            }
        }
        B.f[u] = cf;
    }
}

template <int U>
__device__ __forceinline__ void sp_consume(const SortedBatch<U>& B, uint32_t& cur, uint32_t& cur_f, uint64_t& ic,
                                           const FrameMeta6* meta, uint8_t* rows, uint32_t* sums_ic, uint32_t k) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (B.s[u] >= 16u) continue;  // uniform
        if (B.s[u] != cur) {          // uniform: a new step begins in this slot
            if (cur < 16u) {
                const uint32_t r = row_sum_dpp(fold64(ic));
                if (k == 15u) sums_ic[cur_f] = r;
            }
            cur = B.s[u];
            cur_f = B.f[u];
            ic = 0;
        }
        const FrameMeta6 fm = meta[B.f[u]];
        const uint32_t rowhi = fm.rowhi, off = fm.packed & 0xFFu;
        const uint32_t ro = 256u * B.j[u] + 16u * k;
        const u32x4 x = B.v[u];
        if (B.j[u] == 0u) {
            if (k < 4u) *(u32x4*)(rows + B.f[u] * kWin + ro) = x;  // the 64-B header window
            ic += sum_range(x, (int)ro, (int)off + 34, (int)rowhi);
        } else {
            const int nb = (int)(rowhi - min(ro, rowhi));
            u32x4 y = x;
            y.x &= dw_mask(nb);
            y.y &= dw_mask(nb - 4);
            y.z &= dw_mask(nb - 8);
            y.w &= dw_mask(nb - 12);
            ic += sum_dw(y);
        }
    }
}

template <int U, bool FAST>
__device__ __forceinline__ void stream_tile_sorted_pl(const EchoArgs& a, __amdgpu_buffer_rsrc_t rsrc,
                                                      const FrameMeta6* meta, uint32_t* sort, uint8_t* rows,
                                                      uint32_t* sums_ic, uint32_t nit_own, uint32_t lane) {
    const uint32_t q = lane >> 4, k = lane & 15u;
    uint32_t rank = 0;
    for (uint32_t j = 0; j < 64u; ++j) {
        const uint32_t nj = rdlane(nit_own, j);
        rank += (nj < nit_own || (nj == nit_own && j < lane)) ? 1u : 0u;
    }
    sort[rank] = lane;
    if ((rank & 3u) == 3u) sort[64u + (rank >> 2)] = nit_own;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const uint32_t stepns = sort[64u + (lane & 15u)];
    uint32_t s = 0, j = 0;
    while (s < 16u && rdlane(stepns, s) == 0u) ++s;
    uint32_t cs = 16u, cf = 0u, crel = 0u, clim = 0u;
    uint64_t ca16 = 0;
    uint32_t cur = 16u, cur_f = 0u;
    uint64_t ic = 0;
    SortedBatch<U> A, B;
    sp_issue<U, FAST>(A, s, j, stepns, cs, cf, crel, clim, ca16, sort, meta, rsrc, a, q, k);
    while (true) {  // ping-pong: issue the next batch, then consume the older one
        if (A.s[0] >= 16u) break;
        sp_issue<U, FAST>(B, s, j, stepns, cs, cf, crel, clim, ca16, sort, meta, rsrc, a, q, k);
        sp_consume<U>(A, cur, cur_f, ic, meta, rows, sums_ic, k);
        if (B.s[0] >= 16u) break;
        sp_issue<U, FAST>(A, s, j, stepns, cs, cf, crel, clim, ca16, sort, meta, rsrc, a, q, k);
        sp_consume<U>(B, cur, cur_f, ic, meta, rows, sums_ic, k);
    }
    if (cur < 16u) {
        const uint32_t r = row_sum_dpp(fold64(ic));
        if (k == 15u) sums_ic[cur_f] = r;
    }
}


// ================================================================================================
// Wire-format header phase (xsk_gpu_echo_dev_opts; spec: include/xsk_gpu.h).
// Lane = frame.  `row` is the frame's 16-B aligned 128-B window in LDS (frame byte i at row[off + i]),
// `far_raw` the stream's folded sum of row bytes [128, off + len) (absolute-alignment domain).  Parses
// VLAN tags / IHL / tot_len / fragments, sums the IPv4 header and the in-window part of the ICMP message
// from LDS, completes the message sum (re-reading [128, off + end) from memory in the rare case that
// STRICT cuts a message short of the frame beyond the window), decides, patches the reply in LDS.
// Returns true when the patched 64-B window should leave as a whole sector (aligned, rewrite < 64 B).
// ================================================================================================
__device__ __forceinline__ uint32_t wbe16(const uint8_t* p, uint32_t i) {
    return ((uint32_t)p[i] << 8) | (uint32_t)p[i + 1];
}

__device__ __forceinline__ bool wire_header_phase(const EchoArgs& a, uint8_t* row, uint32_t far_raw, uint64_t addr,
                                                  uint32_t len, bool ok, bool live, uint32_t wend, Counters& cnt,
                                                  u32x4* rec_out, uint32_t* verd_out) {
    const bool strict = (a.opts & XSK_GPU_OPT_STRICT_IPV4) != 0u;
    const bool vlan = (a.opts & XSK_GPU_OPT_VLAN) != 0u;
    const bool verify = (a.opts & XSK_GPU_OPT_VERIFY_CSUM) != 0u;
    const uint32_t off = (uint32_t)addr & 15u;
    uint8_t* p = row + off;  // frame byte i = p[i] for off + i < wend
    uint32_t verdict = XSK_GPU_TX_REPLY;
    uint32_t l3 = 14, hl = 20, end = len, et = 0, tags = 0;
    bool hdrs = false;  // all three headers inside the frame: the record is filled
    if (!ok) verdict = XSK_GPU_DROP_BAD_DESC;
    else if (len < 14) verdict = XSK_GPU_DROP_SHORT;
    else {
        et = wbe16(p, 12);
        bool cut = false;
        if (vlan) {
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                if (!cut && (et == 0x8100u || et == 0x88A8u) && tags == (uint32_t)g) {
                    if (len < l3 + 4) cut = true;
                    else {
                        et = wbe16(p, l3 + 2);
                        l3 += 4;
                        tags++;
                    }
                }
            }
        }
        if (cut) verdict = XSK_GPU_DROP_SHORT;
        else if (et != 0x0800u) verdict = XSK_GPU_DROP_NOT_IPV4;
        else if (len < l3 + 20) verdict = XSK_GPU_DROP_SHORT;
        else {
            bool bad = false;
            if (strict) {
                const uint32_t vihl = p[l3];
                if ((vihl >> 4) != 4u || (vihl & 15u) < 5u) bad = true;
                else {
                    hl = 4u * (vihl & 15u);
                    const uint32_t tot = wbe16(p, l3 + 2);
                    if (tot < hl + 8 || l3 + tot > len) bad = true;
                    else if (wbe16(p, l3 + 6) & 0x3FFFu) bad = true;
                    else end = l3 + tot;
                }
            }
            if (bad) verdict = XSK_GPU_DROP_BAD_IP;
            else if (p[l3 + 9] != 1u) verdict = XSK_GPU_DROP_NOT_ICMP;
            else if (len < l3 + hl + 8) verdict = XSK_GPU_DROP_SHORT;
            else hdrs = true;
        }
    }
    const uint32_t l4 = l3 + hl;
    uint32_t ip_sum = 0, ic_sum = 0, itype = 0, icode = 0, csum_in = 0, flags = 0;
    if (hdrs) {
        // in-window sums (absolute-alignment domain: LE dwords of the 16-B aligned row)
        const uint32_t ic_end = off + end, ic_hi_w = min(ic_end, 128u);
        uint64_t ip_acc = 0, ic_acc = 0;
        const uint32_t* r32 = (const uint32_t*)row;
#pragma unroll 8
        for (int d = 0; d < 32; ++d) {
            const uint32_t x = r32[d];
            ip_acc += keep_bytes(x, 4 * d, (int)(off + l3), (int)(off + l4));
            ic_acc += keep_bytes(x, 4 * d, (int)(off + l4), (int)ic_hi_w);
        }
        uint64_t far = 0;
        if (ic_end > 128u) {
            if (end == len) {
                far = far_raw;  // the stream summed exactly [128, off + len)
            } else {            // STRICT message ending before the frame does, beyond the window: re-read
                const uint8_t* fb = a.umem + (addr & ~15ull);
                for (uint32_t o = 128u; o < ic_end; o += 4u)
                    far += keep_bytes(*(const uint32_t*)(fb + o), (int)o, 128, (int)ic_end);
            }
        }
        ip_sum = fold64(ip_acc);
        ic_sum = fold64(ic_acc + far);
        if (!((uint32_t)addr & 1u)) {
            ip_sum = bswap16(ip_sum);
            ic_sum = bswap16(ic_sum);
        }
        itype = p[l4];
        icode = p[l4 + 1];
        csum_in = wbe16(p, l4 + 2);
        if (ip_sum == 0xFFFFu) flags |= XSK_GPU_F_IP_CSUM_OK;
        if (ic_sum == 0xFFFFu) flags |= XSK_GPU_F_ICMP_CSUM_OK;
        if (tags) flags |= XSK_GPU_F_VLAN;
        if (hl > 20u) flags |= XSK_GPU_F_IP_OPTIONS;
        if (itype != 8u || (strict && icode != 0u)) verdict = XSK_GPU_DROP_NOT_ECHO;
        else if (verify && (ip_sum != 0xFFFFu || ic_sum != 0xFFFFu)) verdict = XSK_GPU_DROP_BAD_CSUM;
    }
    const bool tx = hdrs && verdict == XSK_GPU_TX_REPLY;
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
#pragma unroll
        for (int i = 0; i < 6; ++i) {  // xsk_receive.c:148-157 at the parsed offsets, in LDS
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
        p[l4] = 0;
        p[l4 + 2] = (uint8_t)csum_new_le;
        p[l4 + 3] = (uint8_t)(csum_new_le >> 8);
        if (off == 0u && l4 + 4u <= 64u && wend >= 64u) {
            wb = true;  // whole 64-B sector, stored in the write phase
        } else {        // byte-exact: only the rewritten bytes
            uint8_t* pkt = a.umem + addr;
#pragma unroll
            for (int i = 0; i < 12; ++i) pkt[i] = p[i];
#pragma unroll
            for (int i = 0; i < 8; ++i) pkt[l3 + 12 + i] = p[l3 + 12 + i];
            pkt[l4] = 0;
            pkt[l4 + 2] = p[l4 + 2];
            pkt[l4 + 3] = p[l4 + 3];
        }
    }
    const uint32_t vihl = hdrs ? p[l3] : 0u, proto = hdrs ? 1u : 0u;
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

// SYNC: how a wave enters its write phase.  0: at once; 1: workgroup barrier (all waves read, then
// all write); 2: a wave at least half of whose frames this round had >= HEAVY bytes (template parameter; default
// kHeavyLen, the shipped reference-mode kernel 512 -- with write-through write phases c4's waves gain from
// waiting too: DESIGN.md §4) waits until every wave of
// the workgroup has finished reading the round (LDS arrival counter), lighter waves go ahead -- the
// phase separation pays where reads dominate, and costs latency hiding where frames are short.
// 3 / 4 (tuning only): a chip-wide barrier before (3) or around (4) every write phase, on a counter the
// host zeroes at partials + 64 Ki (measured 4-80 % slower).
constexpr uint32_t kHeavyLen = 1024;
// STREAM: 0 = per-step row streams (stream_frame), 1 = sorted step-packed streams (stream_tile_sorted),
// 2 = per tile: per-step streams when every parsed frame needs the same number (>= U) of row-loads
// (uniform long frames: nothing to sort, every step fills a batch), sorted step-packed streams otherwise;
// 3 = sorted step-packed streams with software-pipelined batches (stream_tile_sorted_pl) for every
// tile; 4 = as 2 with the pipelined version.
// PF: load the descriptors of the wave's next tile while the current one streams.
// WGT (tuning only): record each workgroup's start / end wall clock (100 MHz) after the counter
// partials in the workspace (u64 [8192 + 2 g], [8192 + 2 g + 1]).
// WIRE: the wire-format mode (a.opts != 0): 128-B windows (so TPW 1), wire_header_phase.
// NTS (tuning): write-phase stores nontemporal.  NOWR (tuning, wrong results): skip the write phase,
// to time the read phase alone.
// MID: tiles whose frames all lie within 128 B of their 16-B aligned starts (pings) are read by 8-lane
// groups, 8 frames per wave-load, all 8 loads in flight.
// D2: sums of 16-bit halves with v_dot2_u32_u16 in the per-step streams, the short and ping-size paths;
// the header phase's IPv4 sum with fixed masks when every frame has its whole header.
// SKM: ranked streams mask only slots where a frame ends and rank small-row tiles by counting; uniform
// short / ping-size tiles compute their ICMP byte masks once per tile.
// Dynamic round schedule (DYN, tuning): the batch's units of kWaves6 tiles (one tile per wave) are cut
// into 8 contiguous regions, one per XCD (workgroup g is taken to sit on XCD g % 8 -- a speed heuristic
// only, nothing depends on it).  A workgroup's first round takes TPW units of its home region statically;
// later rounds claim TPW consecutive units of the home region with one atomicAdd on the region's head
// and, once it is exhausted, move on to the next regions in turn (stealing from slower XCDs).  The last
// workgroup to leave zeroes the counters for the next launch (queue: head[8], exits).  Thread 0 only.
struct DynQueue {
    uint32_t* q;
    uint32_t units, ntiles, home, k, nwg, first;
    __device__ __forceinline__ void init(const EchoArgs& a, int tpw) {
        q = a.queue;
        ntiles = (a.n + kTile - 1) / kTile;
        units = (ntiles + kWaves6 - 1) / kWaves6;
        home = blockIdx.x & 7u;
        k = 0;
        nwg = gridDim.x;
        first = 1;
        (void)tpw;
    }
    __device__ __forceinline__ uint32_t rbeg(uint32_t x) const { return (uint32_t)(((uint64_t)units * x) >> 3); }
    // workgroups whose home region is x
    __device__ __forceinline__ uint32_t nhome(uint32_t x) const { return nwg > x ? (nwg - x + 7u) >> 3 : 0u; }
    template <int TPW>
    __device__ __forceinline__ void claim_round(uint32_t (*out)[2]) {
        uint32_t u0 = 0, nu = 0;  // claimed units [u0, u0 + nu)
        if (first) {              // static first round: TPW units of the home region, no atomics
            first = 0;
            const uint32_t rb = rbeg(home), re = rbeg(home + 1);
            const uint32_t b = rb + (blockIdx.x >> 3) * (uint32_t)TPW;
            if (b < re) {
                u0 = b;
                nu = min((uint32_t)TPW, re - b);
            }
        }
        while (!nu && k < 8u) {
            const uint32_t x = (home + k) & 7u;
            const uint32_t rb = rbeg(x), re = rbeg(x + 1);
            const uint32_t ns = min(nhome(x) * (uint32_t)TPW, re - rb);  // units the first round took
            const uint32_t old = __hip_atomic_fetch_add(q + x, (uint32_t)TPW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t b = rb + ns + old;
            if (b < re) {
                u0 = b;
                nu = min((uint32_t)TPW, re - b);
            } else {
                ++k;  // region exhausted for good
            }
        }
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const bool v = (uint32_t)i < nu;
            out[i][0] = v ? (u0 + (uint32_t)i) * kWaves6 : 0u;
            out[i][1] = v ? min((u0 + (uint32_t)i + 1u) * kWaves6, ntiles) : 0u;
        }
    }
    __device__ __forceinline__ void leave() {
        if (__hip_atomic_fetch_add(q + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1u) {
            for (int x = 0; x < 9; ++x) __hip_atomic_store(q + x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
};

// LDS of one round-kernel workgroup (152.5 KiB of the CU's 160 KiB in reference mode).  NW waves, SLOTS
// LDS header-window tiles per wave (= TPW unless some tiles of a round are held in VGPRs, echo6_body VT).
template <int TPW, bool WIRE, int STREAM, int NW = kWaves6, int SLOTS = TPW>
struct Echo6Smem {
    static constexpr uint32_t kRowW = WIRE ? 128u : (uint32_t)kWin;
    __attribute__((aligned(16))) uint8_t hdr[NW][SLOTS][kTile * kRowW];  // 128 KiB: header windows
    __attribute__((aligned(16))) FrameMeta6 meta[NW][kTile];            // 16 KiB (NW 16)
    uint32_t sum[NW][2][kTile];                                          // 8 KiB
    uint32_t sort[STREAM >= 1 ? NW : 1][80];                            // 5 KiB (STREAM 1, 2)
    unsigned long long cnt[NW][4];
    uint32_t arrive;
    uint32_t claim[TPW][2];  // DYN: this round's units [begin, end) in tiles
    u32x4 desc[kTile];       // DLDS: the descriptors of a batch of <= 64 frames, delivered with its doorbell
};

// The round kernel's work over the tiles [t_begin, t_end) of one workgroup (every wave of the
// workgroup calls it with the same range): rounds of kWaves6 * TPW tiles, read phase, write phase, and
// the counters (store_partials).  echo_kernel6 runs it once per workgroup on its static share; the
// low-latency persistent kernel (xsk_lowlat.hip) once per doorbell.
// One frame's descriptor checks and stream geometry (reference mode), as the round body computes them.
struct FrameIn {
    uint64_t addr, a16;
    uint32_t len, off, rowhi, lim;
    bool ok, parse;
};
__device__ __forceinline__ FrameIn frame_in(const EchoArgs& a, u32x4 dsc, bool in_n) {
    FrameIn F;
    F.addr = (uint64_t)dsc.x | ((uint64_t)dsc.y << 32);
    F.len = dsc.z;
    const uint64_t need = F.len >= 20 ? (F.len > 38 ? F.len : 38) : F.len;  // xsk_receive.c:120-157
    F.ok = in_n && F.len <= kMaxLen && F.addr <= a.umem_size && need <= a.umem_size - F.addr;
    F.parse = F.ok && F.len >= 20u;
    F.a16 = F.addr & ~15ull;
    F.off = (uint32_t)F.addr & 15u;
    F.rowhi = F.parse ? F.off + F.len : 0u;
    const uint32_t wend = F.ok ? (uint32_t)min(a.umem_size - F.a16, (uint64_t)kWin) : 0u;
    F.lim = max(F.rowhi, F.parse ? wend : 0u);
    return F;
}

// PAIR: both tiles of a wave's round read at once when every frame of both fits its 64-B window (c2:
// minimum-size frames).  The two descriptor loads go out together, then all eight 16-B frame loads of the
// two tiles (4 lanes per frame, 16 frames per wave-load; a frame's address and limit come from its owner
// lane by bpermute, so neither tile needs the LDS metadata), and only then are they summed -- the round
// pays two memory round trips instead of four, with twice the bytes in flight.  The windows go to the two
// LDS slots, the ICMP sums to the two sum rows (the IPv4 header sum comes from the window: IPH), then the
// header phase of each tile.  Returns false (nothing written) when either tile has a longer frame.
template <bool SYNC2>
__device__ __forceinline__ bool read_round_short2(const EchoArgs& a, uint32_t t0, uint32_t t1, uint8_t* rows0,
                                                  uint8_t* rows1, uint32_t* sums0, uint32_t* sums1, uint32_t lane,
                                                  Counters& cnt, u32x4* rec, uint32_t* verd, uint32_t* alo,
                                                  uint32_t* ahi, uint64_t* wbm, uint32_t& round_long,
                                                  const u32x4* pre = nullptr) {
    if (a.front) return false;
    const uint32_t fi0 = t0 * kTile + lane, fi1 = t1 * kTile + lane;
    const bool in0 = fi0 < a.n, in1 = fi1 < a.n;
    u32x4 d0 = u32x4{0u, 0u, 0u, 0u}, d1 = u32x4{0u, 0u, 0u, 0u};
    if (pre) {  // RPF: the round's descriptors were prefetched during the previous round
        if (in0) d0 = pre[0];
        if (in1) d1 = pre[1];
    } else {
        if (in0) d0 = *(const u32x4*)(a.descs + fi0);
        if (in1) d1 = *(const u32x4*)(a.descs + fi1);
    }
    const FrameIn F0 = frame_in(a, d0, in0), F1 = frame_in(a, d1, in1);
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
    bool wb = header_phase5<true, true, true>(a, rows0 + lane * kWin, 0u, sums0[lane], F0.addr, F0.len, in0, F0.ok,
                                             F0.parse, fi0, cnt, &rec[0], &verd[0]);
    wbm[0] = __ballot(wb);
    wb = header_phase5<true, true, true>(a, rows1 + lane * kWin, 0u, sums1[lane], F1.addr, F1.len, in1, F1.ok,
                                        F1.parse, fi1, cnt, &rec[1], &verd[1]);
    wbm[1] = __ballot(wb);
    alo[0] = d0.x;
    ahi[0] = d0.y;
    alo[1] = d1.x;
    ahi[1] = d1.y;
    if (SYNC2)
        round_long += (uint32_t)__popcll(__ballot(in0 && F0.len >= kHeavyLen)) +
                      (uint32_t)__popcll(__ballot(in1 && F1.len >= kHeavyLen));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // the sums / windows are rewritten by the next round
    return true;
}

// NW: waves per workgroup.  VT: the first VT tiles of a wave's round keep their patched header windows in
// VGPRs (lane = frame, 64 B) instead of an LDS slot -- they stream through slot 0 and are copied out after
// their header phase -- so a round holds TPW tiles per wave in TPW - VT LDS slots (the one-round kernel,
// echo_kernel8: 8 waves x 8 tiles = a whole 4096-frame CU share, written in ONE write phase at its end).
template <int U, int TPW, int SYNC = 1, int STREAM = 0, bool PF = false, bool WGT = false, bool WIRE = false,
          bool NTS = false, bool NOWR = false, bool MID = false, bool D2 = false, bool SKM = false, bool SUBT = false,
          bool DYN = false, bool TRACE = false, bool DLDS = false, int NW = kWaves6, int VT = 0, int ULONG = 0,
          bool PAIR = false, bool RD2 = false, bool CARRY = false, int DEFW = 0, int RPF = 0, int DIAG = 0, int WT = 0,
          int HEAVY = (int)kHeavyLen>
__device__ __forceinline__ void echo6_body(const EchoArgs& a, uint32_t t_begin, uint32_t t_end, uint32_t tiles_per_wg,
                                           Echo6Smem<TPW, WIRE, STREAM, NW, TPW - VT>& sm) {
    static_assert(!DYN || (!PF && SYNC < 3 && !SUBT && NW == kWaves6), "the dynamic schedule takes no prefetch / grid barrier / sub-tiles");
    static_assert(!WIRE || TPW == 1, "wire windows are 128 B: one tile per wave per round");
    static_assert(VT == 0 || (!WIRE && !PF && TPW - VT >= 1 && VT <= TPW - VT), "VGPR tiles: reference mode, LDS slots for them to pass through");
    constexpr uint32_t kRowW = WIRE ? 128u : (uint32_t)kWin;  // LDS row (header window) bytes
    const uint64_t wgt_start = WGT ? wall_clock64() : 0ull;
    auto& s_hdr = sm.hdr;
    auto& s_sort = sm.sort;
    auto& s_cnt = sm.cnt;
    uint32_t& s_arrive = sm.arrive;
    if (SYNC == 2) {
        if (threadIdx.x == 0) s_arrive = 0u;
        __syncthreads();
    }
    uint32_t rounds_done = 0;

    const uint32_t wave = uniform(threadIdx.x >> 6);
    FrameMeta6* meta = sm.meta[wave];
    uint32_t* sums_ic = sm.sum[wave][0];
    uint32_t* sums_ip = sm.sum[wave][1];
    constexpr uint32_t kRound = (uint32_t)NW * TPW;
    Counters cnt;
    uint32_t lane = threadIdx.x & 63u;
    u32x4 dnext = u32x4{0u, 0u, 0u, 0u};  // PF: descriptor of this lane's frame in the wave's next tile
    if (PF) {
        const uint32_t f0 = (t_begin + wave) * kTile + lane;
        if (t_begin + wave < t_end && f0 < a.n) dnext = *(const u32x4*)(a.descs + f0);
    }

    // SYNC 3/4 (tuning only): chip-wide barriers around every write phase, on a counter the host zeroes
    // before the launch (u32 at partials + 64 Ki); every workgroup runs the same number of rounds.
    uint32_t* gbar = (SYNC >= 3 && a.partials) ? (uint32_t*)(a.partials + 65536) : nullptr;
    uint32_t gbar_n = 0;
    const uint32_t r_end = SYNC >= 3 ? t_begin + tiles_per_wg : t_end;
    DynQueue dq;
    if (DYN && threadIdx.x == 0) dq.init(a, TPW);
    // CARRY: the last tile of a round that is not the workgroup's last keeps its patched windows, record and
    // verdict in VGPRs and is written in the NEXT round's write phase, so a two-round share (c3) writes a
    // quarter of its header sectors in mid-kernel instead of half (writes that meet the other workgroups'
    // reads cost about twice as much as the ones at the end: wexp modes 62 / 65)
    static_assert(!CARRY || (!DYN && VT == 0 && !SUBT && !WIRE && SYNC < 3), "carry: static shares, reference mode");
    u32x4 cwin[4], crec = u32x4{0u, 0u, 0u, 0u};
    uint32_t cverd = 0, calo = 0, cahi = 0, cfi = 0;
    uint64_t cwbm = 0;
    bool carried = false;  // wave-uniform
    // DEFW: the windows of the penultimate round of the share are not written in its write phase but re-read,
    // re-patched and written after the last round's, so a two-round share (c3) has no write phase in mid-kernel
    // (wexp: one write phase at the end of a share 250 us, one after each half 275 us).  DEFW 1: only waves
    // whose round was heavy (SYNC 2's test) defer; 2: every wave.  Records and verdicts are written as usual.
    static_assert(!DEFW || (!DYN && VT == 0 && !SUBT && !WIRE && SYNC < 3 && !CARRY), "deferred windows: static shares, reference mode");
    uint64_t dwbm[TPW];
    uint32_t dalo[TPW], dahi[TPW];
    bool have_def = false;  // wave-uniform
    // RPF: the descriptors of a wave's next-round tiles are loaded at the start of the current round (one
    // 16-B load per lane and tile), so a round's first memory round trip is its frames, not its descriptors
    static_assert(!RPF || (!PF && !DYN && !SUBT && !DLDS && VT == 0 && SYNC < 3), "round prefetch: static shares");
    u32x4 rnext[TPW], rcur[TPW];
    auto phys_tile = [&](uint32_t t) -> uint32_t {  // the read / write phases' tile mapping; ~0u: none
        if (!SUBT && !DYN && a.front) {
            t = front_tile(a, t);
            if (t >= (a.n + kTile - 1) / kTile) return ~0u;
        }
        if (!SUBT && !DYN && a.rot) t = rot_tile(a, t, t_begin, t_end);
        return t;
    };
    auto prefetch_round = [&](uint32_t rb) {
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            rnext[i] = u32x4{0u, 0u, 0u, 0u};
            const uint32_t tl = rb + (uint32_t)i * NW + wave;
            if (tl < t_end) {
                const uint32_t t = phys_tile(tl);
                const uint32_t fi = t * (uint32_t)kTile + lane;
                if (t != ~0u && fi < a.n) rnext[i] = *(const u32x4*)(a.descs + fi);
            }
        }
    };
    // RPF 2 (adaptive): only a wave whose round streamed a ragged tile (ranked stream) prefetches the next
    // round's descriptors -- ragged tiles are short enough for a descriptor round trip to show
    bool have_pf = false;  // wave-uniform: rnext holds the next round's descriptors
    if (RPF == 1) {
        prefetch_round(t_begin);
        have_pf = true;
    }
    // WT: write-phase stores write-through (sc1: the line leaves the XCD's L2 at once instead of staying
    // dirty until the next round's reads evict it, so the write phase really is one); 1 = windows, 2 = windows
    // and records.  They are raw buffer stores (the only 16-B store that takes a cache policy): a tile's
    // windows through a buffer based at the 4 GiB-aligned UMEM region its frames share (32-bit offsets; a tile
    // whose windows straddle regions takes plain stores), its records through a buffer at the tile's first record.
    uint32_t r0 = t_begin;
    for (;;) {  // rounds, workgroup-uniform
        // slot i of this round: wave w streams tile ub[i] + w when it is below ue[i]
        uint32_t ub[TPW], ue[TPW];
        if (DYN) {
            if (threadIdx.x == 0) dq.claim_round<TPW>(sm.claim);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                ub[i] = uniform(sm.claim[i][0]);
                ue[i] = uniform(sm.claim[i][1]);
            }
            __syncthreads();  // the claim slots are rewritten next round
            if (ub[0] >= ue[0]) break;  // claims go in order: slot 0 empty = every region exhausted
        } else {
            if (r0 >= r_end) break;
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                ub[i] = r0 + (uint32_t)i * NW;
                ue[i] = t_end;
            }
            r0 += kRound;
        }
        // RPF: the next round's descriptors are loaded once this round's own loads are out -- before the last
        // tile's stream, or after the paired short tiles' reads -- so waiting for them never waits for the prefetch
        bool rpf_due = false, cur_pf = false, ragged = false;
        if (RPF) {
#pragma unroll
            for (int i = 0; i < TPW; ++i) rcur[i] = rnext[i];
            cur_pf = have_pf;
            have_pf = false;
            rpf_due = r0 < r_end;
        }
        // CARRY: the tile carried out of the previous round is written in this round's write phase
        const bool carried_prev = CARRY && carried;
        u32x4 pwin[4], prec = crec;
        const uint32_t pverd = cverd, palo = calo, pahi = cahi, pfi = cfi;
        const uint64_t pwbm = cwbm;
#pragma unroll
        for (int c = 0; c < 4; ++c) pwin[c] = cwin[c];
        carried = false;
        u32x4 rec[TPW];
        u32x4 vwin[VT > 0 ? VT : 1][4];  // VT: patched windows of the VGPR tiles (lane = frame, 64 B)
        uint32_t verd[TPW], alo[TPW], ahi[TPW];
        uint64_t wbm[TPW];
        uint32_t round_long = 0;  // SYNC 2: frames of >= kHeavyLen bytes this wave read this round (uniform)
        // ================= read phase =================
        // VT == 0: the TPW slots unrolled, every tile's outputs straight into the per-slot arrays; VT > 0 (8
        // tiles per wave): a rolled loop whose outputs are pushed onto register queues with constant indices
        // (dynamically indexed VGPR arrays would live in scratch memory)
        static_assert(!PAIR || (TPW == 2 && !WIRE && !SUBT && !PF && !DYN && VT == 0 && D2 && STREAM >= 1),
                      "paired short tiles: two-tile rounds in reference mode with dot2 sums and IPH");
        bool paired = false;
        if (PAIR && ub[0] + wave < ue[0] && ub[1] + wave < ue[1])  // wave-uniform
            paired = read_round_short2<SYNC == 2>(a, (!SUBT && !DYN && a.rot) ? rot_tile(a, ub[0] + wave, t_begin, t_end) : ub[0] + wave,
                                                  (!SUBT && !DYN && a.rot) ? rot_tile(a, ub[1] + wave, t_begin, t_end) : ub[1] + wave, s_hdr[wave][0], s_hdr[wave][TPW > 1 ? 1 : 0],
                                                  sm.sum[wave][0], sm.sum[wave][1], lane, cnt, rec, verd, alo, ahi,
                                                  wbm, round_long, (RPF && cur_pf) ? rcur : nullptr);
        if (RPF == 1 && paired && rpf_due) {
            prefetch_round(r0);
            have_pf = true;
            rpf_due = false;
        }
        constexpr int kReadUnroll = VT > 0 ? 1 : TPW;
#pragma unroll kReadUnroll
        for (int i = 0; i < TPW; ++i) {
            if (PAIR && paired) continue;  // wave-uniform: both tiles are done
            const uint32_t ub_i = VT > 0 ? ub[0] + (uint32_t)i * NW : ub[i], ue_i = VT > 0 ? ue[0] : ue[i];
            u32x4 rec_o;
            uint32_t verd_o, alo_o, ahi_o;
            uint64_t wbm_o;
            u32x4 vcur[4];
            do {  // one tile; `break` = the slot has no tile for this wave
                uint32_t t = ub_i + wave;
                wbm_o = 0ull;
                rec_o = u32x4{0u, 0u, 0u, 0u};
                verd_o = 0u;
                alo_o = 0u;
                ahi_o = 0u;
                if (t >= ue_i) break;  // wave-uniform
                if (!SUBT && !DYN && a.front) {
                    t = front_tile(a, t);
                    if (t >= (a.n + kTile - 1) / kTile) break;
                }
                if (!SUBT && !DYN && a.rot) t = rot_tile(a, t, t_begin, t_end);
                asm volatile("" : "+v"(lane));
                uint8_t* rows = s_hdr[wave][i < VT ? 0 : i - VT];  // VGPR tiles pass through slot 0
                const uint32_t q = lane >> 4, k = lane & 15u;
                static_assert(!(SUBT && PF), "sub-tiles take no descriptor prefetch");
                const uint32_t fi = t * (SUBT ? a.tile_live : (uint32_t)kTile) + lane;
                const bool in_n = (!SUBT || lane < a.tile_live) && fi < a.n;  // a live frame of the batch
                // ---- 1. descriptors (xsk_receive.c:222-223): lane i <- frame t*64+i ----------------------
                u32x4 dsc = u32x4{0u, 0u, 0u, 0u};
                if (RPF && cur_pf) {
                    if (in_n) dsc = rcur[i];
                } else if (PF) {
                    dsc = dnext;
                    const uint32_t tn = i + 1 < TPW ? t + (uint32_t)NW : r0 + wave;  // next tile (r0: next round)
                    const uint32_t fn = tn * kTile + lane;
                    dnext = u32x4{0u, 0u, 0u, 0u};
                    if (tn < t_end && fn < a.n) dnext = *(const u32x4*)(a.descs + fn);
                } else if (DLDS && a.desc_in_lds) {
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
                const bool mid_tile = MID && !WIRE && !short_tile && __ballot(lim > 128u) == 0ull;
                // SKM: every frame of the tile at the same 16-B offset with the same end (c2, pings): the ICMP
                // byte masks of a lane's block are the same for all its frames -> computed once per tile
                const uint32_t ukey = (off << 24) ^ rowhi;
                const bool uni_tile = SKM && !WIRE && (short_tile || mid_tile) && __ballot(ukey != uniform(ukey)) == 0ull;
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

                if (RPF && i == TPW - 1 && rpf_due && (RPF == 1 || ragged)) {  // the last tile's descriptors are in:
                    prefetch_round(r0);                                          // prefetch the next round's
                    have_pf = true;
                    rpf_due = false;
                }
                if (TRACE && threadIdx.x == 0 && i == 0) a.trace[0] = wall_clock64();  // descriptors parsed
                // ---- 2. stream every row byte once; windows -> LDS rows, row sums -> LDS -----------------
                if (__ballot(nit != 0u) != 0ull) {
                    __builtin_amdgcn_wave_barrier();
                    WinLoader ld;
                    ld.r = __builtin_amdgcn_make_buffer_rsrc((void*)(a.umem + (fast ? wlo : 0ull)), (short)0,
                                                             fast ? (int)((span + 15u) & ~15ull) : 0, kRsrcFlags);
                    if (WIRE && short_tile) {
                        // every frame within its 128-B window: 8 lanes per frame, 8 frames per wave-load;
                        // nothing lies past byte 128, so the streamed part of every sum is zero
                        const uint32_t kk = lane & 7u, ro = 16u * kk;
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
                            const u32x4 v = ro < meta[f].lim ? x[r] : u32x4{0u, 0u, 0u, 0u};
                            *(u32x4*)(rows + f * kRowW + ro) = v;
                        }
                        sums_ic[lane] = 0u;
                    } else if (short_tile) {
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
                            const uint32_t f_packed = fm.packed;
                            const u32x4 v = ro < fm.lim ? x[r] : u32x4{0u, 0u, 0u, 0u};
                            *(u32x4*)(rows + f * kRowW + ro) = v;
                            const int f_off = (int)(f_packed & 0xFFu), f_iphi = (int)((f_packed >> 8) & 0xFFu);
                            // D2: the IPv4 header sum comes from the window in the header phase (STREAM >= 1)
                            constexpr bool kRip = !(D2 && STREAM >= 1);
                            uint32_t rip = 0u;
                            if (kRip) rip = fold64(sum_range(v, (int)ro, f_off + 14, f_iphi));
                            uint32_t ric = (SKM && uni_tile) ? sum_halves(v & umk, 0u)
                                         : D2 ? sum_range_h(v, (int)ro, f_off + 34, (int)fm.rowhi)
                                              : fold64(sum_range(v, (int)ro, f_off + 34, (int)fm.rowhi));
                            if (kRip) rip += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rip, 0xB1, 0xF, 0xF, false);
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0xB1, 0xF, 0xF, false);
                            if (kRip) rip += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rip, 0x4E, 0xF, 0xF, false);
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x4E, 0xF, 0xF, false);
                            if (kk == 0u) {
                                sums_ic[f] = ric;
                                if (kRip) sums_ip[f] = rip;
                            }
                        }
                    } else if (MID && !WIRE && mid_tile) {
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
                            uint32_t ric = (SKM && uni_tile) ? sum_halves(v & umk, 0u)
                                         : D2 ? sum_range_h(v, (int)ro, (int)(fm.packed & 0xFFu) + 34, (int)fm.rowhi)
                                              : fold64(sum_range(v, (int)ro, (int)(fm.packed & 0xFFu) + 34, (int)fm.rowhi));
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0xB1, 0xF, 0xF, false);   // xor 1
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x4E, 0xF, 0xF, false);   // xor 2
                            ric += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ric, 0x141, 0xF, 0xF, false);  // half-row mirror
                            if (kk == 0u) sums_ic[f] = ric;
                        }
                    } else if (STREAM == 3 ||
                               (STREAM == 4 && (__ballot(nit != 0u && nit != uniform(max_nit_lane(nit))) != 0ull ||
                                                uniform(max_nit_lane(nit)) < (uint32_t)U))) {
                        static_assert(!WIRE || STREAM < 3, "wire mode uses the non-pipelined streams");
                        if (fast) stream_tile_sorted_pl<U, true>(a, ld.r, meta, s_sort[wave], rows, sums_ic, nit, lane);
                        else stream_tile_sorted_pl<U, false>(a, ld.r, meta, s_sort[wave], rows, sums_ic, nit, lane);
                    } else if (STREAM == 1 ||
                               (STREAM == 2 && (__ballot(nit != 0u && nit != uniform(max_nit_lane(nit))) != 0ull ||
                                                uniform(max_nit_lane(nit)) < (uint32_t)U))) {
                        // (the dot2 sums measured ~1 % slower in the ranked streams: the 64-bit adds stay there)
                        ragged = true;
                        if (fast) stream_tile_sorted<U, true, WIRE, RD2 && !WIRE, SKM>(a, ld.r, meta, s_sort[wave], rows, sums_ic, nit, lane);
                        else stream_tile_sorted<U, false, WIRE, RD2 && !WIRE, SKM>(a, ld.r, meta, s_sort[wave], rows, sums_ic, nit, lane);
                    } else if (ULONG && (WIRE || STREAM >= 1) && fast && __ballot(!parse) == 0ull &&
                               __ballot(ukey != uniform(ukey)) == 0ull) {
                        if (ULONG == 2 && !WIRE)
                            stream_tile_uniform_pl<U>(ld.r, meta, rows, sums_ic, uniform(nit), uniform(off) + 34u,
                                                      uniform(rowhi), lane);
                        else
                            stream_tile_uniform<U, WIRE>(ld.r, meta, rows, sums_ic, uniform(nit),
                                                         WIRE ? 128u : uniform(off) + 34u, uniform(rowhi), lane,
                                                         a.srot ? (wave * a.srot + blockIdx.x) & 15u : 0u);
                    } else {
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
                                stream_frame<U, WinLoader, WIRE, D2>(ld, ns, f_rowhi, f_lim, f_off, f_iphi, k, rows + f * kRowW, rs);
                            } else {  // frames of one tile more than 2 GiB apart (never in AF_XDP layouts)
                                FarLoader fl;
                                fl.fbase = a.umem + (f_nit ? meta6_a16(fm) : 0ull);
                                stream_frame<U, FarLoader, WIRE, D2>(fl, ns, f_rowhi, f_lim, f_off, f_iphi, k, rows + f * kRowW, rs);
                            }
                            const uint32_t ric = row_sum_dpp(fold64(rs.ic));
                            const uint32_t rip = row_sum_dpp(fold64(rs.ip));
                            if (k == 15u) {
                                sums_ic[f] = ric;
                                sums_ip[f] = rip;
                            }
                        }
                    }
                }

                // ---- 3. header phase (lane = frame); the window stays patched in LDS ---------------------
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (TRACE && threadIdx.x == 0 && i == 0) a.trace[1] = wall_clock64();  // frames streamed
                __builtin_amdgcn_wave_barrier();
                const uint32_t ic_raw = nit ? sums_ic[lane] : 0u;
                const uint32_t ip_raw = nit ? sums_ip[lane] : 0u;
                bool wb = false;
                if (DIAG & 1) {  // diagnostic (wrong results): no header phase at all
                    rec_o = u32x4{ic_raw, ip_raw, 0u, 0u};
                } else if (WIRE)
                    wb = wire_header_phase(a, rows + lane * kRowW, ic_raw, addr, len, ok, in_n, wend, cnt, &rec_o,
                                           &verd_o);
                else
                    wb = header_phase5<true, STREAM >= 1, D2>(a, rows + lane * kWin, ip_raw, ic_raw, addr, len, in_n, ok,
                                                           parse, fi, cnt, &rec_o, &verd_o);
                wbm_o = __ballot(wb);
                if (VT > 0 && i < VT) {  // keep the patched window in VGPRs; slot 0 streams the next tile
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_wave_barrier();
                    const u32x4* rw = (const u32x4*)(rows + lane * kRowW);
    #pragma unroll
                    for (int c = 0; c < 4; ++c) vcur[c] = rw[c];
                }
            } while (0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();  // meta/sums are rewritten by the next tile
            if constexpr (VT == 0) {
                rec[i] = rec_o;
                verd[i] = verd_o;
                alo[i] = alo_o;
                ahi[i] = ahi_o;
                wbm[i] = wbm_o;
            } else {
#pragma unroll
                for (int k = TPW - 1; k > 0; --k) {  // queue: tile i ends at index TPW - 1 - i
                    rec[k] = rec[k - 1];
                    verd[k] = verd[k - 1];
                    alo[k] = alo[k - 1];
                    ahi[k] = ahi[k - 1];
                    wbm[k] = wbm[k - 1];
                }
                rec[0] = rec_o;
                verd[0] = verd_o;
                alo[0] = alo_o;
                ahi[0] = ahi_o;
                wbm[0] = wbm_o;
                if (i < VT) {  // window queue: VGPR tile i ends at index VT - 1 - i
#pragma unroll
                    for (int k = (VT > 0 ? VT : 1) - 1; k > 0; --k)
#pragma unroll
                        for (int c = 0; c < 4; ++c) vwin[k][c] = vwin[k - 1][c];
#pragma unroll
                    for (int c = 0; c < 4; ++c) vwin[0][c] = vcur[c];
                }
            }
        }

        if (RPF == 1 && rpf_due) {  // this wave had no last tile this round
            prefetch_round(r0);
            have_pf = true;
        }
        if (TRACE && threadIdx.x == 0) a.trace[2] = wall_clock64();  // header phase done
        // ================= write phase: every wave of the workgroup has finished reading =================
        if (SYNC == 1) __syncthreads();
        if (SYNC >= 3 && gbar) {  // every workgroup of the chip has finished reading this round
            __syncthreads();
            ++gbar_n;
            if (threadIdx.x == 0) {
                __hip_atomic_fetch_add(gbar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // bounded spin (~0.1 s): a workgroup that is not resident can delay, never hang, the launch
                for (uint32_t it = 0; it < (1u << 21) &&
                     __hip_atomic_load(gbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gbar_n * gridDim.x; ++it)
                    __builtin_amdgcn_s_sleep(1);
            }
            __syncthreads();
        }
        if (SYNC == 2) {
            ++rounds_done;
            if (lane == 0) atomicAdd(&s_arrive, 1u);
            if (uniform(round_long) * 2u >= (uint32_t)(kTile * TPW)) {  // at least half its frames long
                while (__hip_atomic_load(&s_arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
                       rounds_done * (uint32_t)NW)
                    __builtin_amdgcn_s_sleep(2);
            }
        }
        // DEFW: this round is the penultimate one of the share (the next is the last): keep its windows
        const bool defer = DEFW && !DYN && r0 < r_end && r0 + kRound >= r_end &&
                           (DEFW == 2 || uniform(round_long) * 2u >= (uint32_t)(kTile * TPW));
        if (defer) {
            have_def = true;
#pragma unroll
            for (int i = 0; i < TPW; ++i) dwbm[i] = 0ull;
        }
#pragma unroll
        for (int ii = 0; ii < TPW; ++ii) {
            const int i = (ii + VT) % TPW;  // the LDS-slot tiles first, then the VGPR tiles (VT) through freed slots
            const int qi = VT > 0 ? TPW - 1 - i : i;          // VT: tile i's outputs on the register queues
            uint32_t t = ub[i] + wave;
            if (NOWR) {  // keep the read phase alive without storing: fold the records into a counter
                if (t < ue[i]) cnt.rxb += rec[qi].x ^ rec[qi].w ^ (uint32_t)wbm[qi];
                continue;
            }
            if (t >= ue[i]) continue;
            if (!SUBT && !DYN && a.front) {
                t = front_tile(a, t);
                if (t >= (a.n + kTile - 1) / kTile) continue;
            }
            if (!SUBT && !DYN && a.rot) t = rot_tile(a, t, t_begin, t_end);
            const uint8_t* rows = s_hdr[wave][i < VT ? i : i - VT];
            if (CARRY && i == TPW - 1 && r0 < r_end) {  // not the last round: keep this tile for the next one
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                const u32x4* rw = (const u32x4*)(rows + lane * kRowW);
#pragma unroll
                for (int c = 0; c < 4; ++c) cwin[c] = rw[c];
                crec = rec[qi];
                cverd = verd[qi];
                calo = alo[qi];
                cahi = ahi[qi];
                cwbm = wbm[qi];
                cfi = t * (uint32_t)kTile + lane;
                carried = true;
                continue;
            }
            if (i < VT && wbm[qi]) {  // a VGPR tile: its windows back into a slot whose stores have read it
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                u32x4* rw = (u32x4*)(s_hdr[wave][i < VT ? i : 0] + lane * kRowW);
#pragma unroll
                for (int c = 0; c < 4; ++c) rw[c] = vwin[i < VT ? VT - 1 - i : 0][c];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
            }
            if (DEFW && defer) {
                dwbm[i] = wbm[qi];
                dalo[i] = alo[qi];
                dahi[i] = ahi[qi];
            }
            if (wbm[qi] && !(DEFW && defer)) {  // patched windows: 16 frames x 64 B per wave-store, whole 64-B sectors
                // WT: the 4 GiB region of the tile's first written window; every written window inside it?
                const uint32_t hi_u = WT ? rdlane(ahi[qi], (uint32_t)__builtin_ctzll(wbm[qi])) : 0u;
                const bool wt_tile = WT && __ballot(((wbm[qi] >> lane) & 1ull) &&
                                                    (ahi[qi] != hi_u || alo[qi] > 0xFFFFFFC0u)) == 0ull;
                const __amdgpu_buffer_rsrc_t wrs =
                    __builtin_amdgcn_make_buffer_rsrc((void*)(a.umem + ((uint64_t)hi_u << 32)), (short)0, -1, kRsrcFlags);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                    const uint32_t kk = lane & 3u;
                    const uint32_t flo = (uint32_t)__shfl((int)alo[qi], (int)f, 64);
                    const uint32_t fhi = (uint32_t)__shfl((int)ahi[qi], (int)f, 64);
                    if ((wbm[qi] >> f) & 1ull) {
                        const uint64_t fa = (uint64_t)flo | ((uint64_t)fhi << 32);
                        const u32x4 w = *(const u32x4*)(rows + f * kRowW + 16u * kk);
                        if (WT && wt_tile) __builtin_amdgcn_raw_buffer_store_b128(w, wrs, (int)(flo + 16u * kk), 0, kAuxSC1);
                        else if (NTS) __builtin_nontemporal_store(w, (u32x4*)(a.umem + fa + 16u * kk));
                        else *(u32x4*)(a.umem + fa + 16u * kk) = w;
                    }
                }
            }
            const uint32_t fi = t * (SUBT ? a.tile_live : (uint32_t)kTile) + lane;
            if ((!SUBT || lane < a.tile_live) && fi < a.n) {
                if (a.recs) {
                    if (WT >= 2)
                        __builtin_amdgcn_raw_buffer_store_b128(
                            rec[qi],
                            __builtin_amdgcn_make_buffer_rsrc((void*)((u32x4*)a.recs + (uint64_t)uniform(t) * (SUBT ? a.tile_live : (uint32_t)kTile)),
                                                              (short)0, -1, kRsrcFlags),
                            (int)(lane * 16u), 0, kAuxSC1);
                    else if (NTS) __builtin_nontemporal_store(rec[qi], (u32x4*)a.recs + fi);
                    else ((u32x4*)a.recs)[fi] = rec[qi];
                }
                if (a.verdicts) a.verdicts[fi] = (uint8_t)verd[qi];
            }
        }
        if (CARRY && carried_prev) {  // the previous round's carried tile, through slot 0 (its stores have read it)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            u32x4* rw = (u32x4*)(s_hdr[wave][0] + lane * kRowW);
#pragma unroll
            for (int c = 0; c < 4; ++c) rw[c] = pwin[c];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            if (pwbm) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                    const uint32_t kk = lane & 3u;
                    const uint32_t flo = (uint32_t)__shfl((int)palo, (int)f, 64);
                    const uint32_t fhi = (uint32_t)__shfl((int)pahi, (int)f, 64);
                    if ((pwbm >> f) & 1ull) {
                        const uint64_t fa = (uint64_t)flo | ((uint64_t)fhi << 32);
                        *(u32x4*)(a.umem + fa + 16u * kk) = *(const u32x4*)(s_hdr[wave][0] + f * kRowW + 16u * kk);
                    }
                }
            }
            if (pfi < a.n) {
                if (a.recs) ((u32x4*)a.recs)[pfi] = prec;
                if (a.verdicts) a.verdicts[pfi] = (uint8_t)pverd;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // LDS rows are rewritten by the next round
        if (SYNC == 4 && gbar) {  // ... and every workgroup has issued its writes before anyone reads on
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            ++gbar_n;
            if (threadIdx.x == 0) {
                __hip_atomic_fetch_add(gbar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // bounded spin (~0.1 s): a workgroup that is not resident can delay, never hang, the launch
                for (uint32_t it = 0; it < (1u << 21) &&
                     __hip_atomic_load(gbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gbar_n * gridDim.x; ++it)
                    __builtin_amdgcn_s_sleep(1);
            }
            __syncthreads();
        }
    }
    // (DEFW 3 / 4 are diagnostics with wrong results: 3 drops the deferred windows, 4 re-reads them only)
    if (DEFW && DEFW != 3 && have_def) {  // the deferred windows: re-read (unchanged since), re-patched, written
        u32x4 x[TPW][4];
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t f = (uint32_t)r * 16u + (lane >> 2), kk = lane & 3u;
                const uint64_t fa = (uint64_t)(uint32_t)__shfl((int)dalo[i], (int)f, 64) |
                                    ((uint64_t)(uint32_t)__shfl((int)dahi[i], (int)f, 64) << 32);
                x[i][r] = u32x4{0u, 0u, 0u, 0u};
                if ((dwbm[i] >> f) & 1ull) x[i][r] = __builtin_nontemporal_load((const u32x4*)(a.umem + fa + 16u * kk));
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t f = (uint32_t)r * 16u + (lane >> 2), kk = lane & 3u;
                *(u32x4*)(s_hdr[wave][i] + f * kWin + 16u * kk) = x[i][r];
            }
        if (DEFW == 4) {
#pragma unroll
            for (int i = 0; i < TPW; ++i) dwbm[i] = 0ull;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < TPW; ++i)
            if ((dwbm[i] >> lane) & 1ull) repatch_window(s_hdr[wave][i] + lane * kWin);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t f = (uint32_t)r * 16u + (lane >> 2), kk = lane & 3u;
                const uint64_t fa = (uint64_t)(uint32_t)__shfl((int)dalo[i], (int)f, 64) |
                                    ((uint64_t)(uint32_t)__shfl((int)dahi[i], (int)f, 64) << 32);
                if ((dwbm[i] >> f) & 1ull)
                    *(u32x4*)(a.umem + fa + 16u * kk) = *(const u32x4*)(s_hdr[wave][i] + f * kWin + 16u * kk);
            }
    }
    if (DYN && threadIdx.x == 0) dq.leave();
    if (TRACE && threadIdx.x == 0) a.trace[3] = wall_clock64();  // write phase issued
    store_partials<NW>(a, cnt, s_cnt, wave, lane);
    if (TRACE && threadIdx.x == 0) a.trace[4] = wall_clock64();  // counters added
    if (WGT && threadIdx.x == 0 && a.partials) {
        a.partials[8192 + 2 * blockIdx.x] = wgt_start;
        a.partials[8192 + 2 * blockIdx.x + 1] = wall_clock64();
    }
}

// One 16-wave workgroup per CU, each the same contiguous share of tiles_per_wg tiles (echo6_geometry).
// SUBT: tiles of a.tile_live frames (small batches, one workgroup).
// DYN: the dynamic round schedule (DynQueue) instead of the static shares.
// TAIL (> 0): the last ntiles / TAIL tiles of the batch are not in the static shares but in a pool the
// workgroups drain once their share is done, in units of 256 frames run as 16 sub-tiles of 16 frames (one
// per wave) -- units a quarter of a tile's time, so the workgroups' end times even out (a.queue: one
// counter, zero on entry, left zero).  The static shares cover the rest (tiles_per_wg is recomputed).
template <int U, int TPW, int SYNC = 1, int STREAM = 0, bool PF = false, bool WGT = false, bool WIRE = false,
          bool NTS = false, bool NOWR = false, bool MID = false, bool D2 = false, bool SKM = false, bool SUBT = false,
          bool DYN = false, int TAIL = 0, int ULONG = 0, bool PAIR = false, bool RD2 = false, bool CARRY = false,
          int DEFW = 0, int RPF = 0, int DIAG = 0, int WT = 0, int HEAVY = (int)kHeavyLen>
__global__ __launch_bounds__(kThreads6, 1) void echo_kernel6(EchoArgs a, uint32_t tiles_per_wg) {
    __shared__ Echo6Smem<TPW, WIRE, STREAM> sm;
    const uint32_t tl = SUBT ? a.tile_live : (uint32_t)kTile;
    const uint32_t ntiles = (a.n + tl - 1) / tl;
    if (TAIL == 0) {
        // wave-front order (a.front): every workgroup runs logical tiles [0, tiles_per_wg = 16 * passes)
        const uint32_t t_begin = a.front ? 0u : blockIdx.x * tiles_per_wg;
        const uint32_t t_end = a.front ? tiles_per_wg : min(ntiles, t_begin + tiles_per_wg);
        echo6_body<U, TPW, SYNC, STREAM, PF, WGT, WIRE, NTS, NOWR, MID, D2, SKM, SUBT, DYN, false, false, kWaves6, 0,
                   ULONG, PAIR, RD2, CARRY, DEFW, RPF, DIAG, WT, HEAVY>(a, t_begin, t_end, tiles_per_wg, sm);
        return;
    }
    static_assert(TAIL == 0 || (!SUBT && !DYN && !PF && SYNC < 3), "the tail pool runs on plain static shares");
    const uint64_t wgt_start = WGT ? wall_clock64() : 0ull;
    __shared__ uint32_t s_unit;
    const uint32_t nt_tail = ntiles / (uint32_t)(TAIL > 0 ? TAIL : 1);
    const uint32_t nt_s = ntiles - nt_tail;
    const uint32_t per = (nt_s + gridDim.x - 1) / gridDim.x;
    const uint32_t t_begin = min(nt_s, blockIdx.x * per);
    const uint32_t t_end = min(nt_s, t_begin + per);
    if (t_begin < t_end)
        echo6_body<U, TPW, SYNC, STREAM, false, false, WIRE, NTS, NOWR, MID, D2, SKM>(a, t_begin, t_end, per, sm);
    // the pool: frames [f0, n) in units of 256 (16 sub-tiles of 16 frames)
    constexpr uint32_t kSub = 16, kUnit = kSub * kWaves6;
    const uint32_t f0 = nt_s * kTile;
    EchoArgs b = a;
    b.descs = a.descs + f0;
    b.verdicts = a.verdicts ? a.verdicts + f0 : nullptr;
    b.recs = a.recs ? a.recs + f0 : nullptr;
    b.n = a.n > f0 ? a.n - f0 : 0u;
    b.tile_live = kSub;
    const uint32_t units = (b.n + kUnit - 1) / kUnit, nsub = (b.n + kSub - 1) / kSub;
    while (true) {
        if (threadIdx.x == 0)
            s_unit = __hip_atomic_fetch_add(a.queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const uint32_t u = uniform(s_unit);
        __syncthreads();  // s_unit is rewritten by the next claim
        if (u >= units) break;
        echo6_body<U, TPW, SYNC, STREAM, false, false, WIRE, NTS, NOWR, MID, D2, SKM, true>(
            b, u * kWaves6, min(nsub, (u + 1) * kWaves6), kWaves6, sm);
    }
    if (threadIdx.x == 0) {  // the last workgroup out zeroes the counters for the next launch
        if (__hip_atomic_fetch_add(a.queue + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u) {
            __hip_atomic_store(a.queue, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.queue + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (WGT && a.partials) {
            a.partials[8192 + 2 * blockIdx.x] = wgt_start;
            a.partials[8192 + 2 * blockIdx.x + 1] = wall_clock64();
        }
    }
}


// The one-round kernel: 8 waves per workgroup (one workgroup per CU, 2 waves per SIMD, so up to 256 VGPRs
// per lane), rounds of TPW tiles per wave of which the first VT keep their patched windows in VGPRs
// (echo6_body VT) -- with TPW 8 / VT 4 a round is 64 tiles = 4096 frames per CU, a whole 1 M-frame batch's
// share, so every byte is read before the first header sector is written, in ONE write phase at the end
// (a write phase after every half share measured 24-26 us slower on c3's layout: wexp modes 62 / 65 / 66).
constexpr int kWaves8 = 8;
constexpr int kThreads8 = kWaves8 * 64;
template <int U, int TPW, int VT, int SYNC = 0, int STREAM = 2, bool WGT = false, bool NOWR = false, bool MID = true,
          bool D2 = true, bool SKM = true, int ULONG = 0>
__global__ __launch_bounds__(kThreads8, 1) void echo_kernel8(EchoArgs a, uint32_t tiles_per_wg) {
    __shared__ Echo6Smem<TPW, false, STREAM, kWaves8, TPW - VT> sm;
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t t_begin = blockIdx.x * tiles_per_wg;
    const uint32_t t_end = min(ntiles, t_begin + tiles_per_wg);
    echo6_body<U, TPW, SYNC, STREAM, false, WGT, false, false, NOWR, MID, D2, SKM, false, false, false, false, kWaves8,
               VT, ULONG>(a, t_begin, t_end, tiles_per_wg, sm);
}

// Launch geometry: one workgroup per kWaves tiles (the dispatcher balances ragged tiles better than
// a persistent grid: 315 vs 347 us at c3), capped so the partials workspace stays <= 512 KiB (the
// kernel's tile loop covers larger batches).
constexpr uint32_t kMaxGrid = 16384;
constexpr uint32_t kMaxCuBound = 1024;  // workspace bound for the round kernel's one-workgroup-per-CU grid
inline uint32_t echo_grid(uint32_t n) {
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    uint32_t g = (ntiles + kWaves - 1) / kWaves;
    if (g > kMaxGrid) g = kMaxGrid;
    return g < 1 ? 1 : g;
}

// Round kernel geometry: one workgroup per CU (fewer for small batches), equal contiguous tile shares.
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
