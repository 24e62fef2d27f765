// xsk_echo.hip — gfx950 (MI355X / CDNA4) kernels + C ABI for the ICMP-echo frame transform.
//
// Replaces, for a whole batch of AF_XDP descriptors at once, the per-frame call
//   process_packet()   /root/reference/src/lib/xsk_receive.c:113-190   (gates, field swap, type 8->0,
//   csum_replace2()    /root/reference/src/lib/xsk_receive.c:101-111    RFC 1624 incremental update)
// and the counter updates of the batch loop at xsk_receive.c:171-172,229,233.
//
// Kernel shape:
//   * one wavefront owns a 64-frame tile (= RX_BATCH_SIZE, xsk_utils.h:8); lane i owns frame i's
//     header fields, verdict, record and counters;
//   * the 64-byte header windows of the tile are loaded with coalesced 16-B loads (4 lanes per frame)
//     and staged in LDS (80-B padded rows: conflict-free ds_read_b128);
//   * the rest of every frame (bytes >= 64 of its 16-B aligned window) is streamed by the whole wave
//     in 1 KiB wave-loads (16 B per lane, nontemporal), P loads kept in flight through a ring over
//     the tile's flattened chunk list; the full-payload one's-complement sum is accumulated per lane
//     in 64 bits and reduced across the wave with a shuffle tree, then handed to the owning lane;
//   * only the 38 header bytes of accepted frames are written back, plus a 16-B record per frame.
// No MFMA: the op is integer byte arithmetic and HBM-read bound.

#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "../../include/xsk_gpu.h"
#include "xsk_echo_kernels.h"

using namespace xskgpu;

namespace {

constexpr int kTile = XSK_GPU_TILE_FRAMES;  // frames per wave tile
constexpr int kWaves = 4;                   // waves per workgroup
constexpr int kThreads = kTile * kWaves;    // 256
constexpr int kWin = 64;                    // header window [a16, a16 + 64)
constexpr int kPrefetch = 4;                // v2: 1 KiB wave-loads in flight per wave
constexpr int kShipU = 4;                   // v5 (shipped): row-loads in flight per lane
constexpr uint32_t kMaxLen = 1u << 30;      // build-added descriptor sanity bound (XSK_GPU_MAX_LEN)

struct EchoArgs {
    uint8_t* umem;
    uint64_t umem_size;
    const xsk_gpu_desc* descs;
    uint32_t n;
    uint8_t* verdicts;
    xsk_gpu_rec* recs;
    unsigned long long* partials;  // [gridDim.x][4]: rx_packets, rx_bytes, tx_packets, tx_bytes
};

// One slot of the streaming ring.
struct Slot {
    u32x4 v;         // 16 payload bytes of this lane
    uint32_t nv;     // valid bytes of v (0..16)
    uint32_t frame;  // owning frame (lane index in the tile), wave-uniform
    uint32_t last;   // 1 if this chunk closes its frame, wave-uniform
};

// Buffer-resource word 3 for gfx950 raw buffers (cdna_hip_programming.md §5.5 T8).
constexpr int kRsrcFlags = 0x00020000;
constexpr int kAuxNT = 2;  // nontemporal: payload bytes are read exactly once

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);  // keep it unsigned: no sign-extension
}

// Wave-wide u32 sum with DPP row shifts + row broadcasts (no LDS traffic): after the four row_shr
// steps lane 15 of each 16-lane row holds the row's inclusive sum; row_bcast:15 and row_bcast:31
// carry rows 0..2 into lane 63.  Returns the total (wave-uniform, SGPR).
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return rdlane(x, 63);
}

// Issue the 16-B load of this lane for chunk g of the tile's flattened chunk list.  Branch-free on
// the vector side: a raw buffer load whose descriptor (wave-uniform, SGPRs) spans exactly the bytes of
// the chunk that lie inside the frame, so lanes past the frame end read zeros without touching memory,
// and nothing forces a wait before the data is consumed P chunks later.
template <int WIN>
__device__ __forceinline__ void issue_chunk(Slot& s, uint32_t g, uint32_t T, uint32_t end, uint32_t nch,
                                            uint32_t a16_lo, uint32_t a16_hi, uint32_t rowhi, const uint8_t* umem,
                                            uint32_t lane) {
    uint32_t f = 0, nrec = 0, last = 0, c = 0, f_rowhi = 0;
    uint64_t base = 0;
    if (g < T) {  // wave-uniform
        // chunk g belongs to the first frame whose inclusive chunk-prefix end exceeds g
        f = (uint32_t)__popcll(__ballot(end <= g));
        const uint32_t f_end = rdlane(end, f);
        const uint32_t f_nch = rdlane(nch, f);
        c = g - (f_end - f_nch);
        base = ((uint64_t)rdlane(a16_hi, f) << 32) | (uint64_t)rdlane(a16_lo, f);
        f_rowhi = rdlane(rowhi, f);
        const uint32_t cstart = (uint32_t)WIN + c * 1024u;  // row coordinates
        const uint32_t rem = f_rowhi - cstart;             // > 0 by construction
        nrec = rem >= 1024u ? 1024u : ((rem + 15u) & ~15u);
        last = (c + 1 == f_nch) ? 1u : 0u;
        base += cstart;
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(umem + base), (short)0, (int)nrec, kRsrcFlags);
    s.v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(lane * 16u), 0, kAuxNT);
    const int32_t rem = (int32_t)(f_rowhi - ((uint32_t)WIN + c * 1024u + lane * 16u));
    s.nv = g < T ? (rem <= 0 ? 0u : (rem >= 16 ? 16u : (uint32_t)rem)) : 0u;
    s.frame = f;
    s.last = last;
}

// P    : 1 KiB wave-loads kept in flight per wave (ring depth)
// LITE : ablation / layout ceiling — stream every frame byte from offset 0 and sum it, nothing else
// ABL (ablation bits, tuning sweep only; 0 in every shipped launch): 1 = skip header write-back,
// 2 = skip records/verdicts, 4 = skip header DMA (header from stale LDS)
template <int P, bool LITE, int MINW = 1, int ABL = 0>
__global__ __launch_bounds__(kThreads, MINW) void echo_kernel(EchoArgs a) {
    constexpr int WIN = LITE ? 0 : kWin;
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[kWaves][kTile * kWin];
    __shared__ unsigned long long s_cnt[kWaves][4];

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = uniform(threadIdx.x >> 6);
    uint8_t* rows = s_hdr[wave];
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t nwaves = gridDim.x * kWaves;

    uint64_t c_rxp = 0, c_rxb = 0, c_txp = 0, c_txb = 0;

    uint32_t t = blockIdx.x * kWaves + wave;
    // descriptor of this lane's frame in the first tile (next tiles are prefetched one tile ahead)
    u32x4 dsc = *(const u32x4*)(a.descs + min(t * kTile + lane, a.n - 1));
    for (; t < ntiles; t += nwaves) {
        // ---- 1. descriptors (xsk_receive.c:222-223): lane i <- frame t*64+i ------------------------
        const uint32_t fi = t * kTile + lane;
        const bool live = fi < a.n;
        const uint64_t addr = live ? ((uint64_t)dsc.x | ((uint64_t)dsc.y << 32)) : 0;
        const uint32_t len = live ? dsc.z : 0u;
        {
            const uint32_t tn = t + nwaves;  // prefetch the next tile's descriptors
            dsc = *(const u32x4*)(a.descs + min(tn * kTile + lane, a.n - 1));
        }
        // build-added bounds check; the reference reads bytes [0,38) whenever len >= 20
        const uint64_t need = len >= 20 ? (len > 38 ? len : 38) : len;
        const bool ok = live && len <= kMaxLen && addr <= a.umem_size && need <= a.umem_size - addr;
        const bool parse = ok && (LITE || len >= 20);
        const uint32_t a16_lo = (uint32_t)addr & ~15u;
        const uint32_t a16_hi = (uint32_t)(addr >> 32);
        const uint32_t off = (uint32_t)addr & 15u;
        // frame end in row coordinates (row 0 = a16); < 2^31 because len <= kMaxLen
        const uint32_t rowhi = parse ? off + len : 0u;

        // ---- 2. streaming chunk list of the tile: bytes [WIN, rowhi) of each frame, 1 KiB chunks ----
        const uint32_t nch = rowhi > (uint32_t)WIN ? (rowhi - (uint32_t)WIN + 1023u) >> 10 : 0u;
        uint32_t end = nch;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)end, o, 64);
            if (lane >= (uint32_t)o) end += y;
        }
        const uint32_t T = rdlane(end, 63);
        Slot ring[P];
#pragma unroll
        for (int u = 0; u < P; ++u)
            issue_chunk<WIN>(ring[u], (uint32_t)u, T, end, nch, a16_lo, a16_hi, rowhi, a.umem, lane);

        // ---- 3. header windows -> LDS by DMA (global_load_lds): 16 frames x 64 B per instruction ----
        if (!LITE && !(ABL & 4)) {
            const uint32_t row_need = parse ? min(off + (uint32_t)need, (uint32_t)kWin) : 0u;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int f = r * 16 + (int)(lane >> 2);
                const uint32_t k = lane & 3u;
                const uint32_t f_lo = (uint32_t)__shfl((int)a16_lo, f, 64);
                const uint32_t f_hi = (uint32_t)__shfl((int)a16_hi, f, 64);
                const uint32_t f_need = (uint32_t)__shfl((int)row_need, f, 64);
                // unneeded blocks read the (always mapped) UMEM base; those LDS bytes are never used
                const uint64_t src = 16u * k < f_need ? ((((uint64_t)f_hi) << 32) | (uint64_t)f_lo) + 16u * k : 0ull;
                __builtin_amdgcn_global_load_lds((const void*)(a.umem + src),
                                                 (__attribute__((address_space(3))) void*)(rows + r * 1024), 16, 0, 0);
            }
        }

        // ---- 4. drain the stream: per-lane 64-bit sums, one DPP wave reduction per frame ------------
        uint64_t acc = 0;
        uint32_t sres = 0;  // this lane's frame: stream part of the ICMP sum (absolute domain)
        for (uint32_t g0 = 0; g0 < T; g0 += P) {
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const uint32_t g = g0 + (uint32_t)u;
                if (g < T) {
                    u32x4 v = ring[u].v;
                    const uint32_t nv = ring[u].nv;
                    if (nv < 16u) {
                        v.x = keep_bytes(v.x, 0, 0, (int)nv);
                        v.y = keep_bytes(v.y, 4, 0, (int)nv);
                        v.z = keep_bytes(v.z, 8, 0, (int)nv);
                        v.w = keep_bytes(v.w, 12, 0, (int)nv);
                    }
                    acc += (uint64_t)v.x + (uint64_t)v.y + (uint64_t)v.z + (uint64_t)v.w;
                    if (ring[u].last) {
                        const uint32_t tot = wave_sum_dpp(fold64(acc));
                        sres = lane == ring[u].frame ? tot : sres;  // hand the sum to the owning lane
                        acc = 0;
                    }
                }
                issue_chunk<WIN>(ring[u], g + (uint32_t)P, T, end, nch, a16_lo, a16_hi, rowhi, a.umem, lane);
            }
        }

        if (LITE) {
            if (live) {
                c_rxp += 1;
                c_rxb += len;
                c_txb += sres;  // keeps the stream live
            }
            continue;
        }

        // ---- 5. header fields from LDS (the DMA is older than every stream load: already landed) ----
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const uint8_t* row = rows + lane * kWin;
        const uint32_t* rw = (const uint32_t*)(row + (off & ~3u));
        const uint32_t sh = off & 3u;
        uint32_t h[10];  // frame-relative dwords: h[k] = bytes [4k, 4k+4) of the frame
#pragma unroll
        for (int k = 0; k < 10; ++k) h[k] = __builtin_amdgcn_alignbyte(rw[k + 1], rw[k], sh);
        uint32_t d[16];  // absolute (16-B aligned) dwords of the window
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32x4 x = ((const u32x4*)row)[q];
            d[4 * q + 0] = x.x;
            d[4 * q + 1] = x.y;
            d[4 * q + 2] = x.z;
            d[4 * q + 3] = x.w;
        }
        // one's-complement partials in the absolute-alignment domain (RFC 1071 byte-order rule)
        const int ip_lo = (int)off + 14;
        const int ip_hi = parse ? (int)off + (int)min(len, 34u) : ip_lo;
        const int ic_lo = (int)off + 34;
        const int ic_hi = parse ? (int)min(rowhi, (uint32_t)kWin) : 0;
        uint32_t s_ip = 0, s_ic = 0;
#pragma unroll
        for (int j = 3; j < 13; ++j) s_ip += halves(keep_bytes(d[j], 4 * j, ip_lo, ip_hi));
#pragma unroll
        for (int j = 8; j < 16; ++j) s_ic += halves(keep_bytes(d[j], 4 * j, ic_lo, ic_hi));

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
        c16 += c16 < 0xFFF7u ? 1u : 0u;   // end-around carry
        // csum += new (new = 0) and its carry test are no-ops
        const uint32_t csum_new_le = tx ? (~c16) & 0xFFFFu : csum_le;

        // ---- 6. checksums of the input frame (build-added verification fields) --------------------
        const uint32_t odd = (uint32_t)addr & 1u;
        uint32_t ip_sum = fold32(s_ip);
        uint32_t ic_sum = fold32(s_ic + sres);
        if (!odd) {
            ip_sum = bswap16(ip_sum);
            ic_sum = bswap16(ic_sum);
        }
        uint32_t flags = 0;
        if (parse && len >= 34 && ip_sum == 0xFFFFu) flags |= XSK_GPU_F_IP_CSUM_OK;
        if (parse && len >= 42 && ic_sum == 0xFFFFu) flags |= XSK_GPU_F_ICMP_CSUM_OK;

        // ---- 7. echo-reply rewrite, xsk_receive.c:148-157 (bytes 0-11, 26-34, 36-37) -------------
        if (tx && !(ABL & 1)) {
            const uint32_t n0 = (h[1] >> 16) | (h[2] << 16);              // s0 s1 s2 s3
            const uint32_t n1 = (h[2] >> 16) | (h[0] << 16);              // s4 s5 d0 d1
            const uint32_t n2 = (h[0] >> 16) | (h[1] << 16);              // d2 d3 d4 d5
            const uint32_t n6 = (h[6] & 0xFFFFu) | (h[7] & 0xFFFF0000u);  // csum(ip) | daddr[0:2]
            const uint32_t n7 = (h[8] & 0xFFFFu) | (h[6] & 0xFFFF0000u);  // daddr[2:4] | saddr[0:2]
            const uint32_t n8 = (h[7] & 0xFFFFu) | (h[8] & 0xFF000000u);  // saddr[2:4] | type=0 | code
            uint8_t* pkt = a.umem + addr;
            if ((addr & 3u) == 0) {
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

        // ---- 8. verdicts, records, counters --------------------------------------------------------
        if (live) {
            if (a.verdicts && !(ABL & 2)) a.verdicts[fi] = (uint8_t)verdict;
            if (a.recs && !(ABL & 2)) {
                u32x4 r;
                r.x = verdict | (flags << 8) | (proto << 16) | (itype << 24);
                r.y = icode | (vihl << 8) | (eth_proto << 16);
                r.z = (parse ? bswap16(csum_le) : 0u) | ((parse ? bswap16(csum_new_le) : 0u) << 16);
                r.w = (parse ? ip_sum : 0u) | ((parse ? ic_sum : 0u) << 16);
                ((u32x4*)a.recs)[fi] = r;
            }
            c_rxp += 1;
            c_rxb += len;
            if (tx) {
                c_txp += 1;
                c_txb += len;
            }
        }
        __builtin_amdgcn_wave_barrier();  // LDS rows are rewritten by the next tile's DMA
    }

    // ---- counters: wave -> workgroup -> one partial row per workgroup (no atomics) -----------------
    if (a.partials) {
        c_rxp = wave_sum_u64(c_rxp);
        c_rxb = wave_sum_u64(c_rxb);
        c_txp = wave_sum_u64(c_txp);
        c_txb = wave_sum_u64(c_txb);
        if (lane == 0) {
            s_cnt[wave][0] = c_rxp;
            s_cnt[wave][1] = c_rxb;
            s_cnt[wave][2] = c_txp;
            s_cnt[wave][3] = c_txb;
        }
        __syncthreads();
        if (threadIdx.x < 4) {
            unsigned long long s = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) s += s_cnt[w][threadIdx.x];
            a.partials[blockIdx.x * 4 + threadIdx.x] = s;
        }
    }
}

// ================================================================================================
// v3: continuous ring.  The chunk sequence of a wave runs through all of its tiles without a break:
// while tile `cur` is drained, tile `nxt` is already described (per-lane metadata, chunk prefix) and
// its header windows are DMA'd into the other LDS buffer, so the ring keeps issuing nxt's chunks
// across the boundary and cur's header phase runs with P stream loads still in flight.
// ================================================================================================
struct TileLane {       // this lane's frame in one tile
    uint32_t addr_lo, addr_hi, len;
    uint32_t rowhi;     // parse ? (addr & 15) + len : 0     (row coordinates, row 0 = addr & ~15)
    uint32_t nch;       // 1 KiB chunks covering [64, rowhi)
    uint32_t end;       // inclusive prefix of nch over the tile's 64 lanes
    uint32_t flags;     // 1 live, 2 ok, 4 parse
};

__device__ __forceinline__ void make_tile(TileLane& m, uint32_t& T, uint32_t t, const u32x4& dsc, const EchoArgs& a,
                                          uint32_t lane) {
    const uint32_t fi = t * kTile + lane;
    const bool live = fi < a.n;  // false for every lane when t >= ntiles
    const uint64_t addr = live ? ((uint64_t)dsc.x | ((uint64_t)dsc.y << 32)) : 0;
    const uint32_t len = live ? dsc.z : 0u;
    const uint64_t need = len >= 20 ? (len > 38 ? len : 38) : len;
    const bool ok = live && len <= kMaxLen && addr <= a.umem_size && need <= a.umem_size - addr;
    const bool parse = ok && len >= 20;
    m.addr_lo = (uint32_t)addr;
    m.addr_hi = (uint32_t)(addr >> 32);
    m.len = len;
    m.rowhi = parse ? ((uint32_t)addr & 15u) + len : 0u;
    m.nch = m.rowhi > (uint32_t)kWin ? (m.rowhi - (uint32_t)kWin + 1023u) >> 10 : 0u;
    m.flags = (live ? 1u : 0u) | (ok ? 2u : 0u) | (parse ? 4u : 0u);
    uint32_t end = m.nch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)end, o, 64);
        if (lane >= (uint32_t)o) end += y;
    }
    m.end = end;
    T = rdlane(end, 63);
}

// One LDS-DMA wave-instruction: 16 B per lane from `src` into LDS [dst, dst + 1 KiB).  Issued from
// inline asm on purpose: a compiler-visible LDS-DMA in the loop makes LLVM treat vmcnt as out of order
// and emit vmcnt(0) before every stream-slot use (draining the ring).  Completion is covered by the
// kernel's own counted s_waitcnt before the header rows are read (§5.7 item 1, M0 saved/restored).
__device__ __forceinline__ void glds16(const uint8_t* src, uint8_t* dst) {
    const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)dst;
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(uniform(lds))
        : "memory");
}

// The tile's 64-byte header windows -> LDS rows (64 B each), 16 frames per DMA instruction.
__device__ __forceinline__ void dma_headers(const TileLane& m, uint8_t* rows, const EchoArgs& a, uint32_t lane) {
    const uint32_t need = (m.flags & 4u) ? (m.len > 38 ? m.len : 38u) : 0u;
    const uint32_t row_need = min((m.addr_lo & 15u) + need, (uint32_t)kWin);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int f = r * 16 + (int)(lane >> 2);
        const uint32_t k = lane & 3u;
        const uint32_t f_lo = (uint32_t)__shfl((int)(m.addr_lo & ~15u), f, 64);
        const uint32_t f_hi = (uint32_t)__shfl((int)m.addr_hi, f, 64);
        const uint32_t f_need = (uint32_t)__shfl((int)row_need, f, 64);
        // unneeded blocks read the (always mapped) UMEM base; those LDS bytes are never used
        const uint64_t src = 16u * k < f_need ? ((((uint64_t)f_hi) << 32) | (uint64_t)f_lo) + 16u * k : 0ull;
        glds16(a.umem + src, rows + r * 1024);
    }
}

struct Slot3 {
    u32x4 v;
    uint32_t nv;     // valid bytes (per lane)
    uint32_t frame;  // wave-uniform
    uint32_t flags;  // wave-uniform: 1 = holds a chunk, 2 = chunk closes its frame, 4 = owning tile parity
};

// Refill a slot with the next issuable chunk position I (in cur = [cs, cs+cT) or nxt = the cT..cT+nT
// that follow); beyond the described tiles the slot stays empty.  Exactly ONE buffer load is issued
// either way (an empty slot loads zero bytes), so every refill costs the same vmcnt step and the
// compiler's wait counting stays exact.
__device__ __forceinline__ void refill3(Slot3& s, uint32_t& I, uint32_t cs, uint32_t cT, uint32_t nT, uint32_t cpar,
                                        const TileLane& cur, const TileLane& nxt, const uint8_t* umem,
                                        uint32_t lane) {
    uint32_t f = 0, nrec = 0, flags = 0, cstart = 0, f_rowhi = 0;
    uint64_t base = 0;
    const uint32_t rel = I - cs;
    if (rel < cT + nT) {  // wave-uniform
        const bool in_cur = rel < cT;
        const uint32_t g = in_cur ? rel : rel - cT;
        uint32_t f_end, f_nch, lo, hi;
        if (in_cur) {
            f = (uint32_t)__popcll(__ballot(cur.end <= g));
            f_end = rdlane(cur.end, f);
            f_nch = rdlane(cur.nch, f);
            lo = rdlane(cur.addr_lo, f);
            hi = rdlane(cur.addr_hi, f);
            f_rowhi = rdlane(cur.rowhi, f);
        } else {
            f = (uint32_t)__popcll(__ballot(nxt.end <= g));
            f_end = rdlane(nxt.end, f);
            f_nch = rdlane(nxt.nch, f);
            lo = rdlane(nxt.addr_lo, f);
            hi = rdlane(nxt.addr_hi, f);
            f_rowhi = rdlane(nxt.rowhi, f);
        }
        const uint32_t c = g - (f_end - f_nch);
        cstart = (uint32_t)kWin + c * 1024u;
        const uint32_t rem = f_rowhi - cstart;
        nrec = rem >= 1024u ? 1024u : ((rem + 15u) & ~15u);
        flags = 1u | ((c + 1 == f_nch) ? 2u : 0u) | ((in_cur ? cpar : cpar ^ 1u) ? 4u : 0u);
        base = ((((uint64_t)hi) << 32) | (uint64_t)(lo & ~15u)) + cstart;
        ++I;
    }
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)(umem + base), (short)0, (int)nrec, kRsrcFlags);
    s.v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(lane * 16u), 0, kAuxNT);
    const int32_t rem = (int32_t)(f_rowhi - (cstart + lane * 16u));
    s.nv = rem <= 0 ? 0u : (rem >= 16 ? 16u : (uint32_t)rem);
    s.frame = f;
    s.flags = flags;
}

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

// Stores hidden from hipcc's wait-count bookkeeping.  On gfx950 vmcnt retires loads, stores and
// LDS-DMA in issue order (MI355X_MICROARCH.md, s_waitcnt), but LLVM treats a counter with both loads
// and stores pending as out-of-order and would drain the whole stream ring (vmcnt(0)) after every
// header phase.  Nothing in the kernel reads these bytes back, so no wait is needed for them at all;
// `s_nop 1` ends each statement so the next VALU cannot overwrite the data VGPRs early (§5.7 item 1).
__device__ __forceinline__ void st_hdr_aligned(uint8_t* p, u32x3 w012, u32x3 w678, uint32_t csum) {
    asm volatile(
        "global_store_dwordx3 %0, %1, off\n\t"
        "global_store_dwordx3 %0, %2, off offset:24\n\t"
        "global_store_short %0, %3, off offset:36\n\t"
        "s_nop 1" ::"v"(p),
        "v"(w012), "v"(w678), "v"(csum)
        : "memory");
}
__device__ __forceinline__ void st_byte(uint8_t* p, uint32_t v) {
    asm volatile("global_store_byte %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_b128(void* p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ u32x4 load_desc(const xsk_gpu_desc* d, uint32_t i) {
    const u32x3 x = *(const u32x3*)(d + i);  // 12 bytes: addr, len (options unused)
    return u32x4{x.x, x.y, x.z, 0u};
}

template <int P>
__global__ __launch_bounds__(kThreads) void echo_kernel3(EchoArgs a) {
    constexpr uint32_t K = P + 6;  // counted wait: younger VM ops allowed to stay in flight
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[kWaves][2][kTile * kWin];
    __shared__ __attribute__((aligned(16))) uint8_t s_dsc[kWaves][kTile * 16];  // prefetched descriptors
    __shared__ unsigned long long s_cnt[kWaves][4];

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = uniform(threadIdx.x >> 6);
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t nw = gridDim.x * kWaves;
    uint64_t c_rxp = 0, c_rxb = 0, c_txp = 0, c_txb = 0;

    uint32_t tc = blockIdx.x * kWaves + wave;  // cur tile index
    if (tc < ntiles) {
        const uint32_t nmax = a.n - 1;
        const u32x4 d0 = load_desc(a.descs, min(tc * kTile + lane, nmax));
        const u32x4 d1 = load_desc(a.descs, min((tc + nw) * kTile + lane, nmax));
        TileLane cur, nxt;
        uint32_t cT, nT;
        make_tile(cur, cT, tc, d0, a, lane);
        dma_headers(cur, s_hdr[wave][0], a, lane);
        make_tile(nxt, nT, tc + nw, d1, a, lane);
        if (tc + nw < ntiles) dma_headers(nxt, s_hdr[wave][1], a, lane);
        // descriptors of the tile after nxt arrive by LDS-DMA (one 1 KiB wave-instruction)
        glds16((const uint8_t*)(a.descs + min((tc + 2 * nw) * kTile + lane, nmax)), s_dsc[wave]);
        // VM ops issued after DMA(cur) / DMA(nxt) / the descriptor DMA (stores are not counted: an
        // undercount only makes the counted waits stricter)
        uint32_t vm_cur = 4 + 1 + (tc + nw < ntiles ? 4u : 0u);
        uint32_t vm_nxt = 1;
        uint32_t vm_dsc = 0;
        uint32_t cpar = 0;   // parity of cur (selects LDS buffer and stream-sum register)
        uint32_t cs = 0;     // global chunk position where cur starts
        uint32_t I = 0;      // next chunk position to issue
        uint32_t Gc = 0;     // chunks consumed
        uint32_t sres0 = 0, sres1 = 0;
        uint64_t acc = 0;

        Slot3 ring[P];
#pragma unroll
        for (int u = 0; u < P; ++u) refill3(ring[u], I, cs, cT, nT, cpar, cur, nxt, a.umem, lane);
        vm_cur += P;
        vm_nxt += P;
        vm_dsc += P;

        while (true) {
            // ---- one round over the ring: consume every slot in issue order, refill it ----
#pragma unroll
            for (int u = 0; u < P; ++u) {
                if (ring[u].flags & 1u) {
                    u32x4 v = ring[u].v;
                    const uint32_t nv = ring[u].nv;
                    if (nv < 16u) {
                        v.x = keep_bytes(v.x, 0, 0, (int)nv);
                        v.y = keep_bytes(v.y, 4, 0, (int)nv);
                        v.z = keep_bytes(v.z, 8, 0, (int)nv);
                        v.w = keep_bytes(v.w, 12, 0, (int)nv);
                    }
                    acc += (uint64_t)v.x + (uint64_t)v.y + (uint64_t)v.z + (uint64_t)v.w;
                    if (ring[u].flags & 2u) {
                        const uint32_t tot = wave_sum_dpp(fold64(acc));
                        const bool mine = lane == ring[u].frame;
                        if (ring[u].flags & 4u) sres1 = mine ? tot : sres1;
                        else sres0 = mine ? tot : sres0;
                        acc = 0;
                    }
                    ++Gc;
                }
                refill3(ring[u], I, cs, cT, nT, cpar, cur, nxt, a.umem, lane);
            }
            vm_cur += P;
            vm_nxt += P;
            vm_dsc += P;

            // ---- tiles whose chunks are all consumed: header phase, then shift ----
            while (Gc >= cs + cT && tc < ntiles) {
                // DMA(cur) must have landed: all but the K youngest VM ops are complete
                if (vm_cur >= K) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                const uint8_t* row = s_hdr[wave][cpar] + lane * kWin;
                const uint32_t sres = cpar ? sres1 : sres0;
                {
                    const uint32_t flags = cur.flags;
                    const bool live = flags & 1u, ok = flags & 2u, parse = flags & 4u;
                    const uint32_t len = cur.len;
                    const uint32_t off = cur.addr_lo & 15u;
                    const uint32_t* rw = (const uint32_t*)(row + (off & ~3u));
                    uint32_t h[10];
#pragma unroll
                    for (int k = 0; k < 10; ++k) h[k] = __builtin_amdgcn_alignbyte(rw[k + 1], rw[k], off & 3u);
                    const uint32_t* d = (const uint32_t*)row;
                    const int ip_lo = (int)off + 14;
                    const int ip_hi = parse ? (int)off + (int)min(len, 34u) : ip_lo;
                    const int ic_lo = (int)off + 34;
                    const int ic_hi = parse ? (int)min(cur.rowhi, (uint32_t)kWin) : 0;
                    uint32_t s_ip = 0, s_ic = 0;
#pragma unroll
                    for (int j = 3; j < 13; ++j) s_ip += halves(keep_bytes(d[j], 4 * j, ip_lo, ip_hi));
#pragma unroll
                    for (int j = 8; j < 16; ++j) s_ic += halves(keep_bytes(d[j], 4 * j, ic_lo, ic_hi));
                    const uint32_t eth_proto = parse ? (((h[3] & 0xFFu) << 8) | ((h[3] >> 8) & 0xFFu)) : 0u;
                    const uint32_t vihl = parse ? (h[3] >> 16) & 0xFFu : 0u;
                    const uint32_t proto = parse ? h[5] >> 24 : 0u;
                    const uint32_t itype = parse ? (h[8] >> 16) & 0xFFu : 0u;
                    const uint32_t icode = parse ? h[8] >> 24 : 0u;
                    const uint32_t csum_le = parse ? h[9] & 0xFFFFu : 0u;
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
                    c16 = (c16 + 0xFFF7u) & 0xFFFFu;
                    c16 += c16 < 0xFFF7u ? 1u : 0u;
                    const uint32_t csum_new_le = tx ? (~c16) & 0xFFFFu : csum_le;
                    uint32_t ip_sum = fold32(s_ip);
                    uint32_t ic_sum = fold32(s_ic + sres);
                    if (!(cur.addr_lo & 1u)) {
                        ip_sum = bswap16(ip_sum);
                        ic_sum = bswap16(ic_sum);
                    }
                    uint32_t rflags = 0;
                    if (parse && len >= 34 && ip_sum == 0xFFFFu) rflags |= XSK_GPU_F_IP_CSUM_OK;
                    if (parse && len >= 42 && ic_sum == 0xFFFFu) rflags |= XSK_GPU_F_ICMP_CSUM_OK;
                    if (tx) {  // xsk_receive.c:148-157
                        const uint32_t n0 = (h[1] >> 16) | (h[2] << 16);
                        const uint32_t n1 = (h[2] >> 16) | (h[0] << 16);
                        const uint32_t n2 = (h[0] >> 16) | (h[1] << 16);
                        const uint32_t n6 = (h[6] & 0xFFFFu) | (h[7] & 0xFFFF0000u);
                        const uint32_t n7 = (h[8] & 0xFFFFu) | (h[6] & 0xFFFF0000u);
                        const uint32_t n8 = (h[7] & 0xFFFFu) | (h[8] & 0xFF000000u);
                        uint8_t* pkt = a.umem + ((((uint64_t)cur.addr_hi) << 32) | (uint64_t)cur.addr_lo);
                        if ((cur.addr_lo & 3u) == 0) {
                            st_hdr_aligned(pkt, u32x3{n0, n1, n2}, u32x3{n6, n7, n8}, csum_new_le);
                        } else {
                            const uint32_t w[6] = {n0, n1, n2, n6, n7, n8};
#pragma unroll
                            for (int b = 0; b < 12; ++b) st_byte(pkt + b, w[b >> 2] >> (8 * (b & 3)));
#pragma unroll
                            for (int b = 0; b < 12; ++b) st_byte(pkt + 24 + b, w[3 + (b >> 2)] >> (8 * (b & 3)));
                            st_byte(pkt + 36, csum_new_le);
                            st_byte(pkt + 37, csum_new_le >> 8);
                        }
                    }
                    if (live) {
                        const uint32_t fi = tc * kTile + lane;
                        if (a.verdicts) st_byte(a.verdicts + fi, verdict);
                        if (a.recs) {
                            u32x4 r;
                            r.x = verdict | (rflags << 8) | (proto << 16) | (itype << 24);
                            r.y = icode | (vihl << 8) | (eth_proto << 16);
                            r.z = (parse ? bswap16(csum_le) : 0u) | ((parse ? bswap16(csum_new_le) : 0u) << 16);
                            r.w = (parse ? ip_sum : 0u) | ((parse ? ic_sum : 0u) << 16);
                            st_b128((u32x4*)a.recs + fi, r);
                        }
                        c_rxp += 1;
                        c_rxb += len;
                        if (tx) {
                            c_txp += 1;
                            c_txb += len;
                        }
                    }
                }
                if (cpar) sres1 = 0;
                else sres0 = 0;
                // ---- shift: cur <- nxt, describe the tile after it and start its header DMA ----
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS reads of cur done
                __builtin_amdgcn_wave_barrier();
                cs += cT;
                tc += nw;
                cur = nxt;
                cT = nT;
                cpar ^= 1u;
                vm_cur = vm_nxt;
                if (vm_dsc >= K) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                const u32x4 dp = ((const u32x4*)s_dsc[wave])[lane];
                make_tile(nxt, nT, tc + nw, dp, a, lane);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // descriptor row read before reuse
                __builtin_amdgcn_wave_barrier();
                if (tc + nw < ntiles) {
                    dma_headers(nxt, s_hdr[wave][cpar ^ 1u], a, lane);
                    vm_cur += 4;
                    vm_dsc += 4;
                    vm_nxt = 0;
                }
                glds16((const uint8_t*)(a.descs + min((tc + 2 * nw) * kTile + lane, nmax)), s_dsc[wave]);
                vm_dsc = 0;
                ++vm_cur;
                ++vm_nxt;
            }
            if (tc >= ntiles) break;
        }
    }

    // ---- counters: wave -> workgroup -> one partial row per workgroup (no atomics) -----------------
    if (a.partials) {
        c_rxp = wave_sum_u64(c_rxp);
        c_rxb = wave_sum_u64(c_rxb);
        c_txp = wave_sum_u64(c_txp);
        c_txb = wave_sum_u64(c_txb);
        if (lane == 0) {
            s_cnt[wave][0] = c_rxp;
            s_cnt[wave][1] = c_rxb;
            s_cnt[wave][2] = c_txp;
            s_cnt[wave][3] = c_txb;
        }
        __syncthreads();
        if (threadIdx.x < 4) {
            unsigned long long s = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) s += s_cnt[w][threadIdx.x];
            a.partials[blockIdx.x * 4 + threadIdx.x] = s;
        }
    }
}

// ================================================================================================
// v4: row streaming.  The wave still owns a 64-frame tile (lane f = frame f for descriptor, header,
// verdict, record and counters), but the payload is streamed by the four 16-lane DPP rows of the
// wave: in step s, row q streams frame 4s+q with 256-B row-loads (16 B per lane), so a 1500-B frame
// takes 6 loads at 98 % lane utilisation and its partial sum is folded inside the row by 4 DPP row
// shifts instead of a whole-wave reduction.  Latency is hidden by occupancy (<= 64 VGPRs, 8 waves
// per SIMD) plus U loads in flight per lane, not by a cross-frame ring.
// ================================================================================================
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

// One frame's header work (lane = frame): gates, rewrite, checksums, verdict, record, counters.
// `row` is the frame's 64-B header window [a16, a16 + 64) in LDS; `sres` the folded stream sum of
// row bytes [64, rowhi) in the absolute-alignment domain.
struct Counters {
    uint64_t rxp = 0, rxb = 0, txp = 0, txb = 0;
};

// WB64: a 16-B aligned reply is patched into its LDS row instead of memory and the function returns
// true; the caller then stores the whole 64-B window with coalesced full-sector writes (bytes other
// than [0,38) are rewritten with the values they held).  Unaligned replies are stored byte-exact here.
template <bool WB64>
__device__ __forceinline__ bool header_phase(const EchoArgs& a, uint8_t* row, uint32_t sres, uint64_t addr,
                                             uint32_t len, bool live, bool ok, bool parse, uint32_t fi,
                                             Counters& cnt) {
    const uint32_t off = (uint32_t)addr & 15u;
    const uint32_t rowhi = parse ? off + len : 0u;
    const uint32_t* rw = (const uint32_t*)(row + (off & ~3u));
    uint32_t h[10];  // frame-relative dwords: h[k] = bytes [4k, 4k+4) of the frame
#pragma unroll
    for (int k = 0; k < 10; ++k) h[k] = __builtin_amdgcn_alignbyte(rw[k + 1], rw[k], off & 3u);
    uint32_t d[16];  // absolute (16-B aligned) dwords of the window
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const u32x4 x = ((const u32x4*)row)[q];
        d[4 * q + 0] = x.x;
        d[4 * q + 1] = x.y;
        d[4 * q + 2] = x.z;
        d[4 * q + 3] = x.w;
    }
    const int ip_lo = (int)off + 14;
    const int ip_hi = parse ? (int)off + (int)min(len, 34u) : ip_lo;
    const int ic_lo = (int)off + 34;
    const int ic_hi = parse ? (int)min(rowhi, (uint32_t)kWin) : 0;
    uint32_t s_ip = 0, s_ic = 0;
#pragma unroll
    for (int j = 3; j < 13; ++j) s_ip += halves(keep_bytes(d[j], 4 * j, ip_lo, ip_hi));
#pragma unroll
    for (int j = 8; j < 16; ++j) s_ic += halves(keep_bytes(d[j], 4 * j, ic_lo, ic_hi));

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
    uint32_t ip_sum = fold32(s_ip);
    uint32_t ic_sum = fold32(s_ic + sres);
    if (!((uint32_t)addr & 1u)) {
        ip_sum = bswap16(ip_sum);
        ic_sum = bswap16(ic_sum);
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
        uint8_t* pkt = a.umem + addr;
        if (WB64 && (addr & 15u) == 0 && a.umem_size - addr >= (uint64_t)kWin) {
            uint32_t* r32 = (uint32_t*)row;  // row 0 == frame byte 0
            r32[0] = n0;
            r32[1] = n1;
            r32[2] = n2;
            r32[6] = n6;
            r32[7] = n7;
            r32[8] = n8;
            r32[9] = (h[9] & 0xFFFF0000u) | csum_new_le;
            wb = true;
        } else if ((addr & 3u) == 0) {
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
    if (live) {
        if (a.verdicts) a.verdicts[fi] = (uint8_t)verdict;
        if (a.recs) {
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

// Counters: wave -> workgroup -> one partial row per workgroup (no atomics).
__device__ __forceinline__ void store_partials(const EchoArgs& a, Counters c, unsigned long long (*s_cnt)[4],
                                               uint32_t wave, uint32_t lane) {
    if (!a.partials) return;
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
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long s = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s += s_cnt[w][threadIdx.x];
        a.partials[blockIdx.x * 4 + threadIdx.x] = s;
    }
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
struct FarLoader {  // 64-bit addresses; lanes past the frame re-read its first block (masked to zero)
    static constexpr bool kZeroFill = false;
    const uint8_t* fbase;
    __device__ __forceinline__ u32x4 load(uint32_t ro, bool in) const {
        return __builtin_nontemporal_load((const u32x4*)(fbase + (in ? ro : 0u)));
    }
};

// Sum (64-bit, of LE dwords) of row bytes [64, f_rowhi) of this lane's frame: lane k of the row takes
// bytes [64 + 256 j + 16 k, +16) for j < ns.  U loads are issued before the first is consumed.
template <int U, class L>
__device__ __forceinline__ uint64_t stream_row(const L& ld, uint32_t ns, uint32_t f_rowhi, uint32_t k) {
    uint64_t acc = 0;
    for (uint32_t j0 = 0; j0 < ns; j0 += U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t ro = (uint32_t)kWin + 256u * (j0 + (uint32_t)u) + 16u * k;
            v[u] = ld.load(ro, ro < f_rowhi);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t ro = (uint32_t)kWin + 256u * (j0 + (uint32_t)u) + 16u * k;
            const int nb = (int)(f_rowhi - min(ro, f_rowhi));  // valid bytes of this block (0..)
            u32x4 x = v[u];
            const bool fix = L::kZeroFill ? (nb > 0 && nb < 16) : (nb < 16);
            if (__ballot(fix) != 0ull) {  // wave-uniform: only blocks that end (or miss) a frame
                x.x &= dw_mask(nb);
                x.y &= dw_mask(nb - 4);
                x.z &= dw_mask(nb - 8);
                x.w &= dw_mask(nb - 12);
            }
            acc += (uint64_t)x.x + (uint64_t)x.y + (uint64_t)x.z + (uint64_t)x.w;
        }
    }
    return acc;
}

template <int U, int MINW, bool WB64 = true>
__global__ __launch_bounds__(kThreads, MINW) void echo_kernel4(EchoArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[kWaves][kTile * kWin];
    __shared__ uint32_t s_sum[kWaves][kTile];
    __shared__ unsigned long long s_cnt[kWaves][4];

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = uniform(threadIdx.x >> 6);
    const uint32_t q = lane >> 4, k = lane & 15u;
    uint8_t* rows = s_hdr[wave];
    uint32_t* sums = s_sum[wave];
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t nwaves = gridDim.x * kWaves;
    Counters cnt;

    for (uint32_t t = blockIdx.x * kWaves + wave; t < ntiles; t += nwaves) {
        // ---- 1. descriptors (xsk_receive.c:222-223): lane i <- frame t*64+i ----------------------------
        const uint32_t fi = t * kTile + lane;
        const bool live = fi < a.n;
        u32x4 dsc = u32x4{0u, 0u, 0u, 0u};
        if (live) dsc = *(const u32x4*)(a.descs + fi);
        const uint64_t addr = (uint64_t)dsc.x | ((uint64_t)dsc.y << 32);
        const uint32_t len = dsc.z;
        // build-added bounds check; the reference reads bytes [0,38) whenever len >= 20
        const uint64_t need = len >= 20 ? (len > 38 ? len : 38) : len;
        const bool ok = live && len <= kMaxLen && addr <= a.umem_size && need <= a.umem_size - addr;
        const bool parse = ok && len >= 20;
        const uint32_t off = (uint32_t)addr & 15u;
        const uint32_t a16_lo = (uint32_t)addr & ~15u;
        const uint32_t a16_hi = (uint32_t)(addr >> 32);
        const uint32_t rowhi = parse ? off + len : 0u;  // frame end, row coordinates (row 0 = a16)

        // ---- 2. header windows -> LDS by DMA: 16 frames x 64 B per wave-instruction -----------------
        {
            // the whole window when it lies in the UMEM (the write-back of step 5 stores all of it)
            const uint64_t room = a.umem_size - (addr & ~15ull);
            const uint32_t row_need = parse ? (uint32_t)min(room, (uint64_t)kWin) : 0u;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int f = r * 16 + (int)(lane >> 2);
                const uint32_t kk = lane & 3u;
                const uint32_t f_lo = (uint32_t)__shfl((int)a16_lo, f, 64);
                const uint32_t f_hi = (uint32_t)__shfl((int)a16_hi, f, 64);
                const uint32_t f_need = (uint32_t)__shfl((int)row_need, f, 64);
                // unneeded blocks read the (always mapped) UMEM base; those LDS bytes are never used
                const uint64_t src =
                    16u * kk < f_need ? ((((uint64_t)f_hi) << 32) | (uint64_t)f_lo) + 16u * kk : 0ull;
                glds16(a.umem + src, rows + r * 1024);  // asm: keeps LLVM's vmcnt bookkeeping in order
            }
        }

        // ---- 3. stream row bytes [64, rowhi): row q of step s owns frame 4s+q -----------------------
        const uint32_t nit = rowhi > (uint32_t)kWin ? (rowhi - (uint32_t)kWin + 255u) >> 8 : 0u;
        if (__ballot(nit != 0u) != 0ull) {
            // one buffer window [wlo, whi) over every streamed byte of the tile; lanes past their
            // frame's end get an out-of-range offset and load zeros without touching memory
            const uint64_t a16 = addr & ~15ull;
            const uint64_t wlo = wave_min_u64(nit ? a16 : ~0ull);
            const uint64_t whi = wave_max_u64(nit ? addr + len : 0ull);
            const uint64_t span = (whi - wlo + 15u) & ~15ull;  // <= umem_size - wlo (size % 16 == 0)
            if (span < 0x80000000ull) {
                WinLoader ld;
                ld.r = __builtin_amdgcn_make_buffer_rsrc((void*)(a.umem + wlo), (short)0, (int)span, kRsrcFlags);
                const uint32_t rel = nit ? (uint32_t)(a16 - wlo) : 0u;
                for (uint32_t s = 0; s < 16; ++s) {
                    const int f = (int)(4u * s + q);
                    const uint32_t f_nit = (uint32_t)__shfl((int)nit, f, 64);
                    const uint32_t ns = max(max(rdlane(f_nit, 0), rdlane(f_nit, 16)), max(rdlane(f_nit, 32), rdlane(f_nit, 48)));
                    if (ns == 0) continue;
                    ld.rel = (uint32_t)__shfl((int)rel, f, 64);
                    const uint32_t f_rowhi = (uint32_t)__shfl((int)rowhi, f, 64);
                    const uint32_t r = row_sum_dpp(fold64(stream_row<U>(ld, ns, f_rowhi, k)));
                    if (k == 15u) sums[f] = r;
                }
            } else {  // frames of one tile more than 2 GiB apart: 64-bit addresses, clamped loads
                for (uint32_t s = 0; s < 16; ++s) {
                    const int f = (int)(4u * s + q);
                    const uint32_t f_nit = (uint32_t)__shfl((int)nit, f, 64);
                    const uint32_t ns = max(max(rdlane(f_nit, 0), rdlane(f_nit, 16)), max(rdlane(f_nit, 32), rdlane(f_nit, 48)));
                    if (ns == 0) continue;
                    const uint32_t f_lo = (uint32_t)__shfl((int)a16_lo, f, 64);
                    const uint32_t f_hi = (uint32_t)__shfl((int)a16_hi, f, 64);
                    FarLoader ld;
                    ld.fbase = a.umem + (f_nit ? ((((uint64_t)f_hi) << 32) | (uint64_t)f_lo) : 0ull);
                    const uint32_t f_rowhi = (uint32_t)__shfl((int)rowhi, f, 64);
                    const uint32_t r = row_sum_dpp(fold64(stream_row<U>(ld, ns, f_rowhi, k)));
                    if (k == 15u) sums[f] = r;
                }
            }
        }

        // ---- 4. header phase (lane = frame); the DMA is older than every stream load --------------
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const uint32_t sres = nit ? sums[lane] : 0u;
        const bool wb = header_phase<WB64>(a, rows + lane * kWin, sres, addr, len, live, ok, parse, fi, cnt);
        if (WB64) {
            // ---- 5. patched windows -> UMEM: 16 frames x 64 B per wave-store, whole 64-B sectors ----
            const uint64_t wbm = __ballot(wb);
            if (wbm) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int f = r * 16 + (int)(lane >> 2);
                    const uint32_t kk = lane & 3u;
                    const uint32_t f_lo = (uint32_t)__shfl((int)a16_lo, f, 64);
                    const uint32_t f_hi = (uint32_t)__shfl((int)a16_hi, f, 64);
                    if ((wbm >> f) & 1ull) {
                        const u32x4 w = *(const u32x4*)(rows + f * kWin + 16u * kk);
                        *(u32x4*)(a.umem + ((((uint64_t)f_hi) << 32) | (uint64_t)f_lo) + 16u * kk) = w;
                    }
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // LDS rows are rewritten by the next tile's DMA
    }
    store_partials(a, cnt, s_cnt, wave, lane);
}

// ================================================================================================
// v5: one read of every byte.  Like v4 the payload is streamed by 16-lane DPP rows (row q of step s
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
template <int U>
__device__ __forceinline__ void stream_frame(const WinLoader& ld, uint32_t ns, uint32_t f_rowhi, uint32_t f_lim,
                                             uint32_t f_off, uint32_t f_iphi, uint32_t k, uint8_t* hdr_row,
                                             RowSums& rs) {
    if (ns == 1u) {
        const uint32_t ro = 16u * k;
        const u32x4 x = ld.load(ro, ro < f_lim);
        if (k < 4u) *(u32x4*)(hdr_row + ro) = x;
        rs.ip += k < 4u ? sum_range(x, (int)ro, (int)f_off + 14, (int)f_iphi) : 0ull;
        rs.ic += sum_range(x, (int)ro, (int)f_off + 34, (int)f_rowhi);
        return;
    }
    for (uint32_t j0 = 0; j0 < ns; j0 += U) {
        u32x4 v[U];
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
                rs.ic += sum_range(x, (int)ro, (int)f_off + 34, (int)f_rowhi);
            } else {
                const int nb = (int)(f_rowhi - min(ro, f_rowhi));      // frame bytes in this block
                if (__ballot(nb > 0 && nb < 16) != 0ull) {             // a block that ends a frame
                    u32x4 y = x;
                    y.x &= dw_mask(nb);
                    y.y &= dw_mask(nb - 4);
                    y.z &= dw_mask(nb - 8);
                    y.w &= dw_mask(nb - 12);
                    rs.ic += sum_dw(y);
                } else {
                    rs.ic += sum_dw(x);  // whole block in the frame, or zeros past it
                }
            }
        }
    }
}

// Header work of one frame (lane = frame) from its LDS row and its two folded row sums.
__device__ __forceinline__ bool header_phase5(const EchoArgs& a, uint8_t* row, uint32_t ip_raw, uint32_t ic_raw,
                                              uint64_t addr, uint32_t len, bool live, bool ok, bool parse,
                                              uint32_t fi, Counters& cnt) {
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
    if (live) {
        if (a.verdicts) a.verdicts[fi] = (uint8_t)verdict;
        if (a.recs) {
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

template <int U, int MINW>
__global__ __launch_bounds__(kThreads, MINW) void echo_kernel5(EchoArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[kWaves][kTile * kWin];
    __shared__ __attribute__((aligned(16))) FrameMeta s_meta[kWaves][kTile];
    __shared__ uint32_t s_sum[kWaves][2][kTile];  // [ic, ip] folded row sums per frame
    __shared__ unsigned long long s_cnt[kWaves][4];

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = uniform(threadIdx.x >> 6);
    const uint32_t q = lane >> 4, k = lane & 15u;
    uint8_t* rows = s_hdr[wave];
    FrameMeta* meta = s_meta[wave];
    uint32_t* sums_ic = s_sum[wave][0];
    uint32_t* sums_ip = s_sum[wave][1];
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t nwaves = gridDim.x * kWaves;
    Counters cnt;

    for (uint32_t t = blockIdx.x * kWaves + wave; t < ntiles; t += nwaves) {
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
                // wave-load, quad DPP reduction; no row stream
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                    const uint32_t kk = lane & 3u;
                    const FrameMeta& fm = meta[f];
                    const uint32_t f_lim = fm.lim, f_rowhi = fm.rowhi, f_packed = fm.packed;
                    const uint32_t ro = 16u * kk;
                    u32x4 x;
                    if (fast) {
                        ld.rel = fm.rel;
                        x = ld.load(ro, ro < f_lim);
                    } else {
                        const uint64_t fa = (((uint64_t)fm.addr_hi) << 32) | (uint64_t)fm.addr_lo;
                        x = __builtin_nontemporal_load((const u32x4*)(a.umem + (ro < f_lim ? (fa & ~15ull) + ro : 0ull)));
                        if (ro >= f_lim) x = u32x4{0u, 0u, 0u, 0u};
                    }
                    *(u32x4*)(rows + f * kWin + ro) = x;
                    const int f_off = (int)(f_packed & 0xFFu), f_iphi = (int)((f_packed >> 8) & 0xFFu);
                    uint32_t rip = fold64(sum_range(x, (int)ro, f_off + 14, f_iphi));
                    uint32_t ric = fold64(sum_range(x, (int)ro, f_off + 34, (int)f_rowhi));
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
                    const uint8_t* fb =
                        a.umem + (f_nit ? ((((uint64_t)fm.addr_hi) << 32) | (uint64_t)fm.addr_lo) & ~15ull : 0ull);
                    for (uint32_t j = 0; j < ns; ++j) {
                        const uint32_t ro = 256u * j + 16u * k;
                        u32x4 x = __builtin_nontemporal_load((const u32x4*)(fb + (ro < f_lim ? ro : 0u)));
                        if (ro >= f_lim) x = u32x4{0u, 0u, 0u, 0u};
                        if (j == 0 && k < 4u) {
                            *(u32x4*)(rows + f * kWin + ro) = x;
                            rs.ip += sum_range(x, (int)ro, (int)f_off + 14, (int)f_iphi);
                        }
                        rs.ic += sum_range(x, (int)ro, (int)f_off + 34, (int)f_rowhi);
                    }
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

// ------------------------------------------------------------------------------------------------
// Synthetic frames: one wave per frame, bit-identical to oracle_synth_frame().
// ------------------------------------------------------------------------------------------------
struct SynthArgs {
    uint8_t* umem;
    uint64_t umem_size;
    xsk_gpu_desc* descs;
    uint32_t n;
    uint64_t base_off, stride, seed, first, step;
    int mode;
    uint32_t len_lo, len_hi;
};

__device__ __constant__ uint32_t k_short_lens[13] = {0, 1, 13, 14, 19, 20, 21, 33, 34, 37, 38, 41, 42};

__global__ __launch_bounds__(256) void synth_kernel(SynthArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t j = blockIdx.x * 4u + uniform(threadIdx.x >> 6);
    if (j >= a.n) return;
    const uint64_t gidx = a.first + (uint64_t)j * a.step;
    const uint64_t K = mix64(a.seed ^ mix64(gidx));
    const uint64_t r1 = mix64(K + 1), r2 = mix64(K + 2), r3 = mix64(K + 3), r4 = mix64(K + 4), r5 = mix64(K + 5);
    uint32_t L = a.len_lo == a.len_hi ? a.len_lo : a.len_lo + (uint32_t)(r5 % (uint64_t)(a.len_hi - a.len_lo + 1));
    const uint32_t s = a.mode == 1 ? (uint32_t)(r4 >> 32) % 20u : 0u;
    if (s == 18) L = k_short_lens[(r5 >> 40) % 13];
    const uint32_t W = ((L > 64 ? L : 64) + 15u) & ~15u;  // fill extent: whole 16-B blocks
    const uint64_t addr = a.base_off + (uint64_t)j * a.stride;
    uint8_t* frame = a.umem + addr;

    // header dwords (little-endian), checksum fields zero for now
    uint32_t hw[11];
    const uint32_t eth = s == 6 ? 0x86DDu : s == 7 ? 0x8100u : 0x0800u;
    const uint32_t vihl = s == 12 ? 0x46u : s == 13 ? 0x65u : 0x45u;
    const uint32_t tl = (L >= 14 ? L - 14 : 0u) & 0xFFFFu;
    const uint32_t frag = s == 14 ? 0x2000u : 0x4000u;
    const uint32_t proto = s == 8 ? 6u : 1u;
    const uint32_t itype = s == 9 ? 0u : s == 10 ? 13u : 8u;
    const uint32_t icode = s == 11 ? 5u : 0u;
    hw[0] = (uint32_t)r1;
    hw[1] = ((uint32_t)(r1 >> 32) & 0xFFFFu) | ((uint32_t)r2 << 16);
    hw[2] = (uint32_t)(r2 >> 16);
    hw[3] = bswap16(eth) | (vihl << 16);
    hw[4] = bswap16(tl) | ((uint32_t)(r2 >> 48) << 16);
    hw[5] = bswap16(frag) | (64u << 16) | (proto << 24);
    hw[6] = (uint32_t)r3 << 16;
    hw[7] = (uint32_t)(r3 >> 16);
    hw[8] = (uint32_t)(r3 >> 48) | (itype << 16) | (icode << 24);
    hw[9] = ((uint32_t)r4 & 0xFFFFu) << 16;
    hw[10] = ((uint32_t)r4 >> 16) & 0xFFFFu;
    const bool garbage = s == 19;
    const bool zero_icmp = s == 17;

    // Build this lane's blocks (<= 4096/16/64 = 4 per lane) and the ICMP partial sum over [34, L).
    const uint32_t nblk = (W + 15) / 16;
    u32x4 blk[4];
    uint32_t s_ic = 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const uint32_t b = lane + 64u * (uint32_t)it;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        if (b < nblk) {
            const uint64_t p0 = mix64(K + 16 + 2 * (uint64_t)b), p1 = mix64(K + 16 + 2 * (uint64_t)b + 1);
            uint32_t w[4] = {(uint32_t)p0, (uint32_t)(p0 >> 32), (uint32_t)p1, (uint32_t)(p1 >> 32)};
            if (!garbage) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t k = 4 * b + (uint32_t)i;  // frame dword index
                    if (k < 10) w[i] = hw[k];
                    else if (k == 10) w[i] = (w[i] & 0xFFFF0000u) | hw[10];
                    if (zero_icmp) {  // bytes [38, L) zero
                        const int base = 4 * (int)k;
                        const uint32_t z = keep_bytes(0xFFFFFFFFu, base, 38, (int)L);
                        w[i] &= ~z;
                    }
                    s_ic += halves(keep_bytes(w[i], 4 * (int)k, 34, (int)L));
                }
            }
            v = u32x4{w[0], w[1], w[2], w[3]};
        }
        blk[it] = v;
    }
    if (!garbage) {
        const uint32_t tot = wave_sum_u32(s_ic);
        uint32_t icc = (~bswap16(fold32(tot))) & 0xFFFFu;
        if (s == 15) icc ^= 0x1234u;
        uint32_t sip = (hw[3] >> 16) + halves(hw[4]) + halves(hw[5]) + halves(hw[6]) + halves(hw[7]) + (hw[8] & 0xFFFFu);
        uint32_t ipc = (~bswap16(fold32(sip))) & 0xFFFFu;
        if (s == 16) ipc ^= 0x5A5Au;
        // bytes 24-25 live in block 1 (.z low half), bytes 36-37 in block 2 (.y low half); lanes 1, 2
        if (lane == 1) blk[0].z = (blk[0].z & 0xFFFF0000u) | bswap16(ipc);
        if (lane == 2) blk[0].y = (blk[0].y & 0xFFFF0000u) | bswap16(icc);
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const uint32_t b = lane + 64u * (uint32_t)it;
        if (b < nblk) ((u32x4*)frame)[b] = blk[it];
    }
    if (lane == 0) {
        xsk_gpu_desc dd;
        dd.addr = addr;
        dd.len = L;
        dd.options = 0;
        a.descs[j] = dd;
    }
}

// Staged host mode: gather the 38 rewritten header bytes of every TX_REPLY frame into a packed
// [n][48] array so the host can scatter them back into its UMEM (never touching unowned bytes).
__global__ __launch_bounds__(256) void pack_headers_kernel(const uint8_t* umem, const xsk_gpu_desc* descs,
                                                           const uint8_t* verdicts, uint32_t n, uint8_t* pack) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n || verdicts[i] != XSK_GPU_TX_REPLY) return;
    const uint8_t* p = umem + descs[i].addr;
    uint8_t* q = pack + (uint64_t)i * 48u;
    for (int k = 0; k < 38; ++k) q[k] = p[k];
}

// Re-arm TX_REPLY frames (lane per frame, byte granular: bench utility, not the hot path).
__global__ __launch_bounds__(256) void rearm_kernel(uint8_t* umem, const xsk_gpu_desc* descs, const uint8_t* verdicts,
                                                    uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n || verdicts[i] != XSK_GPU_TX_REPLY) return;
    uint8_t* p = umem + descs[i].addr;
    uint8_t t[6];
    for (int k = 0; k < 6; ++k) t[k] = p[k];
    for (int k = 0; k < 6; ++k) p[k] = p[6 + k];
    for (int k = 0; k < 6; ++k) p[6 + k] = t[k];
    for (int k = 0; k < 4; ++k) {
        const uint8_t x = p[26 + k];
        p[26 + k] = p[30 + k];
        p[30 + k] = x;
    }
    p[34] = 8;
    // csum_replace2(csum, 0, 8) on the LE-loaded field
    uint32_t c = (uint32_t)p[36] | ((uint32_t)p[37] << 8);
    uint32_t x = (~c) & 0xFFFFu;
    x = (x + 0xFFFFu) & 0xFFFFu;
    x += x < 0xFFFFu ? 1u : 0u;
    x = (x + 8u) & 0xFFFFu;
    x += x < 8u ? 1u : 0u;
    x = (~x) & 0xFFFFu;
    p[36] = (uint8_t)x;
    p[37] = (uint8_t)(x >> 8);
}

// Read-only streaming ceiling: every byte loaded once with 16-B nontemporal loads.
__global__ __launch_bounds__(256) void stream_read_kernel(const u32x4* src, uint64_t nvec, unsigned long long* out) {
    uint64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + 3 * stride < nvec; i += 4 * stride) {
        const u32x4 a0 = __builtin_nontemporal_load(src + i);
        const u32x4 a1 = __builtin_nontemporal_load(src + i + stride);
        const u32x4 a2 = __builtin_nontemporal_load(src + i + 2 * stride);
        const u32x4 a3 = __builtin_nontemporal_load(src + i + 3 * stride);
        acc += (uint64_t)a0.x + a0.y + a0.z + a0.w + a1.x + a1.y + a1.z + a1.w;
        acc += (uint64_t)a2.x + a2.y + a2.z + a2.w + a3.x + a3.y + a3.z + a3.w;
    }
    for (; i < nvec; i += stride) {
        const u32x4 a0 = __builtin_nontemporal_load(src + i);
        acc += (uint64_t)a0.x + a0.y + a0.z + a0.w;
    }
    acc = wave_sum_u64(acc);
    if ((threadIdx.x & 63u) == 0) atomicAdd(out, (unsigned long long)acc);
}

// ------------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------------
thread_local const char* g_last_error = "ok";

int hip_fail(hipError_t e) {
    g_last_error = hipGetErrorName(e);
    return e == hipErrorOutOfMemory ? -ENOMEM : -EIO;
}

#define HIP_TRY(expr)                              \
    do {                                           \
        const hipError_t e__ = (expr);             \
        if (e__ != hipSuccess) return hip_fail(e__); \
    } while (0)

constexpr int kMaxDevices = 64;
struct DevInfo {
    bool init = false;
    uint32_t max_wg = 0;  // resident echo workgroups on the whole device
};
DevInfo g_dev[kMaxDevices];
std::mutex g_dev_mu;

int dev_info(int device, DevInfo** out) {
    if (device < 0 || device >= kMaxDevices) return -ENODEV;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    DevInfo& di = g_dev[device];
    if (!di.init) {
        int cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        int per_cu = 0;
        int cur = 0;
        HIP_TRY(hipGetDevice(&cur));
        if (cur != device) HIP_TRY(hipSetDevice(device));
        const hipError_t e =
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&echo_kernel<kPrefetch, false>),
                                                         kThreads, 0);
        if (cur != device) (void)hipSetDevice(cur);
        if (e != hipSuccess) return hip_fail(e);
        if (per_cu < 1) per_cu = 1;
        di.max_wg = (uint32_t)cus * (uint32_t)per_cu;
        di.init = true;
    }
    *out = &di;
    return 0;
}

// One workgroup per kWaves tiles (the dispatcher balances ragged tiles better than a persistent
// grid: 315 vs 347 us at c3), capped so the partials workspace stays <= 512 KiB; the kernels loop.
constexpr uint32_t kMaxGrid = 16384;
uint32_t echo_grid(const DevInfo*, uint32_t n) {
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    uint32_t g = (ntiles + kWaves - 1) / kWaves;
    if (g > kMaxGrid) g = kMaxGrid;
    return g < 1 ? 1 : g;
}

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

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

int xsk_gpu_abi_version(void) { return XSK_GPU_ABI_VERSION; }
const char* xsk_gpu_last_error(void) { return g_last_error; }

size_t xsk_gpu_workspace_size(int device, uint32_t n) {
    DevInfo* di = nullptr;
    if (dev_info(device, &di) != 0) return 0;
    return (size_t)echo_grid(di, n) * 4 * sizeof(unsigned long long);
}

int xsk_gpu_echo_dev(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                     uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, struct xsk_gpu_stats* d_stats,
                     void* d_workspace, void* stream) {
    if (n == 0) return 0;
    if (!d_umem || !d_descs || ((uintptr_t)d_umem & 15u) || (umem_size & 15u) || ((uintptr_t)d_descs & 15u) ||
        ((uintptr_t)d_recs & 15u))
        return -EINVAL;
    if (d_stats && !d_workspace) return -EINVAL;
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    DevInfo* di = nullptr;
    const int rc = dev_info(device, &di);
    if (rc) return rc;
    const uint32_t grid = echo_grid(di, n);
    hipStream_t s = (hipStream_t)stream;
    EchoArgs args;
    args.umem = (uint8_t*)d_umem;
    args.umem_size = umem_size;
    args.descs = d_descs;
    args.n = n;
    args.verdicts = d_verdicts;
    args.recs = d_recs;
    args.partials = d_stats ? (unsigned long long*)d_workspace : nullptr;

    int slot = -1;
    {
        std::lock_guard<std::mutex> lk(g_timer_mu);
        if (g_timer.on && g_timer.count < kTimerCap) {
            slot = g_timer.count++;
            g_timer.dev[slot] = device;
        }
    }
    if (slot >= 0) HIP_TRY(hipEventRecord(g_timer.ev[slot][0], s));
    echo_kernel5<kShipU, 1><<<dim3(grid), dim3(kThreads), 0, s>>>(args);
    HIP_TRY(hipGetLastError());
    if (slot >= 0) HIP_TRY(hipEventRecord(g_timer.ev[slot][1], s));
    if (d_stats) {
        hipLaunchKernelGGL(fold_counters_kernel, dim3(1), dim3(1024), 0, s, (const unsigned long long*)d_workspace, grid,
                           d_stats);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}

// Internal (not in include/xsk_gpu.h): kernel variants for the tuning sweep in tools/kbench.py.
//   variant: 0 <P=4>, 1 <P=8>, 2 <P=2>, 3 <P=6>, 10+x = LITE (stream-only ceiling) of the same P
//   max_grid: 0 = library default, else cap on workgroups
int xsk_gpu__echo_variant(int variant, uint32_t max_grid, void* d_umem, uint64_t umem_size,
                          const struct xsk_gpu_desc* d_descs, uint32_t n, uint8_t* d_verdicts,
                          struct xsk_gpu_rec* d_recs, void* d_workspace, void* stream) {
    if (n == 0) return 0;
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    DevInfo* di = nullptr;
    const int rc = dev_info(device, &di);
    if (rc) return rc;
    uint32_t grid = echo_grid(di, n);
    if (max_grid) {
        const uint32_t full = ((n + kTile - 1) / kTile + kWaves - 1) / kWaves;
        grid = max_grid < full ? max_grid : full;
    }
    EchoArgs args;
    args.umem = (uint8_t*)d_umem;
    args.umem_size = umem_size;
    args.descs = d_descs;
    args.n = n;
    args.verdicts = d_verdicts;
    args.recs = d_recs;
    args.partials = (unsigned long long*)d_workspace;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g(grid), b(kThreads);
    switch (variant) {
        case 0: echo_kernel<4, false><<<g, b, 0, s>>>(args); break;
        case 1: echo_kernel<8, false><<<g, b, 0, s>>>(args); break;
        case 2: echo_kernel<2, false><<<g, b, 0, s>>>(args); break;
        case 3: echo_kernel<6, false><<<g, b, 0, s>>>(args); break;
        case 4: echo_kernel<4, false, 8><<<g, b, 0, s>>>(args); break;
        case 5: echo_kernel<2, false, 8><<<g, b, 0, s>>>(args); break;
        case 6: echo_kernel<8, false, 6><<<g, b, 0, s>>>(args); break;
        case 21: echo_kernel<4, false, 1, 1><<<g, b, 0, s>>>(args); break;
        case 22: echo_kernel<4, false, 1, 2><<<g, b, 0, s>>>(args); break;
        case 24: echo_kernel<4, false, 1, 4><<<g, b, 0, s>>>(args); break;
        case 27: echo_kernel<4, false, 1, 7><<<g, b, 0, s>>>(args); break;
        case 30: echo_kernel3<4><<<g, b, 0, s>>>(args); break;
        case 31: echo_kernel3<8><<<g, b, 0, s>>>(args); break;
        case 32: echo_kernel3<2><<<g, b, 0, s>>>(args); break;
        case 33: echo_kernel3<6><<<g, b, 0, s>>>(args); break;
        case 40: echo_kernel4<6, 1><<<g, b, 0, s>>>(args); break;
        case 41: echo_kernel4<6, 8><<<g, b, 0, s>>>(args); break;
        case 42: echo_kernel4<3, 8><<<g, b, 0, s>>>(args); break;
        case 43: echo_kernel4<6, 6><<<g, b, 0, s>>>(args); break;
        case 44: echo_kernel4<4, 8><<<g, b, 0, s>>>(args); break;
        case 45: echo_kernel4<6, 1, false><<<g, b, 0, s>>>(args); break;
        case 50: echo_kernel5<6, 1><<<g, b, 0, s>>>(args); break;
        case 51: echo_kernel5<3, 1><<<g, b, 0, s>>>(args); break;
        case 52: echo_kernel5<4, 1><<<g, b, 0, s>>>(args); break;
        case 53: echo_kernel5<6, 6><<<g, b, 0, s>>>(args); break;
        case 54: echo_kernel5<3, 8><<<g, b, 0, s>>>(args); break;
        case 10: echo_kernel<4, true><<<g, b, 0, s>>>(args); break;
        case 11: echo_kernel<8, true><<<g, b, 0, s>>>(args); break;
        case 12: echo_kernel<2, true><<<g, b, 0, s>>>(args); break;
        case 13: echo_kernel<6, true><<<g, b, 0, s>>>(args); break;
        default: return -EINVAL;
    }
    HIP_TRY(hipGetLastError());
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

int xsk_gpu_synth_dev(void* d_umem, uint64_t umem_size, struct xsk_gpu_desc* d_descs, uint32_t n, uint64_t base_off,
                      uint64_t stride, uint64_t seed, uint64_t first, uint64_t step, int mode, uint32_t len_lo,
                      uint32_t len_hi, void* stream) {
    if (n == 0) return 0;
    if (!d_umem || !d_descs || (base_off & 15u) || (stride & 15u) || len_lo > len_hi || (mode != 0 && mode != 1) ||
        ((uintptr_t)d_umem & 15u))
        return -EINVAL;
    const uint64_t w = ((len_hi > 64 ? len_hi : 64) + 15u) & ~15ull;
    if (stride < w || w > 4096) return -EINVAL;
    if (base_off + (uint64_t)(n - 1) * stride + w > umem_size) return -EINVAL;
    SynthArgs a;
    a.umem = (uint8_t*)d_umem;
    a.umem_size = umem_size;
    a.descs = d_descs;
    a.n = n;
    a.base_off = base_off;
    a.stride = stride;
    a.seed = seed;
    a.first = first;
    a.step = step;
    a.mode = mode;
    a.len_lo = len_lo;
    a.len_hi = len_hi;
    hipLaunchKernelGGL(synth_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
    HIP_TRY(hipGetLastError());
    return 0;
}

int xsk_gpu_rearm_dev(void* d_umem, const struct xsk_gpu_desc* d_descs, const uint8_t* d_verdicts, uint32_t n,
                      void* stream) {
    if (n == 0) return 0;
    if (!d_umem || !d_descs || !d_verdicts) return -EINVAL;
    hipLaunchKernelGGL(rearm_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (uint8_t*)d_umem, d_descs,
                       d_verdicts, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

// Internal (not in include/xsk_gpu.h): used by the host-UMEM staged mode in xsk_gpu_host.c.
int xsk_gpu__pack_headers_dev(const void* d_umem, const struct xsk_gpu_desc* d_descs, const uint8_t* d_verdicts,
                              uint32_t n, uint8_t* d_pack, void* stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(pack_headers_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)d_umem, d_descs, d_verdicts, n, d_pack);
    HIP_TRY(hipGetLastError());
    return 0;
}

int xsk_gpu_stream_read_dev(const void* d_src, uint64_t bytes, uint64_t* d_out, void* stream) {
    if (!d_src || !d_out || (bytes & 15u) || ((uintptr_t)d_src & 15u)) return -EINVAL;
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    hipLaunchKernelGGL(stream_read_kernel, dim3((unsigned)cus * 8u), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)d_src, bytes / 16, (unsigned long long*)d_out);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"
