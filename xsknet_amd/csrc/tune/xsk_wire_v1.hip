// xsk_wire_v1.hip — TUNING LIBRARY ONLY (libxsknet_amd_tune.so): the first wire-format kernel,
// superseded by the round kernel's WIRE mode (echo_kernel6<.., WIRE = true>, launched by
// xsk_gpu_echo_dev_opts in xsk_echo.hip), kept for same-session comparisons (tools/wireab.py).
//
// Wire-format widening (build-added): with nonzero XSK_GPU_OPT_* the kernel works
// instead of the reference-exact round kernel: the headers are parsed (802.1Q/802.1ad tags, IHL, tot_len, fragments) instead of read
// at the fixed offsets of process_packet() (src/lib/xsk_receive.c:120-121), checksums can gate the
// reply, and the reply rewrite of xsk_receive.c:148-157 lands at the parsed offsets.  The spec is the
// comment block above XSK_GPU_OPT_STRICT_IPV4 in include/xsk_gpu.h; oracle_echo_batch_opts() restates it
// on the CPU.
//
// Layout: the round structure of echo_kernel6 (one 16-wave workgroup per CU, one tile per wave per
// round, heavy waves write after the round; see the template comment).  One wave per 64-frame tile,
// lane = frame.  Each lane loads its frame's 128-B header window
// (16-B aligned, 8 x 16 B) into an LDS row, parses it with byte reads, and sums the IPv4 header and the
// part of the ICMP message inside the window from LDS (absolute-alignment domain, like the round
// kernel).  The rest of the message, row bytes [128, off + end), is streamed by 16-lane rows (one frame
// per row per step, 256-B row-loads).  Patched windows of 16-B aligned replies whose rewrite ends
// inside the first 64 bytes leave as whole 64-B sectors; every other reply is patched byte-exact.
#include <errno.h>

#include "xsk_echo_lab.h"
#include "../xsk_hip_util.h"

using namespace xskgpu;

namespace {

constexpr int kWinW = 128;  // wire-mode header window
constexpr int kWireU = 4;   // row-loads in flight per lane in the payload stream

__device__ __forceinline__ uint32_t be16_at(const uint8_t* row, uint32_t i) {
    return ((uint32_t)row[i] << 8) | (uint32_t)row[i + 1];
}

// NW waves per workgroup.  ROUND = false: a grid of small workgroups, each wave a tile at a time,
// writes at the tile's end.  ROUND = true: the round structure of echo_kernel6 (one 16-wave workgroup
// per CU, equal contiguous tile shares, one tile per wave per round); a wave whose tile averaged
// >= kHeavyLen bytes per frame holds its header sectors, records and verdicts until every wave of the
// workgroup has finished reading the round, so HBM sees read phases and write bursts, not a mix.
template <int U, int NW, bool ROUND>
__global__ __launch_bounds__(NW * 64) void echo_wire_kernel(EchoArgs a, uint32_t opts, uint32_t tiles_per_wg) {
    __shared__ __attribute__((aligned(16))) uint8_t s_row[NW][kTile * kWinW];  // 8 KiB per wave
    __shared__ uint64_t s_a16[NW][kTile];
    __shared__ uint32_t s_hi[NW][kTile];   // row coordinate of the message end when it passes the window
    __shared__ uint32_t s_sum[NW][kTile];  // streamed part of the ICMP sum (row-reduced)
    __shared__ unsigned long long s_cnt[NW][4];
    __shared__ uint32_t s_arrive;
    if (ROUND) {
        if (threadIdx.x == 0) s_arrive = 0u;
        __syncthreads();
    }

    const uint32_t wave = uniform(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t q = lane >> 4, k = lane & 15u;
    uint8_t* rows = s_row[wave];
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const bool strict = (opts & XSK_GPU_OPT_STRICT_IPV4) != 0u;
    const bool vlan = (opts & XSK_GPU_OPT_VLAN) != 0u;
    const bool verify = (opts & XSK_GPU_OPT_VERIFY_CSUM) != 0u;
    Counters cnt;
    // tile loop: ROUND -> workgroup-uniform rounds over the share [t_begin, t_end); else grid-stride
    const uint32_t t_begin = ROUND ? blockIdx.x * tiles_per_wg : blockIdx.x * NW + wave;
    const uint32_t t_end = ROUND ? min(ntiles, t_begin + tiles_per_wg) : ntiles;
    const uint32_t t_step = ROUND ? (uint32_t)NW : gridDim.x * NW;
    uint32_t rounds_done = 0;

    for (uint32_t it = t_begin; it < t_end; it += t_step) {
        const uint32_t t = ROUND ? it + wave : it;
        const bool have = t < t_end;  // wave-uniform (always true without ROUND)
        uint64_t wbm = 0;
        uint32_t verdict = XSK_GPU_TX_REPLY, len = 0;
        u32x4 recv = u32x4{0u, 0u, 0u, 0u};
        const uint32_t fi = t * kTile + lane;
        if (have) {
        // ---- descriptor (xsk_receive.c:222-223) and the 128-B window -> LDS row ------------------
        u32x4 dsc = u32x4{0u, 0u, 0u, 0u};
        if (fi < a.n) dsc = *(const u32x4*)(a.descs + fi);
        const uint64_t addr = (uint64_t)dsc.x | ((uint64_t)dsc.y << 32);
        len = dsc.z;
        const bool ok = fi < a.n && len <= kMaxLen && addr <= a.umem_size && len <= a.umem_size - addr;
        const uint64_t a16 = addr & ~15ull;
        const uint32_t off = (uint32_t)addr & 15u;
        const uint32_t wend = ok ? (uint32_t)min(a.umem_size - a16, (uint64_t)kWinW) : 0u;  // multiple of 16
        uint8_t* row = rows + lane * kWinW;
        {
            u32x4 w[kWinW / 16];
#pragma unroll
            for (int c = 0; c < kWinW / 16; ++c)
                w[c] = 16u * c < wend ? __builtin_nontemporal_load((const u32x4*)(a.umem + a16 + 16u * c))
                                      : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
            for (int c = 0; c < kWinW / 16; ++c) *(u32x4*)(row + 16 * c) = w[c];
        }
        s_a16[wave][lane] = a16;

        // ---- parse (spec: include/xsk_gpu.h, XSK_GPU_OPT_*) ----------------------------------------
        const uint8_t* p = row + off;  // frame byte i = p[i] for i < wend - off
        uint32_t l3 = 14, hl = 20, end = len, et = 0, tags = 0;
        bool hdrs = false;  // all three headers inside the frame: the record is filled
        if (!ok) verdict = XSK_GPU_DROP_BAD_DESC;
        else if (len < 14) verdict = XSK_GPU_DROP_SHORT;
        else {
            et = be16_at(p, 12);
            bool cut = false;
            if (vlan) {
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    if (!cut && (et == 0x8100u || et == 0x88A8u) && tags == (uint32_t)g) {
                        if (len < l3 + 4) cut = true;
                        else {
                            et = be16_at(p, l3 + 2);
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
                        const uint32_t tot = be16_at(p, l3 + 2);
                        if (tot < hl + 8 || l3 + tot > len) bad = true;
                        else if (be16_at(p, l3 + 6) & 0x3FFFu) bad = true;
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

        // ---- sums inside the window (absolute-alignment domain: LE dwords of the row) --------------
        const uint32_t ip_lo = off + l3, ip_hi = off + l4;
        const uint32_t ic_lo = off + l4, ic_end = off + end;
        const uint32_t ic_hi_w = hdrs ? min(ic_end, (uint32_t)kWinW) : 0u;
        uint64_t ip_acc = 0, ic_acc = 0;
        if (hdrs) {
            const uint32_t* r32 = (const uint32_t*)row;
#pragma unroll 8
            for (int d = 0; d < kWinW / 4; ++d) {
                const uint32_t x = r32[d];
                ip_acc += keep_bytes(x, 4 * d, (int)ip_lo, (int)ip_hi);
                ic_acc += keep_bytes(x, 4 * d, (int)ic_lo, (int)ic_hi_w);
            }
        }
        s_hi[wave][lane] = hdrs && ic_end > (uint32_t)kWinW ? ic_end : 0u;
        s_sum[wave][lane] = 0u;

        // ---- the message beyond the window: 16-lane rows, one frame per row per step ----------------
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        for (uint32_t s = 0; s < 16; ++s) {
            const uint32_t f = 4u * s + q;
            const uint32_t hi = s_hi[wave][f];
            const uint32_t nrow = hi ? (hi - (uint32_t)kWinW + 255u) >> 8 : 0u;
            const uint32_t ns = max(max(rdlane(nrow, 0), rdlane(nrow, 16)), max(rdlane(nrow, 32), rdlane(nrow, 48)));
            if (ns == 0) continue;
            const uint8_t* fb = a.umem + s_a16[wave][f];
            uint64_t acc = 0;
            for (uint32_t j0 = 0; j0 < ns; j0 += U) {
                u32x4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t ro = (uint32_t)kWinW + 256u * (j0 + (uint32_t)u) + 16u * k;
                    v[u] = ro < hi ? __builtin_nontemporal_load((const u32x4*)(fb + ro)) : u32x4{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t ro = (uint32_t)kWinW + 256u * (j0 + (uint32_t)u) + 16u * k;
                    const int nb = (int)(hi - min(ro, hi));
                    u32x4 y = v[u];
                    y.x &= dw_mask(nb);
                    y.y &= dw_mask(nb - 4);
                    y.z &= dw_mask(nb - 8);
                    y.w &= dw_mask(nb - 12);
                    acc += sum_dw(y);
                }
            }
            const uint32_t r = row_sum_dpp(fold64(acc));
            if (k == 15u && hi) s_sum[wave][f] = r;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();

        // ---- checksums, verdict, rewrite (lane = frame) ---------------------------------------------
        uint32_t ip_sum = fold64(ip_acc);
        uint32_t ic_sum = fold32(fold64(ic_acc) + s_sum[wave][lane]);
        if (!((uint32_t)addr & 1u)) {
            ip_sum = bswap16(ip_sum);
            ic_sum = bswap16(ic_sum);
        }
        uint32_t itype = 0, icode = 0, csum_in = 0, flags = 0;
        if (hdrs) {
            itype = p[l4];
            icode = p[l4 + 1];
            csum_in = be16_at(p, l4 + 2);
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
            uint8_t* w = row + off;  // patch the LDS copy (xsk_receive.c:148-157 at the parsed offsets)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const uint8_t x = w[i];
                w[i] = w[6 + i];
                w[6 + i] = x;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint8_t x = w[l3 + 12 + i];
                w[l3 + 12 + i] = w[l3 + 16 + i];
                w[l3 + 16 + i] = x;
            }
            w[l4] = 0;
            w[l4 + 2] = (uint8_t)csum_new_le;
            w[l4 + 3] = (uint8_t)(csum_new_le >> 8);
            if (off == 0u && l4 + 4u <= 64u && wend >= 64u) {
                wb = true;  // whole 64-B sector, stored below 16 frames per wave-store
            } else {        // byte-exact: only the rewritten bytes
                uint8_t* pkt = a.umem + addr;
#pragma unroll
                for (int i = 0; i < 12; ++i) pkt[i] = w[i];
#pragma unroll
                for (int i = 0; i < 8; ++i) pkt[l3 + 12 + i] = w[l3 + 12 + i];
                pkt[l4] = 0;
                pkt[l4 + 2] = w[l4 + 2];
                pkt[l4 + 3] = w[l4 + 3];
            }
        }
        wbm = __ballot(wb);
        {
            const uint32_t vihl = hdrs ? p[l3] : 0u, proto = hdrs ? 1u : 0u;
            recv.x = verdict | (flags << 8) | (proto << 16) | (itype << 24);
            recv.y = icode | (vihl << 8) | ((hdrs ? et : 0u) << 16);
            recv.z = csum_in | (csum_out << 16);
            recv.w = (hdrs ? ip_sum : 0u) | ((hdrs ? ic_sum : 0u) << 16);
        }
        if (fi < a.n) {
            cnt.rxp += 1;
            cnt.rxb += len;
            if (tx) {
                cnt.txp += 1;
                cnt.txb += len;
            }
        }
        }  // have
        if (ROUND) {  // heavy waves wait until the whole workgroup has read this round
            ++rounds_done;
            const uint32_t bytes = uniform(wave_sum_u32(have && fi < a.n ? min(len, 65536u) : 0u));
            if (lane == 0) atomicAdd(&s_arrive, 1u);
            if (bytes >= kHeavyLen * kTile) {
                while (__hip_atomic_load(&s_arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
                       rounds_done * (uint32_t)NW)
                    __builtin_amdgcn_s_sleep(2);
            }
        }
        if (have) {
            if (wbm) {  // patched 64-B sectors, 16 frames per wave-store
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                    const uint32_t kk = lane & 3u;
                    if ((wbm >> f) & 1ull)
                        *(u32x4*)(a.umem + s_a16[wave][f] + 16u * kk) = *(const u32x4*)(rows + f * kWinW + 16u * kk);
                }
            }
            if (fi < a.n) {
                if (a.verdicts) a.verdicts[fi] = (uint8_t)verdict;
                if (a.recs) ((u32x4*)a.recs)[fi] = recv;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();  // LDS rows are rewritten by the next tile
    }
    store_partials<NW>(a, cnt, s_cnt, wave, lane);
}

}  // namespace

extern "C" {

uint32_t xsk_gpu__num_cu(int device);  // xsk_echo.hip (product library)

// Wire-mode kernels for comparison: impl 1 = echo_wire_kernel (window first, then the stream), 2 = the
// round kernel's WIRE mode with dot2 sums in the per-step streams.  Counters by device atomics into
// d_stats (device memory) or none.  Validation is the caller's (tools only).
int xsk_gpu__echo_wire_variant(int impl, void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs,
                               uint32_t n, uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs,
                               struct xsk_gpu_stats* d_stats, void* stream) {
    if (n == 0) return 0;
    if (!opts || (opts & ~XSK_GPU_OPT_ALL)) return -EINVAL;
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    const uint32_t ncu = xsk_gpu__num_cu(device);
    if (!ncu) return -ENODEV;
    uint32_t grid = 0, tiles_per_wg = 0;
    echo6_geometry(n, ncu, &grid, &tiles_per_wg);
    EchoArgs args;
    args.umem = (uint8_t*)d_umem;
    args.umem_size = umem_size;
    args.descs = d_descs;
    args.n = n;
    args.verdicts = d_verdicts;
    args.recs = d_recs;
    args.partials = nullptr;
    args.opts = opts;
    args.stats_direct = d_stats ? (unsigned long long*)&d_stats->rx_packets : nullptr;
    if (impl == 2)
        echo_kernel6<kShip6U, 1, 2, 2, false, false, true, false, false, false, true>
            <<<dim3(grid), dim3(kThreads6), 0, (hipStream_t)stream>>>(args, tiles_per_wg);
    else if (impl == 1)
        echo_wire_kernel<kWireU, kWaves6, true><<<dim3(grid), dim3(kThreads6), 0, (hipStream_t)stream>>>(args, opts,
                                                                                                       tiles_per_wg);
    else
        return -EINVAL;
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"
