// xsk_tune.hip — kernel variants for the tuning sweep (tools/kbench.py) and the parity test of every
// variant (tests/test_gpu_parity.py::test_kernel_variants_parity).  Not on the product path.
//
//   0-6   v2 "wave per frame": one wave streams each frame of its 64-frame tile in 1 KiB wave-loads,
//         P loads in flight through a ring over the tile's chunk list, header windows by LDS-DMA,
//         one whole-wave DPP reduction per frame, 38-B partial header stores (the first design;
//         DESIGN.md §3 has the measurements that replaced it)
//   10-13 v2 LITE: stream and sum every frame byte, nothing else (a layout read ceiling)
//   21-27 v2 ablations (ABL bits: 1 no header store, 2 no records/verdicts, 4 no header DMA)
//   50-54 the shipped row-streaming kernel at other U (loads in flight) / occupancy settings
#include <errno.h>

#include "xsk_echo_lab.h"
#include "../xsk_hip_util.h"
#include "xsk_echo_variants.h"

using namespace xskgpu;

namespace {

// One slot of the streaming ring.
struct Slot {
    u32x4 v;         // 16 payload bytes of this lane
    uint32_t nv;     // valid bytes of v (0..16)
    uint32_t frame;  // owning frame (lane index in the tile), wave-uniform
    uint32_t last;   // 1 if this chunk closes its frame, wave-uniform
};

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

}  // namespace

// 170-172 (round 3): the shipped kernel's switches (variant 158) in workgroups of NWV = 8 waves, two per CU (half
// the LDS each), so that one workgroup's round tail and write phase overlap the other's reads on the same CU instead
// of leaving the CU's loads to the last waves of a 16-wave round.  172: heavy threshold 1024 B.
template <int NWV, int HV>
__global__ __launch_bounds__(NWV * 64, 2) void echo_kernel6w(EchoArgs a, uint32_t tiles_per_wg) {
    __shared__ Echo6Smem<2, false, 2, NWV> sm;
    static_assert(sizeof(sm) <= 81920, "two workgroups per CU");
    const uint32_t ntiles = (a.n + kTile - 1) / kTile;
    const uint32_t t_begin = blockIdx.x * tiles_per_wg;
    const uint32_t t_end = min(ntiles, t_begin + tiles_per_wg);
    echo6_body<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, false, false, NWV, 0, 1,
               true, false, false, 0, 0, 0, 2, HV>(a, t_begin, t_end, tiles_per_wg, sm);
}

extern "C" {

uint32_t xsk_gpu__num_cu(int device);  // xsk_echo.hip

// Internal (not in include/xsk_gpu.h): kernel variants for the tuning sweep in tools/kbench.py.
//   variant: 0 <P=4>, 1 <P=8>, 2 <P=2>, 3 <P=6>, 10+x = LITE (stream-only ceiling) of the same P
//   50-54 = echo_kernel5 <U, min waves>, 60-64 = the round kernel echo_kernel6 <U, tiles per wave>
//   max_grid: 0 = library default, else cap on workgroups
int xsk_gpu__echo_variant(int variant, uint32_t max_grid, void* d_umem, uint64_t umem_size,
                          const struct xsk_gpu_desc* d_descs, uint32_t n, uint8_t* d_verdicts,
                          struct xsk_gpu_rec* d_recs, void* d_workspace, void* stream) {
    if (n == 0) return 0;
    uint32_t grid = echo_grid(n);
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
    if (variant >= 60 && variant < 200) {  // round kernel: max_grid = workgroups (0: one per CU)
        int device = 0;
        HIP_TRY(hipGetDevice(&device));
        uint32_t g6 = 0, per = 0;
        echo6_geometry(n, max_grid ? max_grid : xsk_gpu__num_cu(device), &g6, &per);
        const dim3 gg(g6), bb(kThreads6);
        if (variant >= 170 && variant <= 172) {  // two 8-wave workgroups per CU
            echo6_geometry(n, 2u * (max_grid ? max_grid : xsk_gpu__num_cu(device)), &g6, &per);
            if (variant == 172) echo_kernel6w<8, 1024><<<dim3(g6), dim3(512), 0, s>>>(args, per);
            else echo_kernel6w<8, 512><<<dim3(g6), dim3(512), 0, s>>>(args, per);
            HIP_TRY(hipGetLastError());
            return 0;
        }
        if ((variant >= 93 && variant <= 95) || (variant >= 99 && variant <= 102)) {  // queue counters at workspace + 768 KiB: zero, left zero
            if (!d_workspace) return -EINVAL;
            args.queue = (uint32_t*)((uint8_t*)d_workspace + (768u << 10));
        }
        if (variant == 103 || variant == 104) {  // 92 in the wave-front tile order (front_mode 1 / 2)
            const uint32_t ntiles = (n + kTile - 1) / kTile, front = 16u * g6;
            args.front = front;
            args.front_mode = variant == 103 ? 1u : 2u;
            per = 16u * ((ntiles + front - 1) / front);
        }
        if (variant == 134 || variant == 136) args.rot = 37;  // 131 with rotated shares
        if (variant == 135 || variant == 136) args.srot = 5;  // 131 with rotated uniform-stream steps
        if (variant >= 160 && variant <= 162) args.opts = XSK_GPU_OPT_ALL;  // the wire-mode kernel, every option
        if (variant == 90 || variant == 91 || variant == 128 || variant == 129) {  // chip-wide barrier counter (workspace + 512 KiB), zeroed
            if (!d_workspace) return -EINVAL;
            HIP_TRY(hipMemsetAsync((uint8_t*)d_workspace + 65536 * 8, 0, 64, s));
        }
        switch (variant) {
            case 60: echo_kernel6<4, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 61: echo_kernel6<6, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 62: echo_kernel6<8, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 63: echo_kernel6<4, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 64: echo_kernel6<2, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 65: echo_kernel7<4, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 66: echo_kernel7<6, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 67: echo_kernel7<3, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 68: echo_kernel7<4, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 69: echo_kernel7<2, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 70: echo_kernel6<4, 2, 0><<<gg, bb, 0, s>>>(args, per); break;
            case 71: echo_kernel6<4, 1, 0><<<gg, bb, 0, s>>>(args, per); break;
            case 72: echo_kernel6<4, 2, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 73: echo_kernel6<4, 2, 2, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 74: echo_kernel6<6, 2, 2, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 75: echo_kernel6<8, 2, 2, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 76: echo_kernel6<4, 2, 2, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 77: echo_kernel6<6, 2, 2, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 78: echo_kernel6<4, 2, 2, 2, true><<<gg, bb, 0, s>>>(args, per); break;
            case 79: echo_kernel6<4, 2, 2, 2, false, true><<<gg, bb, 0, s>>>(args, per); break;
            case 80: echo_kernel6<4, 2, 2, 3><<<gg, bb, 0, s>>>(args, per); break;
            case 84: echo_kernel6<4, 2, 2, 2, false, false, false, true><<<gg, bb, 0, s>>>(args, per); break;
            case 85: echo_kernel6<4, 2, 2, 2, false, false, false, false, true><<<gg, bb, 0, s>>>(args, per); break;
            case 86: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true><<<gg, bb, 0, s>>>(args, per); break;
            case 87: echo_kernel6<4, 2, 2, 2, true, false, false, false, false, true><<<gg, bb, 0, s>>>(args, per); break;
            case 88: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 89: echo_kernel6<4, 2, 2, 2, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 90: echo_kernel6<4, 2, 3, 2, false, false, false, false, false, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 91: echo_kernel6<4, 2, 4, 2, false, false, false, false, false, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 92: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            // 93-95: the dynamic round schedule (per-XCD regions, atomic claims, stealing); 94 + WGT
            // end-time probes, 95 with one tile per wave per round
            case 93: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, true><<<gg, bb, 0, s>>>(args, per); break;
            case 94: echo_kernel6<4, 2, 2, 2, false, true, false, false, false, true, true, true, false, true><<<gg, bb, 0, s>>>(args, per); break;
            case 95: echo_kernel6<4, 1, 2, 2, false, false, false, false, false, true, true, true, false, true><<<gg, bb, 0, s>>>(args, per); break;
            case 96: echo_kernel6<4, 1, 2, 2, false, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            // 97 / 98: the shipped kernel with 6 / 8 row-loads in flight per lane (a 1500-B frame in one batch)
            case 97: echo_kernel6<6, 2, 2, 2, false, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 98: echo_kernel6<8, 2, 2, 2, false, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            // 99-102: the shipped kernel + a tail pool of ntiles / TAIL tiles in 256-frame units (TAIL 8, 16, 4;
            // 102 = TAIL 8 with WGT end-time probes)
            case 99: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 8><<<gg, bb, 0, s>>>(args, per); break;
            case 100: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 16><<<gg, bb, 0, s>>>(args, per); break;
            case 101: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 4><<<gg, bb, 0, s>>>(args, per); break;
            case 102: echo_kernel6<4, 2, 2, 2, false, true, false, false, false, true, true, true, false, false, 8><<<gg, bb, 0, s>>>(args, per); break;
            // 105: 92 without the write phase (read phase alone, wrong results); 106: 105 with no round
            // waits (SYNC 0); 107: 92 with SYNC 0 (every wave writes as soon as it has read)
            case 105: echo_kernel6<4, 2, 2, 2, false, false, false, false, true, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 106: echo_kernel6<4, 2, 0, 2, false, false, false, false, true, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 107: echo_kernel6<4, 2, 0, 2, false, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            // 108-111: the one-round kernel echo_kernel8 (8 waves, TPW tiles per wave, VT of them in VGPRs):
            // 108 <4, 8, 4> SYNC 0; 109 = 108 NOWR; 110 <4, 8, 4> SYNC 2; 111 <4, 4, 0> (LDS only, 2 rounds at c3)
            case 108: echo_kernel8<4, 8, 4><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            case 109: echo_kernel8<4, 8, 4, 0, 2, false, true><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            case 110: echo_kernel8<4, 8, 4, 2><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            case 111: echo_kernel8<4, 4, 0><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            // 112 / 113: 108 with 6 / 8 row-loads in flight per lane; 114 / 115 their read phases alone
            // 116: 92 with the next tile's descriptors prefetched while the current one streams (PF)
            case 116: echo_kernel6<4, 2, 2, 2, true, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            // 117 / 118: 92 with software-pipelined ranked streams for every tile (STREAM 3) / ragged tiles (4)
            case 117: echo_kernel6<4, 2, 2, 3, false, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 118: echo_kernel6<4, 2, 2, 4, false, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            // 119: 92 with the uniform long-tile stream (ULONG: per-tile byte masks, no per-block mask logic);
            // 120: 119 without the write phase
            case 119: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 120: echo_kernel6<4, 2, 2, 2, false, false, false, false, true, true, true, true, false, false, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            // 121 / 122: the one-round kernel (112 / 108) with the uniform long-tile stream (ULONG)
            case 121: echo_kernel8<6, 8, 4, 0, 2, false, false, true, true, true, 1><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            case 122: echo_kernel8<4, 8, 4, 0, 2, false, false, true, true, true, 1><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            // 123: 119 with the pipelined uniform stream (ULONG 2); 124: 123 without the write phase;
            // 125: the one-round kernel (121) with it
            case 123: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 124: echo_kernel6<4, 2, 2, 2, false, false, false, false, true, true, true, true, false, false, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 125: echo_kernel8<4, 8, 4, 0, 2, false, false, true, true, true, 2><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            // 126: 119 with paired short tiles (PAIR); 127: 126 without the write phase
            case 126: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true><<<gg, bb, 0, s>>>(args, per); break;
            case 127: echo_kernel6<4, 2, 2, 2, false, false, false, false, true, true, true, true, false, false, 0, 1, true><<<gg, bb, 0, s>>>(args, per); break;
            // 128 / 129: 119 with a chip-wide barrier before (SYNC 3) / around (SYNC 4) every write phase
            case 128: echo_kernel6<4, 2, 3, 2, false, false, false, false, false, true, true, true, false, false, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 129: echo_kernel6<4, 2, 4, 2, false, false, false, false, false, true, true, true, false, false, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            // 130: the shipped kernel (ULONG + PAIR) with nontemporal write-phase stores (NTS); 131: shipped
            case 130: echo_kernel6<4, 2, 2, 2, false, false, false, true, false, true, true, true, false, false, 0, 1, true><<<gg, bb, 0, s>>>(args, per); break;
            case 131: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true><<<gg, bb, 0, s>>>(args, per); break;
            // 132: shipped + dot2 sums in the ranked streams (RD2)
            case 132: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, true><<<gg, bb, 0, s>>>(args, per); break;
            // 133: shipped + the cross-round carry of each round's last tile (CARRY)
            case 133: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, true><<<gg, bb, 0, s>>>(args, per); break;
            // 134: shipped with rotated shares (EchoArgs::rot); 135: with rotated uniform-stream steps (srot); 136: both
            case 134:
            case 135:
            case 136: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true><<<gg, bb, 0, s>>>(args, per); break;
            // 137 / 138: shipped + the penultimate round's windows deferred to the end (DEFW 1: heavy waves; 2: all)
            case 137: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 138: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 2><<<gg, bb, 0, s>>>(args, per); break;
            // 139 / 140: diagnostics (wrong results): 137 dropping the deferred windows / re-reading them only
            case 139: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 3><<<gg, bb, 0, s>>>(args, per); break;
            case 140: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 4><<<gg, bb, 0, s>>>(args, per); break;
            // 141-143: the shipped kernel's read phase alone (NOWR, wrong results) with the next tile's descriptors
            // prefetched (141), without the round waits (142: SYNC 0), both (143); 144: 131 + PF
            case 141: echo_kernel6<4, 2, 2, 2, true, false, false, false, true, true, true, true, false, false, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 142: echo_kernel6<4, 2, 0, 2, false, false, false, false, true, true, true, true, false, false, 0, 1, true><<<gg, bb, 0, s>>>(args, per); break;
            case 143: echo_kernel6<4, 2, 0, 2, true, false, false, false, true, true, true, true, false, false, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 144: echo_kernel6<4, 2, 2, 2, true, false, false, false, false, true, true, true, false, false, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 145: echo_kernel6<4, 2, 2, 2, false, false, false, false, true, true, true, true, false, false, 0, 1, true><<<gg, bb, 0, s>>>(args, per); break;
            // 146: 131 + the round-level descriptor prefetch (RPF); 147: its read phase alone (NOWR)
            case 146: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, true><<<gg, bb, 0, s>>>(args, per); break;
            case 147: echo_kernel6<4, 2, 2, 2, false, false, false, false, true, true, true, true, false, false, 0, 1, true, false, false, 0, true><<<gg, bb, 0, s>>>(args, per); break;
            // 148: 145 (read phase alone) without the header phase; 149: 141 (+ PF) without it (diagnostics)
            case 148: echo_kernel6<4, 2, 2, 2, false, false, false, false, true, true, true, true, false, false, 0, 1, true, false, false, 0, false, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 149: echo_kernel6<4, 2, 2, 2, true, false, false, false, true, true, true, true, false, false, 0, 1, false, false, false, 0, false, 1><<<gg, bb, 0, s>>>(args, per); break;
            // 151: 131 + the adaptive round prefetch (RPF 2: waves that streamed a ragged tile this round)
            case 151: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            // 152 / 153: 131 with write-through (sc1) window stores / window and record stores (WT 1 / 2)
            case 152: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 153: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            // 154-157: the shipped kernel (153, write-through) with SYNC 0 / SYNC 1 / PF instead of PAIR / one
            // tile per wave per round; 160 / 161: the wire-mode kernel (opts = all) plain / write-through
            case 154: echo_kernel6<4, 2, 0, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 155: echo_kernel6<4, 2, 1, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 156: echo_kernel6<4, 2, 2, 2, true, false, false, false, false, true, true, true, false, false, 0, 1, false, false, false, 0, 0, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            case 157: echo_kernel6<4, 1, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, false, false, false, 0, 0, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            // 158 / 159: the shipped kernel with the SYNC 2 heavy-frame length at 512 / 256 B (c4's waves then wait)
            case 158: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            case 159: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2, 256><<<gg, bb, 0, s>>>(args, per); break;
            case 160: echo_kernel6<4, 1, 2, 2, false, false, true, false, false, false, false, false, false, false, 0, 1><<<gg, bb, 0, s>>>(args, per); break;
            case 161: echo_kernel6<4, 1, 2, 2, false, false, true, false, false, false, false, false, false, false, 0, 1, false, false, false, 0, 0, 0, 2><<<gg, bb, 0, s>>>(args, per); break;
            // 162: 161 (wire mode, write-through) with the 512-B heavy threshold
            case 162: echo_kernel6<4, 1, 2, 2, false, false, true, false, false, false, false, false, false, false, 0, 1, false, false, false, 0, 0, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            // 163: the shipped kernel (write-through, 512-B heavy threshold) as a tuning variant; 164 / 165 with
            // the round-level descriptor prefetch (RPF 1 / 2); 166 with PF instead of PAIR
            case 163: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            case 164: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 1, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            case 165: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 2, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            case 166: echo_kernel6<4, 2, 2, 2, true, false, false, false, false, true, true, true, false, false, 0, 1, false, false, false, 0, 0, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            // 173-175 (round 3): the shipped kernel (158) with U = 2 / 3 / 6 row-loads per batch in the streams
            case 173: echo_kernel6<2, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            case 174: echo_kernel6<3, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            case 175: echo_kernel6<6, 2, 2, 2, false, false, false, false, false, true, true, true, false, false, 0, 1, true, false, false, 0, 0, 0, 2, 512><<<gg, bb, 0, s>>>(args, per); break;
            case 112: echo_kernel8<6, 8, 4><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            case 113: echo_kernel8<8, 8, 4><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            case 114: echo_kernel8<6, 8, 4, 0, 2, false, true><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            case 115: echo_kernel8<8, 8, 4, 0, 2, false, true><<<gg, dim3(kThreads8), 0, s>>>(args, per); break;
            case 103:
            case 104: echo_kernel6<4, 2, 2, 2, false, false, false, false, false, true, true, true><<<gg, bb, 0, s>>>(args, per); break;
            case 81: echo_kernel6<4, 2, 2, 4><<<gg, bb, 0, s>>>(args, per); break;
            case 82: echo_kernel6<3, 2, 2, 3><<<gg, bb, 0, s>>>(args, per); break;
            case 83: echo_kernel6<5, 2, 2, 3><<<gg, bb, 0, s>>>(args, per); break;
            default: return -EINVAL;
        }
        HIP_TRY(hipGetLastError());
        return 0;
    }
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
        case 50: echo_kernel5<6, 1><<<g, b, 0, s>>>(args); break;
        case 51: echo_kernel5<3, 1><<<g, b, 0, s>>>(args); break;
        case 52: echo_kernel5<4, 1><<<g, b, 0, s>>>(args); break;
        case 53: echo_kernel5<4, 6><<<g, b, 0, s>>>(args); break;
        case 54: echo_kernel5<3, 6><<<g, b, 0, s>>>(args); break;
        case 10: echo_kernel<4, true><<<g, b, 0, s>>>(args); break;
        case 11: echo_kernel<8, true><<<g, b, 0, s>>>(args); break;
        case 12: echo_kernel<2, true><<<g, b, 0, s>>>(args); break;
        case 13: echo_kernel<6, true><<<g, b, 0, s>>>(args); break;
        default: return -EINVAL;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"

// The tuning library's own copy of the error hook (the product library's is hidden).
extern "C" __attribute__((visibility("hidden"))) int xsk_gpu__hip_fail(hipError_t e) {
    return e == hipErrorOutOfMemory ? -ENOMEM : -EIO;
}
