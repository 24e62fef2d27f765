// xsk_aux.hip — bench / test utilities of the C ABI (not on the hot path): the synthetic frame
// generator (bit-identical to oracle/echo_oracle.c), re-arm, the staged-mode copy-in gather and header gather, and
// the read-only streaming ceiling.
#include <errno.h>

#include "../../include/xsk_gpu.h"
#include "xsk_echo_kernels.h"
#include "xsk_gpu_internal.h"
#include "xsk_hip_util.h"

using namespace xskgpu;

namespace {

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

// Staged host mode: gather the rewritten header bytes of every TX_REPLY frame into a packed [n][96]
// array so the host can scatter them back into its UMEM (never touching unowned bytes): bytes [0, 38)
// in reference mode, [0, min(len, 96)) in wire mode (its rewrite ends at l4 + 4 <= 86 <= len).
constexpr uint32_t kPack = 96;
__global__ __launch_bounds__(256) void pack_headers_kernel(const uint8_t* umem, const xsk_gpu_desc* descs,
                                                           const uint8_t* verdicts, uint32_t n, uint8_t* pack,
                                                           uint32_t wire) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n || verdicts[i] != XSK_GPU_TX_REPLY) return;
    const uint8_t* p = umem + descs[i].addr;
    uint8_t* q = pack + (uint64_t)i * kPack;
    const uint32_t w = wire ? min(descs[i].len, kPack) : 38u;
    for (uint32_t k = 0; k < w; ++k) q[k] = p[k];
}

// Staged host mode, scattered descriptors: copy every frame's read span into the device mirror at the same offset.
// One 16-lane row per frame (4 frames per wave), 256-B row-loads, four in flight per lane before the stores -- a batch's
// PCIe reads overlap like the zerocopy kernel's.  Only the bytes the transform will read move (xsk_gpu__read_span),
// never the gaps between frames.  Two sources:
//   offs == nullptr: the mapped host UMEM (its device alias), read across PCIe at the frame's own offset (the gather);
//   offs != nullptr: a device staging buffer the host packed the spans into (no alias on this device): frame f's span
//                    starts at src + offs[f]; offs[f] == UINT32_MAX marks a frame the host copied by itself.
__global__ __launch_bounds__(256) void stage_gather_kernel(const uint8_t* src, const uint32_t* offs, uint8_t* dst,
                                                           uint64_t umem_size, const xsk_gpu_desc* descs, uint32_t n,
                                                           uint32_t wire) {
    const uint32_t f = (blockIdx.x * 256u + threadIdx.x) >> 4, k = threadIdx.x & 15u;
    if (f >= n) return;
    const xsk_gpu_desc d = descs[f];
    uint64_t a16 = 0;
    const uint64_t span = xsk_gpu__read_span(d.addr, d.len, umem_size, (int)wire, &a16);
    uint64_t from = a16;
    if (offs) {
        const uint32_t o = offs[f];
        if (o == UINT32_MAX) return;
        from = o;
    }
    const u32x4* s = (const u32x4*)(src + from);
    u32x4* t = (u32x4*)(dst + a16);
    const uint64_t nv = span >> 4;  // 16-B vectors
    for (uint64_t v0 = 0; v0 < nv; v0 += 64u) {
        u32x4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t v = v0 + 16u * (uint32_t)u + k;
            if (v < nv) x[u] = __builtin_nontemporal_load(s + v);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t v = v0 + 16u * (uint32_t)u + k;
            if (v < nv) t[v] = x[u];
        }
    }
}

// csum_replace2(csum, 0, 8) on the LE-loaded field: the inverse of the transform's (8 -> 0) patch
__device__ __forceinline__ uint32_t rearm_csum(uint32_t c) {
    uint32_t x = (~c) & 0xFFFFu;
    x = (x + 0xFFFFu) & 0xFFFFu;
    x += x < 0xFFFFu ? 1u : 0u;
    x = (x + 8u) & 0xFFFFu;
    x += x < 8u ? 1u : 0u;
    return (~x) & 0xFFFFu;
}

// Re-arm TX_REPLY frames (lane per frame; bench utility, not the hot path).  A 16-B aligned frame (every
// frame the bench generates) is re-armed as its whole 64-B sector -- four 16-B loads, the swaps as dword
// shuffles, four 16-B stores: no partial-sector writes (the frame owns [addr, addr + max(len, 64)),
// include/xsk_gpu.h); any other frame byte by byte.
__global__ __launch_bounds__(256) void rearm_kernel(uint8_t* umem, const xsk_gpu_desc* descs, const uint8_t* verdicts,
                                                    uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n || verdicts[i] != XSK_GPU_TX_REPLY) return;
    uint8_t* p = umem + descs[i].addr;
    if ((descs[i].addr & 15u) == 0) {
        u32x4* q = (u32x4*)p;
        u32x4 a = q[0], b = q[1], c = q[2];
        const u32x4 d = q[3];
        // bytes 0-11: MACs swapped back (the same shuffle as the transform's, xsk_receive.c:148-151)
        const uint32_t n0 = (a.y >> 16) | (a.z << 16), n1 = (a.z >> 16) | (a.x << 16), n2 = (a.x >> 16) | (a.y << 16);
        a.x = n0;
        a.y = n1;
        a.z = n2;
        // dwords 6, 7, 8 = bytes 24-35: IPv4 addresses swapped back (:153-155), type 0 -> 8 (byte 34)
        const uint32_t h6 = b.z, h7 = b.w, h8 = c.x;
        b.z = (h6 & 0xFFFFu) | (h7 & 0xFFFF0000u);
        b.w = (h8 & 0xFFFFu) | (h6 & 0xFFFF0000u);
        c.x = (h7 & 0xFFFFu) | (h8 & 0xFF000000u) | (8u << 16);
        c.y = (c.y & 0xFFFF0000u) | rearm_csum(c.y & 0xFFFFu);  // bytes 36-37
        q[0] = a;
        q[1] = b;
        q[2] = c;
        q[3] = d;
        return;
    }
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
    const uint32_t x = rearm_csum((uint32_t)p[36] | ((uint32_t)p[37] << 8));
    p[36] = (uint8_t)x;
    p[37] = (uint8_t)(x >> 8);
}

// Read-only streaming ceiling: every byte loaded once with 16-B nontemporal loads, in the pattern that measured
// fastest for a plain read (profiles/r01/read_order_ceilings_*.log: 6.8 TB/s on 1.5 GB): one 16-wave workgroup per
// CU over a contiguous share, each step four 1-KiB wave-loads per wave (64 KiB per workgroup) in flight.
__global__ __launch_bounds__(1024, 1) void stream_read_kernel(const u32x4* src, uint64_t nvec, unsigned long long* out) {
    const uint64_t per = (nvec + gridDim.x - 1) / gridDim.x;  // 16-B vectors of this workgroup's share
    const uint64_t b = (uint64_t)blockIdx.x * per;
    const uint64_t e = b + per < nvec ? b + per : nvec;
    uint64_t acc = 0;
    uint64_t i = b + threadIdx.x;
    for (; i + 3 * 1024 < e; i += 4 * 1024) {
        const u32x4 a0 = __builtin_nontemporal_load(src + i);
        const u32x4 a1 = __builtin_nontemporal_load(src + i + 1024);
        const u32x4 a2 = __builtin_nontemporal_load(src + i + 2048);
        const u32x4 a3 = __builtin_nontemporal_load(src + i + 3072);
        acc += (uint64_t)a0.x + a0.y + a0.z + a0.w + a1.x + a1.y + a1.z + a1.w;
        acc += (uint64_t)a2.x + a2.y + a2.z + a2.w + a3.x + a3.y + a3.z + a3.w;
    }
    for (; i < e; i += 1024) {
        const u32x4 a0 = __builtin_nontemporal_load(src + i);
        acc += (uint64_t)a0.x + a0.y + a0.z + a0.w;
    }
    acc = wave_sum_u64(acc);
    if ((threadIdx.x & 63u) == 0) atomicAdd(out, (unsigned long long)acc);
}

}  // namespace

extern "C" {

int xsk_gpu_synth_dev(void* d_umem, uint64_t umem_size, struct xsk_gpu_desc* d_descs, uint32_t n, uint64_t base_off,
                      uint64_t stride, uint64_t seed, uint64_t first, uint64_t step, int mode, uint32_t len_lo,
                      uint32_t len_hi, void* stream) {
    if (n == 0) return 0;
    if (n > XSK_GPU_MAX_BATCH) return -EINVAL;
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
    // at most 4 M frames (1 M workgroups) per launch: a grid's thread count must stay below 2^32
    constexpr uint32_t kChunk = 1u << 22;
    for (uint32_t c0 = 0; c0 < n; c0 += kChunk) {
        SynthArgs b = a;
        b.n = n - c0 < kChunk ? n - c0 : kChunk;
        b.descs = d_descs + c0;
        b.base_off = base_off + (uint64_t)c0 * stride;
        b.first = first + (uint64_t)c0 * step;
        hipLaunchKernelGGL(synth_kernel, dim3((b.n + 3) / 4), dim3(256), 0, (hipStream_t)stream, b);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}

int xsk_gpu_rearm_dev(void* d_umem, const struct xsk_gpu_desc* d_descs, const uint8_t* d_verdicts, uint32_t n,
                      void* stream) {
    if (n == 0) return 0;
    if (n > XSK_GPU_MAX_BATCH) return -EINVAL;
    if (!d_umem || !d_descs || !d_verdicts) return -EINVAL;
    hipLaunchKernelGGL(rearm_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (uint8_t*)d_umem, d_descs,
                       d_verdicts, n);
    HIP_TRY(hipGetLastError());
    return 0;
}

int xsk_gpu__pack_headers_dev(const void* d_umem, const struct xsk_gpu_desc* d_descs, const uint8_t* d_verdicts,
                              uint32_t n, uint8_t* d_pack, uint32_t wire, void* stream) {
    if (n == 0) return 0;
    if (n > XSK_GPU_MAX_BATCH) return -EINVAL;
    hipLaunchKernelGGL(pack_headers_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)d_umem, d_descs, d_verdicts, n, d_pack, wire);
    HIP_TRY(hipGetLastError());
    return 0;
}

static int stage_gather_launch(const void* src, const uint32_t* d_offs, void* d_mirror, uint64_t umem_size,
                               const struct xsk_gpu_desc* d_descs, uint32_t n, uint32_t wire, void* stream) {
    if (n == 0) return 0;
    if (n > XSK_GPU_MAX_BATCH || !src || !d_mirror || !d_descs) return -EINVAL;
    // <= 2^24 frames (2^22 workgroups) per launch
    constexpr uint32_t kChunk = 1u << 24;
    for (uint32_t c0 = 0; c0 < n; c0 += kChunk) {
        const uint32_t m = n - c0 < kChunk ? n - c0 : kChunk;
        hipLaunchKernelGGL(stage_gather_kernel, dim3((m + 15u) / 16u), dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t*)src, d_offs ? d_offs + c0 : nullptr, (uint8_t*)d_mirror, umem_size,
                           d_descs + c0, m, wire);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}

int xsk_gpu__stage_gather_dev(const void* m_umem, void* d_mirror, uint64_t umem_size, const struct xsk_gpu_desc* d_descs,
                              uint32_t n, uint32_t wire, void* stream) {
    return stage_gather_launch(m_umem, nullptr, d_mirror, umem_size, d_descs, n, wire, stream);
}

int xsk_gpu__stage_unpack_dev(const void* d_stage, const uint32_t* d_offs, void* d_mirror, uint64_t umem_size,
                              const struct xsk_gpu_desc* d_descs, uint32_t n, uint32_t wire, void* stream) {
    if (!d_offs) return -EINVAL;
    return stage_gather_launch(d_stage, d_offs, d_mirror, umem_size, d_descs, n, wire, stream);
}

int xsk_gpu_stream_read_dev(const void* d_src, uint64_t bytes, uint64_t* d_out, void* stream) {
    if (!d_src || !d_out || (bytes & 15u) || ((uintptr_t)d_src & 15u)) return -EINVAL;
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    hipLaunchKernelGGL(stream_read_kernel, dim3((unsigned)cus), dim3(1024), 0, (hipStream_t)stream,
                       (const u32x4*)d_src, bytes / 16, (unsigned long long*)d_out);
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"
