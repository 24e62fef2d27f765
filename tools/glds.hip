// glds.hip — read-ceiling micro-experiment (GPU box, tuning only): register loads vs LDS-DMA
// (global_load_lds_dwordx4) for the frame layouts of the echo transform.
//
// A "piece" is one wave-instruction's 1 KiB.  Layout 0: contiguous slab (piece p = bytes [1024p, 1024p+1024)).
// Layout 1: row streams as in the round kernel — piece p covers row r = p % R of the four frames 4g..4g+3
// (g = p / R, R = ceil(len / 256)); lane l reads frame 4g + l/16 at r*256 + (l%16)*16, masked beyond len.
// Layout 2: frame-major 1 KiB pieces (two per frame up to 2 KiB); layout 3: 128-B rows of 8 frames.
// Every wave walks pieces p = w, w + W, ... (W = all waves), U pieces in flight.
//   reg<U>      : __builtin_nontemporal_load into VGPRs, then sum
//   glds<U,AUX> : global_load_lds_dwordx4 into a per-wave LDS ring of U KiB, s_waitcnt vmcnt(0), ds_read of
//                 the lane's own 16 B (the DMA image is lane-linear), sum.  AUX 2 = nt, 0 = default policy.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Geo {
    const uint8_t* base;
    uint64_t npieces;
    uint32_t layout, len, stride, rows;
};

__device__ __forceinline__ const uint8_t* piece_src(const Geo& g, uint64_t p, uint32_t lane, bool& in) {
    if (g.layout == 0) {
        in = true;
        return g.base + p * 1024u + lane * 16u;
    }
    if (g.layout == 2) {  // frame-major: piece p = 1 KiB part p % 2 of frame p / 2 (len <= 2048)
        const uint64_t f = p >> 1;
        const uint32_t off = (uint32_t)(p & 1u) * 1024u + lane * 16u;
        in = off < g.len;
        return g.base + f * g.stride + (in ? off : 0u);
    }
    if (g.layout == 3) {  // 128-B rows of 8 frames: piece p = row p % R8 of frames 8g..8g+7
        const uint32_t r8 = (g.len + 127u) / 128u;
        const uint64_t grp = p / r8;
        const uint32_t r = (uint32_t)(p - grp * r8);
        const uint64_t f = grp * 8u + (lane >> 3);
        const uint32_t off = r * 128u + (lane & 7u) * 16u;
        in = off < g.len;
        return g.base + f * g.stride + (in ? off : 0u);
    }
    const uint64_t grp = p / g.rows;
    const uint32_t r = (uint32_t)(p - grp * g.rows);
    const uint64_t f = grp * 4u + (lane >> 4);
    const uint32_t off = r * 256u + (lane & 15u) * 16u;
    uint32_t len = g.len;
    if (g.layout == 4) {  // c4-like: len of frame f uniform in [64, 1500] (hash of f), rows up to 6
        uint32_t h = (uint32_t)f * 0x9E3779B1u;
        h ^= h >> 15;
        h *= 0x85EBCA77u;
        h ^= h >> 13;
        len = 64u + h % 1437u;
    }
    in = off < len;
    return g.base + f * g.stride + (in ? off : 0u);
}

template <int U>
__global__ __launch_bounds__(256) void reg_read(Geo g, unsigned long long* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t W = (uint64_t)gridDim.x * 4u, w = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    uint64_t acc = 0;
    for (uint64_t p0 = w; p0 < g.npieces; p0 += U * W) {
        u32x4 x[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t p = p0 + u * W;
            bool in = false;
            const uint8_t* s = p < g.npieces ? piece_src(g, p, lane, in) : g.base;
            ok[u] = in && p < g.npieces;
            x[u] = __builtin_nontemporal_load((const u32x4*)s);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) acc += (uint64_t)x[u].x + x[u].y + x[u].z + x[u].w;
    }
    if (acc == 0x123456789ull) out[0] = acc;
}

template <int U, int AUX>
__global__ __launch_bounds__(256) void glds_read(Geo g, unsigned long long* out) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[4][U][1024];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t W = (uint64_t)gridDim.x * 4u, w = (uint64_t)blockIdx.x * 4u + wv;
    uint64_t acc = 0;
    for (uint64_t p0 = w; p0 < g.npieces; p0 += U * W) {
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t p = p0 + u * W;
            bool in = false;
            const uint8_t* s = p < g.npieces ? piece_src(g, p, lane, in) : g.base;
            ok[u] = in && p < g.npieces;
            __builtin_amdgcn_global_load_lds((const void*)s, (__attribute__((address_space(3))) void*)&ring[wv][u][0],
                                             16, 0, AUX);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32x4 y = *(const u32x4*)&ring[wv][u][lane * 16u];
            if (ok[u]) acc += (uint64_t)y.x + y.y + y.z + y.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring reads done before the next DMA overwrites
    }
    if (acc == 0x123456789ull) out[0] = acc;
}

// Per-workgroup contiguous shares (persistent, one 1024-thread workgroup per CU): workgroup b streams
// pieces [b * P / G, (b + 1) * P / G); its 16 waves take consecutive pieces (wave w: base + k * 16 + w).
template <int U>
__global__ __launch_bounds__(1024) void reg_read_wg(Geo g, unsigned long long* out) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t per = (g.npieces + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < g.npieces ? b0 + per : g.npieces;
    uint64_t acc = 0;
    for (uint64_t p0 = b0 + wv; p0 < b1; p0 += U * 16u) {
        u32x4 x[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t p = p0 + u * 16u;
            bool in = false;
            const uint8_t* s = p < b1 ? piece_src(g, p, lane, in) : g.base;
            ok[u] = in && p < b1;
            x[u] = __builtin_nontemporal_load((const u32x4*)s);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) acc += (uint64_t)x[u].x + x[u].y + x[u].z + x[u].w;
    }
    if (acc == 0x123456789ull) out[0] = acc;
}

extern "C" int glds_run(int kind, const void* base, uint64_t npieces, uint32_t layout, uint32_t len, uint32_t stride,
                        uint32_t grid, void* out, void* stream) {
    Geo g{(const uint8_t*)base, npieces, layout, len, stride, (len + 255u) / 256u};
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* o = (unsigned long long*)out;
    switch (kind) {
        case 0: reg_read<4><<<grid, 256, 0, s>>>(g, o); break;
        case 1: reg_read<8><<<grid, 256, 0, s>>>(g, o); break;
        case 2: glds_read<4, 2><<<grid, 256, 0, s>>>(g, o); break;
        case 3: glds_read<8, 2><<<grid, 256, 0, s>>>(g, o); break;
        case 4: glds_read<4, 0><<<grid, 256, 0, s>>>(g, o); break;
        case 5: glds_read<8, 0><<<grid, 256, 0, s>>>(g, o); break;
        case 6: glds_read<16, 2><<<grid, 256, 0, s>>>(g, o); break;
        case 7: reg_read_wg<4><<<grid, 1024, 0, s>>>(g, o); break;
        case 8: reg_read_wg<8><<<grid, 1024, 0, s>>>(g, o); break;
        case 9: reg_read_wg<2><<<grid, 1024, 0, s>>>(g, o); break;
        default: return -22;
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}
