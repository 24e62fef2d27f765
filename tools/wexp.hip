// wexp.hip — write-pattern micro-experiment (tuning tool, not the product).
// Streams 1500-B frames at a fixed stride like the echo kernel's row streaming (16 lanes per frame,
// 16 B per lane per load) and writes back a header-sized piece of every frame in different ways, to
// price in-place header write-back against the read stream.  Writes store the bytes just read, so
// every run leaves the buffer unchanged.
//   mode 0: read only
//   mode 1: + 64 B per frame (4 lanes x 16 B, right after the frame's loads)
//   mode 2: + 128 B per frame (8 lanes x 16 B)
//   mode 3: + 38 B per frame as dwordx3 + dwordx3 + short from one lane (the reference's bytes)
//   mode 4: + 64 B per frame, deferred to the end of the 64-frame tile (staged in LDS)
//   mode 5: write only, 64 B per frame (no payload reads)
//   mode 6: mode 1 with default-policy (not nt) loads
//   mode 7: mode 4 with nontemporal stores
//   mode 8: + 64 B per frame into a contiguous side buffer (coalesced), not in place
//   mode 9: header read only, 64 B per frame (4 lanes), no payload
//   mode 10: + 64 B per frame of constant data stored right after the frame's loads are ISSUED
//            (before they return): the write reaches the DRAM page the reads just opened
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

template <int MODE>
__global__ __launch_bounds__(256) void wexp_kernel(uint8_t* buf, uint32_t n, uint32_t stride, uint32_t len,
                                                   unsigned long long* out, uint8_t* side) {
    __shared__ __attribute__((aligned(16))) uint8_t s_row[4][64 * 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t q = lane >> 4, k = lane & 15u;
    const uint32_t ntiles = (n + 63) / 64, nw = gridDim.x * 4;
    uint64_t acc = 0;
    for (uint32_t t = blockIdx.x * 4 + wave; t < ntiles; t += nw) {
        for (uint32_t s = 0; s < 16; ++s) {
            const uint32_t f = t * 64 + 4 * s + q;
            if (f >= n) break;
            uint8_t* fr = buf + (uint64_t)f * stride;
            u32x4 v[6];
            if (MODE == 10) {  // unconditional loads (stride >= 1536), then the store, then the waits
#pragma unroll
                for (int u = 0; u < 6; ++u) v[u] = __builtin_nontemporal_load((const u32x4*)(fr + 256u * u + 16u * k));
                if (k < 4) {
                    const u32x4 c = u32x4{f, 0x5A5A5A5Au, f, 0x01234567u};
                    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(fr + 16u * k), "v"(c) : "memory");
                }
#pragma unroll
                for (int u = 0; u < 6; ++u) acc += (uint64_t)v[u].x + v[u].y + v[u].z + v[u].w;
            } else if (MODE == 9) {
                v[0] = k < 4 ? __builtin_nontemporal_load((const u32x4*)(fr + 16u * k)) : u32x4{0, 0, 0, 0};
                acc += (uint64_t)v[0].x + v[0].y + v[0].z + v[0].w;
            } else if (MODE != 5) {
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    const uint32_t ro = 256u * u + 16u * k;
                    v[u] = u32x4{0, 0, 0, 0};
                    if (ro < len) {
                        if (MODE == 6) v[u] = *(const u32x4*)(fr + ro);
                        else v[u] = __builtin_nontemporal_load((const u32x4*)(fr + ro));
                    }
                }
#pragma unroll
                for (int u = 0; u < 6; ++u) acc += (uint64_t)v[u].x + v[u].y + v[u].z + v[u].w;
            } else {
                v[0] = *(const u32x4*)(buf + 16u * k);  // same bytes for every frame: L2 hits
            }
            if ((MODE == 1 || MODE == 5 || MODE == 6) && k < 4) *(u32x4*)(fr + 16u * k) = v[0];
            if (MODE == 2 && k < 8) *(u32x4*)(fr + 16u * k) = v[0];
            if (MODE == 3) {
                const uint32_t x0 = (uint32_t)__shfl((int)v[0].x, q * 16 + 0), x1 = (uint32_t)__shfl((int)v[0].y, q * 16 + 0),
                               x2 = (uint32_t)__shfl((int)v[0].z, q * 16 + 0);
                const uint32_t y0 = (uint32_t)__shfl((int)v[0].z, q * 16 + 1), y1 = (uint32_t)__shfl((int)v[0].w, q * 16 + 1),
                               y2 = (uint32_t)__shfl((int)v[0].x, q * 16 + 2), c = (uint32_t)__shfl((int)v[0].y, q * 16 + 2);
                if (k == 0) {
                    *(u32x3*)fr = u32x3{x0, x1, x2};
                    *(u32x3*)(fr + 24) = u32x3{y0, y1, y2};
                    *(uint16_t*)(fr + 36) = (uint16_t)c;
                }
            }
            if (MODE == 8 && k < 4) *(u32x4*)(side + (uint64_t)f * 64 + 16u * k) = v[0];
            if ((MODE == 4 || MODE == 7) && k < 4) *(u32x4*)(&s_row[wave][(4 * s + q) * 64 + 16 * k]) = v[0];
        }
        if (MODE == 4 || MODE == 7) {
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t f = t * 64 + r * 16 + (lane >> 2);
                if (f < n) {
                    u32x4* dst = (u32x4*)(buf + (uint64_t)f * stride + 16u * (lane & 3u));
                    const u32x4 w = *(const u32x4*)(&s_row[wave][(r * 16 + (lane >> 2)) * 64 + 16 * (lane & 3u)]);
                    if (MODE == 7) __builtin_nontemporal_store(w, dst);
                    else *dst = w;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (acc == 0x123456789ull) out[0] = acc;  // keeps the loads alive
}

extern "C" int wexp_run(int mode, void* buf, uint32_t n, uint32_t stride, uint32_t len, void* out, uint32_t grid,
                        void* stream, void* side_) {
    uint8_t* side = (uint8_t*)side_;
    const dim3 g(grid), b(256);
    hipStream_t s = (hipStream_t)stream;
    uint8_t* p = (uint8_t*)buf;
    unsigned long long* o = (unsigned long long*)out;
    switch (mode) {
        case 0: wexp_kernel<0><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 1: wexp_kernel<1><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 2: wexp_kernel<2><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 3: wexp_kernel<3><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 4: wexp_kernel<4><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 5: wexp_kernel<5><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 6: wexp_kernel<6><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 7: wexp_kernel<7><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 8: wexp_kernel<8><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 9: wexp_kernel<9><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 10: wexp_kernel<10><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
