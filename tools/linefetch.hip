// linefetch.hip — what a partially read 128-B line costs on gfx950 (do loads that touch
// only the first 64 B of a line fetch 64 B or 128 B?).  Cold 4 GiB buffers, each mode one launch per buffer:
//   0  every byte of every 128-B line (1 KiB per wave-load)
//   1  the first 64 B of every 128-B line (16 lines per wave-load)
//   2  the first 16 B of every 128-B line (64 lines per wave-load)
//   3  c4's read pattern: 1 M frames at a 2 KiB stride, frame j's bytes [0, L_j) with L_j uniform in 64..1500,
//      16-lane rows streaming 256-B row-loads, lanes past the frame end not loading (buffer out-of-range)
//   4  the same with every frame's read rounded up to whole 128-B lines
//   5  c4's frame bytes read in address order: the slab swept by 1-KiB wave-loads (grid-stride), a lane loading its
//      16-B block only if it lies inside its 2-KiB slot's frame [0, L_j) -- the DRAM sees c4's exact lines in order
//   6  the same sweep over contiguous per-workgroup shares (the read-ceiling kernel's pattern, 1 workgroup per CU)
//   7  every byte, contiguous per-workgroup shares (the read ceiling itself on this buffer)
//   8  c4's frames, one LANE per frame: every lane streams its own frame with 16-B loads, eight in flight, so each
//      wave-load instruction reaches 64 frames at once -- DRAM parallelism far above any row-stream's (L2 merges the
//      four 16-B loads of a sector); how fast can the memory system deliver c4's lines at all?
// (round 4: is c4's read phase at the floor of its access pattern, or is the contiguous read ceiling reachable?)
// Every lane sums what it read into one atomic per wave (no dead-code elimination, negligible traffic).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t flen(uint32_t j) {  // deterministic U{64..1500}
    uint64_t z = (uint64_t)j * 0x9E3779B97F4A7C15ull + 0x5EED0004ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return 64u + (uint32_t)(z % 1437u);
}

__device__ __forceinline__ uint32_t max_lane(uint32_t x) {
    for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
    return x;
}

template <int MODE>
__global__ __launch_bounds__(1024) void linefetch(const uint8_t* buf, uint64_t bytes, unsigned long long* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 16u + (threadIdx.x >> 6), nwaves = (uint64_t)gridDim.x * 16u;
    uint32_t acc = 0;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, 0x7FFFFFF0, 0x00020000);
    if (MODE <= 2) {
        // per wave-load: MODE 0 -> 1 KiB contiguous, 1 -> 16 lines x 64 B, 2 -> 64 lines x 16 B
        constexpr uint64_t span = MODE == 0 ? 1024u : MODE == 1 ? 2048u : 8192u;
        const uint64_t off_l = MODE == 0 ? 16u * lane : MODE == 1 ? 128u * (lane >> 2) + 16u * (lane & 3u) : 128u * lane;
        const uint64_t units = bytes / span;
        for (uint64_t u = wave * 4u; u < units; u += nwaves * 4u) {
            u32x4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint64_t o = (u + i) * span + off_l;
                v[i] = u + i < units ? __builtin_nontemporal_load((const u32x4*)(buf + o)) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) acc += v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        }
    } else if (MODE == 8) {
        const uint64_t nframes = bytes / 2048u;
        for (uint64_t t = wave; t * 64u < nframes; t += nwaves) {
            const uint64_t f = t * 64u + lane;
            const uint32_t L = f < nframes ? flen((uint32_t)f) : 0u;
            const uint8_t* fb = buf + f * 2048u;
            const uint32_t nv = (L + 15u) >> 4, mx = __builtin_amdgcn_readfirstlane(max_lane(nv));
            for (uint32_t j0 = 0; j0 < mx; j0 += 8) {
                u32x4 v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    v[i] = u32x4{0u, 0u, 0u, 0u};
                    if (j0 + i < nv) v[i] = __builtin_nontemporal_load((const u32x4*)(fb + 16u * (j0 + i)));
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) acc += v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
            }
        }
    } else if (MODE >= 5) {
        const uint64_t units = bytes / 1024u;  // 1-KiB wave-loads
        uint64_t u0, u1, step;
        if (MODE == 5) {
            u0 = wave * 4u;
            u1 = units;
            step = nwaves * 4u;
        } else {  // contiguous share of the workgroup, its 16 waves interleaved by wave-load
            const uint64_t per = (units + gridDim.x - 1) / gridDim.x;
            u0 = (uint64_t)blockIdx.x * per + (threadIdx.x >> 6) * 4u;
            u1 = min(units, (uint64_t)blockIdx.x * per + per);
            step = 64u;
        }
        for (uint64_t u = u0; u < u1; u += step) {
            u32x4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint64_t o = (u + i) * 1024u + 16u * lane;
                const uint32_t L = MODE == 7 ? 2048u : flen((uint32_t)(o >> 11));
                v[i] = u32x4{0u, 0u, 0u, 0u};
                if (u + i < u1 && (o & 2047u) < L) v[i] = __builtin_nontemporal_load((const u32x4*)(buf + o));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) acc += v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        }
    } else {
        const uint32_t q = lane >> 4, k = lane & 15u;
        const uint64_t nframes = bytes / 2048u;
        for (uint64_t f0 = wave * 4u; f0 < nframes; f0 += nwaves * 4u) {  // 4 frames per wave-step, one per row
            const uint64_t f = f0 + q;
            uint32_t L = f < nframes ? flen((uint32_t)f) : 0u;
            if (MODE == 4) L = (L + 127u) & ~127u;
            const uint32_t ns = (L + 255u) >> 8;
            const uint32_t nsw = __builtin_amdgcn_readfirstlane(max(max(__shfl(ns, 0), __shfl(ns, 16)), max(__shfl(ns, 32), __shfl(ns, 48))));
            const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc((void*)(buf + f0 * 2048u), (short)0, 0x7FFFFFF0, 0x00020000);
            for (uint32_t j0 = 0; j0 < nsw; j0 += 4) {
                u32x4 v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t ro = 256u * (j0 + i) + 16u * k;
                    v[i] = __builtin_amdgcn_raw_buffer_load_b128(rf, (int)(ro < L ? q * 2048u + ro : 0x80000000u), 0, 2);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) acc += v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
            }
        }
        (void)r;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) atomicAdd(out, (unsigned long long)acc);
}

extern "C" int linefetch_run(int mode, const void* buf, uint64_t bytes, void* out, uint32_t grid, void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    unsigned long long* o = (unsigned long long*)out;
    const uint8_t* b = (const uint8_t*)buf;
    switch (mode) {
        case 0: linefetch<0><<<grid, 1024, 0, s>>>(b, bytes, o); break;
        case 1: linefetch<1><<<grid, 1024, 0, s>>>(b, bytes, o); break;
        case 2: linefetch<2><<<grid, 1024, 0, s>>>(b, bytes, o); break;
        case 3: linefetch<3><<<grid, 1024, 0, s>>>(b, bytes, o); break;
        case 4: linefetch<4><<<grid, 1024, 0, s>>>(b, bytes, o); break;
        case 5: linefetch<5><<<grid, 1024, 0, s>>>(b, bytes, o); break;
        case 6: linefetch<6><<<grid / 4, 1024, 0, s>>>(b, bytes, o); break;  // one workgroup per CU
        case 7: linefetch<7><<<grid / 4, 1024, 0, s>>>(b, bytes, o); break;
        case 8: linefetch<8><<<grid / 4, 1024, 0, s>>>(b, bytes, o); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
