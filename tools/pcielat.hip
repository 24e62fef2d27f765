// pcielat.hip — how fast one wave reads pinned host memory across PCIe (diagnostics for the LOWLAT
// doorbell path).  One workgroup of one wave; each pattern runs `reps` times over fresh
// host lines (the host rewrites the buffer between launches), timed with the 100-MHz wall clock:
//   pattern 0: one 8-byte read (the doorbell)
//   pattern 1: 64 x 64-B reads at a 4-KiB stride, 4 instructions of 16 frames x 4 lanes (the short-tile
//              header windows), non-temporal loads (what the round kernel issues)
//   pattern 2: the same with plain loads;  pattern 3: with sc0|sc1 (system-coherent) buffer loads
//   pattern 4: 64 x 64-B reads at a 64-B stride (one contiguous 4-KiB run)
//   pattern 5: 1 x 16-B per lane, 64 lanes contiguous (the descriptors of a 64-frame batch)
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libpcielat.so tools/pcielat.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void pcielat_kernel(const uint8_t* host, uint32_t pattern, uint32_t stride,
                                                     unsigned long long* out) {
    const uint32_t lane = threadIdx.x;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint64_t t0 = wall_clock64();
    uint32_t acc = 0;
    if (pattern == 0) {
        acc = (uint32_t)__hip_atomic_load((const uint64_t*)host, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (pattern <= 4) {
        const uint32_t kk = lane & 3u;
        u32x4 x[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
            const u32x4* p = (const u32x4*)(host + (uint64_t)f * stride + 16u * kk);
            if (pattern == 1) x[r] = __builtin_nontemporal_load(p);
            else if (pattern == 2) x[r] = *p;
            else {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)host, (short)0, 0x7FFFFFFF,
                                                                                   0x00020000);
                x[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(f * stride + 16u * kk), 0, 1 | 16);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) acc += x[r].x ^ x[r].y ^ x[r].z ^ x[r].w;
    } else {
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)(host + 16u * lane));
        acc = v.x ^ v.w;
    }
    // make the loaded data live, then stop the clock
    acc = __builtin_amdgcn_readfirstlane(acc) | 1u;
    const uint64_t t1 = wall_clock64();
    if (lane == 0) {
        out[0] = t1 - t0;
        out[1] = acc;
    }
}

extern "C" int pcielat_run(const void* d_host_alias, uint32_t pattern, uint32_t stride, unsigned long long* d_out) {
    hipLaunchKernelGGL(pcielat_kernel, dim3(1), dim3(64), 0, 0, (const uint8_t*)d_host_alias, pattern, stride, d_out);
    if (hipGetLastError() != hipSuccess) return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
