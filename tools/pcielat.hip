// pcielat.hip — how fast one wave reads and writes pinned host memory across PCIe (diagnostics for the
// LOWLAT doorbell path).  One workgroup of one wave; each pattern runs `reps` times over
// fresh host lines (the host rewrites the buffer between launches), timed with the 100-MHz wall clock
// (every timed region ends with an explicit wait for the memory operations it times):
//   pattern 0: one 8-byte system-coherent read (the doorbell)
//   pattern 1: 64 x 64-B reads at a 4-KiB stride, 4 instructions of 16 frames x 4 lanes (the short-tile
//              header windows), non-temporal loads (what the round kernel issues)
//   pattern 2: the same with plain loads;  pattern 3: with sc0|sc1 (system-coherent) buffer loads
//   pattern 4: 64 x 64-B reads at a 64-B stride (one contiguous 4-KiB run)
//   pattern 5: 1 x 16-B per lane, 64 lanes contiguous (the descriptors of a 64-frame batch)
//   pattern 6: 16 dependent 8-B system-coherent reads of one word (time / 16 = one round trip)
//   pattern 7: 16 dependent 8-B system-coherent reads of 16 different lines
//   pattern 8: 64 x 64-B plain stores at a 4-KiB stride, then a system-scope release fence
//   pattern 9: the same stores with sc0|sc1, then only a wait for the stores' acknowledgements
//   pattern 10: a system-scope release fence alone (nothing stored)
//   pattern 11: 64 x 64-B plain stores, then only a wait for their acknowledgements
//   pattern 12: 64 x 64-B non-temporal stores, then only a wait for their acknowledgements
//   pattern 13: a system-scope L2 + L1 invalidation (buffer_inv sc0 sc1), then pattern 1's reads
//   pattern 14: the invalidation alone, waited for
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libpcielat.so tools/pcielat.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <time.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t = wall_clock64();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return t;
}

__global__ __launch_bounds__(64) void pcielat_kernel(uint8_t* host, uint32_t pattern, uint32_t stride,
                                                     unsigned long long* out) {
    const uint32_t lane = threadIdx.x;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)host, (short)0, 0x7FFFFFFF, 0x00020000);
    const uint32_t kk = lane & 3u;
    uint32_t acc = 0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const uint64_t t0 = stamp();
    if (pattern == 0) {
        acc = (uint32_t)__hip_atomic_load((const uint64_t*)host, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (pattern <= 4 || pattern == 13) {
        if (pattern == 13) asm volatile("buffer_inv sc0 sc1" ::: "memory");
        u32x4 x[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
            const u32x4* p = (const u32x4*)(host + (uint64_t)f * stride + 16u * kk);
            if (pattern == 1 || pattern == 13) x[r] = __builtin_nontemporal_load(p);
            else if (pattern == 2) x[r] = *p;
            else x[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(f * stride + 16u * kk), 0, 1 | 16);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) acc += x[r].x ^ x[r].y ^ x[r].z ^ x[r].w;
    } else if (pattern == 14) {
        asm volatile("buffer_inv sc0 sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
    } else if (pattern == 5) {
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)(host + 16u * lane));
        acc = v.x ^ v.w;
    } else if (pattern == 6 || pattern == 7) {
        uint64_t off = 0;
        for (int r = 0; r < 16; ++r) {
            const uint64_t v = __hip_atomic_load((const uint64_t*)(host + off), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            acc += (uint32_t)v;
            // the next address depends on the value read (at most 64 B further: stays in the buffer)
            off = (pattern == 7 ? (uint64_t)(r + 1) * stride : 0ull) + (((uint32_t)v >> 31) << 6);
        }
    } else if (pattern <= 12) {
        if (pattern != 10) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t f = (uint32_t)r * 16u + (lane >> 2);
                const u32x4 w = u32x4{lane, f, pattern, 7u};
                u32x4* p = (u32x4*)(host + (uint64_t)f * stride + 16u * kk);
                if (pattern == 9) __builtin_amdgcn_raw_buffer_store_b128(w, rs, (int)(f * stride + 16u * kk), 0, 1 | 16);
                else if (pattern == 12) __builtin_nontemporal_store(w, p);
                else *p = w;
            }
        }
        if (pattern == 8 || pattern == 10) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // make the loaded data live and wait for every memory operation, then stop the clock
    acc = __builtin_amdgcn_readfirstlane(acc) | 1u;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const uint64_t t1 = stamp();
    if (lane == 0) {
        out[0] = t1 - t0;
        out[1] = acc;
    }
}

extern "C" int pcielat_run(void* d_host_alias, uint32_t pattern, uint32_t stride, unsigned long long* d_out) {
    hipLaunchKernelGGL(pcielat_kernel, dim3(1), dim3(64), 0, 0, (uint8_t*)d_host_alias, pattern, stride, d_out);
    if (hipGetLastError() != hipSuccess) return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

// Ping-pong: one wave polls word 0 of `flags` (fine-grained host memory) for i = 1 .. iters and answers
// each with a store of i to word 16 (another line); the host posts i and spins on the answer.  The host's
// round-trip time per exchange is the floor of a doorbell + completion handshake.  mode 0: one poll in
// flight, relaxed answer; 1: relaxed answer after a system release fence; 2: two polls in flight (the
// word and a copy at word 8 ... kept equal by the host).  Every wave leaves after iters or 100 ms idle.
__global__ __launch_bounds__(64) void pingpong_kernel(uint64_t* flags, uint32_t iters, uint32_t mode) {
    uint64_t last = wall_clock64();
    for (uint32_t i = 1; i <= iters;) {
        uint64_t v = __hip_atomic_load(flags + ((mode == 2 && (i & 1u)) ? 8 : 0), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
        v = __builtin_amdgcn_readfirstlane((uint32_t)v);
        if (v >= i) {
            if (mode == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __hip_atomic_store(flags + 16, (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            ++i;
            last = wall_clock64();
        } else if (wall_clock64() - last > 10000000ull) {
            break;  // 100 ms without a post: the host is gone
        }
    }
}

extern "C" int pcielat_pingpong(void* d_flags, volatile uint64_t* h_flags, uint32_t iters, uint32_t mode,
                                double* ns_per_exchange) {
    for (int k = 0; k < 24; ++k) h_flags[k] = 0;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -1;
    hipLaunchKernelGGL(pingpong_kernel, dim3(1), dim3(64), 0, s, (uint64_t*)d_flags, iters, mode);
    if (hipGetLastError() != hipSuccess) return -1;
    // the first exchange also waits for the launch: time the rest
    struct timespec t0, t1;
    int rc = 0;
    for (uint32_t i = 1; i <= iters; ++i) {
        if (i == 2) clock_gettime(CLOCK_MONOTONIC, &t0);
        __atomic_store_n(&h_flags[8], (uint64_t)i, __ATOMIC_SEQ_CST);
        __atomic_store_n(&h_flags[0], (uint64_t)i, __ATOMIC_SEQ_CST);
        uint64_t spins = 0;
        while (__atomic_load_n(&h_flags[16], __ATOMIC_ACQUIRE) < i) {
            __builtin_ia32_pause();
            if (++spins > 400000000ull) { rc = -2; break; }
        }
        if (rc) break;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    *ns_per_exchange = ((t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec)) / (double)(iters - 1);
    if (hipStreamSynchronize(s) != hipSuccess) rc = -1;
    (void)hipStreamDestroy(s);
    return rc;
}
