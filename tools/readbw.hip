// readbw.hip -- HBM read-rate probe (tool, not the product): how fast can ANY kernel read a slab once on this MI355X?
// the bench's read ceiling (xsk_gpu_stream_read_dev: one 1024-thread workgroup per CU,
// a contiguous share each, four 16-B nontemporal loads in flight per lane) is one read pattern; these are others.  Each
// variant reads every 16-B vector of the slab once and folds it into a sum (so no load is dead), one atomic per wave.
//   shape 0: contiguous share per workgroup, `wg_per_cu` workgroups of `threads` per CU, U loads in flight per lane
//   shape 1: grid-stride (consecutive workgroups read consecutive chunks of threads * U vectors, round after round)
// Built by tools/readbw.py (hipcc --offload-arch=gfx950 -shared); driven from Python with torch device buffers.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int U, bool NT, int SHAPE>
__global__ void read_kernel(const u32x4* __restrict__ src, uint64_t nvec, unsigned long long* out) {
    const uint64_t T = blockDim.x;
    uint64_t acc = 0;
    if constexpr (SHAPE == 0) {
        const uint64_t per = (nvec + gridDim.x - 1) / gridDim.x;
        const uint64_t b = (uint64_t)blockIdx.x * per;
        const uint64_t e = b + per < nvec ? b + per : nvec;
        uint64_t i = b + threadIdx.x;
        for (; i + (U - 1) * T < e; i += U * T) {
            u32x4 a[U];
#pragma unroll
            for (int k = 0; k < U; ++k) a[k] = ld<U, NT>(src + i + k * T);
#pragma unroll
            for (int k = 0; k < U; ++k) acc += (uint64_t)a[k].x + a[k].y + a[k].z + a[k].w;
        }
        for (; i < e; i += T) {
            const u32x4 a = ld<U, NT>(src + i);
            acc += (uint64_t)a.x + a.y + a.z + a.w;
        }
    } else {
        const uint64_t chunk = U * T;
        const uint64_t stride = chunk * gridDim.x;
        uint64_t i = (uint64_t)blockIdx.x * chunk + threadIdx.x;
        for (; i + (U - 1) * T < nvec; i += stride) {
            u32x4 a[U];
#pragma unroll
            for (int k = 0; k < U; ++k) a[k] = ld<U, NT>(src + i + k * T);
#pragma unroll
            for (int k = 0; k < U; ++k) acc += (uint64_t)a[k].x + a[k].y + a[k].z + a[k].w;
        }
        for (; i < nvec; i += T) {
            const u32x4 a = ld<U, NT>(src + i);
            acc += (uint64_t)a.x + a.y + a.z + a.w;
        }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63u) == 0) atomicAdd(out, (unsigned long long)acc);
}

#define CASE(U, NT, S)                                                                                  \
    if (u == U && nt == NT && shape == S) {                                                           \
        hipLaunchKernelGGL((read_kernel<U, NT, S>), dim3(grid), dim3(threads), 0, (hipStream_t)stream, \
                           (const u32x4*)src, bytes / 16, (unsigned long long*)out);                   \
        return hipGetLastError() == hipSuccess ? 0 : -5;                                               \
    }

extern "C" int readbw_launch(const void* src, uint64_t bytes, void* out, int shape, int u, int nt, unsigned grid,
                             unsigned threads, void* stream) {
    if (!src || !out || (bytes & 15u) || threads == 0 || threads > 1024 || grid == 0) return -22;
    CASE(4, 1, 0) CASE(4, 0, 0) CASE(8, 1, 0) CASE(8, 0, 0) CASE(16, 1, 0) CASE(16, 0, 0)
    CASE(4, 1, 1) CASE(4, 0, 1) CASE(8, 1, 1) CASE(8, 0, 1) CASE(16, 1, 1) CASE(16, 0, 1)
    return -22;
}
