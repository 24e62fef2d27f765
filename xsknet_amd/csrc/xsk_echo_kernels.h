// xsk_echo_kernels.h — device helpers shared by the echo, synth and rearm kernels (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xskgpu {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Keep bytes [lo, hi) of the little-endian dword whose first byte sits at `base` (all in one
// coordinate system); bytes outside become zero.
__device__ __forceinline__ uint32_t keep_bytes(uint32_t v, int base, int lo, int hi) {
    int s = lo - base;
    int e = hi - base;
    s = s < 0 ? 0 : s;
    e = e > 4 ? 4 : e;
    const uint32_t ms = s >= 4 ? 0u : (0xFFFFFFFFu << (8 * s));
    const uint32_t me = e <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - e)));
    return e > s ? (v & ms & me) : 0u;
}

// Sum of the two little-endian 16-bit halves of a dword (one's-complement partial, < 2^17).
__device__ __forceinline__ uint32_t halves(uint32_t v) { return (v & 0xFFFFu) + (v >> 16); }

// Fold a 64-bit sum of 16-bit words (or of dwords) to 16 bits, end-around carry (RFC 1071 §4.1).
__device__ __forceinline__ uint32_t fold64(uint64_t a) {
    uint64_t t = (a & 0xFFFFFFFFull) + (a >> 32);
    t = (t & 0xFFFFFFFFull) + (t >> 32);
    uint32_t x = (uint32_t)t;
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return x;
}
__device__ __forceinline__ uint32_t fold32(uint32_t x) {
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return x;
}
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// Wave-wide (64-lane) sum; every lane receives the total.  Butterfly over ds_swizzle/bpermute —
// the __shfl_down tree of the north star, run as xor so no final broadcast is needed.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// splitmix64 output function (oracle/echo_oracle.c:oracle_mix64).
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

}  // namespace xskgpu
