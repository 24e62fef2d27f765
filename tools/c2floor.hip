// Floors for c2's traffic shape (packed 64-B frames): what a plain streaming kernel with no rounds, no LDS and no
// header phase takes to read each frame's descriptor and 64 bytes and write the 64 bytes back (unchanged), a 16-B
// record and a verdict byte.  Used to decide whether a lane-per-frame path for short frames could beat the round kernel on c2.
//   mode 0: four lanes per frame (lane q moves bytes 16q..16q+15), desc read by every lane of the frame
//   mode 1: one lane per frame, four 16-B loads and stores per lane
//   mode 2: frames only (no descriptors, records or verdicts): 64 MB in place, the copy floor
//   mode 3: mode 0 with the frame address taken from the descriptor (dependent load, as the product must)
#include <hip/hip_runtime.h>
#include <stdint.h>

struct Desc {
    uint64_t addr;
    uint32_t len;
    uint32_t options;
};

template <int MODE>
__global__ __launch_bounds__(256) void c2floor(uint8_t* umem, const Desc* descs, uint8_t* verd, uint4* recs,
                                               uint32_t n) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (MODE == 1) {
        if (t >= n) return;
        const Desc d = descs[t];
        uint4* f = (uint4*)(umem + d.addr);
        uint4 v0 = f[0], v1 = f[1], v2 = f[2], v3 = f[3];
        asm volatile("" : "+v"(v0.x), "+v"(v1.x), "+v"(v2.x), "+v"(v3.x));  // stored back unchanged, not elided
        f[0] = v0; f[1] = v1; f[2] = v2; f[3] = v3;
        recs[t] = make_uint4(v0.x + v1.x, v2.x + v3.x, d.len, 3u);
        verd[t] = 1;
        return;
    }
    const uint32_t fi = t >> 2, q = t & 3u;
    if (fi >= n) return;
    uint4* f;
    uint32_t len = 64;
    if (MODE == 2) {
        f = (uint4*)(umem + (uint64_t)fi * 64u);
    } else if (MODE == 0) {
        const uint4 dd = ((const uint4*)descs)[fi];
        len = dd.z;
        f = (uint4*)(umem + (uint64_t)fi * 64u);
    } else {
        const uint4 dd = ((const uint4*)descs)[fi];
        len = dd.z;
        f = (uint4*)(umem + ((uint64_t)dd.y << 32 | dd.x));
    }
    uint4 v = f[q];
    asm volatile("" : "+v"(v.x));  // stored back unchanged, not elided
    const uint32_t s = v.x + v.y + v.z + v.w;
    const uint32_t s4 = s + __shfl_xor(s, 1) + __shfl_xor(s, 2);
    f[q] = v;
    if (MODE != 2 && q == 0) {
        recs[fi] = make_uint4(s4, len, 0u, 3u);
        verd[fi] = 1;
    }
}

extern "C" int c2floor_run(int mode, void* umem, const void* descs, void* verd, void* recs, uint32_t n,
                           void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    uint8_t* u = (uint8_t*)umem;
    const Desc* d = (const Desc*)descs;
    uint8_t* v = (uint8_t*)verd;
    uint4* r = (uint4*)recs;
    const uint32_t g4 = (n * 4u + 255u) / 256u, g1 = (n + 255u) / 256u;
    switch (mode) {
        case 0: c2floor<0><<<g4, 256, 0, s>>>(u, d, v, r, n); break;
        case 1: c2floor<1><<<g1, 256, 0, s>>>(u, d, v, r, n); break;
        case 2: c2floor<2><<<g4, 256, 0, s>>>(u, d, v, r, n); break;
        case 3: c2floor<3><<<g4, 256, 0, s>>>(u, d, v, r, n); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
