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
//   mode 11: + 128 B per frame (the whole first line), deferred to the end of the tile (LDS-staged)
//   mode 12: mode 0, then a second launch that re-reads and rewrites every frame's 64-B window
//            (two-phase: the whole read stream first, all header writes after it)
//   mode 13: the second launch of mode 12 alone (64-B window read + write, cold)
//   mode 14: mode 12 with the 64-B window loaded with the default (cacheable) policy in the first pass
//   mode 15: phase-separated rounds: a persistent grid (one 1024-thread workgroup per CU) reads 2048
//            frames per workgroup per round, holding their 64-B windows in LDS (128 KiB), then all
//            workgroups write their windows back at once; the read stream never meets a write
//   mode 16: mode 15 without the write phase (the structure's read rate)
//   mode 17: mode 15 with tiles interleaved across workgroups (step s of every workgroup reads one
//            compact front of consecutive frames), mode 18: mode 17 without the write phase
//   mode 19/20: mode 15/16 with two steps (8 frames, 12 loads per lane) in flight per wave
//   mode 21/22: mode 15/16 with 1024-frame rounds (64 KiB LDS, two workgroups per CU: grid 512)
//   mode 23/24: mode 21/22 with two steps in flight
//   mode 25 / 26: write only, 48 / 32 B per frame (3 / 2 lanes x 16 B), no payload reads
//   mode 30-35: read-only persistent layouts (grid = workgroups of 1024 threads, each a contiguous share
//            of the frames): 30 = waves share a 64-frame chunk per step (= mode 16), 31 = every wave
//            streams its own 64-frame tile (row q of step s: frame 4s+q), 32 = 31 with each workgroup
//            starting at a rotated tile of its share, 33 = 30 rotated, 34 = 31 with 512-thread
//            workgroups (grid 2x), 35 = 31 with 8 loads per lane in flight (two frames per row)
//   mode 36: 31 with 256-thread workgroups (grid = workgroups); 37: 31 in the wave-front order (pass p: tiles
//            [p * 16 * grid, ...), wave w of workgroup g tile 16 g + w); 38: 36 in the wave-front order
//   mode 40-47: the read ladder (wexp_ladder): 40 <4 waves, front, 6 loads>, 41 <16, front, 6>, 42 <16,
//            contiguous, 6>, 43 <16, contiguous, 4+2>, 44 <16, contiguous, 12 pipelined>, 45 <16, front, 12>,
//            46 <4, contiguous, 6>, 47 <16, front, 4+2>
//   mode 50-53: two-phase (12) with Infinity-Cache policies for the window line in the first pass: 50 the
//            first 128-B line default-policy, the rest nt; 51 everything default; 52 = 50 via raw buffer
//            loads; 53 = 50's first pass alone
//   mode 60-64: ladder with 8 waves (512-thread workgroups): 60 <8, contiguous, 12 pipelined>, 61 <8, contiguous,
//            6>; and with every window written once at the END of the workgroup's share (ENDW): 62 <16,
//            contiguous, 4+2>, 63 <8, contiguous, 12>, 64 <16, contiguous, 12>; 65: 62 with the windows of
//            every 2 tiles of a wave written after them (2 write phases per share, no sync); 66: 65 with a
//            workgroup barrier before each write phase
//   mode 68 / 69: 65 with a grid barrier before / before and after the mid-share write phase
//   mode 67: 62 with every wave's second tile's windows written mid-share (a quarter), the rest at the end
//   mode 74 (REREAD): 62's single end phase, the first half share's windows read again (64 B per frame) right before
//            they are stored in it -- the kernel form would keep only sums and verdicts of round 0 and redo its rewrite
//   mode 70-73 (DEFER): 62's single end phase with the first half share's windows parked in a contiguous side buffer
//            between (70 default stores, 71 nontemporal, 72 write-through, 73 = 70 without the end barrier)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

template <int MODE>
__global__ __launch_bounds__(256) void wexp_kernel(uint8_t* buf, uint32_t n, uint32_t stride, uint32_t len,
                                                   unsigned long long* out, uint8_t* side) {
    __shared__ __attribute__((aligned(16))) uint8_t s_row[4][64 * 64];
    __shared__ __attribute__((aligned(16))) uint8_t s_row2[MODE == 11 ? 4 : 1][MODE == 11 ? 64 * 128 : 16];
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
            } else if (MODE != 5 && MODE != 25 && MODE != 26) {
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    const uint32_t ro = 256u * u + 16u * k;
                    v[u] = u32x4{0, 0, 0, 0};
                    if (ro < len) {
                        if (MODE == 6 || MODE == 51 || (MODE == 14 && u == 0 && k < 4) || (MODE == 50 && u == 0 && k < 8))
                            v[u] = *(const u32x4*)(fr + ro);
                        else if (MODE == 52 && u == 0 && k < 8)
                            v[u] = __builtin_amdgcn_raw_buffer_load_b128(
                                __builtin_amdgcn_make_buffer_rsrc((void*)fr, (short)0, 256, 0x00020000), (int)ro, 0, 0);
                        else v[u] = __builtin_nontemporal_load((const u32x4*)(fr + ro));
                    }
                }
#pragma unroll
                for (int u = 0; u < 6; ++u) acc += (uint64_t)v[u].x + v[u].y + v[u].z + v[u].w;
            } else {
                v[0] = *(const u32x4*)(buf + 16u * k);  // same bytes for every frame: L2 hits
            }
            if ((MODE == 1 || MODE == 5 || MODE == 6) && k < 4) *(u32x4*)(fr + 16u * k) = v[0];
            if (MODE == 25 && k < 3) *(u32x4*)(fr + 16u * k) = v[0];
            if (MODE == 26 && k < 2) *(u32x4*)(fr + 16u * k) = v[0];
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
            if (MODE == 11 && k < 8) *(u32x4*)(&s_row2[wave][(4 * s + q) * 128 + 16 * k]) = v[0];
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
        if (MODE == 11) {
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const uint32_t f = t * 64 + r * 8 + (lane >> 3);
                if (f < n) {
                    u32x4* dst = (u32x4*)(buf + (uint64_t)f * stride + 16u * (lane & 7u));
                    *dst = *(const u32x4*)(&s_row2[wave][(r * 8 + (lane >> 3)) * 128 + 16 * (lane & 7u)]);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (acc == 0x123456789ull) out[0] = acc;  // keeps the loads alive
}

// Second pass of modes 12-14: 4 lanes per frame re-read the 64-B window and store it back.
__global__ __launch_bounds__(256) void wexp_patch(uint8_t* buf, uint32_t n, uint32_t stride) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const uint32_t f = i >> 2, k = i & 3u;
    if (f >= n) return;
    u32x4* p = (u32x4*)(buf + (uint64_t)f * stride + 16u * k);
    u32x4 v = *p;
    v.x ^= 0u;
    asm volatile("" : "+v"(v));
    *p = v;
}

// Modes 15/16.  grid = workgroups (normally one per CU), 1024 threads each, 2048 frames per round.
template <bool WRITE, bool IL, uint32_t R = 2048, int ST = 1>
__global__ __launch_bounds__(1024) void wexp_rounds(uint8_t* buf, uint32_t n, uint32_t stride, uint32_t len,
                                                    unsigned long long* out) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[R * 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t q = lane >> 4, k = lane & 15u;
    const uint32_t per = IL ? R : (n + gridDim.x - 1) / gridDim.x;
    const uint32_t G = gridDim.x;
    const uint32_t nrounds = IL ? (n + G * R - 1) / (G * R) : 1u;
    uint64_t acc = 0;
    const uint64_t t_start = wall_clock64();
    for (uint32_t rr = 0; rr < nrounds; ++rr)
    for (uint32_t r0 = IL ? 0u : blockIdx.x * per, f0 = r0, f1 = IL ? R : min(n, f0 + per); r0 < f1; r0 += R) {
        // frame of local index j (0..R-1) in this round
        auto gf = [&](uint32_t j) -> uint32_t {
            return IL ? (rr * G * (R / 64) + (j >> 6) * G + blockIdx.x) * 64u + (j & 63u) : r0 + j;
        };
        // read phase: wave w takes frames r0 + 4*(w + 16*s) + q
        for (uint32_t s0 = 0; s0 < R / 64; s0 += ST) {
            u32x4 v[ST][6];
#pragma unroll
            for (int t = 0; t < ST; ++t) {
                const uint32_t j = 4u * (wave + 16u * (s0 + t)) + q;
                const uint32_t f = gf(j);
                const bool live = IL ? f < n : f < f1;
                const uint8_t* fr = buf + (uint64_t)(live ? f : 0u) * stride;
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    const uint32_t ro = 256u * u + 16u * k;
                    v[t][u] = (live && ro < len) ? __builtin_nontemporal_load((const u32x4*)(fr + ro)) : u32x4{0, 0, 0, 0};
                }
            }
#pragma unroll
            for (int t = 0; t < ST; ++t) {
                const uint32_t j = 4u * (wave + 16u * (s0 + t)) + q;
#pragma unroll
                for (int u = 0; u < 6; ++u) acc += (uint64_t)v[t][u].x + v[t][u].y + v[t][u].z + v[t][u].w;
                if (WRITE && k < 4) *(u32x4*)(&s_win[j * 64 + 16 * k]) = v[t][0];
            }
        }
        if (WRITE) {
            __syncthreads();
#pragma unroll
            for (int r = 0; r < (int)(R * 4 / 1024); ++r) {
                const uint32_t idx = (uint32_t)r * 1024u + threadIdx.x;  // 16-B piece
                const uint32_t j = idx >> 2, kk = idx & 3u;
                const uint32_t f = gf(j);
                if (IL ? f < n : f < f1) *(u32x4*)(buf + (uint64_t)f * stride + 16u * kk) = *(const u32x4*)(&s_win[j * 64 + 16 * kk]);
            }
            __syncthreads();
        }
    }
    if (acc == 0x123456789ull) out[0] = acc;
    __syncthreads();
    if (threadIdx.x == 0 && gridDim.x <= 2048) {
        out[8 + 2 * blockIdx.x] = t_start;
        out[9 + 2 * blockIdx.x] = wall_clock64();
    }
}

template <int PAT, bool ROT, int NW, bool FRONT = false>
__global__ __launch_bounds__(NW * 64) void wexp_pers(const uint8_t* buf, uint32_t n, uint32_t stride, uint32_t len,
                                                     unsigned long long* out) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t q = lane >> 4, k = lane & 15u;
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t per = (ntiles + gridDim.x - 1) / gridDim.x;  // tiles per workgroup
    const uint32_t t0 = blockIdx.x * per;
    const uint32_t rot = ROT ? (blockIdx.x * 37u) % per : 0u;
    uint64_t acc = 0;
    if (PAT == 0) {  // waves share chunk c: wave w takes frames 4w+q of it
        for (uint32_t c = 0; c < per; ++c) {
            const uint32_t t = t0 + (c + rot) % per;
            if (t >= ntiles) continue;
            const uint32_t f = t * 64 + 4 * wave + q;
            if (f >= n) continue;
            const uint8_t* fr = buf + (uint64_t)f * stride;
            u32x4 v[6];
#pragma unroll
            for (int u = 0; u < 6; ++u) {
                const uint32_t ro = 256u * u + 16u * k;
                v[u] = ro < len ? __builtin_nontemporal_load((const u32x4*)(fr + ro)) : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < 6; ++u) acc += (uint64_t)v[u].x + v[u].y + v[u].z + v[u].w;
        }
    } else {  // every wave its own tile
        for (uint32_t c = wave; c < per; c += NW) {
            // FRONT: the grid's waves sweep the batch in passes of (grid * NW) consecutive tiles
            const uint32_t t = FRONT ? (c / NW) * gridDim.x * NW + blockIdx.x * NW + wave : t0 + (c + rot) % per;
            if (t >= ntiles) continue;
            for (uint32_t s = 0; s < 16; s += (PAT == 2 ? 2 : 1)) {
                constexpr int NF = PAT == 2 ? 2 : 1;
                u32x4 v[NF][6];
#pragma unroll
                for (int h = 0; h < NF; ++h) {
                    const uint32_t f = t * 64 + 4 * (s + h) + q;
                    const uint8_t* fr = buf + (uint64_t)(f < n ? f : 0u) * stride;
#pragma unroll
                    for (int u = 0; u < 6; ++u) {
                        const uint32_t ro = 256u * u + 16u * k;
                        v[h][u] = (f < n && ro < len) ? __builtin_nontemporal_load((const u32x4*)(fr + ro)) : u32x4{0, 0, 0, 0};
                    }
                }
#pragma unroll
                for (int h = 0; h < NF; ++h)
#pragma unroll
                    for (int u = 0; u < 6; ++u) acc += (uint64_t)v[h][u].x + v[h][u].y + v[h][u].z + v[h][u].w;
            }
        }
    }
    if (acc == 0x123456789ull) out[0] = acc;
}

// Read ladder (modes 40-46): a clean read-only kernel between wexp_kernel<0> and the round kernel's read
// pattern.  Frames of a tile are read through a tile-wide raw buffer (out-of-range offsets -> zeros, no
// branches), 16 lanes per frame (row q of step s: frame 4s+q), 256-B row-loads.  NW waves per workgroup;
// FRONT: the grid's waves sweep the batch in passes of grid * NW tiles, else contiguous per-workgroup
// shares; LM 0: a step's 6 row-loads in one batch, 1: batches of 4 + 2 (the shipped U = 4), 2: step
// s + 1's 6 loads issued before step s is summed (12 in flight).
// Grid-wide barrier of a persistent grid (every workgroup resident: one per CU) on a counter that is never reset:
// each use adds gridDim.x arrivals, so the target is the next multiple of gridDim.x.  Stores before it are waited for.
__device__ __forceinline__ void grid_barrier(unsigned long long* ctr) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long old = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long target = (old / gridDim.x + 1ull) * gridDim.x;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(2);
    }
    __syncthreads();
}

template <int NW, bool FRONT, int LM, int ENDW = 0>
__global__ __launch_bounds__(NW * 64) void wexp_ladder(uint8_t* buf, uint32_t n, uint32_t stride, uint32_t len,
                                                       unsigned long long* out, uint8_t* side = nullptr) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t q = lane >> 4, k = lane & 15u;
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    uint64_t acc = 0;
    for (uint32_t c = wave; c < per; c += NW) {
        // ENDW 4-7 (DEFER): the windows of the share's first half ("round 0", c < 2 NW) go to a contiguous side
        // buffer right after the tile (4 KiB per tile, coalesced); every window is scattered in one end phase
        if (ENDW >= 4 && ENDW <= 7 && c >= 2u * NW && c < 4u * NW) {
            const uint32_t tp = blockIdx.x * per + c - 2u * NW;  // the round-0 tile this wave read two tiles ago
            const u32x4 w = u32x4{(uint32_t)acc, (uint32_t)(acc >> 32), lane, wave};
            if (tp < ntiles) {
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    u32x4* dst = (u32x4*)(side + (uint64_t)tp * 4096u + (uint32_t)rr * 1024u + lane * 16u);
                    if (ENDW == 5) __builtin_nontemporal_store(w, dst);
                    else if (ENDW == 6) __builtin_amdgcn_raw_buffer_store_b128(w, __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, 16, 0x00020000), 0, 0, 16);
                    else *dst = w;
                }
            }
        }
        const uint32_t t = FRONT ? (c / NW) * gridDim.x * NW + blockIdx.x * NW + wave : blockIdx.x * per + c;
        if (ENDW == 8 && c >= 3u * NW && c < 4u * NW) {  // ENDW 8: only tile 1 of the wave written mid-share
            const u32x4 w = u32x4{(uint32_t)acc, (uint32_t)(acc >> 32), lane, wave};
            const uint32_t tt = blockIdx.x * per + c - 2u * NW;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const uint32_t f = tt * 64u + (uint32_t)rr * 16u + (lane >> 2);
                if (tt < ntiles && f < n) *(u32x4*)(buf + (uint64_t)f * stride + 16u * (lane & 3u)) = w;
            }
        }
        if ((ENDW == 2 || ENDW == 3 || ENDW == 9 || ENDW == 10) && c >= 2u * NW && ((c / NW) & 1u) == 0u) {  // a write phase after every 2 tiles
            if (ENDW == 3) __syncthreads();
            if (ENDW >= 9) grid_barrier(out + 1);  // 9 / 10: every workgroup has read its first half before any writes
            const u32x4 w = u32x4{(uint32_t)acc, (uint32_t)(acc >> 32), lane, wave};
            for (uint32_t cc = c - 2u * NW; cc < c; cc += NW) {
                const uint32_t tt = blockIdx.x * per + cc;
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const uint32_t f = tt * 64u + (uint32_t)rr * 16u + (lane >> 2);
                    if (tt < ntiles && f < n) *(u32x4*)(buf + (uint64_t)f * stride + 16u * (lane & 3u)) = w;
                }
            }
            if (ENDW == 10) grid_barrier(out + 1);  // ... and no workgroup reads again before every write phase is done
        }
        if (t >= ntiles) continue;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(buf + (uint64_t)t * 64u * stride),
                                                                           (short)0, (int)(64u * stride), 0x00020000);
        auto ld = [&](uint32_t s, uint32_t u) -> u32x4 {
            const uint32_t ro = 256u * u + 16u * k;
            const uint32_t o = (4u * s + q) * stride + ro;
            return __builtin_amdgcn_raw_buffer_load_b128(r, (int)(ro < len ? o : 0x80000000u), 0, 2);
        };
        if (LM == 2) {
            u32x4 a[6], b[6];
#pragma unroll
            for (int u = 0; u < 6; ++u) a[u] = ld(0, u);
            for (uint32_t s = 0; s < 16; s += 2) {
#pragma unroll
                for (int u = 0; u < 6; ++u) b[u] = ld(s + 1, u);
#pragma unroll
                for (int u = 0; u < 6; ++u) acc += (uint64_t)a[u].x + a[u].y + a[u].z + a[u].w;
                if (s + 2 < 16) {
#pragma unroll
                    for (int u = 0; u < 6; ++u) a[u] = ld(s + 2, u);
                }
#pragma unroll
                for (int u = 0; u < 6; ++u) acc += (uint64_t)b[u].x + b[u].y + b[u].z + b[u].w;
            }
        } else {
            for (uint32_t s = 0; s < 16; ++s) {
                u32x4 v[6];
                if (LM == 0) {
#pragma unroll
                    for (int u = 0; u < 6; ++u) v[u] = ld(s, u);
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) v[u] = ld(s, u);
#pragma unroll
                    for (int u = 0; u < 4; ++u) acc += (uint64_t)v[u].x + v[u].y + v[u].z + v[u].w;
                    v[0] = ld(s, 4);
                    v[1] = ld(s, 5);
                    v[2] = v[3] = v[4] = v[5] = u32x4{0, 0, 0, 0};
                }
#pragma unroll
                for (int u = 0; u < 6; ++u) acc += (uint64_t)v[u].x + v[u].y + v[u].z + v[u].w;
            }
        }
    }
    if (ENDW) {  // every frame's 64-B window written once, after the workgroup has read its whole share
        if (ENDW != 2 && ENDW != 7) __syncthreads();
        const u32x4 w = u32x4{(uint32_t)acc, (uint32_t)(acc >> 32), lane, wave};
        for (uint32_t c = (ENDW == 2 || ENDW == 3 || ENDW == 9 || ENDW == 10) ? wave + ((per - wave + NW - 1) / NW - 1) / 2 * 2 * NW : wave; c < per;
             c += NW) {
            const uint32_t t = FRONT ? (c / NW) * gridDim.x * NW + blockIdx.x * NW + wave : blockIdx.x * per + c;
            if (t >= ntiles) continue;
            if (ENDW == 8 && c >= NW && c < 2u * NW) continue;  // tile 1: written mid-share
            u32x4 ws[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                ws[r] = w;
                if (ENDW >= 4 && ENDW <= 7 && c < 2u * NW) ws[r] = *(const u32x4*)(side + (uint64_t)t * 4096u + (uint32_t)r * 1024u + lane * 16u);
                if (ENDW == 11 && c < 2u * NW) {  // REREAD: the first half share's windows read again before they go out
                    const uint32_t f = t * 64u + (uint32_t)r * 16u + (lane >> 2);
                    if (f < n) ws[r] = *(const u32x4*)(buf + (uint64_t)f * stride + 16u * (lane & 3u));
                    ws[r].x ^= w.x;
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t f = t * 64u + (uint32_t)r * 16u + (lane >> 2);
                if (f < n) *(u32x4*)(buf + (uint64_t)f * stride + 16u * (lane & 3u)) = ws[r];
            }
        }
    }
    if (acc == 0x123456789ull) out[0] = acc;
}

extern "C" int wexp_run(int mode, void* buf, uint32_t n, uint32_t stride, uint32_t len, void* out, uint32_t grid,
                        void* stream, void* side_) {
    uint8_t* side = (uint8_t*)side_;
    if (!side && (mode == 8 || (mode >= 70 && mode <= 73))) return -1;  // modes that write or read the side buffer
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
        case 11: wexp_kernel<11><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 25: wexp_kernel<25><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 26: wexp_kernel<26><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;
        case 12: wexp_kernel<0><<<g, b, 0, s>>>(p, n, stride, len, o, side);
                 wexp_patch<<<(n * 4 + 255) / 256, 256, 0, s>>>(p, n, stride); break;
        case 15: wexp_rounds<true, false><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 16: wexp_rounds<false, false><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 17: wexp_rounds<true, true><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 18: wexp_rounds<false, true><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 19: wexp_rounds<true, false, 2048, 2><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 20: wexp_rounds<false, false, 2048, 2><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 21: wexp_rounds<true, false, 1024, 1><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 22: wexp_rounds<false, false, 1024, 1><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 23: wexp_rounds<true, false, 1024, 2><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 24: wexp_rounds<false, false, 1024, 2><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 30: wexp_pers<0, false, 16><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 31: wexp_pers<1, false, 16><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 32: wexp_pers<1, true, 16><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 33: wexp_pers<0, true, 16><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 34: wexp_pers<1, false, 8><<<2 * grid, 512, 0, s>>>(p, n, stride, len, o); break;
        case 35: wexp_pers<2, false, 16><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        // 36: 31 with 256-thread workgroups (grid = workgroups); 37: 31 in the wave-front order; 38: 36 + front
        case 36: wexp_pers<1, false, 4><<<g, 256, 0, s>>>(p, n, stride, len, o); break;
        case 37: wexp_pers<1, false, 16, true><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 38: wexp_pers<1, false, 4, true><<<g, 256, 0, s>>>(p, n, stride, len, o); break;
        case 40: wexp_ladder<4, true, 0><<<g, 256, 0, s>>>(p, n, stride, len, o); break;
        case 41: wexp_ladder<16, true, 0><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 42: wexp_ladder<16, false, 0><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 43: wexp_ladder<16, false, 1><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 44: wexp_ladder<16, false, 2><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 45: wexp_ladder<16, true, 2><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 46: wexp_ladder<4, false, 0><<<g, 256, 0, s>>>(p, n, stride, len, o); break;
        case 47: wexp_ladder<16, true, 1><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 60: wexp_ladder<8, false, 2><<<g, 512, 0, s>>>(p, n, stride, len, o); break;
        case 61: wexp_ladder<8, false, 0><<<g, 512, 0, s>>>(p, n, stride, len, o); break;
        case 62: wexp_ladder<16, false, 1, 1><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 63: wexp_ladder<8, false, 2, 1><<<g, 512, 0, s>>>(p, n, stride, len, o); break;
        case 64: wexp_ladder<16, false, 2, 1><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 65: wexp_ladder<16, false, 1, 2><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 66: wexp_ladder<16, false, 1, 3><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        // 70-73 (DEFER): 62's single end phase, the first half share's windows parked in a contiguous side buffer
        // between (70 default stores, 71 nontemporal, 72 sc1 write-through, 73 = 70 without the end barrier)
        // 68 / 69: 65 with a grid barrier before (68) / before and after (69) the mid-share write phase (the grid must be
        // resident at once: at most one 1024-lane workgroup per CU)
        case 68: if (grid > 256) return -1; wexp_ladder<16, false, 1, 9><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 69: if (grid > 256) return -1; wexp_ladder<16, false, 1, 10><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        // 67: 62 with a quarter of the windows (every wave's second tile) written mid-share, the rest at the end
        case 67: wexp_ladder<16, false, 1, 8><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 70: wexp_ladder<16, false, 1, 4><<<g, 1024, 0, s>>>(p, n, stride, len, o, side); break;
        case 71: wexp_ladder<16, false, 1, 5><<<g, 1024, 0, s>>>(p, n, stride, len, o, side); break;
        case 72: wexp_ladder<16, false, 1, 6><<<g, 1024, 0, s>>>(p, n, stride, len, o, side); break;
        case 73: wexp_ladder<16, false, 1, 7><<<g, 1024, 0, s>>>(p, n, stride, len, o, side); break;
        case 74: wexp_ladder<16, false, 1, 11><<<g, 1024, 0, s>>>(p, n, stride, len, o); break;
        case 13: wexp_patch<<<(n * 4 + 255) / 256, 256, 0, s>>>(p, n, stride); break;
        case 14: wexp_kernel<14><<<g, b, 0, s>>>(p, n, stride, len, o, side);
                 wexp_patch<<<(n * 4 + 255) / 256, 256, 0, s>>>(p, n, stride); break;
        // 50-52: two-phase (12) with the first pass loading each frame's first 128-B line with the default
        // policy (50; 52: a raw buffer load, aux 0) and the rest nontemporal, or everything default (51):
        // can the windows stay in the Infinity Cache for the second pass?
        case 50: wexp_kernel<50><<<g, b, 0, s>>>(p, n, stride, len, o, side);
                 wexp_patch<<<(n * 4 + 255) / 256, 256, 0, s>>>(p, n, stride); break;
        case 51: wexp_kernel<51><<<g, b, 0, s>>>(p, n, stride, len, o, side);
                 wexp_patch<<<(n * 4 + 255) / 256, 256, 0, s>>>(p, n, stride); break;
        case 52: wexp_kernel<52><<<g, b, 0, s>>>(p, n, stride, len, o, side);
                 wexp_patch<<<(n * 4 + 255) / 256, 256, 0, s>>>(p, n, stride); break;
        case 53: wexp_kernel<50><<<g, b, 0, s>>>(p, n, stride, len, o, side); break;  // 50's first pass alone
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
