// xsk_classify.hip — the XDP ingress filter of the reference as a device pass over a batch:
// xdp_sock_prog() (src/kern/inner_xdp.c:26-61; phy_xdp.c:39-81 makes the same tests) decides per frame
// DROP / PASS / REDIRECT, and the REDIRECT frames are compacted in order into a descriptor list that
// feeds xsk_gpu_echo_dev() ("XDP pre-filter parity").
//
// Three launches, all HBM/latency bound (no MFMA):
//   1. classify: lane per frame — descriptor, bounds check, bytes 12-13 and 23 of the frame, action;
//      per-workgroup count of REDIRECT frames (wave ballots);
//   2. scan: one 1024-thread workgroup turns the per-workgroup counts into exclusive offsets and the
//      total;
//   3. scatter: lane per frame again — wave ballot prefix + workgroup offset -> output slot.
#include <errno.h>

#include "../../include/xsk_gpu.h"
#include "xsk_echo_kernels.h"
#include "xsk_hip_util.h"

using namespace xskgpu;

namespace {

constexpr int kCT = 256;  // frames per workgroup
constexpr uint32_t kMaxLen = XSK_GPU_MAX_LEN;

__device__ __forceinline__ uint32_t classify_one(const uint8_t* umem, uint64_t umem_size, const xsk_gpu_desc& d,
                                                 int bound) {
    const uint64_t a = d.addr;
    const uint32_t len = d.len;
    const uint32_t need = len < 34 ? (len < 14 ? 0u : 14u) : 34u;
    if (len > kMaxLen || a > umem_size || need > umem_size - a) return XSK_GPU_XDP_DROP;  // build-added
    if (len < 14) return XSK_GPU_XDP_DROP;                                               // :35-36
    // the three bytes the program reads, loaded together (one round trip; byte 23 only when the IPv4
    // header is inside the frame, so nothing past the frame is read)
    const uint8_t* p = umem + a;
    const uint32_t e0 = p[12], e1 = p[13];
    const uint32_t pr = len >= 34 ? (uint32_t)p[23] : 0u;
    if (e0 != 0x08 || e1 != 0x00) return XSK_GPU_XDP_PASS;                              // :38-39
    if (len < 34) return XSK_GPU_XDP_DROP;                                               // :41-42
    if (pr != 1) return XSK_GPU_XDP_PASS;                                                // :44-45
    return bound ? XSK_GPU_XDP_REDIRECT : XSK_GPU_XDP_DROP;                              // :57-60
}

__global__ __launch_bounds__(kCT) void classify_kernel(const uint8_t* umem, uint64_t umem_size,
                                                       const xsk_gpu_desc* descs, uint32_t n, int bound,
                                                       uint8_t* actions, uint32_t* wg_count) {
    __shared__ uint32_t s_w[kCT / 64];
    const uint32_t i = blockIdx.x * kCT + threadIdx.x;
    uint32_t act = 0;
    if (i < n) {
        act = classify_one(umem, umem_size, descs[i], bound);
        actions[i] = (uint8_t)act;
    }
    const uint64_t m = __ballot(act == XSK_GPU_XDP_REDIRECT);
    if ((threadIdx.x & 63u) == 0) s_w[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) wg_count[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// Exclusive scan of nwg counts in place (one workgroup of 1024): thread t owns a contiguous run.
__global__ __launch_bounds__(1024) void scan_kernel(uint32_t* wg_count, uint32_t nwg, uint32_t* d_total) {
    __shared__ uint32_t s[1024];
    const uint32_t per = (nwg + 1023u) / 1024u;
    const uint32_t b = threadIdx.x * per, e = min(b + per, nwg);
    uint32_t sum = 0;
    for (uint32_t j = b; j < e; ++j) sum += wg_count[j];
    s[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t o = 1; o < 1024u; o <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t v = threadIdx.x >= o ? s[threadIdx.x - o] : 0u;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = s[threadIdx.x] - sum;  // exclusive prefix of this run
    for (uint32_t j = b; j < e; ++j) {
        const uint32_t c = wg_count[j];
        wg_count[j] = run;
        run += c;
    }
    if (threadIdx.x == 1023u) *d_total = s[1023];
}

__global__ __launch_bounds__(kCT) void scatter_kernel(const xsk_gpu_desc* descs, uint32_t n, const uint8_t* actions,
                                                      const uint32_t* wg_off, xsk_gpu_desc* out) {
    __shared__ uint32_t s_w[kCT / 64];
    const uint32_t i = blockIdx.x * kCT + threadIdx.x;
    const bool r = i < n && actions[i] == XSK_GPU_XDP_REDIRECT;
    const uint64_t m = __ballot(r);
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t base = wg_off[blockIdx.x];
    for (uint32_t k = 0; k < w; ++k) base += s_w[k];
    if (r) {
        const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        out[base + below] = descs[i];
    }
}

}  // namespace

extern "C" {

size_t xsk_gpu_classify_workspace_size(uint32_t n) { return (size_t)((n + kCT - 1) / kCT + 1) * sizeof(uint32_t); }

int xsk_gpu_classify_dev(const void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                         int target_bound, uint8_t* d_actions, struct xsk_gpu_desc* d_out, uint32_t* d_nout,
                         void* d_workspace, void* stream) {
    if (n == 0) {
        if (d_nout) HIP_TRY(hipMemsetAsync(d_nout, 0, sizeof(uint32_t), (hipStream_t)stream));
        return 0;
    }
    if (!d_umem || !d_descs || !d_actions || !d_workspace || (d_out && !d_nout) || ((uintptr_t)d_descs & 15u) ||
        ((uintptr_t)d_out & 15u) || n > XSK_GPU_MAX_BATCH)
        return -EINVAL;
    const uint32_t nwg = (n + kCT - 1) / kCT;
    hipStream_t s = (hipStream_t)stream;
    uint32_t* wg = (uint32_t*)d_workspace;
    hipLaunchKernelGGL(classify_kernel, dim3(nwg), dim3(kCT), 0, s, (const uint8_t*)d_umem, umem_size, d_descs, n,
                       target_bound, d_actions, wg);
    HIP_TRY(hipGetLastError());
    if (d_out) {
        hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, s, wg, nwg, d_nout);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(scatter_kernel, dim3(nwg), dim3(kCT), 0, s, d_descs, n, (const uint8_t*)d_actions,
                           (const uint32_t*)wg, d_out);
        HIP_TRY(hipGetLastError());
    }
    return 0;
}

}  // extern "C"
