// xsk_tune_slack.hip — the product round kernel with the round-4 candidate SLACK: a heavy wave enters its write phase
// once all but SLACK waves of its workgroup have read the round (SLACK < 0: only waves that streamed a ragged tile
// get the -SLACK slack).  The product header is left as shipped: the Makefile applies tools/slack_header.patch to a
// copy of it, ../xsk_echo_device_slack.gen.h (not tracked).  For in-process A/B (tools/abbench.py variants >= 2000);
// tuning library only.
#include <errno.h>

#include "../xsk_echo_device_slack.gen.h"
#include "../xsk_gpu_internal.h"
#include "../xsk_hip_util.h"

using namespace xskgpu;

extern "C" uint32_t xsk_gpu__num_cu(int device);

//   0: SLACK 0 (as shipped)   2 / 4: SLACK 2 / 4   1: SLACK 2 for ragged-tile waves only
extern "C" int xsk_gpu__slack_variant(int variant, uint32_t grid_force, void* d_umem, uint64_t umem_size,
                                      const struct xsk_gpu_desc* d_descs, uint32_t n, uint8_t* d_verdicts,
                                      struct xsk_gpu_rec* d_recs, void* d_workspace, void* stream) {
    if (n == 0) return 0;
    if (n <= XSK_GPU_LOWLAT_MAX || !d_workspace) return -EINVAL;
    int device = 0;
    HIP_TRY(hipGetDevice(&device));
    uint32_t grid = 0, per = 0;
    echo6_geometry(n, grid_force ? grid_force : xsk_gpu__num_cu(device), &grid, &per);
    EchoArgs args;
    args.umem = (uint8_t*)d_umem;
    args.umem_size = umem_size;
    args.descs = d_descs;
    args.n = n;
    args.verdicts = d_verdicts;
    args.recs = d_recs;
    args.partials = (unsigned long long*)d_workspace;
    const hipStream_t s = (hipStream_t)stream;
    const dim3 gg(grid), bb(kThreads6);
    switch (variant) {
        case 0: echo_round_kernel<false, false, kUR, true, true, 0><<<gg, bb, 0, s>>>(args, per); break;
        case 1: echo_round_kernel<false, false, kUR, true, true, -2><<<gg, bb, 0, s>>>(args, per); break;
        case 2: echo_round_kernel<false, false, kUR, true, true, 2><<<gg, bb, 0, s>>>(args, per); break;
        case 4: echo_round_kernel<false, false, kUR, true, true, 4><<<gg, bb, 0, s>>>(args, per); break;
        default: return -EINVAL;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}
