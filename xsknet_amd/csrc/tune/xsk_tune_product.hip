// xsk_tune_product.hip — the PRODUCT round kernel (../xsk_echo_device.h, the same source libxsknet_amd.so
// compiles) at alternative values of its remaining template switches, for in-process A/B against the shipped
// instance (tools/abbench.py variants >= 1000, bench.py --variant).  Tuning library only.
//   0  as shipped (reference mode)            2  wire mode as shipped (every option)
// (round 3 also measured RMETA -- ranked streams reading their step's metadata rows in rank order, one LDS read
// per step instead of two dependent ones: c4 195.5 vs 187.2 us, profiles/r03/ab_rank_ordered_meta_*.log -- and
// ROLL, the tiles of a round in a rolled loop so the kernel's code shrinks from 78 to 46 KB: c4 185.9 vs 185.9 us,
// c3 275.8 vs 276.0, profiles/r03/ab_rolled_tile_loop_*.log; neither shipped.  New candidates get the free slots.)
// (round 3 measured RAGGED 2 here -- ragged tiles with their ICMP masks computed once per frame -- against the
// shipped ranked streams: c4 193.0 vs 185.7 us, profiles/r03/ab_ragged_masks_once_*.log; not shipped)
#include <errno.h>

#include "../xsk_echo_device.h"
#include "../xsk_gpu_internal.h"
#include "../xsk_hip_util.h"

using namespace xskgpu;

extern "C" uint32_t xsk_gpu__num_cu(int device);

extern "C" int xsk_gpu__product_variant(int variant, uint32_t grid_force, void* d_umem, uint64_t umem_size,
                                        const struct xsk_gpu_desc* d_descs, uint32_t n, uint8_t* d_verdicts,
                                        struct xsk_gpu_rec* d_recs, void* d_workspace, void* stream) {
    if (n == 0) return 0;
    if (n <= XSK_GPU_LOWLAT_MAX || !d_workspace) return -EINVAL;  // large batches: the round kernel's geometry
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
    args.partials = (unsigned long long*)d_workspace;  // counters as per-workgroup partial rows
    const hipStream_t s = (hipStream_t)stream;
    const dim3 gg(grid), bb(kThreads6);
    switch (variant) {
        case 0: echo_round_kernel<false, false><<<gg, bb, 0, s>>>(args, per); break;
        case 2: args.opts = XSK_GPU_OPT_ALL; echo_round_kernel<true, false><<<gg, bb, 0, s>>>(args, per); break;
        default: return -EINVAL;
    }
    HIP_TRY(hipGetLastError());
    return 0;
}
