/*
 * xsk_gpu_host.c — host-UMEM drop-in for the client's RX loop (C11 + HIP runtime C API).
 *
 * The reference's RX path (src/lib/xsk_receive.c:192-237) peeks up to RX_BATCH_SIZE descriptors
 * and calls process_packet() on each frame of the UMEM (a posix_memalign'd host buffer,
 * src/lib/xsk_utils.c:132-135).  xsk_gpu_process() takes that batch of descriptors and runs the
 * whole batch through the gfx950 kernel (xsk_gpu_echo_dev), leaving the UMEM exactly as the
 * per-frame loop would have, and returns per-frame verdicts plus the stats_record counters.
 *
 *   ZEROCOPY: the UMEM is registered as mapped pinned memory; the kernel reads and rewrites frames
 *             over PCIe in place.  One launch per batch; nothing but descriptors and results moves.
 *   STAGED:   frames are copied host->device into a device mirror of the UMEM (one strided 2-D copy
 *             when the batch has a uniform frame stride, else the batch's byte span), transformed in
 *             HBM, and only the 38 rewritten header bytes of TX_REPLY frames are copied back and
 *             scattered into the UMEM — bytes the batch does not own are never written.
 */
#define _GNU_SOURCE
#define __HIP_PLATFORM_AMD__ 1
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/xsk_gpu.h"

int xsk_gpu__pack_headers_dev(const void* d_umem, const struct xsk_gpu_desc* d_descs, const uint8_t* d_verdicts,
                              uint32_t n, uint8_t* d_pack, void* stream);

struct xsk_gpu_ctx {
    int device;
    int mode;
    uint8_t* umem;
    uint64_t umem_size;
    uint32_t max_batch;
    uint8_t* d_umem; /* mapped alias of umem (ZEROCOPY) or device mirror (STAGED) */
    struct xsk_gpu_desc* d_descs;
    uint8_t* d_verdicts;
    struct xsk_gpu_rec* d_recs;
    struct xsk_gpu_stats* d_stats;
    void* d_ws;
    uint8_t* d_pack;  /* STAGED: [max_batch][48] rewritten headers */
    uint8_t* h_pack;  /* STAGED: pinned host copy of d_pack */
    uint8_t* h_verd;  /* pinned verdict staging */
    struct xsk_gpu_stats* h_stats;
    hipStream_t stream;
    int registered;
};

static int fail(hipError_t e) { return e == hipErrorOutOfMemory ? -ENOMEM : -EIO; }
#define TRY(expr)                           \
    do {                                    \
        const hipError_t e_ = (expr);       \
        if (e_ != hipSuccess) {             \
            rc = fail(e_);                  \
            goto out;                       \
        }                                   \
    } while (0)

void xsk_gpu_fini(xsk_gpu_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->mode == XSK_GPU_MODE_STAGED && c->d_umem) (void)hipFree(c->d_umem);
    if (c->registered) (void)hipHostUnregister(c->umem);
    (void)hipFree(c->d_descs);
    (void)hipFree(c->d_verdicts);
    (void)hipFree(c->d_recs);
    (void)hipFree(c->d_stats);
    (void)hipFree(c->d_ws);
    (void)hipFree(c->d_pack);
    if (c->h_pack) (void)hipHostFree(c->h_pack);
    if (c->h_verd) (void)hipHostFree(c->h_verd);
    if (c->h_stats) (void)hipHostFree(c->h_stats);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    free(c);
}

int xsk_gpu_init(xsk_gpu_ctx** out, int device, void* umem, uint64_t umem_size, uint32_t max_batch, int mode) {
    int rc = 0;
    if (!out || !umem || umem_size == 0 || ((uintptr_t)umem & 15u) || (umem_size & 15u) || max_batch == 0 ||
        (mode != XSK_GPU_MODE_ZEROCOPY && mode != XSK_GPU_MODE_STAGED))
        return -EINVAL;
    *out = NULL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -ENODEV;
    xsk_gpu_ctx* c = (xsk_gpu_ctx*)calloc(1, sizeof *c);
    if (!c) return -ENOMEM;
    c->device = device;
    c->mode = mode;
    c->umem = (uint8_t*)umem;
    c->umem_size = umem_size;
    c->max_batch = max_batch;
    TRY(hipSetDevice(device));
    TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    TRY(hipHostRegister(umem, umem_size, mode == XSK_GPU_MODE_ZEROCOPY ? hipHostRegisterMapped : hipHostRegisterDefault));
    c->registered = 1;
    if (mode == XSK_GPU_MODE_ZEROCOPY) {
        TRY(hipHostGetDevicePointer((void**)&c->d_umem, umem, 0));
    } else {
        TRY(hipMalloc((void**)&c->d_umem, umem_size));
        TRY(hipMalloc((void**)&c->d_pack, (size_t)max_batch * 48u));
        TRY(hipHostMalloc((void**)&c->h_pack, (size_t)max_batch * 48u, hipHostMallocDefault));
    }
    TRY(hipMalloc((void**)&c->d_descs, (size_t)max_batch * sizeof(struct xsk_gpu_desc)));
    TRY(hipMalloc((void**)&c->d_verdicts, max_batch));
    TRY(hipMalloc((void**)&c->d_recs, (size_t)max_batch * sizeof(struct xsk_gpu_rec)));
    TRY(hipMalloc((void**)&c->d_stats, sizeof(struct xsk_gpu_stats)));
    {
        const size_t ws = xsk_gpu_workspace_size(device, max_batch);
        if (ws == 0) {
            rc = -EIO;
            goto out;
        }
        TRY(hipMalloc(&c->d_ws, ws));
    }
    TRY(hipHostMalloc((void**)&c->h_verd, max_batch, hipHostMallocDefault));
    TRY(hipHostMalloc((void**)&c->h_stats, sizeof(struct xsk_gpu_stats), hipHostMallocDefault));
    *out = c;
    return 0;
out:
    xsk_gpu_fini(c);
    return rc;
}

/* Uniform stride S (>= 64, multiple of 16) when addr[i] = addr[0] + i*S for the whole batch. */
static uint64_t uniform_stride(const struct xsk_gpu_desc* d, uint32_t n) {
    if (n < 2) return 0;
    if (d[1].addr <= d[0].addr) return 0;
    const uint64_t s = d[1].addr - d[0].addr;
    if (s < 64 || (s & 15u)) return 0;
    for (uint32_t i = 2; i < n; i++)
        if (d[i].addr != d[0].addr + (uint64_t)i * s) return 0;
    return s;
}

static int stage_in(xsk_gpu_ctx* c, const struct xsk_gpu_desc* d, uint32_t n) {
    /* Bytes the kernel may read: [align16(addr), align16(addr)+64) u [addr, addr+len), clipped. */
    uint64_t lo = UINT64_MAX, hi = 0, width = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t a = d[i].addr;
        if (a >= c->umem_size) continue; /* BAD_DESC: the kernel reads nothing */
        const uint64_t a16 = a & ~15ull;
        uint64_t e = a + (d[i].len > 48 ? d[i].len : 48);
        if (e < a16 + 64) e = a16 + 64;
        e = (e + 15) & ~15ull;
        if (e > c->umem_size) e = c->umem_size;
        if (a16 < lo) lo = a16;
        if (e > hi) hi = e;
        if (e - a16 > width) width = e - a16;
    }
    if (hi <= lo) return 0;
    const uint64_t s = uniform_stride(d, n);
    if (s && width <= s && (d[0].addr & ~15ull) + (uint64_t)(n - 1) * s + width <= c->umem_size) {
        const uint64_t base = d[0].addr & ~15ull;
        if (hipMemcpy2DAsync(c->d_umem + base, s, c->umem + base, s, width, n, hipMemcpyHostToDevice, c->stream) !=
            hipSuccess)
            return -EIO;
        return 0;
    }
    if (hipMemcpyAsync(c->d_umem + lo, c->umem + lo, hi - lo, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return -EIO;
    return 0;
}

int xsk_gpu_process(xsk_gpu_ctx* c, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                    struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats) {
    int rc = 0;
    if (!c || (!descs && n)) return -EINVAL;
    if (n == 0) return 0;
    if (n > c->max_batch) return -EINVAL;
    TRY(hipSetDevice(c->device));
    TRY(hipMemcpyAsync(c->d_descs, descs, (size_t)n * sizeof *descs, hipMemcpyHostToDevice, c->stream));
    TRY(hipMemsetAsync(c->d_stats, 0, sizeof(struct xsk_gpu_stats), c->stream));
    if (c->mode == XSK_GPU_MODE_STAGED) {
        rc = stage_in(c, descs, n);
        if (rc) goto out;
    }
    rc = xsk_gpu_echo_dev(c->d_umem, c->umem_size, c->d_descs, n, c->d_verdicts, recs ? c->d_recs : NULL, c->d_stats,
                          c->d_ws, c->stream);
    if (rc) goto out;
    if (c->mode == XSK_GPU_MODE_STAGED) {
        rc = xsk_gpu__pack_headers_dev(c->d_umem, c->d_descs, c->d_verdicts, n, c->d_pack, c->stream);
        if (rc) goto out;
        TRY(hipMemcpyAsync(c->h_pack, c->d_pack, (size_t)n * 48u, hipMemcpyDeviceToHost, c->stream));
    }
    TRY(hipMemcpyAsync(c->h_verd, c->d_verdicts, n, hipMemcpyDeviceToHost, c->stream));
    if (recs) TRY(hipMemcpyAsync(recs, c->d_recs, (size_t)n * sizeof *recs, hipMemcpyDeviceToHost, c->stream));
    TRY(hipMemcpyAsync(c->h_stats, c->d_stats, sizeof *c->h_stats, hipMemcpyDeviceToHost, c->stream));
    TRY(hipStreamSynchronize(c->stream));
    if (c->mode == XSK_GPU_MODE_STAGED) {
        for (uint32_t i = 0; i < n; i++)
            if (c->h_verd[i] == XSK_GPU_TX_REPLY) memcpy(c->umem + descs[i].addr, c->h_pack + (size_t)i * 48u, 38);
    }
    if (verdicts) memcpy(verdicts, c->h_verd, n);
    if (stats) {
        stats->rx_packets += c->h_stats->rx_packets;
        stats->rx_bytes += c->h_stats->rx_bytes;
        stats->tx_packets += c->h_stats->tx_packets;
        stats->tx_bytes += c->h_stats->tx_bytes;
    }
out:
    return rc;
}
