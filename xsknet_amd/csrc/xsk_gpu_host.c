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
 *             over PCIe in place, reads the descriptors from a mapped pinned staging buffer and writes
 *             verdicts and counters straight into mapped pinned host memory: a batch is one kernel
 *             launch (two when it spans more than one workgroup) and one synchronisation, no copies.
 *   LOWLAT:   ZEROCOPY, but batches of <= XSK_GPU_LOWLAT_MAX frames go to a resident polling kernel
 *             through a doorbell in mapped host memory (xsk_lowlat.hip): no launch, no synchronisation.
 *   STAGED:   the bytes the transform reads are copied host->device into a device mirror of the UMEM (one
 *             strided 2-D DMA copy when the chunk has a uniform frame stride, one copy of the chunk's span when its
 *             frames cover it densely, else -- AF_XDP's recycled, scattered descriptors -- a gather kernel that
 *             moves each frame's own bytes across PCIe, or, on a device without a mapped alias of the UMEM, a host
 *             pack of those bytes into pinned staging; xsk_stage_plan.h decides), transformed in HBM, and only the
 *             38 rewritten header bytes of TX_REPLY frames are copied back and scattered into the UMEM — bytes the
 *             batch does not own are never written.  Batches of more than one chunk run as a two-stream pipeline: a
 *             copy stream takes every chunk's copy-in back to back and a compute stream each chunk's transform,
 *             header pack and copy-back once its copy-in has landed; a copy-in that may write mirror bytes of an
 *             earlier chunk's frames (xsk_stage_plan.h, `contained`) first waits for the previous chunk's pack.  The
 *             last chunks halve in size, and the host scatters chunk i while later chunks are still in flight.
 */
#define _GNU_SOURCE
#define __HIP_PLATFORM_AMD__ 1
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#include "xsk_gpu_internal.h"
#include "xsk_stage_plan.h"

#define NSTREAMS 2
#define CHUNK_FRAMES 32768u /* staged pipeline granule: ~49 MB of 1500-B frames per copy-in */
#define TAIL_FRAMES 4096u   /* staged: the last chunks halve down to this, so the work left after the last copy-in
                             * (transform, pack, copy-back, host scatter of one chunk) is short */
#define PACK 96u            /* staged: bytes per frame of the packed rewritten headers (wire mode <= 86) */
#define STAGE_HALF (32u << 20) /* staged without a mapped alias: default bytes per half of the host-pack staging */

struct xsk_gpu_ctx {
    int device;
    int mode;
    uint32_t opts;  /* XSK_GPU_OPT_* for xsk_gpu_echo_dev_opts() */
    uint8_t* umem;
    uint64_t umem_size;
    uint32_t max_batch;
    uint32_t max_chunks;
    uint8_t* d_umem; /* mapped alias of umem (ZEROCOPY) or device mirror (STAGED) */
    struct xsk_gpu_desc* d_descs;
    uint8_t* d_verdicts;
    struct xsk_gpu_rec* d_recs;
    struct xsk_gpu_stats* d_stats; /* [max_chunks] */
    void* d_ws[NSTREAMS];
    size_t ws_size; /* bytes of each d_ws */
    uint8_t* d_pack;  /* STAGED: [max_batch][PACK] rewritten headers */
    uint8_t* h_pack;  /* STAGED: pinned host copy of d_pack */
    uint8_t* h_verd;  /* pinned (mapped) verdict staging */
    struct xsk_gpu_stats* h_stats; /* [max_chunks], pinned (mapped) */
    struct xsk_gpu_desc* h_descs;  /* ZEROCOPY: pinned (mapped) descriptor staging; STAGED: pinned descriptor staging
                                    * (the copy stream's descriptor copies are then true DMA copies, not the runtime's
                                    * synchronous pageable path) */
    struct xsk_gpu_desc* m_descs;  /* ZEROCOPY: device aliases of h_descs / h_verd / h_stats */
    uint8_t* m_verd;
    struct xsk_gpu_stats* m_stats;
    uint8_t* m_umem;  /* STAGED: the mapped alias of umem (the gather kernel's source) */
    hipStream_t stream[NSTREAMS];
    hipEvent_t* done; /* [max_chunks]: chunk's results are in host memory */
    hipEvent_t* packed; /* STAGED [max_chunks]: chunk's rewritten headers are packed (its mirror bytes are free) */
    hipEvent_t* in_done; /* STAGED [max_chunks]: chunk's copy-in has landed in the mirror */
    uint64_t staged[XSK_GPU__STAGED_STATS]; /* STAGED: the copy-in record (xsk_gpu__staged_stats) */
    uint8_t* h_stage;   /* STAGED without an alias: pinned host staging, two halves of STAGE_HALF (allocated on first use) */
    uint8_t* d_stage;   /* its device copy */
    hipEvent_t stage_ev[2]; /* the DMA copy that last read each host half ... */
    int stage_rec[2];       /* ... once one has */
    int stage_half;     /* the half the next host pack fills */
    uint64_t stage_bytes; /* bytes per half (STAGE_HALF; xsk_gpu__staged_noalias sets others for tests) */
    void* reg_base;   /* the registration this context holds a reference of (xsk_gpu__umem_ref), or NULL */
    xsk_gpu__lowlat* ll; /* LOWLAT: the doorbell channel */
    int ll_slot;         /* holds one of the device's XSK_GPU_LOWLAT_PER_DEVICE LOWLAT slots */
    uint64_t ll_outcome[4]; /* LOWLAT doorbell batches that missed their timeout: all, completed through the launch path
                             * after a partial service, returned -ETIMEDOUT, completed late (every slice served,
                             * found after STOP) -- xsk_gpu__lowlat_outcomes */
    /* the batch xsk_gpu__submit put in flight and xsk_gpu__complete has not taken back yet */
    uint32_t pend_n;      /* its frames; 0: none */
    int pend_bell;        /* on the doorbell (else launched) */
    uint32_t pend_w;      /* doorbell: its serving workgroups */
    uint32_t pend_chunks; /* launched: its chunks */
    int pend_recs;        /* records asked for */
    /* the last failed submit / complete: 1 when every frame of its batch is known untouched (it may be submitted
     * again), 0 when some may have been transformed (xsk_gpu__failed_untouched) */
    int fail_untouched;
};

/* LOWLAT contexts per device in this process (include/xsk_gpu.h, XSK_GPU_LOWLAT_PER_DEVICE): a slot is taken at
 * init and given back at fini; a LOWLAT request without a free slot runs as ZEROCOPY.  The cap is the runtime's
 * highest-priority hardware queues -- min(XSK_GPU_LOWLAT_PER_DEVICE, GPU_MAX_HW_QUEUES), read once -- less the queues
 * the application reserved for its own highest-priority streams (xsk_gpu_lowlat_reserve). */
#define LL_MAX_DEV 64
static atomic_int g_ll_slots[LL_MAX_DEV];
static atomic_int g_ll_reserved[LL_MAX_DEV];
static atomic_int g_hw_queues; /* 0: not read yet */

static int hw_queues(void) {
    int q = atomic_load(&g_hw_queues);
    if (q > 0) return q;
    /* the HIP runtime's own variable (its hardware queues per process and priority; HIP's default is 4): not a
     * switch of this library */
    const char* e = getenv("GPU_MAX_HW_QUEUES");
    q = 4; /* unset: the runtime's default */
    if (e && *e) {
        char* end = NULL;
        const long v = strtol(e, &end, 10);
        if (end != e && v >= 1) q = v < XSK_GPU_LOWLAT_PER_DEVICE ? (int)v : XSK_GPU_LOWLAT_PER_DEVICE;
    }
    atomic_store(&g_hw_queues, q);
    return q;
}

static int ll_cap(int device) {
    const int cap = hw_queues() - atomic_load(&g_ll_reserved[device]);
    return cap > 0 ? cap : 0;
}

static int ll_slot_take(int device) {
    if (device < 0 || device >= LL_MAX_DEV) return 0;
    const int cap = ll_cap(device);
    int cur = atomic_load(&g_ll_slots[device]);
    while (cur < cap)
        if (atomic_compare_exchange_weak(&g_ll_slots[device], &cur, cur + 1)) return 1;
    return 0;
}

int xsk_gpu_lowlat_reserve(int device, uint32_t queues) {
    if (device < 0 || device >= LL_MAX_DEV || queues > XSK_GPU_LOWLAT_PER_DEVICE) return -EINVAL;
    atomic_store(&g_ll_reserved[device], (int)queues);
    return ll_cap(device);
}
int xsk_gpu_lowlat_cap(int device) {
    if (device < 0 || device >= LL_MAX_DEV) return -EINVAL;
    return ll_cap(device);
}
static void ll_slot_give(int device) {
    if (device >= 0 && device < LL_MAX_DEV) atomic_fetch_sub(&g_ll_slots[device], 1);
}

int xsk_gpu__ll_busy(int device) {
    return device >= 0 && device < LL_MAX_DEV && atomic_load(&g_ll_slots[device]) > 0;
}

/* STAGED: frames in the next chunk of an n-frame batch with `rem` frames left -- a batch of at most CHUNK_FRAMES is
 * one chunk; a larger one takes CHUNK_FRAMES while two or more chunks' worth remain, then halves (multiples of 16)
 * down to TAIL_FRAMES. */
static uint32_t stage_chunk(uint32_t n, uint32_t rem) {
    if (n <= CHUNK_FRAMES || rem <= TAIL_FRAMES) return rem;
    if (rem >= 2u * CHUNK_FRAMES) return CHUNK_FRAMES;
    const uint32_t half = ((rem / 2u) + 15u) & ~15u;
    return half < TAIL_FRAMES ? TAIL_FRAMES : half;
}
/* an upper bound of the chunks of any batch of at most n frames (the halving tail adds at most 5; checked by
 * tests/test_staged_plan.py's restatement) */
static uint32_t stage_chunks_max(uint32_t n) { return (n + CHUNK_FRAMES - 1) / CHUNK_FRAMES + 5u; }

/* ZEROCOPY and LOWLAT read the UMEM in place through its mapped alias */
static int zerocopy(const xsk_gpu_ctx* c) { return c->mode != XSK_GPU_MODE_STAGED; }

static int fail(hipError_t e) { return e == hipErrorOutOfMemory ? -ENOMEM : -EIO; }
#define TRY(expr)                           \
    do {                                    \
        const hipError_t e_ = (expr);       \
        if (e_ != hipSuccess) {             \
            rc = fail(e_);                  \
            goto out;                       \
        }                                   \
    } while (0)

/* the caller's current device, to put back on return: object lifecycles and per-call paths all select their own
 * device and leave the caller's thread as they found it */
int xsk_gpu__dev_save(void) {
    int d = -1;
    if (hipGetDevice(&d) != hipSuccess) {
        (void)hipGetLastError();
        d = -1;
    }
    return d;
}
void xsk_gpu__dev_restore(int d) {
    int now = -1;
    if (d >= 0 && (hipGetDevice(&now) != hipSuccess || now != d)) (void)hipSetDevice(d);
}

static void fini_impl(xsk_gpu_ctx* c);
void xsk_gpu_fini(xsk_gpu_ctx* c) {
    if (!c) return;
    const int caller_dev = xsk_gpu__dev_save();
    fini_impl(c);
    xsk_gpu__dev_restore(caller_dev);
}

static void fini_impl(xsk_gpu_ctx* c) {
    (void)xsk_gpu__complete(c, NULL, NULL, NULL); /* a batch still in flight: let it finish (results dropped) */
    (void)hipSetDevice(c->device);
    xsk_gpu__lowlat_free(c->ll); /* stops the resident kernel (waits for it) ... */
    if (c->ll_slot) ll_slot_give(c->device); /* ... before its hardware queue is offered to another context */
    for (int s = 0; s < NSTREAMS; s++)
        if (c->stream[s]) (void)hipStreamSynchronize(c->stream[s]);
    const int d = c->device;
    const size_t nd = (size_t)c->max_batch * sizeof(struct xsk_gpu_desc);
    const size_t nst = (size_t)c->max_chunks * sizeof(struct xsk_gpu_stats);
    if (c->mode == XSK_GPU_MODE_STAGED && c->d_umem) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, c->d_umem, c->umem_size);
    xsk_gpu__umem_unref(c->reg_base);
    if (c->d_descs) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, c->d_descs, nd);
    if (c->d_verdicts) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, c->d_verdicts, c->max_batch);
    if (c->d_recs) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, c->d_recs, (size_t)c->max_batch * sizeof(struct xsk_gpu_rec));
    if (c->d_stats) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, c->d_stats, nst);
    for (int s = 0; s < NSTREAMS; s++)
        if (c->d_ws[s]) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, c->d_ws[s], c->ws_size);
    if (c->d_pack) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, c->d_pack, (size_t)c->max_batch * PACK);
    if (c->d_stage) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, c->d_stage, 2u * (size_t)c->stage_bytes);
    if (c->h_stage) xsk_gpu__buf_free(d, XSK_GPU__BUF_HOST, c->h_stage, 2u * (size_t)c->stage_bytes);
    for (int h = 0; h < 2; h++)
        if (c->stage_ev[h]) (void)hipEventDestroy(c->stage_ev[h]);
    if (c->h_pack) xsk_gpu__buf_free(d, XSK_GPU__BUF_HOST, c->h_pack, (size_t)c->max_batch * PACK);
    if (c->h_verd) xsk_gpu__buf_free(d, XSK_GPU__BUF_HOST | hipHostMallocMapped, c->h_verd, c->max_batch);
    if (c->h_stats) xsk_gpu__buf_free(d, XSK_GPU__BUF_HOST | hipHostMallocMapped, c->h_stats, nst);
    if (c->h_descs) xsk_gpu__buf_free(d, XSK_GPU__BUF_HOST | (zerocopy(c) ? hipHostMallocMapped : 0u), c->h_descs, nd);
    xsk_gpu__buf_free(d, 0, NULL, 0); /* (no resident grid left on the device: what was kept goes too) */
    if (c->done) {
        for (uint32_t i = 0; i < c->max_chunks; i++)
            if (c->done[i]) (void)hipEventDestroy(c->done[i]);
        free(c->done);
    }
    if (c->packed) {
        for (uint32_t i = 0; i < c->max_chunks; i++)
            if (c->packed[i]) (void)hipEventDestroy(c->packed[i]);
        free(c->packed);
    }
    if (c->in_done) {
        for (uint32_t i = 0; i < c->max_chunks; i++)
            if (c->in_done[i]) (void)hipEventDestroy(c->in_done[i]);
        free(c->in_done);
    }
    for (int s = 0; s < NSTREAMS; s++)
        if (c->stream[s]) (void)hipStreamDestroy(c->stream[s]);
    free(c);
}

static int init_impl(xsk_gpu_ctx** out, int device, void* umem, uint64_t umem_size, uint32_t max_batch, int mode,
                     int prereg) {
    int rc = 0;
    if (!out || !umem || umem_size == 0 || !xsk_gpu__umem_aligned(umem) || (umem_size & 15u) || max_batch == 0 ||
        max_batch > XSK_GPU_MAX_BATCH ||
        (mode != XSK_GPU_MODE_ZEROCOPY && mode != XSK_GPU_MODE_STAGED && mode != XSK_GPU_MODE_LOWLAT))
        return -EINVAL;
    *out = NULL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -ENODEV;
    xsk_gpu_ctx* c = (xsk_gpu_ctx*)calloc(1, sizeof *c);
    if (!c) return -ENOMEM;
    c->device = device;
    c->mode = mode;
    if (mode == XSK_GPU_MODE_LOWLAT) { /* no free slot: ZEROCOPY, the same data path with a launch per batch */
        c->ll_slot = ll_slot_take(device);
        if (!c->ll_slot) c->mode = XSK_GPU_MODE_ZEROCOPY;
    }
    c->umem = (uint8_t*)umem;
    c->umem_size = umem_size;
    c->max_batch = max_batch;
    c->max_chunks = mode == XSK_GPU_MODE_STAGED ? stage_chunks_max(max_batch) : 1;
    c->stage_bytes = STAGE_HALF;
    TRY(hipSetDevice(device));
    for (int s = 0; s < NSTREAMS; s++) TRY(hipStreamCreateWithFlags(&c->stream[s], hipStreamNonBlocking));
    if (!prereg) { /* mapped in every mode: STAGED's gather kernel reads scattered frames through the alias */
        if ((rc = xsk_gpu__umem_ref(umem, umem_size, &c->reg_base)) != 0) goto out;
    }
    if (zerocopy(c)) {
        TRY(hipHostGetDevicePointer((void**)&c->d_umem, umem, 0));
    } else {
        /* the gather kernel's source; a runtime that gives no device alias on this device (a portable registration
         * made on another one) leaves STAGED with its DMA copies: scattered chunks then copy their span */
        if (hipHostGetDevicePointer((void**)&c->m_umem, umem, 0) != hipSuccess) {
            c->m_umem = NULL;
            (void)hipGetLastError();
        }
        TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_DEV, (void**)&c->d_umem, umem_size));
        TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_DEV, (void**)&c->d_pack, (size_t)max_batch * PACK));
        TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_HOST, (void**)&c->h_pack, (size_t)max_batch * PACK));
    }
    const size_t nd = (size_t)max_batch * sizeof(struct xsk_gpu_desc);
    const size_t nst = (size_t)c->max_chunks * sizeof(struct xsk_gpu_stats);
    TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_DEV, (void**)&c->d_descs, nd));
    TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_DEV, (void**)&c->d_verdicts, max_batch));
    TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_DEV, (void**)&c->d_recs, max_batch * sizeof(struct xsk_gpu_rec)));
    TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_DEV, (void**)&c->d_stats, nst));
    {
        const uint32_t per = max_batch < CHUNK_FRAMES || zerocopy(c) ? max_batch : CHUNK_FRAMES;
        const size_t ws = xsk_gpu_workspace_size(device, per);
        if (ws == 0) {
            rc = -EIO;
            goto out;
        }
        c->ws_size = ws;
        for (int s = 0; s < NSTREAMS; s++) TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_DEV, &c->d_ws[s], ws));
    }
    TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_HOST | hipHostMallocMapped, (void**)&c->h_verd, max_batch));
    TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_HOST | hipHostMallocMapped, (void**)&c->h_stats, nst));
    if (!zerocopy(c)) TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_HOST, (void**)&c->h_descs, nd));
    if (zerocopy(c)) {
        TRY(xsk_gpu__buf_alloc(device, XSK_GPU__BUF_HOST | hipHostMallocMapped, (void**)&c->h_descs, nd));
        TRY(hipHostGetDevicePointer((void**)&c->m_descs, c->h_descs, 0));
        TRY(hipHostGetDevicePointer((void**)&c->m_verd, c->h_verd, 0));
        TRY(hipHostGetDevicePointer((void**)&c->m_stats, c->h_stats, 0));
    }
    c->done = (hipEvent_t*)calloc(c->max_chunks, sizeof(hipEvent_t));
    if (!c->done) {
        rc = -ENOMEM;
        goto out;
    }
    for (uint32_t i = 0; i < c->max_chunks; i++) TRY(hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming));
    if (c->mode == XSK_GPU_MODE_STAGED) {
        c->packed = (hipEvent_t*)calloc(c->max_chunks, sizeof(hipEvent_t));
        if (!c->packed) {
            rc = -ENOMEM;
            goto out;
        }
        c->in_done = (hipEvent_t*)calloc(c->max_chunks, sizeof(hipEvent_t));
        if (!c->in_done) {
            rc = -ENOMEM;
            goto out;
        }
        for (uint32_t i = 0; i < c->max_chunks; i++) {
            TRY(hipEventCreateWithFlags(&c->packed[i], hipEventDisableTiming));
            TRY(hipEventCreateWithFlags(&c->in_done[i], hipEventDisableTiming));
        }
    }
    if (c->mode == XSK_GPU_MODE_LOWLAT) {
        rc = xsk_gpu__lowlat_start(&c->ll, c->d_umem, umem_size, 0);
        if (rc) goto out;
    }
    *out = c;
    return 0;
out:
    xsk_gpu_fini(c);
    return rc;
}

int xsk_gpu_init(xsk_gpu_ctx** out, int device, void* umem, uint64_t umem_size, uint32_t max_batch, int mode) {
    const int caller_dev = xsk_gpu__dev_save();
    const int rc = init_impl(out, device, umem, umem_size, max_batch, mode, 0);
    xsk_gpu__dev_restore(caller_dev);
    return rc;
}

int xsk_gpu__init_prereg(xsk_gpu_ctx** out, int device, void* umem, uint64_t umem_size, uint32_t max_batch, int mode) {
    const int caller_dev = xsk_gpu__dev_save();
    const int rc = init_impl(out, device, umem, umem_size, max_batch, mode, 1);
    xsk_gpu__dev_restore(caller_dev);
    return rc;
}

uint32_t xsk_gpu__ctx_max_batch(const xsk_gpu_ctx* c) { return c ? c->max_batch : 0u; }

void xsk_gpu__ctx_quiesce(xsk_gpu_ctx* c) {
    if (!c || !c->ll || c->pend_n) return; /* (never with a batch in flight: its completion must see it served) */
    const int caller_dev = xsk_gpu__dev_save();
    (void)hipSetDevice(c->device);
    xsk_gpu__lowlat_stop(c->ll);
    xsk_gpu__dev_restore(caller_dev);
}

int xsk_gpu__staged_stats(const xsk_gpu_ctx* c, uint64_t out[XSK_GPU__STAGED_STATS]) {
    if (!c || !out || c->mode != XSK_GPU_MODE_STAGED) return -EINVAL;
    for (int i = 0; i < XSK_GPU__STAGED_STATS; i++) out[i] = c->staged[i];
    return 0;
}
int xsk_gpu__staged_noalias(xsk_gpu_ctx* c, uint32_t half_bytes) {
    if (!c || c->mode != XSK_GPU_MODE_STAGED || (half_bytes && (half_bytes < 4096u || (half_bytes & 15u))) ||
        c->h_stage)
        return -EINVAL;
    c->m_umem = NULL;
    if (half_bytes) c->stage_bytes = half_bytes;
    return 0;
}
int xsk_gpu_ctx_mode(const xsk_gpu_ctx* c) { return c ? c->mode : -EINVAL; }
int xsk_gpu__lowlat_outcomes(const xsk_gpu_ctx* c, uint64_t out[4]) {
    if (!c || !out || !c->ll) return -EINVAL;
    for (int i = 0; i < 4; i++) out[i] = c->ll_outcome[i];
    return 0;
}
xsk_gpu__lowlat* xsk_gpu__ctx_lowlat(xsk_gpu_ctx* c) { return c ? c->ll : NULL; }
int xsk_gpu__umem_view(xsk_gpu_ctx* c, uint64_t off, void* out, uint64_t n) {
    if (!c || !out || !zerocopy(c) || off > c->umem_size || n > c->umem_size - off) return -EINVAL;
    int rc = 0, caller_dev = -1;
    if (hipGetDevice(&caller_dev) != hipSuccess) caller_dev = -1;
    TRY(hipSetDevice(c->device));
    TRY(hipMemcpy(out, c->d_umem + off, n, hipMemcpyDeviceToHost)); /* through the device alias's translation */
out:
    if (caller_dev >= 0 && caller_dev != c->device) (void)hipSetDevice(caller_dev);
    return rc;
}

int xsk_gpu_set_options(xsk_gpu_ctx* c, uint32_t opts) {
    if (!c || (opts & ~XSK_GPU_OPT_ALL)) return -EINVAL;
    if (c->pend_n) return -EBUSY; /* the batch in flight runs under the options it was submitted with */
    if (c->ll) {
        (void)hipSetDevice(c->device);
        const int rc = xsk_gpu__lowlat_set_opts(c->ll, opts);
        if (rc) return rc;
    }
    c->opts = opts;
    return 0;
}

/* STAGED without a mapped alias, scattered frames (XSK_STAGE_HOSTPACK): the host copies the chunk's read spans back
 * to back into a half of the pinned staging -- a table of u32 offsets first, then the spans, each at a 16-B aligned
 * offset -- one DMA copy moves the half, and the unpack kernel puts every span at its offset in the mirror.  A half is
 * refilled once the DMA copy that last read it has finished (its event), so the host packs half h while half h ^ 1 is
 * in flight.  A frame whose span cannot fit a half moves by a DMA copy of its own.  The bytes moved are the spans plus
 * 4 per frame of offsets: never the gaps between frames. */
static int stage_hostpack(xsk_gpu_ctx* c, const struct xsk_gpu_desc* d, const struct xsk_gpu_desc* dd, uint32_t n,
                          hipStream_t st) {
    const int wire = c->opts != 0;
    const uint64_t half = c->stage_bytes;
    if (!c->h_stage) { /* first use: all of it or nothing (a later call retries) */
        uint8_t *hs = NULL, *ds = NULL;
        hipEvent_t ev[2] = {NULL, NULL};
        int rc = 0;
        if (xsk_gpu__buf_alloc(c->device, XSK_GPU__BUF_HOST, (void**)&hs, 2u * (size_t)half) != hipSuccess ||
            xsk_gpu__buf_alloc(c->device, XSK_GPU__BUF_DEV, (void**)&ds, 2u * (size_t)half) != hipSuccess)
            rc = -ENOMEM;
        for (int h = 0; h < 2 && !rc; h++)
            if (hipEventCreateWithFlags(&ev[h], hipEventDisableTiming) != hipSuccess) rc = -EIO;
        if (rc) {
            if (hs) xsk_gpu__buf_free(c->device, XSK_GPU__BUF_HOST, hs, 2u * (size_t)half);
            if (ds) xsk_gpu__buf_free(c->device, XSK_GPU__BUF_DEV, ds, 2u * (size_t)half);
            for (int h = 0; h < 2; h++)
                if (ev[h]) (void)hipEventDestroy(ev[h]);
            return rc;
        }
        c->h_stage = hs;
        c->d_stage = ds;
        c->stage_ev[0] = ev[0];
        c->stage_ev[1] = ev[1];
        c->stage_rec[0] = c->stage_rec[1] = 0;
    }
    for (uint32_t f0 = 0; f0 < n;) {
        uint64_t bytes = 0; /* the frames [f0, f1) whose offsets table and spans fit one half */
        const uint32_t f1 = xsk_gpu__hostpack_split(d, f0, n, c->umem_size, wire, half, &bytes);
        const int h = c->stage_half;
        if (c->stage_rec[h] && hipEventSynchronize(c->stage_ev[h]) != hipSuccess) return -EIO;
        uint8_t* hs = c->h_stage + (size_t)h * half;
        uint8_t* ds = c->d_stage + (size_t)h * half;
        uint32_t* offs = (uint32_t*)hs;
        const uint32_t m = f1 - f0;
        const uint64_t data0 = ((uint64_t)m * 4u + 15u) & ~15ull;
        uint64_t pos = data0;
        for (uint32_t f = f0; f < f1; f++) {
            uint64_t a16 = 0;
            const uint64_t sp = xsk_gpu__read_span(d[f].addr, d[f].len, c->umem_size, wire, &a16);
            if (sp + 16u > half) { /* too large for any half: its own DMA copy */
                if (hipMemcpyAsync(c->d_umem + a16, c->umem + a16, sp, hipMemcpyHostToDevice, st) != hipSuccess)
                    return -EIO;
                c->staged[0] += sp;
                c->staged[6]++;
                offs[f - f0] = UINT32_MAX;
                continue;
            }
            offs[f - f0] = (uint32_t)(pos - data0);
            memcpy(hs + pos, c->umem + a16, sp);
            pos += sp;
        }
        if (hipMemcpyAsync(ds, hs, pos, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipEventRecord(c->stage_ev[h], st) != hipSuccess)
            return -EIO;
        c->stage_rec[h] = 1;
        const int rc = xsk_gpu__stage_unpack_dev(ds + data0, (const uint32_t*)ds, c->d_umem, c->umem_size, dd + f0, m,
                                                 (uint32_t)wire, st);
        if (rc) return rc;
        c->staged[0] += pos; /* the offsets table (padded to 16 B) and the spans */
        c->stage_half ^= 1;
        f0 = f1;
    }
    c->staged[5]++;
    return 0;
}

/* Enqueue the copy-in chunk d[0..n) planned as p (dd: the chunk's descriptors, already on the device) on stream st;
 * c->staged records the bytes (never more than 1.1 x the frames' read spans, plus the host pack's offsets). */
static int stage_issue(xsk_gpu_ctx* c, const struct xsk_stage_plan* p, const struct xsk_gpu_desc* d,
                       const struct xsk_gpu_desc* dd, uint32_t n, hipStream_t st) {
    switch (p->kind) {
        case XSK_STAGE_2D:
            if (hipMemcpy2DAsync(c->d_umem + p->base, p->stride, c->umem + p->base, p->stride, p->width, n,
                                 hipMemcpyHostToDevice, st) != hipSuccess)
                return -EIO;
            c->staged[0] += (uint64_t)n * p->width;
            c->staged[1]++;
            return 0;
        case XSK_STAGE_SPAN:
            if (hipMemcpyAsync(c->d_umem + p->lo, c->umem + p->lo, p->hi - p->lo, hipMemcpyHostToDevice, st) != hipSuccess)
                return -EIO;
            c->staged[0] += p->hi - p->lo;
            c->staged[2]++;
            return 0;
        case XSK_STAGE_GATHER: {
            const int rc = xsk_gpu__stage_gather_dev(c->m_umem, c->d_umem, c->umem_size, dd, n, (uint32_t)(c->opts != 0), st);
            if (rc) return rc;
            c->staged[0] += p->sum;
            c->staged[3]++;
            return 0;
        }
        case XSK_STAGE_HOSTPACK:
            return stage_hostpack(c, d, dd, n, st);
        default:
            return 0;
    }
}

/* Enqueue one chunk [i0, i0+n) of the batch (ZEROCOPY: on stream s); results land in the pinned host buffers
 * and c->done[ci] fires when they are there. */
static int enqueue_chunk(xsk_gpu_ctx* c, const struct xsk_gpu_desc* descs, uint32_t i0, uint32_t n, uint32_t ci,
                         int want_recs, int s, int* prefix_aligned) {
    int rc = 0;
    if (zerocopy(c)) { /* descriptors in, verdicts and counters out: mapped host memory */
        const hipStream_t st = c->stream[s];
        memcpy(c->h_descs + i0, descs + i0, (size_t)n * sizeof *descs);
        memset(&c->h_stats[ci], 0, sizeof c->h_stats[ci]);
        const uint32_t tile = n <= XSK_GPU_LOWLAT_MAX ? xsk_gpu__small_tile_w(descs + i0, n, 256u) : 0u;
        rc = xsk_gpu__echo_dev_opts_hoststats(c->d_umem, c->umem_size, c->m_descs + i0, n, c->opts, c->m_verd + i0,
                                              want_recs ? c->d_recs + i0 : NULL, c->m_stats + ci, c->d_ws[s], st, tile);
        if (rc) goto out;
        TRY(hipEventRecord(c->done[ci], st));
        return 0;
    }
    /* STAGED: the copy stream (stream[0]) takes every chunk's descriptors and copy-in back to back, so the H2D
     * direction of the link never waits for a transform; the compute stream (stream[1]) runs each chunk's
     * transform once its copy-in is in, then its header pack and the copy-back.  A copy-in that may write mirror
     * bytes of an earlier chunk's frames (not contained, xsk_stage_plan.h: an unaligned frame anywhere in the call so
     * far, a span or a 2-D row reaching past the frame's own bytes, the dense-span copy) first waits for the previous
     * chunk's pack, and so for every earlier chunk's (the compute stream is in order); later chunks' transforms
     * follow their own copy-ins, which follow this one on the copy stream.  Contained copy-ins run under the other
     * chunks' transforms. */
    (void)s;
    const hipStream_t sa = c->stream[0], sb = c->stream[1];
    struct xsk_gpu_desc* dd = c->d_descs + i0;
    /* (slot i0.. of the pinned staging is not reused within a call, and the previous call has drained) */
    memcpy(c->h_descs + i0, descs + i0, (size_t)n * sizeof *descs);
    TRY(hipMemcpyAsync(dd, c->h_descs + i0, (size_t)n * sizeof *descs, hipMemcpyHostToDevice, sa));
    const struct xsk_stage_plan p =
        xsk_gpu__stage_plan(descs + i0, n, c->umem_size, c->opts != 0, c->m_umem != NULL, *prefix_aligned);
    *prefix_aligned &= (int)p.aligned;
    if (ci > 0 && !p.contained) TRY(hipStreamWaitEvent(sa, c->packed[ci - 1], 0));
    if (p.contained) c->staged[4]++;
    rc = stage_issue(c, &p, descs + i0, dd, n, sa);
    if (rc) goto out;
    TRY(hipEventRecord(c->in_done[ci], sa));
    TRY(hipStreamWaitEvent(sb, c->in_done[ci], 0));
    TRY(hipMemsetAsync(c->d_stats + ci, 0, sizeof(struct xsk_gpu_stats), sb));
    rc = xsk_gpu_echo_dev_opts(c->d_umem, c->umem_size, dd, n, c->opts, c->d_verdicts + i0,
                               want_recs ? c->d_recs + i0 : NULL, c->d_stats + ci, c->d_ws[1], sb);
    if (rc) goto out;
    rc = xsk_gpu__pack_headers_dev(c->d_umem, dd, c->d_verdicts + i0, n, c->d_pack + (size_t)i0 * PACK, c->opts != 0,
                                   sb);
    if (rc) goto out;
    TRY(hipEventRecord(c->packed[ci], sb));
    TRY(hipMemcpyAsync(c->h_pack + (size_t)i0 * PACK, c->d_pack + (size_t)i0 * PACK, (size_t)n * PACK,
                       hipMemcpyDeviceToHost, sb));
    TRY(hipMemcpyAsync(c->h_verd + i0, c->d_verdicts + i0, n, hipMemcpyDeviceToHost, sb));
    TRY(hipMemcpyAsync(c->h_stats + ci, c->d_stats + ci, sizeof *c->h_stats, hipMemcpyDeviceToHost, sb));
    TRY(hipEventRecord(c->done[ci], sb));
out:
    return rc;
}

int xsk_gpu_process(xsk_gpu_ctx* c, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                    struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats) {
    return xsk_gpu__process_ex(c, descs, n, verdicts, recs, stats, 0);
}

int xsk_gpu__process_ex(xsk_gpu_ctx* c, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                        struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats, int no_doorbell) {
    const int rc = xsk_gpu__submit(c, descs, n, recs != NULL, no_doorbell);
    if (rc) return rc;
    return xsk_gpu__complete(c, verdicts, recs, stats);
}

int xsk_gpu__submit(xsk_gpu_ctx* c, const struct xsk_gpu_desc* descs, uint32_t n, int want_recs, int no_doorbell) {
    int rc = 0;
    if (!c || (!descs && n)) return -EINVAL;
    c->fail_untouched = 1; /* every failure below before a batch is posted or a chunk enqueued */
    if (c->pend_n) return -EBUSY; /* one batch in flight per context */
    if (n == 0) return 0;
    if (n > c->max_batch) return -EINVAL;
    if (c->ll && xsk_gpu__lowlat_broken(c->ll)) {
        /* a timed-out doorbell batch whose kernel has not stopped yet may still write: nothing else runs
         * until it has (-EBUSY), then the context is usable again */
        if (!xsk_gpu__lowlat_recover(c->ll)) return -EBUSY;
    }
    if (c->ll && n <= XSK_GPU_LOWLAT_MAX && !no_doorbell) { /* the doorbell: no launch, no sync, no HIP call */
        memcpy(xsk_gpu__lowlat_descs(c->ll), descs, (size_t)n * sizeof *descs);
        uint32_t w = 0;
        rc = xsk_gpu__lowlat_post(c->ll, n, want_recs, &w);
        if (rc) {
            /* posted, then the relaunch failed: a later instance could still serve it (the channel is broken) */
            c->fail_untouched = !xsk_gpu__lowlat_broken(c->ll);
            return rc;
        }
        c->pend_n = n;
        c->pend_bell = 1;
        c->pend_w = w;
        c->pend_recs = want_recs;
        return 0;
    }
    int caller_dev = -1; /* the caller's current device, restored on return */
    if (hipGetDevice(&caller_dev) != hipSuccess) caller_dev = -1;
    TRY(hipSetDevice(c->device));
    if (c->ll) xsk_gpu__lowlat_stop(c->ll); /* a large batch: the launch path (its streams never wait on it) */
    const int staged = c->mode == XSK_GPU_MODE_STAGED;
    uint32_t nchunks = 0;
    int prefix_aligned = 1; /* every frame of the chunks enqueued so far starts 16-B aligned */
    for (uint32_t i0 = 0; i0 < n; nchunks++) {
        const uint32_t m = staged ? stage_chunk(n, n - i0) : n;
        rc = enqueue_chunk(c, descs, i0, m, nchunks, want_recs, (int)(nchunks % NSTREAMS), &prefix_aligned);
        if (rc) {
            for (int s = 0; s < NSTREAMS; s++) (void)hipStreamSynchronize(c->stream[s]);
            c->fail_untouched = 0; /* chunks before this one, or this one's kernel, may have run */
            goto out;
        }
        i0 += m;
    }
    c->pend_n = n;
    c->pend_bell = 0;
    c->pend_chunks = nchunks;
    c->pend_recs = want_recs;
out:
    if (caller_dev >= 0 && caller_dev != c->device) (void)hipSetDevice(caller_dev);
    return rc;
}

int xsk_gpu__failed_untouched(const xsk_gpu_ctx* c) { return c && c->fail_untouched; }

int xsk_gpu__ready(const xsk_gpu_ctx* c) {
    if (!c || !c->pend_n) return 1;
    if (c->pend_bell) return xsk_gpu__lowlat_ready(c->ll);
    return hipEventQuery(c->done[c->pend_chunks - 1]) == hipSuccess;
}

/* The doorbell batch in flight: wait, then verdicts, records and the counters the kernel's counter phase would add. */
static int complete_doorbell(xsk_gpu_ctx* c, uint32_t n, uint8_t* verdicts, struct xsk_gpu_rec* recs,
                             struct xsk_gpu_stats* stats) {
    const struct xsk_gpu_desc* descs = xsk_gpu__lowlat_descs(c->ll); /* the batch as submitted (options aside) */
    const uint32_t w = c->pend_w;
    if (!c->pend_recs) recs = NULL;
    uint32_t unserved = 0;
    int rc = xsk_gpu__lowlat_wait(c->ll, &unserved);
    /* timed out: untouched frames stay the caller's (-ETIMEDOUT) unless the channel stopped with part of the
     * batch served -- the GPU is evidently alive, so the untouched slices take the launch path and the call
     * completes, every frame transformed exactly once */
    const int partial = rc == -ETIMEDOUT && !xsk_gpu__lowlat_broken(c->ll) && unserved && unserved != (1u << w) - 1u;
    if (rc == -ETIMEDOUT) c->ll_outcome[partial ? 1 : 2]++, c->ll_outcome[0]++;
    if (!rc && xsk_gpu__lowlat_last_late(c->ll)) c->ll_outcome[3]++, c->ll_outcome[0]++;
    if (rc && !partial) {
        /* every slice untouched (the channel stopped without serving any) or the outcome unknown (broken) */
        c->fail_untouched = rc == -ETIMEDOUT && !xsk_gpu__lowlat_broken(c->ll) && unserved == (1u << w) - 1u;
        return rc;
    }
    uint8_t hv[XSK_GPU_LOWLAT_MAX];
    memcpy(hv, xsk_gpu__lowlat_verdicts(c->ll), n);
    if (recs) memcpy(recs, xsk_gpu__lowlat_recs(c->ll), (size_t)n * sizeof *recs);
    for (uint32_t g = 0; partial && g < w; g++) {
        if (!((unserved >> g) & 1u)) continue;
        uint32_t f0 = 0, f1 = 0;
        xsk_gpu__ll_slice(n, w, g, &f0, &f1);
        if (f1 <= f0) continue;
        rc = xsk_gpu__process_ex(c, descs + f0, f1 - f0, hv + f0, recs ? recs + f0 : NULL, NULL, 1);
        if (rc) {
            c->fail_untouched = 0; /* the grid served the other slices */
            return rc;
        }
    }
    if (verdicts) memcpy(verdicts, hv, n);
    if (stats) { /* xsk_receive.c:171-172, 229, 233 -- what the kernel's counter phase would add */
        uint64_t rxb = 0, txp = 0, txb = 0;
        for (uint32_t i = 0; i < n; i++) {
            rxb += descs[i].len;
            if (hv[i] == XSK_GPU_TX_REPLY) {
                txp++;
                txb += descs[i].len;
            }
        }
        stats->rx_packets += n;
        stats->rx_bytes += rxb;
        stats->tx_packets += txp;
        stats->tx_bytes += txb;
    }
    return 0;
}

int xsk_gpu__complete(xsk_gpu_ctx* c, uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats) {
    int rc = 0;
    if (!c) return -EINVAL;
    const uint32_t n = c->pend_n;
    if (!n) return 0;
    c->pend_n = 0;
    c->fail_untouched = 0; /* a failure below: part of the batch may have been transformed */
    if (c->pend_bell) return complete_doorbell(c, n, verdicts, recs, stats);
    if (!c->pend_recs) recs = NULL;
    const struct xsk_gpu_desc* descs = c->h_descs; /* the batch as submitted: every chunk copied it there */
    int caller_dev = -1;
    if (hipGetDevice(&caller_dev) != hipSuccess) caller_dev = -1;
    TRY(hipSetDevice(c->device));
    const int staged = c->mode == XSK_GPU_MODE_STAGED;
    for (uint32_t ci = 0, i0 = 0; ci < c->pend_chunks; ci++) {
        const uint32_t m = staged ? stage_chunk(n, n - i0) : n;
        if (hipEventSynchronize(c->done[ci]) != hipSuccess) {
            rc = -EIO;
            goto drain;
        }
        if (staged) { /* scatter the rewritten bytes of this chunk's replies */
            for (uint32_t i = i0; i < i0 + m; i++) {
                if (c->h_verd[i] != XSK_GPU_TX_REPLY) continue;
                /* reference mode rewrites bytes [0, 38); wire mode bytes below l4 + 4 <= 86 <= len */
                const uint32_t w = c->opts ? (descs[i].len < PACK ? descs[i].len : PACK) : 38u;
                memcpy(c->umem + descs[i].addr, c->h_pack + (size_t)i * PACK, w);
            }
        }
        if (stats) {
            stats->rx_packets += c->h_stats[ci].rx_packets;
            stats->rx_bytes += c->h_stats[ci].rx_bytes;
            stats->tx_packets += c->h_stats[ci].tx_packets;
            stats->tx_bytes += c->h_stats[ci].tx_bytes;
        }
        i0 += m;
    }
    if (verdicts) memcpy(verdicts, c->h_verd, n);
    if (recs) {
        for (int s = 0; s < NSTREAMS; s++) TRY(hipStreamSynchronize(c->stream[s]));
        TRY(hipMemcpy(recs, c->d_recs, (size_t)n * sizeof *recs, hipMemcpyDeviceToHost));
    }
    goto out;
drain:
    for (int s = 0; s < NSTREAMS; s++) (void)hipStreamSynchronize(c->stream[s]);
out:
    if (caller_dev >= 0 && caller_dev != c->device) (void)hipSetDevice(caller_dev);
    return rc;
}
