/*
 * xsk_gpu_multi.c — several GPUs (or several contexts on one GPU) behind one RX loop.
 *
 * Frames are independent: process_packet() reads and writes only its own frame
 * (src/lib/xsk_receive.c:113-190), so a batch of descriptors splits with no exchange step.  Descriptor i
 * goes to context i mod G (round-robin, BASELINE config 5); every context is an ordinary host context
 * (xsk_gpu_host.c) over the SAME caller UMEM — the one posix_memalign'd buffer of xsk_utils.c:132-135 —
 * which is registered with the HIP runtime once, portable and mapped, so every device can read it
 * (ZEROCOPY / LOWLAT) or copy from it (STAGED).  Each context runs on a host thread of its own (context
 * 0 on the caller's thread) with its own streams; the stats_record counters (xsk_utils.h:17-23) are the
 * sum over the contexts, done here on the host.  No collective: nothing crosses between GPUs.
 */
#define _GNU_SOURCE
#define __HIP_PLATFORM_AMD__ 1
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "xsk_gpu_internal.h"

struct multi_worker {
    struct xsk_gpu_multi* m;
    uint32_t g;
    pthread_t th;
    int started;
    xsk_gpu_ctx* ctx;
    struct xsk_gpu_desc* descs; /* [cap] this context's sub-batch */
    uint8_t* verd;              /* [cap] */
    struct xsk_gpu_rec* recs;   /* [cap] */
    uint32_t cap;
    struct xsk_gpu_stats st;
    int rc;
    int inject; /* fault injection (xsk_gpu__multi_inject): the next share fails with this error */
};

struct xsk_gpu_multi {
    uint32_t G;
    uint8_t* umem;
    uint64_t umem_size;
    uint32_t max_batch;
    void* reg_base; /* the UMEM registration this object holds a reference of */
    int reg_device;
    struct multi_worker w[XSK_GPU_MULTI_MAX];
    /* the current job, published under mu */
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    uint64_t gen;
    uint32_t pending;
    int quit;
    const struct xsk_gpu_desc* job_descs;
    uint32_t job_n;
    uint8_t* job_verd;
    struct xsk_gpu_rec* job_recs;
    int job_launch; /* every share takes the launch path (a share above XSK_GPU_LOWLAT_MAX, or not every context
                     * runs LOWLAT) */
    int all_lowlat; /* every context really runs XSK_GPU_MODE_LOWLAT (none was downgraded at init) */
    int status[XSK_GPU_MULTI_MAX]; /* per-context result of the last xsk_gpu_multi_process */
};

/* Context g's share of the batch: descriptors g, g + G, g + 2G, ... */
static void run_share(struct multi_worker* w) {
    struct xsk_gpu_multi* m = w->m;
    const uint32_t G = m->G, g = w->g, n = m->job_n;
    const uint32_t k = n > g ? (n - g + G - 1) / G : 0;
    memset(&w->st, 0, sizeof w->st);
    w->rc = 0;
    if (!k) return;
    if (w->inject) {
        w->rc = w->inject;
        w->inject = 0;
        return;
    }
    for (uint32_t j = 0; j < k; j++) w->descs[j] = m->job_descs[g + (size_t)j * G];
    w->rc = xsk_gpu__process_ex(w->ctx, w->descs, k, w->verd, m->job_recs ? w->recs : NULL, &w->st, m->job_launch);
    if (w->rc) return;
    if (m->job_verd)
        for (uint32_t j = 0; j < k; j++) m->job_verd[g + (size_t)j * G] = w->verd[j];
    if (m->job_recs)
        for (uint32_t j = 0; j < k; j++) m->job_recs[g + (size_t)j * G] = w->recs[j];
}

static void* worker_main(void* arg) {
    struct multi_worker* w = (struct multi_worker*)arg;
    struct xsk_gpu_multi* m = w->m;
    uint64_t seen = 0;
    pthread_mutex_lock(&m->mu);
    for (;;) {
        while (!m->quit && m->gen == seen) pthread_cond_wait(&m->go, &m->mu);
        if (m->quit) break;
        seen = m->gen;
        pthread_mutex_unlock(&m->mu);
        run_share(w);
        pthread_mutex_lock(&m->mu);
        if (--m->pending == 0) pthread_cond_signal(&m->done);
    }
    pthread_mutex_unlock(&m->mu);
    return NULL;
}

void xsk_gpu_multi_fini(xsk_gpu_multi* m) {
    if (!m) return;
    pthread_mutex_lock(&m->mu);
    m->quit = 1;
    pthread_cond_broadcast(&m->go);
    pthread_mutex_unlock(&m->mu);
    for (uint32_t g = 0; g < m->G; g++) {
        struct multi_worker* w = &m->w[g];
        if (w->started) pthread_join(w->th, NULL);
        xsk_gpu_fini(w->ctx);
        free(w->descs);
        free(w->verd);
        free(w->recs);
    }
    if (m->reg_base) {
        const int caller_dev = xsk_gpu__dev_save();
        (void)hipSetDevice(m->reg_device);
        xsk_gpu__umem_unref(m->reg_base);
        xsk_gpu__dev_restore(caller_dev);
    }
    pthread_cond_destroy(&m->go);
    pthread_cond_destroy(&m->done);
    pthread_mutex_destroy(&m->mu);
    free(m);
}

int xsk_gpu_multi_init(xsk_gpu_multi** out, const int* devices, uint32_t ndev, void* umem, uint64_t umem_size,
                       uint32_t max_batch, int mode) {
    if (!out || !devices || ndev == 0 || ndev > XSK_GPU_MULTI_MAX || !umem || umem_size == 0 || !xsk_gpu__umem_aligned(umem) ||
        (umem_size & 15u) || max_batch == 0 || max_batch > XSK_GPU_MAX_BATCH ||
        (mode != XSK_GPU_MODE_ZEROCOPY && mode != XSK_GPU_MODE_STAGED && mode != XSK_GPU_MODE_LOWLAT))
        return -EINVAL;
    *out = NULL;
    int ndevs = 0;
    if (hipGetDeviceCount(&ndevs) != hipSuccess) return -ENODEV;
    for (uint32_t g = 0; g < ndev; g++)
        if (devices[g] < 0 || devices[g] >= ndevs) return -ENODEV;
    xsk_gpu_multi* m = (xsk_gpu_multi*)calloc(1, sizeof *m);
    if (!m) return -ENOMEM;
    m->G = ndev;
    m->umem = (uint8_t*)umem;
    m->umem_size = umem_size;
    m->max_batch = max_batch;
    pthread_mutex_init(&m->mu, NULL);
    pthread_cond_init(&m->go, NULL);
    pthread_cond_init(&m->done, NULL);
    int rc = 0;
    /* one registration of the caller's UMEM for every device (portable) with a device alias (mapped) */
    m->reg_device = devices[0];
    const int caller_dev = xsk_gpu__dev_save();
    /* (shared and counted with every other user of this UMEM: xsk_gpu__umem_ref) */
    rc = hipSetDevice(devices[0]) == hipSuccess ? xsk_gpu__umem_ref(umem, umem_size, &m->reg_base) : -EIO;
    xsk_gpu__dev_restore(caller_dev);
    if (rc) goto fail;
    const uint32_t cap = (max_batch + ndev - 1) / ndev;
    for (uint32_t g = 0; g < ndev; g++) {
        struct multi_worker* w = &m->w[g];
        w->m = m;
        w->g = g;
        w->cap = cap;
        w->descs = (struct xsk_gpu_desc*)malloc((size_t)cap * sizeof *w->descs);
        w->verd = (uint8_t*)malloc(cap);
        w->recs = (struct xsk_gpu_rec*)malloc((size_t)cap * sizeof *w->recs);
        if (!w->descs || !w->verd || !w->recs) {
            rc = -ENOMEM;
            goto fail;
        }
        rc = xsk_gpu__init_prereg(&w->ctx, devices[g], umem, umem_size, cap, mode);
        if (rc) goto fail;
    }
    m->all_lowlat = 1;
    for (uint32_t g = 0; g < ndev; g++) m->all_lowlat &= xsk_gpu_ctx_mode(m->w[g].ctx) == XSK_GPU_MODE_LOWLAT;
    for (uint32_t g = 1; g < ndev; g++) {
        if (pthread_create(&m->w[g].th, NULL, worker_main, &m->w[g]) != 0) {
            rc = -EAGAIN;
            goto fail;
        }
        m->w[g].started = 1;
    }
    *out = m;
    return 0;
fail:
    xsk_gpu_multi_fini(m);
    return rc;
}

int xsk_gpu_multi_set_options(xsk_gpu_multi* m, uint32_t opts) {
    if (!m || (opts & ~XSK_GPU_OPT_ALL)) return -EINVAL;
    for (uint32_t g = 0; g < m->G; g++) {
        const int rc = xsk_gpu_set_options(m->w[g].ctx, opts);
        if (rc) return rc;
    }
    return 0;
}

int xsk_gpu_multi_process(xsk_gpu_multi* m, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                          struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats) {
    if (!m || (!descs && n)) return -EINVAL;
    if (n == 0) return 0;
    if (n > m->max_batch) return -EINVAL;
    m->job_descs = descs;
    m->job_n = n;
    m->job_verd = verdicts;
    m->job_recs = recs;
    /* the path is chosen per batch from the modes the contexts really run, not per share: the doorbell only when
     * every context runs LOWLAT (a LOWLAT request beyond the device's resident-kernel cap runs as ZEROCOPY) and every
     * share fits it; otherwise every context takes the launch path, and every resident kernel has stopped before
     * any share is launched, so no share runs beside a resident kernel that holds a CU */
    m->job_launch = !m->all_lowlat || (n + m->G - 1) / m->G > XSK_GPU_LOWLAT_MAX;
    /* (with a downgraded context no batch ever takes a doorbell, so no resident kernel is ever started: nothing to
     * stop, per call or otherwise -- ADVICE r04) */
    if (m->job_launch && m->all_lowlat)
        for (uint32_t g = 0; g < m->G; g++) xsk_gpu__ctx_quiesce(m->w[g].ctx); /* (each restores the caller's device) */
    if (m->G > 1) {
        pthread_mutex_lock(&m->mu);
        m->pending = m->G - 1;
        m->gen++;
        pthread_cond_broadcast(&m->go);
        pthread_mutex_unlock(&m->mu);
    }
    run_share(&m->w[0]); /* context 0 on the caller's thread */
    if (m->G > 1) {
        pthread_mutex_lock(&m->mu);
        while (m->pending) pthread_cond_wait(&m->done, &m->mu);
        pthread_mutex_unlock(&m->mu);
    }
    struct xsk_gpu_stats st[XSK_GPU_MULTI_MAX];
    for (uint32_t g = 0; g < m->G; g++) {
        m->status[g] = m->w[g].rc;
        st[g] = m->w[g].st;
    }
    return xsk_gpu__multi_fold(m->status, st, m->G, stats);
}

int xsk_gpu_multi_status(const xsk_gpu_multi* m, int* status, uint32_t cap) {
    if (!m || (!status && cap)) return -EINVAL;
    for (uint32_t g = 0; g < m->G && g < cap; g++) status[g] = m->status[g];
    return (int)m->G;
}

xsk_gpu_ctx* xsk_gpu__multi_ctx(xsk_gpu_multi* m, uint32_t g) { return m && g < m->G ? m->w[g].ctx : NULL; }

int xsk_gpu__multi_inject(xsk_gpu_multi* m, uint32_t g, int rc) {
    if (!m || g >= m->G || rc >= 0) return -EINVAL;
    m->w[g].inject = rc;
    return 0;
}
