/*
 * xsk_gpu_internal.h — symbols shared between the translation units of libxsknet_amd.so that are not
 * part of the public C ABI (include/xsk_gpu.h).  C11 and C++ (HIP) both include it.
 */
#ifndef XSK_GPU_INTERNAL_H
#define XSK_GPU_INTERNAL_H

#include <unistd.h>

#include "../../include/xsk_gpu.h"
#include "xsk_lowlat_proto.h"

/* A host UMEM starts on a page of its own (include/xsk_gpu.h): AF_XDP rejects an area that is not page-aligned and the
 * reference allocates one with posix_memalign(getpagesize(), ...) (src/lib/xsk_utils.c:132-135).  The runtime registers
 * whole pages, so a UMEM that began inside a page would share that page's registration -- and its GPU translation --
 * with whatever else lives there. */
static inline int xsk_gpu__umem_aligned(const void* umem) {
    long pg = sysconf(_SC_PAGESIZE);
    if (pg <= 0) pg = 4096;
    return ((uintptr_t)umem % (uintptr_t)pg) == 0;
}

#ifdef __cplusplus
extern "C" {
#endif

#define XSK_GPU__HIDDEN __attribute__((visibility("hidden")))

/* xsk_aux.hip: staged mode's gather of the rewritten header bytes of TX_REPLY frames */
XSK_GPU__HIDDEN int xsk_gpu__pack_headers_dev(const void* d_umem, const struct xsk_gpu_desc* d_descs,
                                              const uint8_t* d_verdicts, uint32_t n, uint8_t* d_pack, uint32_t wire,
                                              void* stream);

/* The bytes the transform reads of one frame, [*a16, *a16 + return value): for a frame it parses (reference mode:
 * len >= 20, wire mode: len >= 14, the descriptor inside the UMEM) its 16-B aligned start up to
 * align16(max(off + len, its 64-B header window inside the UMEM)) -- both modes read the same window since round 4
 * (xsk_echo_device.h, frame_in / echo6_body step 1: lim = max(rowhi, wend)); 0 for a frame it reads nothing of.
 * Host and device (staged mode's copy-in, xsk_gpu_host.c, and its gather kernel). */
#ifdef __HIPCC__
__host__ __device__
#endif
static inline uint64_t xsk_gpu__read_span(uint64_t addr, uint32_t len, uint64_t umem_size, int wire, uint64_t* a16) {
    *a16 = addr & ~15ull;
    const uint64_t need = wire ? len : (len >= 20u ? (len > 38u ? len : 38u) : len);
    if (len > XSK_GPU_MAX_LEN || addr > umem_size || need > umem_size - addr || len < (wire ? 14u : 20u)) return 0;
    const uint64_t off = addr & 15u;
    const uint64_t win = 64u;
    const uint64_t wend = umem_size - *a16 < win ? umem_size - *a16 : win;
    const uint64_t lim = off + len > wend ? off + len : wend;
    return (lim + 15u) & ~15ull;
}

/* xsk_aux.hip: staged mode's per-frame copy-in for descriptor sets that are neither one uniform stride nor one
 * dense span (AF_XDP recycles frames through a LIFO free stack, xsk_receive.c:55-71, so RX addresses scatter over the
 * UMEM): every frame's read span (xsk_gpu__read_span) from the mapped host UMEM into the device mirror at the same
 * offset.  d_descs in device memory. */
XSK_GPU__HIDDEN int xsk_gpu__stage_gather_dev(const void* m_umem, void* d_mirror, uint64_t umem_size,
                                              const struct xsk_gpu_desc* d_descs, uint32_t n, uint32_t wire,
                                              void* stream);
/* xsk_aux.hip: the same per-frame copy from a device staging buffer the host packed the read spans into (a context
 * whose device has no mapped alias of the UMEM): frame f's span is at d_stage + d_offs[f] (16-B aligned), or nowhere
 * when d_offs[f] == UINT32_MAX (the host copied that frame itself). */
XSK_GPU__HIDDEN int xsk_gpu__stage_unpack_dev(const void* d_stage, const uint32_t* d_offs, void* d_mirror,
                                              uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                                              uint32_t wire, void* stream);

/* xsk_echo.hip: xsk_gpu_echo_dev_opts for counters in mapped host memory (no device atomics): d_stats
 * must be a slot zeroed for this call (a one-workgroup launch stores the counters without reading it).
 * tile: frames per wave of a small batch (xsk_gpu__small_tile), 0 = ceil(n / 16). */
XSK_GPU__HIDDEN int xsk_gpu__echo_dev_opts_hoststats(void* d_umem, uint64_t umem_size,
                                                     const struct xsk_gpu_desc* d_descs, uint32_t n, uint32_t opts,
                                                     uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs,
                                                     struct xsk_gpu_stats* d_stats, void* d_workspace, void* stream,
                                                     uint32_t tile);

/* xsk_echo.hip (exported for tests and tools, not part of the ABI): xsk_gpu_echo_dev_opts with the workgroup
 * count forced to `grid` (0 = default): a large batch on `grid` static shares, a small one (n <=
 * XSK_GPU_LOWLAT_MAX) as sub-tiles over `grid` workgroups. */
int xsk_gpu__echo_dev_grid(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                           uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, struct xsk_gpu_stats* d_stats,
                           void* d_workspace, void* stream, uint32_t grid);

/* Frames per wave for a small batch (n <= XSK_GPU_LOWLAT_MAX) whose frames are read across PCIe: about
 * 8 KiB of frame bytes per wave, 1..max_waves waves (a 64-frame batch of minimum-size frames is one wave: its
 * few PCIe reads are better in one wave's hands than queued behind many; 1500-B frames spread over as many
 * waves as their bytes ask for).  A multiple of 4 in [4, 64].  The LOWLAT kernel asks for at most its 16
 * waves, a launched zerocopy batch for up to 256 (16 workgroups: one CU's loads in flight cap a batch's PCIe
 * rate). */
static inline uint32_t xsk_gpu__small_tile_w(const struct xsk_gpu_desc* descs, uint32_t n, uint32_t max_waves) {
    uint64_t bytes = 0;
    for (uint32_t i = 0; i < n; i++) bytes += descs[i].len < 4096u ? descs[i].len : 4096u;
    uint64_t waves = (bytes + 8191u) / 8192u;
    waves = waves < 1 ? 1 : (waves > max_waves ? max_waves : waves);
    uint32_t t = (uint32_t)((n + waves - 1) / waves);
    t = (t + 3u) & ~3u;
    return t < 4u ? 4u : (t > 64u ? 64u : t);
}
static inline uint32_t xsk_gpu__small_tile(const struct xsk_gpu_desc* descs, uint32_t n) {
    return xsk_gpu__small_tile_w(descs, n, 16u);
}

/* xsk_gpu_multi.c: fold the G shares of one xsk_gpu_multi_process call into the caller's counters, all or
 * nothing: when every share succeeded (rc[g] == 0) their counters are added to *out and 0 is returned; when any
 * failed, *out is left untouched and the first failing share's error is returned (xsk_gpu_multi_status() then
 * tells which shares were transformed).  Pure host code, unit-tested on the CPU (tests/c/test_multi_fold.c). */
static inline int xsk_gpu__multi_fold(const int* rc, const struct xsk_gpu_stats* st, uint32_t G,
                                      struct xsk_gpu_stats* out) {
    for (uint32_t g = 0; g < G; g++)
        if (rc[g]) return rc[g];
    if (out) {
        for (uint32_t g = 0; g < G; g++) {
            out->rx_packets += st[g].rx_packets;
            out->rx_bytes += st[g].rx_bytes;
            out->tx_packets += st[g].tx_packets;
            out->tx_bytes += st[g].tx_bytes;
        }
    }
    return 0;
}

/* xsk_gpu_host.c: xsk_gpu_process with the doorbell path of a LOWLAT context disabled for this call
 * (no_doorbell != 0: the batch takes the launch path even when it is small) -- the multi-context path decides
 * per batch, so that shares of one batch never split between the resident kernel and launched grids. */
XSK_GPU__HIDDEN int xsk_gpu__process_ex(xsk_gpu_ctx* ctx, const struct xsk_gpu_desc* descs, uint32_t n,
                                        uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats,
                                        int no_doorbell);

/* xsk_gpu_host.c: xsk_gpu__process_ex in two halves, so that a caller with several contexts keeps a batch in flight on
 * each (the pipelined RX loop, xsk_gpu_pipe.c).  submit enqueues the batch -- posts it on the doorbell, or launches it
 * -- and returns (-EBUSY while the context has one in flight; the descriptors are copied, `descs` may be reused at
 * once); complete waits for it and returns what xsk_gpu_process would have (0 with nothing in flight); ready = complete
 * would not block.  Records come back only when submit asked for them. */
XSK_GPU__HIDDEN int xsk_gpu__submit(xsk_gpu_ctx* ctx, const struct xsk_gpu_desc* descs, uint32_t n, int want_recs,
                                    int no_doorbell);
XSK_GPU__HIDDEN int xsk_gpu__complete(xsk_gpu_ctx* ctx, uint8_t* verdicts, struct xsk_gpu_rec* recs,
                                      struct xsk_gpu_stats* stats);
XSK_GPU__HIDDEN int xsk_gpu__ready(const xsk_gpu_ctx* ctx);
/* After a failed xsk_gpu__submit / xsk_gpu__complete / xsk_gpu_process: 1 when every frame of that batch is known to be
 * untouched -- nothing was posted or launched, or a doorbell batch timed out and the stopped grid had served none of it
 * -- so the batch may be run again; 0 when some frames may have been transformed (a partly served batch whose launch
 * path failed, a launch error, a channel still running after its timeout): running it again could transform a frame
 * twice (a request already turned into a reply reads as DROP_NOT_ECHO), so the RX loops drop such a batch instead. */
XSK_GPU__HIDDEN int xsk_gpu__failed_untouched(const xsk_gpu_ctx* ctx);

/* xsk_gpu_rx.c, shared by xsk_gpu_rx_step and the pipelined loop (xsk_gpu_pipe.c): stock the fill ring from the
 * free-frame stack (src/lib/xsk_receive.c:201-217; returns the frames handed over), and hand a transformed batch on --
 * replies onto the TX ring while it has room, every other frame back to the pool, the counters (:171-186, :226-233);
 * r->replied and r->tx_full accumulate. */
XSK_GPU__HIDDEN uint32_t xsk_gpu__rx_refill(struct xsk_gpu_ring* fill, struct xsk_gpu_frame_pool* pool);
XSK_GPU__HIDDEN void xsk_gpu__rx_drop(const struct xsk_gpu_desc* descs, uint32_t n, struct xsk_gpu_frame_pool* pool);
XSK_GPU__HIDDEN void xsk_gpu__rx_emit(const struct xsk_gpu_desc* descs, const uint8_t* verdict, uint32_t n,
                                      struct xsk_gpu_ring* tx, struct xsk_gpu_frame_pool* pool,
                                      struct xsk_gpu_stats* stats, struct xsk_gpu_rx_result* r);

/* xsk_gpu_pipe.c (tests and tools, not part of the ABI): context i of a pipelined RX loop, or NULL. */
xsk_gpu_ctx* xsk_gpu__rx_pipe_ctx(xsk_gpu_rx_pipe* p, uint32_t i);

/* xsk_gpu_multi.c (exported for the GPU tests, not part of the ABI): context g's next share fails with `rc`
 * without being processed (fault injection for the partial-failure semantics). */
int xsk_gpu__multi_inject(xsk_gpu_multi* m, uint32_t g, int rc);

/* xsk_lowlat.hip: ask every resident LOWLAT grid of the process to leave once idle (delta +1), or stop asking (-1);
 * requests count.  Used around a runtime call that waits for every stream of the device (hipHostUnregister). */
XSK_GPU__HIDDEN void xsk_gpu__ll_yield_all(int delta);
/* xsk_gpu_host.c: 1 while a LOWLAT slot of `device` is taken (a resident grid may run there). */
XSK_GPU__HIDDEN int xsk_gpu__ll_busy(int device);
/* xsk_gpu_mem.c: device (XSK_GPU__BUF_DEV, hipMalloc) and pinned host (XSK_GPU__BUF_HOST | hipHostMalloc flags)
 * buffers of contexts and LOWLAT channels.  A buffer released while a LOWLAT slot of its device is taken is kept for
 * the next allocation of the same device, kind and size instead of freed (the runtime's free would wait for the
 * resident grids), up to 256 buffers and 8 GiB; free(d, 0, NULL, 0) frees what is kept for `d` once no slot is
 * taken.  alloc returns a hipError_t.
 * buf_kept: buffers kept for `device` (tests). */
#define XSK_GPU__BUF_DEV 0u
#define XSK_GPU__BUF_HOST 0x80000000u
XSK_GPU__HIDDEN int xsk_gpu__buf_alloc(int device, unsigned kind, void** p, size_t size);
XSK_GPU__HIDDEN void xsk_gpu__buf_free(int device, unsigned kind, void* p, size_t size);
int xsk_gpu__buf_kept(int device);
/* xsk_gpu_mem.c: the in-process registrations of host UMEMs -- one runtime registration per UMEM, counted (the runtime
 * keeps one per base and does not count).  ref: 0 with *reg_base = the registration referenced (to unref at release),
 * -EBUSY (the range starts inside a registration and runs past it), -ENOMEM or -EIO; unref(reg_base): the last
 * reference unregisters (NULL: no-op).  umem_refs: the references of the registration at `base` (tests). */
XSK_GPU__HIDDEN int xsk_gpu__umem_ref(void* base, uint64_t size, void** reg_base);
XSK_GPU__HIDDEN void xsk_gpu__umem_unref(void* reg_base);
int xsk_gpu__umem_refs(const void* base);
/* xsk_gpu_host.c: xsk_gpu_init over a UMEM the caller has already registered with the HIP runtime
 * (portable + mapped, e.g. the one registration of a multi-GPU object): the context neither registers
 * nor unregisters it. */
XSK_GPU__HIDDEN int xsk_gpu__init_prereg(xsk_gpu_ctx** out, int device, void* umem, uint64_t umem_size,
                                         uint32_t max_batch, int mode);
XSK_GPU__HIDDEN uint32_t xsk_gpu__ctx_max_batch(const xsk_gpu_ctx* ctx);
/* xsk_gpu_host.c: stop the context's resident LOWLAT kernel, if any, and wait for it (the multi-context path stops
 * every context's before a batch whose shares take the launch path). */
XSK_GPU__HIDDEN void xsk_gpu__ctx_quiesce(xsk_gpu_ctx* ctx);
/* xsk_gpu_host.c (exported for the GPU tests and the bench, not part of the ABI): a STAGED context's copy-in record
 * since init -- out[0] bytes copied host->device (frame bytes, plus the staging offsets of the host pack), out[1..3]
 * chunks copied as one 2-D stride / one dense span / by the gather kernel, out[4] chunks whose copy-in was contained
 * (not ordered after the previous chunk's pack), out[5] chunks copied by the host pack (no mapped alias on the
 * context's device), out[6] frames of those copied by a DMA copy of their own (a span larger than a staging half).
 * -EINVAL for other modes. */
#define XSK_GPU__STAGED_STATS 7
int xsk_gpu__staged_stats(const xsk_gpu_ctx* ctx, uint64_t out[XSK_GPU__STAGED_STATS]);
/* xsk_gpu_host.c (test switch, not part of the ABI): a STAGED context forgets its UMEM's mapped device alias, as on a
 * device where the runtime gives none, so its scattered copy-ins take the host pack, with staging halves of half_bytes
 * (0 = the default 32 MiB; else >= 4096 and a multiple of 16, so that tests reach the frames too large for a half).
 * -EINVAL for other modes, bad sizes, or once the host pack has run. */
int xsk_gpu__staged_noalias(xsk_gpu_ctx* ctx, uint32_t half_bytes);
/* xsk_gpu_multi.c (tests and the bench, not part of the ABI): context g of a multi object, or NULL. */
xsk_gpu_ctx* xsk_gpu__multi_ctx(xsk_gpu_multi* m, uint32_t g);

/* xsk_lowlat.hip: the low-latency doorbell channel of a XSK_GPU_MODE_LOWLAT context (doorbell layout and
 * host protocol: xsk_lowlat_proto.h). */
/* Diagnostics of a LOWLAT kernel, in DEVICE memory (a store to host memory would put a PCIe
 * acknowledgement in front of the next doorbell poll), read by xsk_gpu__lowlat_trace().  100-MHz ticks. */
struct xsk_gpu__lldiag {
    uint64_t trace[4];  /* last batch: mean doorbell sampling interval, acquire + barrier, body, release +
                         * barrier + completion */
    uint64_t body[6];   /* wave 0's clock at the body's phase boundaries (descriptors, frames streamed,
                         * header phase, writes issued, counters), then the body's start */
    uint64_t clk[2];    /* shader-clock (s_memtime) ticks and wall ticks over the last body */
    uint64_t polls[3];  /* this kernel instance: batches served, doorbell reads examined, reads that saw a
                         * new doorbell with descriptor slots not yet tagged */
    uint32_t exit_gen;  /* the leader's idle exit: the launch generation that is leaving (the other resident
                         * workgroups poll it and leave too) */
    uint32_t pad;
};
typedef struct xsk_gpu__lowlat xsk_gpu__lowlat;
/* Create the channel on the current device for the (mapped) UMEM alias d_umem: its doorbell, mapped
 * buffers and stream.  The persistent kernel starts with the first batch. */
XSK_GPU__HIDDEN int xsk_gpu__lowlat_start(xsk_gpu__lowlat** out, void* d_umem, uint64_t umem_size, uint32_t opts);
XSK_GPU__HIDDEN void xsk_gpu__lowlat_free(xsk_gpu__lowlat* ll);
/* Post the batch already written into the mapped descriptor buffer and wait for its completion (xsk_gpu__ll_run):
 * *groups = the workgroups it was posted for (its slices: xsk_gpu__ll_slice), and on -ETIMEDOUT *unserved = the
 * slices left untouched (all bits when the channel is broken: unknown). */
XSK_GPU__HIDDEN int xsk_gpu__lowlat_run(xsk_gpu__lowlat* ll, uint32_t n, int want_recs, uint32_t* groups,
                                        uint32_t* unserved);
/* The two halves of xsk_gpu__lowlat_run (xsk_gpu__ll_begin / xsk_gpu__ll_wait): post the batch (-EBUSY while one is in
 * flight), wait for the one in flight; ready = it is complete (never blocks). */
XSK_GPU__HIDDEN int xsk_gpu__lowlat_post(xsk_gpu__lowlat* ll, uint32_t n, int want_recs, uint32_t* groups);
XSK_GPU__HIDDEN int xsk_gpu__lowlat_wait(xsk_gpu__lowlat* ll, uint32_t* unserved);
XSK_GPU__HIDDEN int xsk_gpu__lowlat_ready(const xsk_gpu__lowlat* ll);
XSK_GPU__HIDDEN int xsk_gpu__lowlat_set_opts(xsk_gpu__lowlat* ll, uint32_t opts);
XSK_GPU__HIDDEN void xsk_gpu__lowlat_stop(xsk_gpu__lowlat* ll);
/* 1 while a timed-out batch's instance has not stopped (later calls return -EBUSY). */
XSK_GPU__HIDDEN int xsk_gpu__lowlat_broken(xsk_gpu__lowlat* ll);
/* The last wait returned 0 for a batch past its timeout (a late completion: every slice served, found after STOP). */
XSK_GPU__HIDDEN int xsk_gpu__lowlat_last_late(const xsk_gpu__lowlat* ll);
/* A broken channel whose instance has stopped by now becomes usable again: returns 1 if the channel is usable
 * (never broken, or recovered), 0 while the instance still runs.  Never blocks. */
XSK_GPU__HIDDEN int xsk_gpu__lowlat_recover(xsk_gpu__lowlat* ll);
/* Mapped host buffers the kernel reads / writes: descriptors, verdicts, records. */
XSK_GPU__HIDDEN struct xsk_gpu_desc* xsk_gpu__lowlat_descs(xsk_gpu__lowlat* ll);
XSK_GPU__HIDDEN uint8_t* xsk_gpu__lowlat_verdicts(xsk_gpu__lowlat* ll);
XSK_GPU__HIDDEN struct xsk_gpu_rec* xsk_gpu__lowlat_recs(xsk_gpu__lowlat* ll);
/* Diagnostics (tools/hostlat.py): the phase durations of a LOWLAT context's last doorbell batch, in
 * nanoseconds: out[0..3] the trace[] phases, out[4..8] body[0..4] relative to the body's start; out[9]
 * the shader clock over the last body, in MHz; out[10..11] the host's time from entry to the doorbell
 * store and from there to seeing the completion. */
int xsk_gpu__lowlat_trace(xsk_gpu_ctx* ctx, uint64_t out_ns[15]);
/* Tuning / test knobs of a LOWLAT context (exported for tools/hostlat.py and the GPU tests; not part of the
 * ABI): frames per wave of a doorbell batch (multiple of 4 in [4, 64]; 0 = from the batch's bytes), the
 * workgroups that serve it (1..XSK_GPU__LL_WG; 0 = from its size), and the completion timeout in
 * microseconds (0 = 2 s).  -EINVAL for a non-LOWLAT context or values out of range. */
int xsk_gpu__lowlat_tune(xsk_gpu_ctx* ctx, uint32_t tile_frames, uint32_t groups, uint32_t timeout_us);
XSK_GPU__HIDDEN xsk_gpu__lowlat* xsk_gpu__ctx_lowlat(xsk_gpu_ctx* ctx);
/* xsk_gpu_host.c (exported for the GPU tests, not part of the ABI): a LOWLAT context's doorbell batches that missed their
 * completion timeout since init -- out[0] all of them, out[1] those completed through the launch path after the
 * resident grid had served part of them, out[2] those returned as -ETIMEDOUT.  -EINVAL for other modes. */
int xsk_gpu__lowlat_outcomes(const xsk_gpu_ctx* ctx, uint64_t out[4]);
/* xsk_lowlat.hip (test switch, not part of the ABI): the resident grid is launched with `wgs` workgroups (1 ..
 * XSK_GPU__LL_WG; 0 = all) from the next batch on, while batches are still posted for as many workgroups as their size
 * asks (xsk_gpu__lowlat_tune's `groups`): slices of workgroups that do not exist are never served, which makes a batch
 * time out partly served -- the deterministic test of the partial-timeout path. */
int xsk_gpu__lowlat_test_width(xsk_gpu_ctx* ctx, uint32_t wgs);
/* xsk_lowlat.hip (exported for the GPU tests, not part of the ABI): workgroups of resident LOWLAT grids running on
 * `device` in this process right now (each adds itself when it starts and leaves when it exits): 0 once every LOWLAT
 * context is gone -- no grid outlives its channel. */
int xsk_gpu__lowlat_live(int device, uint32_t* out);
/* xsk_gpu_host.c (exported for the GPU tests' failure reports, not part of the ABI): n bytes of a ZEROCOPY / LOWLAT
 * context's UMEM at `off`, copied through the context's device alias -- what the GPU's translation of those pages
 * holds, to set beside the host's view of the same bytes. */
int xsk_gpu__umem_view(xsk_gpu_ctx* ctx, uint64_t off, void* out, uint64_t n);

/* the caller's current device (-1 when unknown), and putting it back (xsk_gpu_host.c) */
__attribute__((visibility("hidden"))) int xsk_gpu__dev_save(void);
__attribute__((visibility("hidden"))) void xsk_gpu__dev_restore(int device);

#ifdef __cplusplus
}
#endif

#endif /* XSK_GPU_INTERNAL_H */
