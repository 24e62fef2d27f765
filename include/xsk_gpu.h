/*
 * xsk_gpu.h — C ABI of the MI355X (gfx950) ICMP-echo frame transform.
 *
 * This library replaces the per-descriptor call to the reference's
 *   static bool process_packet(struct xsk_socket_info*, uint64_t addr, uint32_t len,
 *                              const struct egress_sock*)          src/lib/xsk_receive.c:113-190
 * inside the RX batch loop
 *   for (i = 0; i < rcvd; i++) { ... process_packet(...) ... }     src/lib/xsk_receive.c:220-230
 * by ONE call per batch of AF_XDP descriptors.  Frames are rewritten in place (echo request ->
 * echo reply) exactly as the reference does, the per-frame decision comes back as a verdict, and
 * the four stats counters of `struct stats_record` (src/lib/xsk_utils.h:17-23) are accumulated
 * exactly as src/lib/xsk_receive.c:171-172,229,233 accumulate them.
 *
 * Plain C, no HIP/torch types: streams and device pointers are passed as `void*`.
 * Every entry point returns 0 or a negative errno value (-EINVAL, -ENOMEM, -EIO, -ENODEV); it never
 * prints and never exits (the reference logs and `exit()`s; per-frame failures are verdicts here).
 *
 * Frame ownership contract (AF_XDP gives every frame its own >= 2048-byte UMEM chunk):
 *   - the UMEM size is a multiple of 16; a device UMEM's base is 16-byte aligned, a host UMEM's base
 *     (xsk_gpu_init, xsk_gpu_multi_init, xsk_gpu_rx_pipe_init) page-aligned, as AF_XDP requires of the area
 *     it registers (the reference: posix_memalign(getpagesize(), ...), src/lib/xsk_utils.c:132-135), so that
 *     no page of a registered UMEM is shared with another allocation -- -EINVAL otherwise;
 *   - every frame exclusively owns the bytes [addr, addr + max(len, 64)) of the UMEM for the duration
 *     of a call (frames of one batch never overlap); the library only changes bytes
 *     [addr, addr + 38) of frames whose verdict is XSK_GPU_TX_REPLY (exactly the bytes the reference
 *     rewrites), and only reads bytes inside [align16(addr), align16(addr) + 64) u [addr, addr + len);
 *   - a 16-B aligned reply whose [addr, addr + 64) lies in the UMEM is stored as that whole 64-byte
 *     window (bytes 38-63 are written back with the values they held), so HBM sees full sectors
 *     instead of read-modify-write partial ones; unaligned replies are stored byte-exact.
 */
#ifndef XSK_GPU_H
#define XSK_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XSK_GPU_ABI_VERSION 1

/* Descriptors with len above this are DROP_BAD_DESC (AF_XDP frames are <= one UMEM chunk). */
#define XSK_GPU_MAX_LEN (1u << 30)

/* Frames per wavefront tile == RX_BATCH_SIZE (src/lib/xsk_utils.h:8). */
#define XSK_GPU_TILE_FRAMES 64

/* Largest n one device-resident call accepts (frame indices stay 32-bit); larger n is -EINVAL. */
#define XSK_GPU_MAX_BATCH 0xFFFFFF00u

/* One RX descriptor. Binary-identical to `struct xdp_desc` of <linux/if_xdp.h>, which the reference
 * reads at src/lib/xsk_receive.c:222-223 (addr = UMEM offset, len = frame length). */
struct xsk_gpu_desc {
    uint64_t addr;
    uint32_t len;
    uint32_t options;
};

/* Counters. Binary-identical to the reference's `struct stats_record` (src/lib/xsk_utils.h:17-23).
 * Accumulated, never reset, by every call:
 *   rx_packets += n                      (xsk_receive.c:233)
 *   rx_bytes   += sum(len)   all frames  (xsk_receive.c:229)
 *   tx_packets += #TX_REPLY              (xsk_receive.c:172; sendto assumed to succeed: see
 *                                         xsk_gpu_stats_tx_failed() to apply the real outcome)
 *   tx_bytes   += sum(len)   TX_REPLY    (xsk_receive.c:171)
 * `timestamp` is never touched (the reference's stats thread owns it, xsk_stats.c:83). */
struct xsk_gpu_stats {
    uint64_t timestamp;
    uint64_t rx_packets;
    uint64_t rx_bytes;
    uint64_t tx_packets;
    uint64_t tx_bytes;
};

/* Per-frame verdict. The reference returns `false` for every frame (xsk_receive.c:124-146,189);
 * these codes say WHICH branch it took. */
enum xsk_gpu_verdict {
    XSK_GPU_TX_REPLY = 0,       /* gates passed, frame rewritten; the reference sendto()s it (:148-172) */
    XSK_GPU_DROP_SHORT = 1,     /* len < 20: the three silent length checks (:123-133)               */
    XSK_GPU_DROP_NOT_IPV4 = 2,  /* bytes 12-13 != 08 00 (:135-138)                                  */
    XSK_GPU_DROP_NOT_ICMP = 3,  /* byte 23 != 1 (:140-143)                                          */
    XSK_GPU_DROP_NOT_ECHO = 4,  /* byte 34 != 8 (:144-147)                                          */
    XSK_GPU_DROP_BAD_DESC = 5,  /* build-added: the frame does not lie inside the UMEM, or
                                   len > XSK_GPU_MAX_LEN (the reference would read out of bounds);
                                   never emitted for valid descriptors */
    XSK_GPU_DROP_BAD_IP = 6,    /* wire mode, XSK_GPU_OPT_STRICT_IPV4 only: see below            */
    XSK_GPU_DROP_BAD_CSUM = 7   /* wire mode, XSK_GPU_OPT_VERIFY_CSUM only: see below            */
};

/* Record flags (build-added verification of the INPUT frame; the reference never verifies). */
#define XSK_GPU_F_IP_CSUM_OK 0x01u   /* len >= 34 and the IPv4 header [14,34) sums to 0xFFFF */
#define XSK_GPU_F_ICMP_CSUM_OK 0x02u /* len >= 42 and the ICMP message [34,len) sums to 0xFFFF */
#define XSK_GPU_F_VLAN 0x04u         /* wire mode: one or two VLAN tags were skipped           */
#define XSK_GPU_F_IP_OPTIONS 0x08u   /* wire mode: IHL > 5 (IPv4 options present)             */

/* ------------------------------------------------------------------------------------------ */
/* Wire-format widening (build-added).  opts == 0 is the reference's gates */
/* exactly (everything above).  Any nonzero opts selects "wire mode", which parses the headers  */
/* instead of assuming the reference's fixed offsets (xsk_receive.c:120-121):                   */
/*   l3 = 14; with XSK_GPU_OPT_VLAN up to two 802.1Q/802.1ad tags (TPID 0x8100 / 0x88A8) are     */
/*        skipped, l3 += 4 each (a tag cut by the frame end: DROP_SHORT);                        */
/*   DROP_SHORT if len < 14; DROP_NOT_IPV4 unless the (inner) ethertype is 0x0800;               */
/*   DROP_SHORT if len < l3 + 20;                                                                */
/*   with XSK_GPU_OPT_STRICT_IPV4: DROP_BAD_IP unless version == 4 and IHL >= 5, unless          */
/*        IHL*4 + 8 <= tot_len and l3 + tot_len <= len, or if MF is set or the fragment offset is */
/*        nonzero; the IPv4 header is IHL*4 bytes and the ICMP message is [l4, l3 + tot_len)     */
/*        (Ethernet padding excluded); without it the header is 20 bytes and the message         */
/*        [l4, len), l4 = l3 + header bytes;                                                     */
/*   DROP_NOT_ICMP unless protocol (byte l3 + 9) == 1; DROP_SHORT if len < l4 + 8;               */
/*   DROP_NOT_ECHO unless type (byte l4) == 8 (and, STRICT, code == 0);                          */
/*   with XSK_GPU_OPT_VERIFY_CSUM: DROP_BAD_CSUM unless both the IPv4 header and the ICMP message */
/*        sum to 0xFFFF;                                                                         */
/*   otherwise TX_REPLY: process_packet's rewrite (xsk_receive.c:148-157) at the parsed offsets: */
/*        MACs swapped, addresses at l3+12 / l3+16 swapped, type = 0, checksum at l4+2 updated   */
/*        by csum_replace2(8 -> 0).                                                              */
/* Wire-mode records: verdict always; every other field only once all three headers lie inside  */
/* the frame (TX_REPLY, DROP_NOT_ECHO, DROP_BAD_CSUM), else zero: eth_proto = inner ethertype,   */
/* ip_vihl / ip_proto / icmp_* from l3 / l4, ip_sum over [l3, l4), icmp_sum over the message,    */
/* flags IP_CSUM_OK / ICMP_CSUM_OK (sum == 0xFFFF), VLAN, IP_OPTIONS.  Wire mode reads only      */
/* [addr, addr + len) plus the 16-B-aligned 64-byte header window (within the UMEM), and a       */
/* descriptor whose [addr, addr + len) leaves the UMEM is DROP_BAD_DESC.                         */
/* ------------------------------------------------------------------------------------------ */
#define XSK_GPU_OPT_STRICT_IPV4 0x1u
#define XSK_GPU_OPT_VLAN 0x2u
#define XSK_GPU_OPT_VERIFY_CSUM 0x4u
#define XSK_GPU_OPT_ALL 0x7u

/* Optional 16-byte per-frame result record. Parsed fields are those the reference reads
 * (xsk_receive.c:135,140,144,157); they are all zero when len < 20 because the reference reads
 * nothing then.  Checksums are RFC 1071 folded one's-complement sums of 16-bit big-endian words,
 * odd tail zero-padded, over the frame's own bytes only (0 for an empty range). */
struct xsk_gpu_rec {
    uint8_t verdict;        /* enum xsk_gpu_verdict                                        */
    uint8_t flags;          /* XSK_GPU_F_*                                                 */
    uint8_t ip_proto;       /* byte 23                                                     */
    uint8_t icmp_type;      /* byte 34 as received                                         */
    uint8_t icmp_code;      /* byte 35                                                     */
    uint8_t ip_vihl;        /* byte 14 (version/IHL; not checked by the reference)         */
    uint16_t eth_proto;     /* bytes 12-13, big-endian value                               */
    uint16_t icmp_csum_in;  /* bytes 36-37 as received, big-endian value                   */
    uint16_t icmp_csum_out; /* bytes 36-37 after the transform (== in unless TX_REPLY)     */
    uint16_t ip_sum;        /* folded sum over [14, min(len, 34))                          */
    uint16_t icmp_sum;      /* folded sum over [34, len)                                   */
};

/* ------------------------------------------------------------------------------------------ */
/* Device-resident entry points (frames, descriptors and outputs already in HBM).             */
/* ------------------------------------------------------------------------------------------ */

/* Bytes of device workspace xsk_gpu_echo_dev() needs for a batch of n frames on `device`
 * (per-workgroup counter partials; 32 B per 64-frame tile, at least 512 B, at most 32 KiB). */
size_t xsk_gpu_workspace_size(int device, uint32_t n);

/* Transform n frames in place on the current HIP device.
 *   d_umem/umem_size : device UMEM (16-B aligned base, size % 16 == 0)
 *   d_descs          : n descriptors (device memory, 16-B aligned)
 *   d_verdicts       : n bytes, or NULL
 *   d_recs           : n records (16-B aligned), or NULL
 *   d_stats          : one xsk_gpu_stats in device memory (not mapped host memory: every workgroup adds
 *                      its counters with device-scope atomics), accumulated; or NULL
 *   d_workspace      : xsk_gpu_workspace_size() bytes of device memory; may be NULL iff d_stats is
 *   stream           : hipStream_t (NULL = default stream)
 * Asynchronous: enqueues the transform kernel on `stream` and returns.  Replaces xsk_receive.c:220-233
 * for one batch. */
int xsk_gpu_echo_dev(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                     uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs, struct xsk_gpu_stats* d_stats,
                     void* d_workspace, void* stream);

/* xsk_gpu_echo_dev() with wire-format options (XSK_GPU_OPT_*; 0 = xsk_gpu_echo_dev() exactly).
 * Unknown option bits are -EINVAL. */
int xsk_gpu_echo_dev_opts(void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                          uint32_t opts, uint8_t* d_verdicts, struct xsk_gpu_rec* d_recs,
                          struct xsk_gpu_stats* d_stats, void* d_workspace, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Host-UMEM entry points: the drop-in for the client's RX loop (xsk_receive.c:192-237).       */
/* ------------------------------------------------------------------------------------------ */

typedef struct xsk_gpu_ctx xsk_gpu_ctx;

enum xsk_gpu_mode {
    /* The kernel reads and rewrites the registered host UMEM directly over PCIe (mapped pinned
     * memory): one launch per batch, no copies of frame bytes.  Best for small RX batches. */
    XSK_GPU_MODE_ZEROCOPY = 0,
    /* The bytes the transform reads are copied host->device (one strided 2-D copy for a uniform stride, one
     * copy of a densely covered span, else a per-frame gather across PCIe: never more than 1.1 x the bytes the
     * frames own), transformed in HBM, and only the rewritten header bytes of replies are copied back.  Best
     * for large batches. */
    XSK_GPU_MODE_STAGED = 1,
    /* ZEROCOPY data path plus a resident polling kernel for the RX loop's small batches: a call with
     * n <= XSK_GPU_LOWLAT_MAX writes the descriptors into mapped host memory, bumps a doorbell the
     * kernel polls, and spins until the kernel publishes completion -- no launch, no stream sync.  The
     * kernel runs the launched kernel's code (bit-identical results), holds one CU while it serves, and
     * exits on xsk_gpu_fini() or after 50 ms without a batch (the next call relaunches it).  Larger
     * batches stop it and take the ZEROCOPY launch path. */
    XSK_GPU_MODE_LOWLAT = 2
};

/* Largest batch the LOWLAT doorbell takes (larger ones are launched). */
#define XSK_GPU_LOWLAT_MAX 1024u

/* Resident LOWLAT kernels per device in one process.  Each waits for batches on a highest-priority stream of its
 * own, and the HIP runtime backs a process's streams of one priority with a few hardware queues (GPU_MAX_HW_QUEUES,
 * 4 by default): a resident kernel that lands on a queue behind another one does not start until that one exits,
 * and its batches would time out (tools/rxqueues: 8 LOWLAT queues on one GPU, 4 of them -ETIMEDOUT).  So a device
 * holds at most min(XSK_GPU_LOWLAT_PER_DEVICE, GPU_MAX_HW_QUEUES) - reserved resident kernels of this process, where
 * `reserved` is what xsk_gpu_lowlat_reserve() set aside; a context created in XSK_GPU_MODE_LOWLAT beyond that runs as
 * XSK_GPU_MODE_ZEROCOPY (same results, a launch per batch); xsk_gpu_ctx_mode() reports the mode a context runs in,
 * and xsk_gpu_fini() releases the slot once its kernel has stopped.
 * The cap assumes the process runs NO other highest-priority streams on that device: an application stream of the
 * highest priority (hipStreamCreateWithPriority with the greatest priority, torch.cuda.Stream(priority=-1)) shares
 * those hardware queues, so its work may wait behind a resident kernel and a resident kernel behind its work.  An
 * application with such streams reserves one queue per stream first.
 * With the runtime's default (GPU_MAX_HW_QUEUES unset or 4) that is 4; a deployment that sets GPU_MAX_HW_QUEUES=8 in
 * its environment gets 8 (round 5, tools/rxring: a depth-8 pipelined RX loop at 64-frame steps 44-45 Mframes/s against
 * 29-30 at depth 4).  Not more: with 16 resident kernels the grids were time-sliced (a depth-16 pipe
 * 0.12 Mframes/s), the device's hardware queue slots oversubscribed.  The cap in force is xsk_gpu_lowlat_cap(device);
 * this constant is only its ceiling. */
#define XSK_GPU_LOWLAT_PER_DEVICE 8

/* Reserve `queues` (<= XSK_GPU_LOWLAT_PER_DEVICE) of `device`'s highest-priority hardware queues for the application's
 * own highest-priority streams: LOWLAT contexts created afterwards stay within the rest (earlier ones keep running).
 * Process-wide, host-only (no device call).  Returns the resident LOWLAT kernels now allowed on the device, or
 * -EINVAL. */
int xsk_gpu_lowlat_reserve(int device, uint32_t queues);

/* The resident LOWLAT kernels a process may run on `device` now: min(XSK_GPU_LOWLAT_PER_DEVICE,
 * GPU_MAX_HW_QUEUES (4 when unset)) less the queues reserved above -- the number to size LOWLAT contexts or a LOWLAT
 * pipe's depth by (XSK_GPU_LOWLAT_PER_DEVICE is only the ceiling).  Host-only, changes nothing; -EINVAL for a negative
 * or out-of-range device index. */
int xsk_gpu_lowlat_cap(int device);

/* Bind a context to GPU `device` and the caller's UMEM (e.g. the posix_memalign'd buffer of
 * xsk_utils.c:132-135; its base must be page-aligned, -EINVAL otherwise).  The UMEM is registered with the HIP
 * runtime (hipHostRegister, portable + mapped) until the last context, multi object or pipe over it is released:
 * several of them may share one UMEM (AF_XDP sockets sharing a UMEM, one context per RX queue), and the library counts
 * its users of each registration (the runtime keeps one per base and does not); a UMEM that is a part of one already
 * registered by the library uses that registration.  -EBUSY for a UMEM that overlaps such a registration without
 * lying inside it (no two registrations ever share a page).  A UMEM the caller registered with the runtime itself is used as it is (it must be mapped) and
 * stays registered.  max_batch bounds n of later calls. */
int xsk_gpu_init(xsk_gpu_ctx** out, int device, void* umem, uint64_t umem_size, uint32_t max_batch, int mode);

/* The mode `ctx` runs in (XSK_GPU_MODE_*): the one it was created with, except a LOWLAT request beyond
 * XSK_GPU_LOWLAT_PER_DEVICE, which runs as ZEROCOPY.  -EINVAL for NULL. */
int xsk_gpu_ctx_mode(const xsk_gpu_ctx* ctx);

/* Synchronously process one batch of host descriptors against the bound UMEM.  Same outputs as
 * xsk_gpu_echo_dev(); `verdicts`, `recs` and `stats` are host pointers (each may be NULL).
 * XSK_GPU_MODE_LOWLAT: if a doorbell batch is not complete within 2 s the call posts STOP and waits (up to 1 s)
 * for the resident kernel to stop.  A workgroup that finds STOP before it took its slice of the batch never serves
 * it, so once the kernel has stopped every slice is either transformed exactly once or untouched: all served -> the
 * call returns 0 after all; some served -> the untouched slices take the launch path and the call returns 0; none
 * served -> -ETIMEDOUT with every frame untouched (a retry transforms them exactly once).  If the kernel had not
 * stopped within the second, the call returns -ETIMEDOUT with the batch's frames in an unknown state, and every
 * later call returns -EBUSY, touching nothing, until it has (xsk_gpu_fini() waits for it). */
int xsk_gpu_process(xsk_gpu_ctx* ctx, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                    struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats);

/* The reference counts a reply in tx_packets / tx_bytes only after its sendto() succeeded
 * (xsk_receive.c:166-172); every entry point above counts each TX_REPLY frame as sent.  A caller that sends the
 * replies itself reports the outcome here: for every i with verdicts[i] == XSK_GPU_TX_REPLY and sent[i] == 0,
 * tx_packets -= 1 and tx_bytes -= descs[i].len, so the counters end where the reference's would.  Host memory
 * only, no device call.  Returns the number of frames taken back (never more than the counters hold), or
 * -EINVAL. */
int xsk_gpu_stats_tx_failed(struct xsk_gpu_stats* stats, const struct xsk_gpu_desc* descs, const uint8_t* verdicts,
                            const uint8_t* sent, uint32_t n);

/* Wire-format options (XSK_GPU_OPT_*) for this context's later xsk_gpu_process() / xsk_gpu_rx_step()
 * calls (0 at init: the reference's gates). */
int xsk_gpu_set_options(xsk_gpu_ctx* ctx, uint32_t opts);

/* Release device buffers and unregister the UMEM. NULL is a no-op. */
void xsk_gpu_fini(xsk_gpu_ctx* ctx);

/* ------------------------------------------------------------------------------------------ */
/* Several GPUs behind one RX loop: one UMEM, G contexts.                       */
/* ------------------------------------------------------------------------------------------ */

typedef struct xsk_gpu_multi xsk_gpu_multi;

#define XSK_GPU_MULTI_MAX 16

/* Bind G = ndev contexts (devices[g], repeats allowed: G contexts on one GPU) to ONE caller UMEM
 * (registered once with the HIP runtime, portable + mapped, for every device).  `mode` and
 * `max_batch` as for xsk_gpu_init(); max_batch bounds the whole batch of later calls.
 * Device memory: a STAGED context holds a full umem_size mirror of the UMEM on its device (a share's frames
 * lie anywhere in it), so contexts that repeat a device need G x umem_size there; ZEROCOPY and LOWLAT
 * contexts read the UMEM in place and hold only per-batch buffers. */
int xsk_gpu_multi_init(xsk_gpu_multi** out, const int* devices, uint32_t ndev, void* umem, uint64_t umem_size,
                       uint32_t max_batch, int mode);

/* xsk_gpu_process() of one batch over the G contexts: descriptor i goes to context i mod G (frames
 * are independent, xsk_receive.c:113-190), each context runs on its own host thread and stream, and
 * verdicts / records land at the descriptors' own positions.  The four counters are the sum over the
 * contexts (xsk_utils.h:17-23), added to *stats like xsk_gpu_process() does.
 * LOWLAT contexts: the path is chosen per batch -- the doorbells only when every context really runs LOWLAT
 * (xsk_gpu_ctx_mode: requests beyond a device's resident-kernel cap run as ZEROCOPY) and no share exceeds
 * XSK_GPU_LOWLAT_MAX; otherwise every resident kernel is stopped first and every share is launched, so shares of one
 * batch never split between resident kernels and launched grids.
 * Partial failure: when any context fails, the call returns the first failing context's error and adds
 * NOTHING to *stats (all or nothing); the shares of the contexts that succeeded are transformed and their
 * verdicts / records written, the failed shares' positions are left as they were -- xsk_gpu_multi_status()
 * says which is which. */
int xsk_gpu_multi_process(xsk_gpu_multi* m, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                          struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats);

/* Per-context result of the last xsk_gpu_multi_process(): status[g] = 0 or that context's negative errno for
 * the share of descriptors i with i mod G == g (at most `cap` entries written).  Returns G. */
int xsk_gpu_multi_status(const xsk_gpu_multi* m, int* status, uint32_t cap);

/* Wire-format options for every context (xsk_gpu_set_options). */
int xsk_gpu_multi_set_options(xsk_gpu_multi* m, uint32_t opts);

/* Stop the worker threads, release every context, unregister the UMEM.  NULL is a no-op. */
void xsk_gpu_multi_fini(xsk_gpu_multi* m);

/* ------------------------------------------------------------------------------------------ */
/* XDP ingress filter on the device (the frames the echo transform sees).                      */
/* ------------------------------------------------------------------------------------------ */

/* XDP actions, values of enum xdp_action (<linux/bpf.h>). */
#define XSK_GPU_XDP_DROP 1
#define XSK_GPU_XDP_PASS 2
#define XSK_GPU_XDP_REDIRECT 4

/* Bytes of zero-or-garbage device workspace xsk_gpu_classify_dev() needs for n frames. */
size_t xsk_gpu_classify_workspace_size(uint32_t n);

/* xdp_sock_prog() of src/kern/inner_xdp.c:26-61 over a device-resident batch (phy_xdp.c:39-81 makes
 * the same tests with a devmap instead of the xsks_map):
 *   d_actions[i] = XSK_GPU_XDP_DROP      if len < 14                        (:35-36)
 *                  XSK_GPU_XDP_PASS      if bytes 12-13 != 08 00            (:38-39)
 *                  XSK_GPU_XDP_DROP      if len < 34                        (:41-42)
 *                  XSK_GPU_XDP_PASS      if byte 23 != 1 (not ICMP)         (:44-45)
 *                  XSK_GPU_XDP_REDIRECT  if target_bound, else XSK_GPU_XDP_DROP (:57-60)
 * (a descriptor outside the UMEM is XSK_GPU_XDP_DROP: build-added).  With d_out (16-B aligned, room
 * for n descriptors) the REDIRECT frames' descriptors are also written there in batch order and
 * their count to *d_nout: the input of xsk_gpu_echo_dev().  Asynchronous on `stream`. */
int xsk_gpu_classify_dev(const void* d_umem, uint64_t umem_size, const struct xsk_gpu_desc* d_descs, uint32_t n,
                         int target_bound, uint8_t* d_actions, struct xsk_gpu_desc* d_out, uint32_t* d_nout,
                         void* d_workspace, void* stream);

/* The UMEM allocation for the host modes: the reference allocates its UMEM with posix_memalign(getpagesize(),
 * NUM_FRAMES * FRAME_SIZE) (src/lib/xsk_utils.c:132-135); this gives the same kind of memory (anonymous, private,
 * page-aligned: AF_XDP registers it as it is) 2 MiB aligned, advised onto transparent huge pages and touched up front.
 * The GPU then walks one translation per 2 MiB instead of one per 4 KiB frame chunk: a 64 x 64-B LOWLAT call 8.8 ->
 * 7.2 us, a scattered 1024 x 64-B call 17.8 -> 12.9 (profiles/r05/hostlat_pages.jsonl).  size: a multiple of 16.
 * *huge_bytes (may be NULL) = how much of it the kernel did back with huge pages (0 without THP).  0 or -errno.
 * Release with xsk_gpu_umem_free(umem, size) after every context over it is gone. */
int xsk_gpu_umem_alloc(void** umem, uint64_t size, uint64_t* huge_bytes);
void xsk_gpu_umem_free(void* umem, uint64_t size);

/* ------------------------------------------------------------------------------------------ */
/* AF_XDP ring loop: the reference's handle_receive_packets() around one xsk_gpu_process().    */
/* ------------------------------------------------------------------------------------------ */

/* An AF_XDP ring, field-compatible with libxdp's struct xsk_ring_prod / struct xsk_ring_cons
 * (<xdp/xsk.h>), so a caller passes &xsk->rx, &xsk->tx, &umem->fq, &umem->cq cast to this type.
 * Descriptor rings (RX, TX) hold struct xsk_gpu_desc entries, address rings (fill, completion)
 * hold uint64_t UMEM offsets. */
struct xsk_gpu_ring {
    uint32_t cached_prod;
    uint32_t cached_cons;
    uint32_t mask;
    uint32_t size;
    uint32_t* producer;
    uint32_t* consumer;
    void* ring;
    uint32_t* flags;
};

/* The client's free-frame stack: struct xsk_socket_info's umem_frame_addr[] / umem_frame_free
 * (src/lib/xsk_utils.h:30-31), popped by xsk_alloc_umem_frame and pushed by xsk_free_umem_frame
 * (src/lib/xsk_receive.c:54-70). */
struct xsk_gpu_frame_pool {
    uint64_t* addr;
    uint32_t n_free;
    uint32_t capacity;
};

struct xsk_gpu_rx_result {
    uint32_t received;   /* RX descriptors consumed                                     */
    uint32_t replied;    /* TX_REPLY frames submitted to the TX ring                    */
    uint32_t tx_full;    /* TX_REPLY frames dropped because the TX ring was full        */
    uint32_t refilled;   /* free frames handed to the fill ring                         */
};

#define XSK_GPU_RX_MAX_STEP 1024u /* frames per xsk_gpu_rx_step() call */

/* One pass of handle_receive_packets() (src/lib/xsk_receive.c:192-237) with the transform on the
 * GPU and the XSK TX path the reference leaves commented out (:174-186) enabled instead of the
 * per-frame sendto() (:166):
 *   1. peek up to min(max_batch, XSK_GPU_RX_MAX_STEP, the context's max_batch) RX descriptors (:196);
 *      none -> return 0;
 *   2. refill the fill ring with min(free fill slots, free frames) frames from `pool` (:201-217;
 *      the reference reserves the free-slot count even when it has fewer free frames);
 *   3. xsk_gpu_process() the batch (replaces the per-frame process_packet() loop :220-230);
 *   4. submit every TX_REPLY frame to the TX ring; a reply that finds the TX ring full is dropped
 *      and its frame freed, like :178-181; every other frame goes back to `pool` (:226-227);
 *   5. release the RX entries (:232).
 * Counters: rx_packets += received (:233), rx_bytes += sum(len) (:229), tx_packets / tx_bytes count
 * the frames actually submitted (:171-172 count successful sends).  The TX kick (sendto on the XSK
 * fd, :86) stays with the caller, which owns the socket.  Returns the number of frames received
 * (0 if the RX ring was empty) or a negative errno; `res` may be NULL.  On an error the batch's frames stay on the RX
 * ring for a retry when every one of them is known untouched (nothing was posted or launched, or a LOWLAT batch timed
 * out unserved); when some may have been transformed (a partly served batch whose launch path failed, a launch error,
 * a LOWLAT kernel still running after its timeout) the batch is dropped instead -- released from the RX ring, every
 * frame back to `pool`, none transmitted, res->received set -- since a retry could transform a frame twice. */
int xsk_gpu_rx_step(xsk_gpu_ctx* ctx, struct xsk_gpu_ring* rx, struct xsk_gpu_ring* fill, struct xsk_gpu_ring* tx,
                    struct xsk_gpu_frame_pool* pool, uint32_t max_batch, struct xsk_gpu_stats* stats,
                    struct xsk_gpu_rx_result* res);

/* complete_tx() (src/lib/xsk_receive.c:77-99) minus the kick: move up to `max` completed TX frames
 * from the completion ring back to `pool`.  Returns the number moved. */
uint32_t xsk_gpu_tx_complete(struct xsk_gpu_ring* comp, struct xsk_gpu_frame_pool* pool, uint32_t max);

/* Pipelined RX loop: xsk_gpu_rx_step with up to `depth` batches in flight, so that one queue's steps overlap their
 * PCIe round trips instead of paying one per step.  The object owns up to `depth` contexts of `mode` over one
 * registration of the UMEM and hands batches to them in turn.  A LOWLAT pipe stops adding contexts at the first one
 * the device has no resident-kernel slot left for (xsk_gpu_ctx_mode): batches complete in RX order, so one launched
 * ZEROCOPY context among doorbell ones holds every batch behind it (4 LOWLAT + 4 ZEROCOPY at 64-frame steps: 5.2
 * Mframes/s against 29 for the 4 LOWLAT alone); xsk_gpu_rx_pipe_depth() says how many it kept.  Only when not even the
 * first context gets a slot are all `depth` contexts ZEROCOPY.  Frames of different batches are different frames, so batches in flight never
 * share a byte (the ownership contract above).
 *
 * xsk_gpu_rx_pipe_step:
 *   1. if a context is free and the RX ring holds descriptors: peek up to min(max_batch, XSK_GPU_RX_MAX_STEP) of them,
 *      submit them and release the RX entries (the object keeps a copy of the descriptors: res->received);
 *   2. complete batches in submission order -- the oldest when every context is busy, any that are already done, and
 *      all of them when step 1 found the RX ring empty -- each like xsk_gpu_rx_step's steps 4 and 5: replies onto the
 *      TX ring (or dropped and freed when it is full), every other frame back to `pool`, counters;
 *   3. refill the fill ring from `pool` (as xsk_gpu_rx_step does, but on every call: frames freed by a step that
 *      received nothing must reach the fill ring too, or with batches in flight it could run dry).
 * Returns the frames completed by this call (not the frames received), or a negative errno.  A batch whose completion
 * fails with every frame untouched stays the oldest in flight, and the next step or flush runs it again through its
 * context (as a caller retries a failed xsk_gpu_rx_step); a batch that may be partly transformed is dropped (its
 * frames back to `pool`, none transmitted) and the pipe moves on.  The call returns the error when it handed no frame
 * on, else its count (the error comes back from a later call if the rerun fails too).  A failed submit leaves its
 * frames on the RX ring, or drops them the same way when some may have been transformed.
 * xsk_gpu_rx_pipe_flush completes every batch in flight (an idle link, teardown); with a failure it stops there, so
 * call it until xsk_gpu_rx_pipe_inflight() is 0.  xsk_gpu_rx_pipe_fini waits for
 * batches still in flight and drops their results: flush first.  Single caller thread, like a context. */
#define XSK_GPU_RX_PIPE_MAX 8u
typedef struct xsk_gpu_rx_pipe xsk_gpu_rx_pipe;
int xsk_gpu_rx_pipe_init(xsk_gpu_rx_pipe** out, int device, void* umem, uint64_t umem_size, uint32_t depth, int mode);
int xsk_gpu_rx_pipe_step(xsk_gpu_rx_pipe* p, struct xsk_gpu_ring* rx, struct xsk_gpu_ring* fill, struct xsk_gpu_ring* tx,
                         struct xsk_gpu_frame_pool* pool, uint32_t max_batch, struct xsk_gpu_stats* stats,
                         struct xsk_gpu_rx_result* res);
int xsk_gpu_rx_pipe_flush(xsk_gpu_rx_pipe* p, struct xsk_gpu_ring* tx, struct xsk_gpu_frame_pool* pool,
                          struct xsk_gpu_stats* stats, struct xsk_gpu_rx_result* res);
/* xsk_gpu_set_options on every context; -EBUSY while a batch is in flight. */
int xsk_gpu_rx_pipe_set_options(xsk_gpu_rx_pipe* p, uint32_t opts);
/* Batches in flight now. */
uint32_t xsk_gpu_rx_pipe_inflight(const xsk_gpu_rx_pipe* p);
/* Contexts the pipe holds (its depth after init; at most the depth asked for).  0 for NULL. */
uint32_t xsk_gpu_rx_pipe_depth(const xsk_gpu_rx_pipe* p);
void xsk_gpu_rx_pipe_fini(xsk_gpu_rx_pipe* p);

/* ------------------------------------------------------------------------------------------ */
/* Bench / test utilities (not on the hot path).                                               */
/* ------------------------------------------------------------------------------------------ */

/* Synthetic frame generator, bit-identical to oracle/echo_oracle.c:oracle_synth_frame().
 * Writes n frames into d_umem at addr = base_off + j*stride and their descriptors into d_descs.
 * Frame j carries global index first + j*step (round-robin sharding: first = rank, step = world).
 * mode 0 = valid ICMP echo requests, mode 1 = mixed edge cases / negatives.
 * len is uniform in [len_lo, len_hi]; each frame's chunk is filled for roundup16(max(len, 64))
 * bytes.  Requires base_off % 16 == 0, stride % 16 == 0, stride >= that extent, extent <= 4096. */
int xsk_gpu_synth_dev(void* d_umem, uint64_t umem_size, struct xsk_gpu_desc* d_descs, uint32_t n,
                      uint64_t base_off, uint64_t stride, uint64_t seed, uint64_t first, uint64_t step, int mode,
                      uint32_t len_lo, uint32_t len_hi, void* stream);

/* Re-arm: turn every TX_REPLY frame of a batch back into the echo request it was generated as
 * (swap fields back, type 0 -> 8, checksum restored).  Used by the bench when it must reuse a batch. */
int xsk_gpu_rearm_dev(void* d_umem, const struct xsk_gpu_desc* d_descs, const uint8_t* d_verdicts, uint32_t n,
                      void* stream);

/* Read-only streaming ceiling: sums `bytes` (multiple of 16) of device memory into *d_out (u64).
 * Used for the measured HBM read ceiling next to the transform. */
int xsk_gpu_stream_read_dev(const void* d_src, uint64_t bytes, uint64_t* d_out, void* stream);

/* Kernel timing with HIP events recorded around every transform-kernel launch on its own stream
 * (bench instrumentation).  enable != 0 starts recording (and clears previous samples);
 * xsk_gpu_timing_read() waits for the recorded launches and returns their summed duration. */
int xsk_gpu_timing_enable(int enable);
int xsk_gpu_timing_read(double* total_ms, uint64_t* launches);

/* ABI version and the name of the last HIP error seen by the library (static string). */
int xsk_gpu_abi_version(void);
const char* xsk_gpu_last_error(void);

/* Build id of the transform kernel in this library: a hash of the sources that define it and of the
 * compiler flags (static string).  Profiles record it so that measured counters are only ever
 * attributed to the build they were taken on. */
const char* xsk_gpu_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* XSK_GPU_H */
