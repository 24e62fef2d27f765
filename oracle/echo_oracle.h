/*
 * echo_oracle.h — CPU oracle for the ICMP-echo frame transform.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code, and only
 * as the checker / the CPU baseline — never as the product path.
 *
 * Parity status: the reference (src/lib/xsk_receive.c) cannot be compiled in this image — its
 * header chain src/lib/xsk_utils.h:3 includes <xdp/xsk.h> (libxdp), which is absent, and stand-in
 * headers are not allowed.  The restatement is pinned instead by (1) the published RFC 1071 and
 * RFC 1624 known-answer examples, (2) the reference-run facts SURVEY.md §8a records (closed form of
 * csum_replace2 over all 65 536 inputs, 0xF7FF -> 0x0000, never 0xFFFF, gate quirks), and (3) golden
 * frames whose expected outputs an independent numpy restatement produced (tests/golden/).
 * See DESIGN.md §Oracle.
 */
#ifndef ECHO_ORACLE_H
#define ECHO_ORACLE_H

#include <stdint.h>
#include "../include/xsk_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* csum_replace2 (xsk_receive.c:101-111), literal u16 restatement on the little-endian-loaded field. */
void oracle_csum_replace2(uint16_t* sum, uint16_t old, uint16_t new_);

/* process_packet (xsk_receive.c:113-157) minus logging and sendto: gates + in-place rewrite.
 * Returns an enum xsk_gpu_verdict (never DROP_BAD_DESC). */
int oracle_process_packet(uint8_t* pkt, uint32_t len);

/* RFC 1071 folded sum of big-endian 16-bit words over pkt[lo, hi), odd tail zero-padded. */
uint16_t oracle_fold_sum(const uint8_t* pkt, uint32_t lo, uint32_t hi);

/* Full contract of xsk_gpu_echo_dev() for one batch (xsk_receive.c:220-233 loop + records). */
void oracle_echo_batch(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n,
                       uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats);

/* Same, split over `threads` pthreads (contiguous frame ranges, per-thread counters). */
void oracle_echo_batch_mt(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n,
                          uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats, int threads);

/* Full contract of xsk_gpu_echo_dev_opts(): opts == 0 is oracle_echo_batch(); otherwise the wire-format
 * widening of include/xsk_gpu.h (XSK_GPU_OPT_*), build-added. */
void oracle_echo_batch_opts(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n,
                            uint32_t opts, uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats);
/* oracle_echo_batch_opts over `threads` pthreads (same bytes, verdicts, records and counters). */
void oracle_echo_batch_opts_mt(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n,
                               uint32_t opts, uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats,
                               int threads);

/* Reference-equivalent work only (gates + rewrite + counters; no full-payload sums, no records):
 * the CPU-baseline variant that does exactly what process_packet does. */
void oracle_echo_batch_hdr(uint8_t* umem, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                           struct xsk_gpu_stats* stats);
void oracle_echo_batch_hdr_mt(uint8_t* umem, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                              struct xsk_gpu_stats* stats, int threads);

/* Synthetic frames (bit-identical to xsk_gpu_synth_dev). Writes roundup16(max(len, 64)) bytes to
 * out (cap must be >= that); returns len, or 0xFFFFFFFF if it does not fit. */
uint32_t oracle_synth_frame(uint64_t seed, uint64_t gidx, int mode, uint32_t len_lo, uint32_t len_hi, uint8_t* out,
                            uint32_t cap);
int oracle_synth_batch(uint8_t* umem, uint64_t umem_size, struct xsk_gpu_desc* descs, uint32_t n, uint64_t base_off,
                       uint64_t stride, uint64_t seed, uint64_t first, uint64_t step, int mode, uint32_t len_lo,
                       uint32_t len_hi);
int oracle_synth_batch_mt(uint8_t* umem, uint64_t umem_size, struct xsk_gpu_desc* descs, uint32_t n, uint64_t base_off,
                          uint64_t stride, uint64_t seed, uint64_t first, uint64_t step, int mode, uint32_t len_lo,
                          uint32_t len_hi, int threads);

/* Re-arm (bit-identical to xsk_gpu_rearm_dev). */
void oracle_rearm(uint8_t* umem, const struct xsk_gpu_desc* descs, const uint8_t* verdicts, uint32_t n);

uint64_t oracle_mix64(uint64_t x);

/* xdp_sock_prog() of src/kern/inner_xdp.c:26-61 (the same tests as xdp_redirect() of
 * src/kern/phy_xdp.c:39-81) on one frame of `len` bytes: XDP_DROP (1) if len < 14 (:35-36),
 * XDP_PASS (2) if the ethertype is not IPv4 (:38-39), XDP_DROP if len < 34 (:41-42), XDP_PASS if the
 * IP protocol is not ICMP (:44-45), else XDP_REDIRECT (4) when a target is bound (xsks_map entry
 * :57-58 / devmap ifindex) and XDP_DROP when none is (:60). */
int oracle_xdp_classify(const uint8_t* pkt, uint32_t len, int target_bound);

/* Batch form: actions[n]; redirect[] receives the REDIRECT descriptors in order; returns their count.
 * A descriptor outside the UMEM is XDP_DROP (build-added: the kernel's data/data_end never are). */
uint32_t oracle_xdp_classify_batch(const uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs,
                                   uint32_t n, int target_bound, uint8_t* actions, struct xsk_gpu_desc* redirect);

#ifdef __cplusplus
}
#endif

#endif
