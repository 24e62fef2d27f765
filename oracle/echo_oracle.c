/*
 * echo_oracle.c — CPU oracle (plain C11) for the ICMP-echo frame transform.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg as the checker / CPU baseline; the product path (xsknet_amd/libxsknet_amd.so) never links it.
 *
 * Each function cites the reference line it restates.  Parity status: see echo_oracle.h (reference
 * unbuildable here: <xdp/xsk.h> absent; pinned by RFC 1071/1624 vectors, SURVEY.md §8a reference-run
 * facts, and independently computed golden frames).
 */
#define _GNU_SOURCE
#include "echo_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------------------------- */
/* The transform                                                                                  */
/* ---------------------------------------------------------------------------------------------- */

/* xsk_receive.c:101-111.  `sum` points at the little-endian load of bytes 36-37; arithmetic is u16
 * with C integer promotion, so `~old` is an int (-9 for old = 8) truncated back to u16 on `+=`. */
void oracle_csum_replace2(uint16_t* sum, uint16_t old, uint16_t new_) {
    uint16_t csum = (uint16_t)~*sum;
    csum = (uint16_t)(csum + (uint16_t)~old);
    csum = (uint16_t)(csum + (csum < (uint16_t)~old));
    csum = (uint16_t)(csum + new_);
    csum = (uint16_t)(csum + (csum < (uint16_t)new_));
    *sum = (uint16_t)~csum;
}

static inline uint16_t ld_le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline void st_le16(uint8_t* p, uint16_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
}
static inline uint16_t ld_be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline void st_be16(uint8_t* p, uint16_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

/* xsk_receive.c:113-157 without logging (:136,141,145,159-163) and sendto (:166).
 * Offsets: ethhdr @0 (14 B), iphdr @14 taken as 20 B regardless of IHL (:120), icmphdr @34 (:121). */
int oracle_process_packet(uint8_t* pkt, uint32_t len) {
    /* :123-133 — three independent checks; len < 20 subsumes them all. */
    if (len < 14) return XSK_GPU_DROP_SHORT;
    if (len < 20) return XSK_GPU_DROP_SHORT;
    if (len < 8) return XSK_GPU_DROP_SHORT;
    /* :135 ntohs(eth->h_proto) != ETH_P_IP */
    if (ld_be16(pkt + 12) != 0x0800) return XSK_GPU_DROP_NOT_IPV4;
    /* :140 ipv4->protocol != IPPROTO_ICMP */
    if (pkt[23] != 1) return XSK_GPU_DROP_NOT_ICMP;
    /* :144 icmp->type != ICMP_ECHO */
    if (pkt[34] != 8) return XSK_GPU_DROP_NOT_ECHO;
    /* :148-151 swap h_dest (0-5) and h_source (6-11) */
    uint8_t tmp[6];
    memcpy(tmp, pkt + 0, 6);
    memcpy(pkt + 0, pkt + 6, 6);
    memcpy(pkt + 6, tmp, 6);
    /* :153-155 swap saddr (26-29) and daddr (30-33) */
    uint8_t ip[4];
    memcpy(ip, pkt + 26, 4);
    memcpy(pkt + 26, pkt + 30, 4);
    memcpy(pkt + 30, ip, 4);
    /* :156 icmp->type = ICMP_ECHOREPLY */
    pkt[34] = 0;
    /* :157 csum_replace2(&icmp->checksum, ICMP_ECHO, ICMP_ECHOREPLY) on the LE-loaded u16 */
    uint16_t c = ld_le16(pkt + 36);
    oracle_csum_replace2(&c, 8, 0);
    st_le16(pkt + 36, c);
    return XSK_GPU_TX_REPLY;
}

/* RFC 1071 §4.1: sum big-endian 16-bit words, pad an odd tail with zero, fold carries. */
uint16_t oracle_fold_sum(const uint8_t* pkt, uint32_t lo, uint32_t hi) {
    uint64_t s = 0;
    uint32_t i = lo;
    for (; i + 1 < hi; i += 2) s += ld_be16(pkt + i);
    if (i < hi) s += (uint64_t)pkt[i] << 8;
    while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
    return (uint16_t)s;
}

static inline uint32_t u32min(uint32_t a, uint32_t b) { return a < b ? a : b; }

/* One frame of the full contract: verdict, record, in-place rewrite.  Descriptor validation is
 * build-added (the reference trusts the kernel's descriptors). */
static int echo_one(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* d, struct xsk_gpu_rec* rec) {
    const uint64_t addr = d->addr;
    const uint32_t len = d->len;
    struct xsk_gpu_rec r;
    memset(&r, 0, sizeof r);
    const uint64_t need = len >= 20 ? (len > 38 ? len : 38) : len;
    if (len > XSK_GPU_MAX_LEN || addr > umem_size || need > umem_size - addr) {
        r.verdict = XSK_GPU_DROP_BAD_DESC;
        if (rec) *rec = r;
        return XSK_GPU_DROP_BAD_DESC;
    }
    uint8_t* pkt = umem + addr;
    if (len >= 20) {
        /* Fields the reference reads (:135,:140,:144,:157), parsed before the rewrite. */
        r.eth_proto = ld_be16(pkt + 12);
        r.ip_vihl = pkt[14];
        r.ip_proto = pkt[23];
        r.icmp_type = pkt[34];
        r.icmp_code = pkt[35];
        r.icmp_csum_in = ld_be16(pkt + 36);
        r.ip_sum = oracle_fold_sum(pkt, 14, u32min(len, 34));
        r.icmp_sum = len > 34 ? oracle_fold_sum(pkt, 34, len) : 0;
        if (len >= 34 && r.ip_sum == 0xFFFF) r.flags |= XSK_GPU_F_IP_CSUM_OK;
        if (len >= 42 && r.icmp_sum == 0xFFFF) r.flags |= XSK_GPU_F_ICMP_CSUM_OK;
    }
    r.verdict = (uint8_t)oracle_process_packet(pkt, len);
    if (len >= 20) r.icmp_csum_out = ld_be16(pkt + 36);
    if (rec) *rec = r;
    return r.verdict;
}

/* The batch loop xsk_receive.c:220-233 with the counter updates of :171-172, :229, :233. */
void oracle_echo_batch(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n,
                       uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats) {
    uint64_t rxb = 0, txp = 0, txb = 0;
    for (uint32_t i = 0; i < n; i++) {
        const int v = echo_one(umem, umem_size, &descs[i], recs ? &recs[i] : NULL);
        if (verdicts) verdicts[i] = (uint8_t)v;
        if (v == XSK_GPU_TX_REPLY) {
            txp++;
            txb += descs[i].len;
        }
        rxb += descs[i].len;
    }
    if (stats) {
        stats->rx_packets += n;
        stats->rx_bytes += rxb;
        stats->tx_packets += txp;
        stats->tx_bytes += txb;
    }
}

void oracle_echo_batch_hdr(uint8_t* umem, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                           struct xsk_gpu_stats* stats) {
    uint64_t rxb = 0, txp = 0, txb = 0;
    for (uint32_t i = 0; i < n; i++) {
        const int v = oracle_process_packet(umem + descs[i].addr, descs[i].len);
        if (verdicts) verdicts[i] = (uint8_t)v;
        if (v == XSK_GPU_TX_REPLY) {
            txp++;
            txb += descs[i].len;
        }
        rxb += descs[i].len;
    }
    if (stats) {
        stats->rx_packets += n;
        stats->rx_bytes += rxb;
        stats->tx_packets += txp;
        stats->tx_bytes += txb;
    }
}

struct mt_job {
    uint8_t* umem;
    uint64_t umem_size;
    const struct xsk_gpu_desc* descs;
    uint32_t n;
    uint8_t* verdicts;
    struct xsk_gpu_rec* recs;
    struct xsk_gpu_stats st;
    int kind;      /* 0 full contract, 1 header-only, 2 wire mode (opts) */
    uint32_t opts;
};

static void* mt_worker(void* arg) {
    struct mt_job* j = (struct mt_job*)arg;
    if (j->kind == 1)
        oracle_echo_batch_hdr(j->umem, j->descs, j->n, j->verdicts, &j->st);
    else if (j->kind == 2)
        oracle_echo_batch_opts(j->umem, j->umem_size, j->descs, j->n, j->opts, j->verdicts, j->recs, &j->st);
    else
        oracle_echo_batch(j->umem, j->umem_size, j->descs, j->n, j->verdicts, j->recs, &j->st);
    return NULL;
}

/* Run jobs[0..threads) on `threads` threads: job 0 on the caller's thread, and any job whose thread cannot be
 * created inline on the caller's thread too; only the threads that started are joined. */
static void run_jobs(void* jobs, size_t job_size, int threads, void* (*fn)(void*)) {
    pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof *tids);
    int* started = (int*)calloc((size_t)threads, sizeof *started);
    for (int t = 1; t < threads; t++)
        started[t] = tids && started && pthread_create(&tids[t], NULL, fn, (char*)jobs + (size_t)t * job_size) == 0;
    for (int t = 0; t < threads; t++)
        if (!started || !started[t]) fn((char*)jobs + (size_t)t * job_size);
    for (int t = 1; t < threads; t++)
        if (started && started[t]) pthread_join(tids[t], NULL);
    free(tids);
    free(started);
}

static void run_mt(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                   struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats, int threads, int kind, uint32_t opts) {
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > n) threads = n ? (int)n : 1;
    struct mt_job* jobs = (struct mt_job*)calloc((size_t)threads, sizeof *jobs);
    if (!jobs) { /* no memory for the job table: one job on this thread */
        struct mt_job one = {umem, umem_size, descs, n, verdicts, recs, {0, 0, 0, 0, 0}, kind, opts};
        mt_worker(&one);
        if (stats) {
            stats->rx_packets += one.st.rx_packets;
            stats->rx_bytes += one.st.rx_bytes;
            stats->tx_packets += one.st.tx_packets;
            stats->tx_bytes += one.st.tx_bytes;
        }
        return;
    }
    uint32_t start = 0;
    for (int t = 0; t < threads; t++) {
        const uint32_t cnt = n / threads + ((uint32_t)t < n % threads ? 1 : 0);
        jobs[t].umem = umem;
        jobs[t].umem_size = umem_size;
        jobs[t].descs = descs + start;
        jobs[t].n = cnt;
        jobs[t].verdicts = verdicts ? verdicts + start : NULL;
        jobs[t].recs = recs ? recs + start : NULL;
        jobs[t].kind = kind;
        jobs[t].opts = opts;
        start += cnt;
    }
    run_jobs(jobs, sizeof *jobs, threads, mt_worker);
    if (stats) {
        for (int t = 0; t < threads; t++) {
            stats->rx_packets += jobs[t].st.rx_packets;
            stats->rx_bytes += jobs[t].st.rx_bytes;
            stats->tx_packets += jobs[t].st.tx_packets;
            stats->tx_bytes += jobs[t].st.tx_bytes;
        }
    }
    free(jobs);
}

void oracle_echo_batch_mt(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n,
                          uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats, int threads) {
    run_mt(umem, umem_size, descs, n, verdicts, recs, stats, threads, 0, 0);
}

void oracle_echo_batch_hdr_mt(uint8_t* umem, const struct xsk_gpu_desc* descs, uint32_t n, uint8_t* verdicts,
                              struct xsk_gpu_stats* stats, int threads) {
    run_mt(umem, 0, descs, n, verdicts, NULL, stats, threads, 1, 0);
}

/* ---------------------------------------------------------------------------------------------- */
/* Synthetic frames: counter-based, so any CPU or GPU regenerates any frame.       */
/* ---------------------------------------------------------------------------------------------- */

/* splitmix64 output function. */
uint64_t oracle_mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static const uint32_t k_short_lens[13] = {0, 1, 13, 14, 19, 20, 21, 33, 34, 37, 38, 41, 42};

static inline uint8_t byte_of(uint64_t v, int i) { return (uint8_t)(v >> (8 * i)); }

/* Frame gidx of a stream: K = mix64(seed ^ mix64(gidx)); header randomness r_k = mix64(K + k),
 * k = 1..5; fill byte at frame offset o = byte (o & 7) of mix64(K + 16 + (o >> 3)).
 * Mixed mode picks a case s = (r4 >> 32) % 20 (0-5 valid; see the switch below). */
uint32_t oracle_synth_frame(uint64_t seed, uint64_t gidx, int mode, uint32_t len_lo, uint32_t len_hi, uint8_t* out,
                            uint32_t cap) {
    const uint64_t K = oracle_mix64(seed ^ oracle_mix64(gidx));
    const uint64_t r1 = oracle_mix64(K + 1), r2 = oracle_mix64(K + 2), r3 = oracle_mix64(K + 3);
    const uint64_t r4 = oracle_mix64(K + 4), r5 = oracle_mix64(K + 5);
    uint32_t L = len_lo == len_hi ? len_lo : len_lo + (uint32_t)(r5 % (uint64_t)(len_hi - len_lo + 1));
    const uint32_t s = mode == 1 ? (uint32_t)(r4 >> 32) % 20u : 0u;
    if (s == 18) L = k_short_lens[(r5 >> 40) % 13];
    const uint32_t W = ((L > 64 ? L : 64) + 15u) & ~15u; /* fill extent: whole 16-B blocks */
    if (W > cap) return 0xFFFFFFFFu;
    for (uint32_t o = 0; o < W; o += 8) { /* W is a multiple of 16 */
        const uint64_t v = oracle_mix64(K + 16 + (o >> 3));
        for (int i = 0; i < 8; i++) out[o + (uint32_t)i] = byte_of(v, i);
    }
    if (s == 19) return L; /* garbage frame: fill pattern only */
    uint8_t* p = out;
    for (int i = 0; i < 6; i++) p[i] = byte_of(r1, i);
    for (int i = 0; i < 6; i++) p[6 + i] = byte_of(r2, i);
    st_be16(p + 12, s == 6 ? 0x86DD : s == 7 ? 0x8100 : 0x0800);
    p[14] = s == 12 ? 0x46 : s == 13 ? 0x65 : 0x45;
    p[15] = 0;
    st_be16(p + 16, (uint16_t)(L >= 14 ? L - 14 : 0));
    p[18] = byte_of(r2, 6);
    p[19] = byte_of(r2, 7);
    st_be16(p + 20, s == 14 ? 0x2000 : 0x4000);
    p[22] = 64;
    p[23] = s == 8 ? 6 : 1;
    p[24] = p[25] = 0;
    for (int i = 0; i < 8; i++) p[26 + i] = byte_of(r3, i);
    p[34] = s == 9 ? 0 : s == 10 ? 13 : 8;
    p[35] = s == 11 ? 5 : 0;
    p[36] = p[37] = 0;
    for (int i = 0; i < 4; i++) p[38 + i] = byte_of(r4, i);
    if (s == 17) { /* all-zero ICMP echo: id, seq and payload zero -> checksum 0xF7FF */
        for (uint32_t o = 38; o < L; o++) p[o] = 0;
    }
    uint16_t ipc = (uint16_t)~oracle_fold_sum(p, 14, 34);
    if (s == 16) ipc ^= 0x5A5A;
    st_be16(p + 24, ipc);
    uint16_t icc = (uint16_t)~oracle_fold_sum(p, 34, L > 34 ? L : 34);
    if (s == 15) icc ^= 0x1234;
    st_be16(p + 36, icc);
    return L;
}

int oracle_synth_batch(uint8_t* umem, uint64_t umem_size, struct xsk_gpu_desc* descs, uint32_t n, uint64_t base_off,
                       uint64_t stride, uint64_t seed, uint64_t first, uint64_t step, int mode, uint32_t len_lo,
                       uint32_t len_hi) {
    for (uint32_t j = 0; j < n; j++) {
        const uint64_t addr = base_off + (uint64_t)j * stride;
        if (addr >= umem_size) return -1;
        const uint64_t room = umem_size - addr;
        const uint32_t cap = (uint32_t)(room < stride ? room : stride);
        const uint32_t L = oracle_synth_frame(seed, first + (uint64_t)j * step, mode, len_lo, len_hi, umem + addr, cap);
        if (L == 0xFFFFFFFFu) return -1;
        descs[j].addr = addr;
        descs[j].len = L;
        descs[j].options = 0;
    }
    return 0;
}

/* oracle_synth_batch over `threads` pthreads (contiguous frame ranges; same bytes). */
struct synth_job {
    uint8_t* umem;
    uint64_t umem_size;
    struct xsk_gpu_desc* descs;
    uint32_t j0, n;
    uint64_t base_off, stride, seed, first, step;
    int mode;
    uint32_t len_lo, len_hi;
    int rc;
};

static void* synth_worker(void* arg) {
    struct synth_job* j = (struct synth_job*)arg;
    j->rc = oracle_synth_batch(j->umem, j->umem_size, j->descs + j->j0, j->n, j->base_off + (uint64_t)j->j0 * j->stride,
                               j->stride, j->seed, j->first + (uint64_t)j->j0 * j->step, j->step, j->mode, j->len_lo,
                               j->len_hi);
    return NULL;
}

int oracle_synth_batch_mt(uint8_t* umem, uint64_t umem_size, struct xsk_gpu_desc* descs, uint32_t n, uint64_t base_off,
                          uint64_t stride, uint64_t seed, uint64_t first, uint64_t step, int mode, uint32_t len_lo,
                          uint32_t len_hi, int threads) {
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > n) threads = n ? (int)n : 1;
    struct synth_job* jobs = (struct synth_job*)calloc((size_t)threads, sizeof *jobs);
    if (!jobs)
        return oracle_synth_batch(umem, umem_size, descs, n, base_off, stride, seed, first, step, mode, len_lo, len_hi);
    uint32_t start = 0;
    for (int t = 0; t < threads; t++) {
        const uint32_t cnt = n / threads + ((uint32_t)t < n % threads ? 1 : 0);
        struct synth_job jb = {umem, umem_size, descs, start, cnt, base_off, stride, seed, first, step, mode, len_lo,
                               len_hi, 0};
        jobs[t] = jb;
        start += cnt;
    }
    run_jobs(jobs, sizeof *jobs, threads, synth_worker);
    int rc = 0;
    for (int t = 0; t < threads; t++)
        if (jobs[t].rc) rc = jobs[t].rc;
    free(jobs);
    return rc;
}

/* Undo one echo transform on TX_REPLY frames: swap back and csum_replace2(csum, 0, 8). */
void oracle_rearm(uint8_t* umem, const struct xsk_gpu_desc* descs, const uint8_t* verdicts, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        if (verdicts[i] != XSK_GPU_TX_REPLY) continue;
        uint8_t* p = umem + descs[i].addr;
        uint8_t tmp[6];
        memcpy(tmp, p, 6);
        memcpy(p, p + 6, 6);
        memcpy(p + 6, tmp, 6);
        uint8_t ip[4];
        memcpy(ip, p + 26, 4);
        memcpy(p + 26, p + 30, 4);
        memcpy(p + 30, ip, 4);
        p[34] = 8;
        uint16_t c = ld_le16(p + 36);
        oracle_csum_replace2(&c, 0, 8);
        st_le16(p + 36, c);
    }
}

/* ---------------------------------------------------------------------------------------------- */
/* Wire-format widening (build-added, the reference has no such mode).        */
/* The spec is include/xsk_gpu.h (XSK_GPU_OPT_*); the rewrite itself is process_packet's           */
/* (xsk_receive.c:148-157) at the parsed offsets.                                                   */
/* ---------------------------------------------------------------------------------------------- */

/* One frame in wire mode.  Returns the verdict; fills *r (zeroed first) and rewrites TX_REPLY frames. */
static int wire_one(uint8_t* p, uint32_t len, uint32_t opts, struct xsk_gpu_rec* r) {
    memset(r, 0, sizeof *r);
    if (len < 14) return XSK_GPU_DROP_SHORT;
    uint32_t l3 = 14;
    uint16_t et = ld_be16(p + 12);
    int tags = 0;
    if (opts & XSK_GPU_OPT_VLAN) {
        while (tags < 2 && (et == 0x8100 || et == 0x88A8)) { /* 802.1Q / 802.1ad tag: TPID, TCI */
            if (len < l3 + 4) return XSK_GPU_DROP_SHORT;
            et = ld_be16(p + l3 + 2);
            l3 += 4;
            tags++;
        }
    }
    if (et != 0x0800) return XSK_GPU_DROP_NOT_IPV4;
    if (len < l3 + 20) return XSK_GPU_DROP_SHORT;
    uint32_t hl = 20, end = len;
    if (opts & XSK_GPU_OPT_STRICT_IPV4) {
        const uint8_t vihl = p[l3];
        if ((vihl >> 4) != 4 || (vihl & 15) < 5) return XSK_GPU_DROP_BAD_IP;
        hl = 4u * (vihl & 15u);
        const uint32_t tot = ld_be16(p + l3 + 2);
        if (tot < hl + 8 || l3 + tot > len) return XSK_GPU_DROP_BAD_IP; /* also covers len < l3 + hl + 8 */
        if (ld_be16(p + l3 + 6) & 0x3FFF) return XSK_GPU_DROP_BAD_IP;  /* MF set or fragment offset != 0 */
        end = l3 + tot;                                                 /* Ethernet padding excluded */
    }
    if (p[l3 + 9] != 1) return XSK_GPU_DROP_NOT_ICMP;
    const uint32_t l4 = l3 + hl;
    if (len < l4 + 8) return XSK_GPU_DROP_SHORT;
    /* every header lies inside the frame from here on: the record is filled */
    r->eth_proto = et;
    r->ip_vihl = p[l3];
    r->ip_proto = p[l3 + 9];
    r->icmp_type = p[l4];
    r->icmp_code = p[l4 + 1];
    r->icmp_csum_in = ld_be16(p + l4 + 2);
    r->ip_sum = oracle_fold_sum(p, l3, l3 + hl);
    r->icmp_sum = oracle_fold_sum(p, l4, end);
    if (r->ip_sum == 0xFFFF) r->flags |= XSK_GPU_F_IP_CSUM_OK;
    if (r->icmp_sum == 0xFFFF) r->flags |= XSK_GPU_F_ICMP_CSUM_OK;
    if (tags) r->flags |= XSK_GPU_F_VLAN;
    if (hl > 20) r->flags |= XSK_GPU_F_IP_OPTIONS;
    int v;
    if (p[l4] != 8 || ((opts & XSK_GPU_OPT_STRICT_IPV4) && p[l4 + 1] != 0)) v = XSK_GPU_DROP_NOT_ECHO;
    else if ((opts & XSK_GPU_OPT_VERIFY_CSUM) && (r->ip_sum != 0xFFFF || r->icmp_sum != 0xFFFF)) v = XSK_GPU_DROP_BAD_CSUM;
    else v = XSK_GPU_TX_REPLY;
    if (v == XSK_GPU_TX_REPLY) { /* xsk_receive.c:148-157 at the parsed offsets */
        uint8_t tmp[6];
        memcpy(tmp, p, 6);
        memcpy(p, p + 6, 6);
        memcpy(p + 6, tmp, 6);
        uint8_t ip[4];
        memcpy(ip, p + l3 + 12, 4);
        memcpy(p + l3 + 12, p + l3 + 16, 4);
        memcpy(p + l3 + 16, ip, 4);
        p[l4] = 0;
        uint16_t c = ld_le16(p + l4 + 2);
        oracle_csum_replace2(&c, 8, 0);
        st_le16(p + l4 + 2, c);
    }
    r->verdict = (uint8_t)v;
    r->icmp_csum_out = ld_be16(p + l4 + 2);
    return v;
}

void oracle_echo_batch_opts(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n,
                            uint32_t opts, uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats) {
    if (opts == 0) {
        oracle_echo_batch(umem, umem_size, descs, n, verdicts, recs, stats);
        return;
    }
    uint64_t rxb = 0, txp = 0, txb = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t a = descs[i].addr;
        const uint32_t len = descs[i].len;
        struct xsk_gpu_rec r;
        int v;
        if (len > XSK_GPU_MAX_LEN || a > umem_size || len > umem_size - a) { /* wire mode reads [addr, addr+len) */
            memset(&r, 0, sizeof r);
            v = XSK_GPU_DROP_BAD_DESC;
            r.verdict = (uint8_t)v;
        } else {
            v = wire_one(umem + a, len, opts, &r);
            r.verdict = (uint8_t)v;
        }
        if (recs) recs[i] = r;
        if (verdicts) verdicts[i] = (uint8_t)v;
        if (v == XSK_GPU_TX_REPLY) {
            txp++;
            txb += len;
        }
        rxb += len;
    }
    if (stats) {
        stats->rx_packets += n;
        stats->rx_bytes += rxb;
        stats->tx_packets += txp;
        stats->tx_bytes += txb;
    }
}

/* oracle_echo_batch_opts over `threads` pthreads (contiguous descriptor ranges; frames never overlap). */
void oracle_echo_batch_opts_mt(uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs, uint32_t n,
                               uint32_t opts, uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats,
                               int threads) {
    run_mt(umem, umem_size, descs, n, verdicts, recs, stats, threads, 2, opts);
}

/* ---------------------------------------------------------------------------------------------- */
/* XDP ingress filter (src/kern/inner_xdp.c:26-61; phy_xdp.c:39-81 applies the same tests)         */
/* ---------------------------------------------------------------------------------------------- */

int oracle_xdp_classify(const uint8_t* pkt, uint32_t len, int target_bound) {
    if (len < 14) return 1;                  /* OVER(eth, data_end) -> XDP_DROP, :35-36            */
    if (ld_be16(pkt + 12) != 0x0800) return 2; /* eth->h_proto != htons(ETH_P_IP) -> XDP_PASS, :38 */
    if (len < 34) return 1;                  /* OVER(iph, data_end) -> XDP_DROP, :41-42            */
    if (pkt[23] != 1) return 2;              /* iph->protocol != IPPROTO_ICMP -> XDP_PASS, :44-45  */
    return target_bound ? 4 : 1;             /* bpf_redirect_map if the queue is bound, :57-60     */
}

uint32_t oracle_xdp_classify_batch(const uint8_t* umem, uint64_t umem_size, const struct xsk_gpu_desc* descs,
                                   uint32_t n, int target_bound, uint8_t* actions, struct xsk_gpu_desc* redirect) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t a = descs[i].addr;
        const uint32_t len = descs[i].len;
        const uint32_t need = len < 34 ? (len < 14 ? 0 : 14) : 34;
        int act;
        if (len > XSK_GPU_MAX_LEN || a > umem_size || need > umem_size - a) act = 1;
        else act = oracle_xdp_classify(umem + a, len, target_bound);
        actions[i] = (uint8_t)act;
        if (act == 4) redirect[k++] = descs[i];
    }
    return k;
}
