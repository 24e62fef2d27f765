/*
 * echo_replay.c — C driver that replays a UMEM image through the GPU echo transform batch by
 * batch, the way the reference client's RX loop does (src/lib/xsk_receive.c:192-237), with the
 * per-descriptor process_packet() call replaced by one xsk_gpu_process() per batch.
 *
 *   echo_replay <umem.bin> <descs.bin> <out_umem.bin> <out_verdicts.bin> [batch] [zerocopy|staged|lowlat]
 *               [gpus=D0,D1,...] [reps=R] [flush=1] [huge=1] [opts=O]
 *
 * With gpus=..., the batches go through xsk_gpu_multi_process() over one context per listed device
 * (repeats allowed): descriptor i of a batch on context i mod G, counters summed on the host.
 * With reps=R (R >= 1), the replay is timed: R passes over the image, the UMEM restored from the input
 * between passes (untimed), and one more key=value pair, us_per_call (wall clock per batch call, the
 * first pass -- which starts the device side -- excluded), is printed; the outputs are those of pass 1.
 * flush=1 evicts the restored UMEM from the CPU caches before each timed pass (frames a NIC delivered);
 * huge=1 puts the UMEM on transparent huge pages.  opts=O sets the wire-format options (XSK_GPU_OPT_*, include/xsk_gpu.h)
 * with xsk_gpu_set_options() / xsk_gpu_multi_set_options() before the first batch.
 *
 * umem.bin: raw UMEM bytes (size multiple of 16).  descs.bin: packed struct xdp_desc records
 * (u64 addr, u32 len, u32 options).  Prints the stats_record counters the reference's stats
 * thread would print (src/lib/xsk_stats.c:37-68) as one line of key=value pairs.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "../include/xsk_gpu.h"

#define RX_BATCH_SIZE 64 /* src/lib/xsk_utils.h:8 */

/* diagnostics hook of libxsknet_amd (not in the public header): LOWLAT phase durations, ns */
int xsk_gpu__lowlat_trace(xsk_gpu_ctx* ctx, uint64_t out_ns[15]);
int xsk_gpu__lowlat_tune(xsk_gpu_ctx* ctx, uint32_t tile_frames, uint32_t groups, uint32_t timeout_us);



static void* slurp(const char* path, size_t* size, size_t align) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void* buf = NULL;
    if (n < 0 || posix_memalign(&buf, align, n > 0 ? (size_t)n : align) != 0) {
        fclose(f);
        return NULL;
    }
    if (n > 0 && fread(buf, 1, (size_t)n, f) != (size_t)n) {
        free(buf);
        fclose(f);
        return NULL;
    }
    fclose(f);
    *size = (size_t)n;
    return buf;
}

/* The UMEM on transparent huge pages (huge=1): 2-MiB aligned anonymous memory with MADV_HUGEPAGE, filled
 * from the image.  AF_XDP accepts any page-aligned UMEM; the reference uses posix_memalign(getpagesize())
 * (xsk_utils.c:135), i.e. 4-KiB pages, whose translations the GPU walks one page per frame. */
static uint8_t* huge_copy(const uint8_t* src, size_t n) {
    const size_t len = (n + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    void* p = mmap(NULL, len + (2u << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return NULL;
    uint8_t* a = (uint8_t*)(((uintptr_t)p + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1));
    madvise(a, len, MADV_HUGEPAGE);
    memcpy(a, src, n);
    return a;
}

/* AnonHugePages (KiB) of the mapping holding p (/proc/self/smaps): whether the kernel did back it with huge pages */
static long huge_kb_at(const void* p) {
    FILE* f = fopen("/proc/self/smaps", "r");
    if (!f) return -1;
    char line[512];
    int in = 0;
    long kb = -1;
    while (fgets(line, sizeof line, f)) {
        unsigned long lo = 0, hi = 0;
        if (sscanf(line, "%lx-%lx ", &lo, &hi) == 2) {
            in = (uintptr_t)p >= lo && (uintptr_t)p < hi;
            continue;
        }
        if (in && sscanf(line, "AnonHugePages: %ld kB", &kb) == 1) break;
    }
    fclose(f);
    return kb;
}

static int dump(const char* path, const void* p, size_t n) {
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    const size_t w = fwrite(p, 1, n, f);
    fclose(f);
    return w == n ? 0 : -1;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr,
                "usage: %s umem.bin descs.bin out_umem.bin out_verdicts.bin [batch] [zerocopy|staged|lowlat] "
                "[gpus=D0,D1,...]\n",
                argv[0]);
        return 2;
    }
    const uint32_t batch = argc > 5 ? (uint32_t)strtoul(argv[5], NULL, 10) : RX_BATCH_SIZE;
    int mode = XSK_GPU_MODE_ZEROCOPY;
    if (argc > 6 && strcmp(argv[6], "staged") == 0) mode = XSK_GPU_MODE_STAGED;
    if (argc > 6 && strcmp(argv[6], "lowlat") == 0) mode = XSK_GPU_MODE_LOWLAT;
    int devices[XSK_GPU_MULTI_MAX];
    uint32_t ndev = 0, reps = 0, flush = 0, huge = 0, tile = 0, groups = 0, opts = 0;
    for (int a = 7; a < argc; a++) {
        if (strncmp(argv[a], "gpus=", 5) == 0) {
            for (char* p = argv[a] + 5; *p && ndev < XSK_GPU_MULTI_MAX;) {
                devices[ndev++] = (int)strtol(p, &p, 10);
                if (*p == ',') p++;
                else break;
            }
        } else if (strncmp(argv[a], "reps=", 5) == 0) {
            reps = (uint32_t)strtoul(argv[a] + 5, NULL, 10);
        } else if (strncmp(argv[a], "flush=", 6) == 0) {
            flush = (uint32_t)strtoul(argv[a] + 6, NULL, 10);
        } else if (strncmp(argv[a], "huge=", 5) == 0) {
            huge = (uint32_t)strtoul(argv[a] + 5, NULL, 10);
        } else if (strncmp(argv[a], "tile=", 5) == 0) { /* LOWLAT: frames per wave (tools/hostlat.py --tiles) */
            tile = (uint32_t)strtoul(argv[a] + 5, NULL, 10);
        } else if (strncmp(argv[a], "groups=", 7) == 0) { /* LOWLAT: serving workgroups (--groups) */
            groups = (uint32_t)strtoul(argv[a] + 7, NULL, 10);
        } else if (strncmp(argv[a], "opts=", 5) == 0) { /* wire-format options (--opts) */
            opts = (uint32_t)strtoul(argv[a] + 5, NULL, 10);
        }
    }
    size_t umem_size = 0, desc_bytes = 0;
    /* page-aligned like the reference's posix_memalign(getpagesize(), ...) (xsk_utils.c:135) */
    uint8_t* umem = (uint8_t*)slurp(argv[1], &umem_size, 4096);
    struct xsk_gpu_desc* descs = (struct xsk_gpu_desc*)slurp(argv[2], &desc_bytes, 16);
    if (!umem || !descs || batch == 0) {
        fprintf(stderr, "cannot read inputs\n");
        return 1;
    }
    if (huge) {
        uint8_t* h = huge_copy(umem, umem_size);
        if (!h) {
            fprintf(stderr, "huge-page UMEM: mmap failed\n");
            return 1;
        }
        free(umem);
        umem = h; /* (never freed: the process ends) */
    }
    const uint32_t n = (uint32_t)(desc_bytes / sizeof *descs);
    uint8_t* verdicts = (uint8_t*)calloc(n ? n : 1, 1);
    uint8_t* scratch = (uint8_t*)calloc(n ? n : 1, 1);
    uint8_t *pristine = NULL, *out1 = NULL;
    if (reps) {
        pristine = (uint8_t*)malloc(umem_size ? umem_size : 1);
        out1 = (uint8_t*)malloc(umem_size ? umem_size : 1);
        if (!pristine || !out1) return 1;
        memcpy(pristine, umem, umem_size);
    }

    xsk_gpu_ctx* ctx = NULL;
    xsk_gpu_multi* multi = NULL;
    int rc = ndev ? xsk_gpu_multi_init(&multi, devices, ndev, umem, umem_size, batch, mode)
                  : xsk_gpu_init(&ctx, 0, umem, umem_size, batch, mode);
    if (rc) {
        fprintf(stderr, "init: %s (%s)\n", strerror(-rc), xsk_gpu_last_error());
        return 1;
    }
    if (opts && (rc = multi ? xsk_gpu_multi_set_options(multi, opts) : xsk_gpu_set_options(ctx, opts))) {
        fprintf(stderr, "options: %s\n", strerror(-rc));
        return 1;
    }
    if ((tile || groups) && ctx && mode == XSK_GPU_MODE_LOWLAT && (rc = xsk_gpu__lowlat_tune(ctx, tile, groups, 0))) {
        fprintf(stderr, "lowlat tune: %s\n", strerror(-rc));
        return 1;
    }
    struct xsk_gpu_stats stats, st_rep;
    memset(&stats, 0, sizeof stats);
    uint64_t freed = 0, tx_ready = 0, timed_calls = 0;
    double timed_s = 0.0;
    const uint32_t passes = reps ? reps : 1;
    for (uint32_t pass = 0; pass < passes; pass++) {
        if (pass) { /* untimed: the frames are requests again */
            memcpy(umem, pristine, umem_size);
            /* flush=1: out of the CPU caches, as frames a NIC wrote by DMA would be (a PCIe read of a line
               dirty in a core's cache waits for the snoop) */
            if (flush)
                for (size_t o = 0; o < umem_size; o += 64) __builtin_ia32_clflush(umem + o);
        }
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        /* handle_receive_packets(): one RX peek of <= batch descriptors per iteration */
        for (uint32_t i = 0; i < n; i += batch) {
            const uint32_t rcvd = n - i < batch ? n - i : batch;
            rc = multi ? xsk_gpu_multi_process(multi, descs + i, rcvd, (pass ? scratch : verdicts) + i, NULL,
                                               pass ? &st_rep : &stats)
                       : xsk_gpu_process(ctx, descs + i, rcvd, (pass ? scratch : verdicts) + i, NULL,
                                         pass ? &st_rep : &stats);
            if (rc) {
                fprintf(stderr, "process: %s (%s)\n", strerror(-rc), xsk_gpu_last_error());
                xsk_gpu_multi_fini(multi);
                xsk_gpu_fini(ctx);
                return 1;
            }
            if (pass) continue;
            /* the reference sendto()s TX_REPLY frames, then frees every frame (:166, :226-227) */
            for (uint32_t k = 0; k < rcvd; k++) {
                if (verdicts[i + k] == XSK_GPU_TX_REPLY) tx_ready++;
                freed++;
            }
        }
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if (pass == 0 && reps) memcpy(out1, umem, umem_size);
        if (pass > 0) {
            timed_s += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
            timed_calls += (n + batch - 1) / batch;
        }
    }
    if (reps) memcpy(umem, out1, umem_size);
    uint64_t tr[15] = {0};
    const int have_trace = ctx && mode == XSK_GPU_MODE_LOWLAT && xsk_gpu__lowlat_trace(ctx, tr) == 0;
    xsk_gpu_multi_fini(multi);
    xsk_gpu_fini(ctx);
    if (dump(argv[3], umem, umem_size) || dump(argv[4], verdicts, n)) {
        fprintf(stderr, "cannot write outputs\n");
        return 1;
    }
    printf("rx_packets=%llu rx_bytes=%llu tx_packets=%llu tx_bytes=%llu freed=%llu tx_ready=%llu",
           (unsigned long long)stats.rx_packets, (unsigned long long)stats.rx_bytes,
           (unsigned long long)stats.tx_packets, (unsigned long long)stats.tx_bytes, (unsigned long long)freed,
           (unsigned long long)tx_ready);
    if (timed_calls) printf(" us_per_call=%.3f calls=%llu", timed_s / (double)timed_calls * 1e6,
                            (unsigned long long)timed_calls);
    if (huge) printf(" huge_kb=%ld", huge_kb_at(umem));
    if (have_trace) {
        printf(" trace_ns=");
        for (int i = 0; i < 15; i++) printf("%s%llu", i ? "," : "", (unsigned long long)tr[i]);
    }
    printf("\n");
    if (!huge) free(umem);
    free(descs);
    free(verdicts);
    free(scratch);
    free(pristine);
    free(out1);
    return 0;
}
