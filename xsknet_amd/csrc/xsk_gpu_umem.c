/*
 * xsk_gpu_umem.c — a UMEM allocation for the host modes: what the reference's init_xsk_socket() gets from
 * posix_memalign(&buffer, getpagesize(), NUM_FRAMES * FRAME_SIZE) (src/lib/xsk_utils.c:132-135), but 2 MiB aligned and
 * advised onto transparent huge pages, and touched up front so the pages exist before the socket registers them.
 * The GPU reads a host-UMEM batch's frames through its own translations; on 4 KiB pages a 64-frame batch of frames one
 * per chunk walks 64 of them.  Measured through the resident kernel (tools/hostlat.py, profiles/r05/hostlat_pages.jsonl):
 * 64 x 64 B 8.8 -> 7.2 us per call, 1024 x 64 B scattered 17.8 -> 12.9, 64 x 1500 B 17.7 -> 15.9.  Host code (C11).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include "xsk_gpu_internal.h"

#define HUGE_2M ((uint64_t)2 << 20)

/* AnonHugePages of the mapping that holds p, in bytes (/proc/self/smaps), or 0 when unknown. */
static uint64_t huge_bytes_at(const void* p) {
    FILE* f = fopen("/proc/self/smaps", "r");
    if (!f) return 0;
    char line[512];
    int in = 0;
    long kb = 0;
    while (fgets(line, sizeof line, f)) {
        unsigned long lo = 0, hi = 0;
        if (sscanf(line, "%lx-%lx ", &lo, &hi) == 2) {
            in = (uintptr_t)p >= lo && (uintptr_t)p < hi;
            continue;
        }
        if (in && sscanf(line, "AnonHugePages: %ld kB", &kb) == 1) break;
    }
    fclose(f);
    return kb > 0 ? (uint64_t)kb << 10 : 0;
}

int xsk_gpu_umem_alloc(void** out, uint64_t size, uint64_t* huge_bytes) {
    if (huge_bytes) *huge_bytes = 0;
    if (!out || size == 0 || (size & 15u) || size > ((uint64_t)1 << 46)) return -EINVAL;
    *out = NULL;
    const uint64_t len = (size + HUGE_2M - 1) & ~(HUGE_2M - 1);
    /* over-allocate by one huge page to align, then give the slack back */
    uint8_t* p = (uint8_t*)mmap(NULL, len + HUGE_2M, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return -ENOMEM;
    uint8_t* a = (uint8_t*)(((uintptr_t)p + HUGE_2M - 1) & ~(uintptr_t)(HUGE_2M - 1));
    if (a > p) munmap(p, (size_t)(a - p));
    if (a + len < p + len + HUGE_2M) munmap(a + len, (size_t)(p + len + HUGE_2M - (a + len)));
    (void)madvise(a, len, MADV_HUGEPAGE); /* advice: a kernel without THP leaves 4 KiB pages */
    memset(a, 0, len);                     /* fault every page in now, as huge pages where the kernel gives them */
    *out = a;
    if (huge_bytes) *huge_bytes = huge_bytes_at(a);
    return 0;
}

void xsk_gpu_umem_free(void* umem, uint64_t size) {
    if (!umem || size == 0) return;
    munmap(umem, (size_t)((size + HUGE_2M - 1) & ~(HUGE_2M - 1)));
}
