/* CPU unit test of the host memory bookkeeping (xsknet_amd/csrc/xsk_gpu_mem.c): the counted table of UMEM registrations
 * and the buffers kept for reuse while a resident LOWLAT grid runs. The HIP runtime calls are stubs that behave as the
 * runtime was measured to (tools/doublereg_probe.py, profiles/r06/doublereg_attributes.jsonl): one registration per
 * base address, a second hipHostRegister of a registered base a silent success, the first hipHostUnregister removing
 * it, hipPointerGetAttributes reporting any address inside a registration as host memory. Checked: one runtime
 * registration per UMEM however many users, parts of a UMEM sharing its registration, -EBUSY for a range overlapping
 * one without lying inside it, a caller's own registration left alone, the table's limit; buffers kept only while the
 * device is busy, reused by exact (device, kind, size), host ones zeroed on reuse, the 256-buffer and 8-GiB limits,
 * everything freed once the device is idle; and, on 8 threads, that no user ever finds its UMEM unregistered while it
 * holds a reference and that every registration and buffer is released at the end. Built and run by
 * tests/test_mem_c.py. */
#include <assert.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../xsknet_amd/csrc/xsk_gpu_mem.c"

/* ---- the runtime, as measured ---- */
#define RT_MAX 4096
static pthread_mutex_t rt_mu = PTHREAD_MUTEX_INITIALIZER;
static struct {
    uintptr_t base;
    size_t size;
} rt_reg[RT_MAX];
static int rt_n;
static atomic_long rt_registers, rt_unregisters, live_dev, live_host;

static int rt_find_base(uintptr_t b) {
    for (int i = 0; i < rt_n; i++)
        if (rt_reg[i].base == b) return i;
    return -1;
}
/* 1 when [p, p + n) lies inside one runtime registration */
static int rt_covers(const void* p, size_t n) {
    pthread_mutex_lock(&rt_mu);
    int ok = 0;
    for (int i = 0; i < rt_n && !ok; i++)
        ok = rt_reg[i].base <= (uintptr_t)p && (uintptr_t)p + n <= rt_reg[i].base + rt_reg[i].size;
    pthread_mutex_unlock(&rt_mu);
    return ok;
}
hipError_t hipHostRegister(void* p, size_t n, unsigned int f) {
    (void)f;
    pthread_mutex_lock(&rt_mu);
    if (rt_find_base((uintptr_t)p) < 0) { /* a second registration of a base: success, nothing changes */
        assert(rt_n < RT_MAX);
        rt_reg[rt_n].base = (uintptr_t)p;
        rt_reg[rt_n].size = n;
        rt_n++;
    }
    pthread_mutex_unlock(&rt_mu);
    atomic_fetch_add(&rt_registers, 1);
    return hipSuccess;
}
hipError_t hipHostUnregister(void* p) {
    pthread_mutex_lock(&rt_mu);
    const int i = rt_find_base((uintptr_t)p);
    if (i >= 0) rt_reg[i] = rt_reg[--rt_n];
    pthread_mutex_unlock(&rt_mu);
    atomic_fetch_add(&rt_unregisters, 1);
    return i >= 0 ? hipSuccess : hipErrorHostMemoryNotRegistered;
}
hipError_t hipPointerGetAttributes(hipPointerAttribute_t* a, const void* p) {
    memset(a, 0, sizeof *a);
    a->type = rt_covers(p, 1) ? hipMemoryTypeHost : hipMemoryTypeUnregistered;
    return hipSuccess;
}
hipError_t hipGetLastError(void) { return hipSuccess; }

/* device buffers are never touched through their pointer here: sizes above 1 MiB get a unique fake address */
static atomic_uintptr_t fake_next = 0x7f0000000000ull;
hipError_t hipMalloc(void** p, size_t n) {
    *p = n > (1u << 20) ? (void*)atomic_fetch_add(&fake_next, (uintptr_t)n + 4096u) : malloc(n ? n : 1);
    atomic_fetch_add(&live_dev, 1);
    return hipSuccess;
}
hipError_t hipFree(void* p) {
    if ((uintptr_t)p < 0x7f0000000000ull || (uintptr_t)p >= 0x7f8000000000ull) free(p);
    atomic_fetch_sub(&live_dev, 1);
    return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned int f) {
    (void)f;
    *p = malloc(n ? n : 1);
    memset(*p, 0, n);
    atomic_fetch_add(&live_host, 1);
    return hipSuccess;
}
hipError_t hipHostFree(void* p) {
    free(p);
    atomic_fetch_sub(&live_host, 1);
    return hipSuccess;
}

static atomic_int g_yield_requests, g_yield_max, g_yield_raises;
void xsk_gpu__ll_yield_all(int delta) {
    if (delta > 0) atomic_fetch_add(&g_yield_raises, 1);
    const int v = atomic_fetch_add(&g_yield_requests, delta) + delta;
    assert(v >= 0);
    int m = atomic_load(&g_yield_max);
    while (v > m && !atomic_compare_exchange_weak(&g_yield_max, &m, v)) {
    }
}

static atomic_int g_busy[4];
int xsk_gpu__ll_busy(int device) { return atomic_load(&g_busy[device]); }

/* ---- registrations ---- */
static void test_registrations(void) {
    static uint8_t u[64 * 4096] __attribute__((aligned(4096)));
    void *ra = NULL, *rb = NULL, *rc = NULL, *rd = NULL;
    const long r0 = rt_registers, u0 = rt_unregisters;
    /* two users of one UMEM: one runtime registration, released by the last */
    assert(xsk_gpu__umem_ref(u, sizeof u, &ra) == 0 && ra == u);
    assert(xsk_gpu__umem_ref(u, sizeof u, &rb) == 0 && rb == u);
    assert(xsk_gpu__umem_refs(u) == 2 && rt_registers == r0 + 1);
    /* a part of it shares the registration; a range starting inside and running past it cannot */
    assert(xsk_gpu__umem_ref(u + 16 * 4096, 32 * 4096, &rc) == 0 && rc == u && xsk_gpu__umem_refs(u) == 3);
    assert(xsk_gpu__umem_ref(u + 48 * 4096, 32 * 4096, &rd) == -EBUSY && rd == NULL);
    xsk_gpu__umem_unref(ra);
    xsk_gpu__umem_unref(rc);
    assert(rt_covers(u, sizeof u) && rt_unregisters == u0); /* still one user */
    xsk_gpu__umem_unref(rb);
    assert(!rt_covers(u, 1) && rt_unregisters == u0 + 1 && xsk_gpu__umem_refs(u) == 0);
    assert(g_yield_requests == 0 && g_yield_max == 1); /* grids asked to yield around the unregistration only */
    xsk_gpu__umem_unref(NULL); /* no-op */

    static uint8_t w[96 * 4096] __attribute__((aligned(4096)));
    void* rw = NULL;
    assert(xsk_gpu__umem_ref(w + 16 * 4096, 32 * 4096, &rw) == 0 && rw == w + 16 * 4096);
    assert(xsk_gpu__umem_ref(w, 32 * 4096, &rd) == -EBUSY && rd == NULL);          /* runs into it from below */
    assert(xsk_gpu__umem_ref(w, sizeof w, &rd) == -EBUSY && rd == NULL);           /* covers it */
    assert(xsk_gpu__umem_ref(w, 16 * 4096, &rd) == 0 && rd == w);                  /* ends where it starts */
    xsk_gpu__umem_unref(rd);
    xsk_gpu__umem_unref(rw);

    /* a caller's own registration: used, left registered */
    assert(hipHostRegister(u, sizeof u, 0) == hipSuccess);
    const long r1 = rt_registers, u1 = rt_unregisters;
    assert(xsk_gpu__umem_ref(u, sizeof u, &ra) == 0 && ra == u && rt_registers == r1);
    xsk_gpu__umem_unref(ra);
    assert(rt_covers(u, sizeof u) && rt_unregisters == u1 && xsk_gpu__umem_refs(u) == 0);
    assert(hipHostUnregister(u) == hipSuccess);

    /* the table holds UMEM_REG_MAX registrations */
    static void* regs[UMEM_REG_MAX];
    uint8_t* big = (uint8_t*)aligned_alloc(4096, (size_t)(UMEM_REG_MAX + 1) * 4096);
    for (int i = 0; i < UMEM_REG_MAX; i++) assert(xsk_gpu__umem_ref(big + (size_t)i * 4096, 4096, &regs[i]) == 0);
    assert(xsk_gpu__umem_ref(big + (size_t)UMEM_REG_MAX * 4096, 4096, &ra) == -ENOMEM && ra == NULL);
    for (int i = 0; i < UMEM_REG_MAX; i++) xsk_gpu__umem_unref(regs[i]);
    assert(g_nreg == 0 && rt_n == 0);
    free(big);
}

/* ---- kept buffers ---- */
static void test_buffers(void) {
    void *a = NULL, *b = NULL, *c = NULL;
    /* idle device: freed at once */
    assert(xsk_gpu__buf_alloc(0, XSK_GPU__BUF_DEV, &a, 4096) == hipSuccess && live_dev == 1);
    xsk_gpu__buf_free(0, XSK_GPU__BUF_DEV, a, 4096);
    assert(live_dev == 0 && xsk_gpu__buf_kept(0) == 0);
    /* busy device: kept, reused by exact (device, kind, size) only */
    atomic_store(&g_busy[0], 1);
    assert(xsk_gpu__buf_alloc(0, XSK_GPU__BUF_HOST | 2u, &a, 1000) == hipSuccess);
    memset(a, 0xAB, 1000);
    xsk_gpu__buf_free(0, XSK_GPU__BUF_HOST | 2u, a, 1000);
    assert(xsk_gpu__buf_kept(0) == 1 && live_host == 1);
    assert(xsk_gpu__buf_alloc(1, XSK_GPU__BUF_HOST | 2u, &b, 1000) == hipSuccess && b != a); /* other device */
    assert(xsk_gpu__buf_alloc(0, XSK_GPU__BUF_HOST, &c, 1000) == hipSuccess && c != a);       /* other kind */
    xsk_gpu__buf_free(1, XSK_GPU__BUF_HOST | 2u, b, 1000); /* device 1 idle: freed */
    xsk_gpu__buf_free(0, XSK_GPU__BUF_HOST, c, 1000);      /* kept */
    assert(xsk_gpu__buf_alloc(0, XSK_GPU__BUF_HOST | 2u, &b, 1000) == hipSuccess && b == a);
    for (int i = 0; i < 1000; i++) assert(((uint8_t*)b)[i] == 0); /* zeroed like a fresh one */
    xsk_gpu__buf_free(0, XSK_GPU__BUF_HOST | 2u, b, 1000);
    assert(xsk_gpu__buf_kept(0) == 2);
    /* the byte limit: two 3-GiB buffers kept, the third freed at once */
    void* g[3];
    for (int i = 0; i < 3; i++) assert(xsk_gpu__buf_alloc(0, XSK_GPU__BUF_DEV, &g[i], 3ull << 30) == hipSuccess);
    const long d0 = live_dev;
    const int r0 = g_yield_raises;
    for (int i = 0; i < 3; i++) xsk_gpu__buf_free(0, XSK_GPU__BUF_DEV, g[i], 3ull << 30);
    assert(xsk_gpu__buf_kept(0) == 4 && live_dev == d0 - 1);
    assert(g_yield_raises == r0 + 1 && g_yield_requests == 0); /* the one free while busy asked the grids aside */
    /* the count limit */
    static void* s[POOL_MAX + 8];
    for (int i = 0; i < POOL_MAX + 8; i++) assert(xsk_gpu__buf_alloc(0, XSK_GPU__BUF_DEV, &s[i], 64) == hipSuccess);
    const int r1 = g_yield_raises;
    for (int i = 0; i < POOL_MAX + 8; i++) xsk_gpu__buf_free(0, XSK_GPU__BUF_DEV, s[i], 64);
    assert(xsk_gpu__buf_kept(0) == POOL_MAX);
    assert(g_yield_raises == r1 + 12 && g_yield_requests == 0); /* 4 kept before + 256 limit: 12 frees past it */
    /* idle again: the next release (or the drain every fini ends with) frees everything kept */
    atomic_store(&g_busy[0], 0);
    xsk_gpu__buf_free(0, 0, NULL, 0);
    assert(xsk_gpu__buf_kept(0) == 0 && g_pool_bytes == 0 && live_dev == 0 && live_host == 0);
}

/* ---- on 8 threads ---- */
#define NTH 8
#define ITERS 20000
static uint8_t g_umem[4][256 * 4096] __attribute__((aligned(4096)));
static atomic_int g_fail;

static uint64_t rnd(uint64_t* s) {
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return *s >> 33;
}

static void* worker(void* arg) {
    uint64_t seed = 0x9E3779B97F4A7C15ull * (uint64_t)(uintptr_t)arg + 1;
    void* held[4] = {NULL, NULL, NULL, NULL};
    const uint8_t* held_at[4] = {NULL, NULL, NULL, NULL};
    size_t held_n[4] = {0, 0, 0, 0};
    for (int it = 0; it < ITERS; it++) {
        const int k = (int)(rnd(&seed) % 4);
        if (held[k]) { /* still registered while held, then released */
            if (!rt_covers(held_at[k], held_n[k])) atomic_fetch_add(&g_fail, 1);
            xsk_gpu__umem_unref(held[k]);
            held[k] = NULL;
        } else { /* the whole UMEM or a page-aligned part of it */
            const size_t first = rnd(&seed) % 2 ? 0 : (rnd(&seed) % 128) * 4096;
            const size_t n = sizeof g_umem[k] - first - (rnd(&seed) % 64) * 4096;
            void* rb = NULL;
            const int rc = xsk_gpu__umem_ref(g_umem[k] + first, n, &rb);
            /* only a part registered first can make a later whole-UMEM user run past it */
            if (rc == 0) {
                held[k] = rb;
                held_at[k] = g_umem[k] + first;
                held_n[k] = n;
                if (!rt_covers(held_at[k], n)) atomic_fetch_add(&g_fail, 1);
            } else if (rc != -EBUSY) {
                atomic_fetch_add(&g_fail, 1);
            }
        }
        /* buffers: busy toggles now and then, sizes from a small set so that reuse happens */
        const int dev = (int)(rnd(&seed) % 2);
        if (rnd(&seed) % 64 == 0) atomic_store(&g_busy[dev], (int)(rnd(&seed) % 2));
        const unsigned kind = rnd(&seed) % 2 ? XSK_GPU__BUF_DEV : XSK_GPU__BUF_HOST;
        const size_t sz = 256u << (rnd(&seed) % 4);
        void* p = NULL;
        if (xsk_gpu__buf_alloc(dev, kind, &p, sz) != hipSuccess || !p) atomic_fetch_add(&g_fail, 1);
        if (kind == XSK_GPU__BUF_HOST) {
            for (size_t i = 0; i < sz; i++)
                if (((uint8_t*)p)[i]) {
                    atomic_fetch_add(&g_fail, 1);
                    break;
                }
            memset(p, 0x5A, sz);
        }
        xsk_gpu__buf_free(dev, kind, p, sz);
    }
    for (int k = 0; k < 4; k++) xsk_gpu__umem_unref(held[k]);
    return NULL;
}

static void test_threads(void) {
    pthread_t th[NTH];
    for (int i = 0; i < NTH; i++) assert(pthread_create(&th[i], NULL, worker, (void*)(uintptr_t)(i + 1)) == 0);
    for (int i = 0; i < NTH; i++) pthread_join(th[i], NULL);
    assert(g_fail == 0);
    for (int k = 0; k < 4; k++) assert(xsk_gpu__umem_refs(g_umem[k]) == 0);
    assert(g_nreg == 0 && rt_n == 0);
    for (int d = 0; d < 2; d++) {
        atomic_store(&g_busy[d], 0);
        xsk_gpu__buf_free(d, 0, NULL, 0);
    }
    assert(g_npool == 0 && live_dev == 0 && live_host == 0);
}

int main(void) {
    test_registrations();
    test_buffers();
    test_threads();
    printf("mem ok: %ld runtime registrations, %ld unregistrations\n", (long)rt_registers, (long)rt_unregisters);
    return 0;
}
