/* xsk_gpu_mem.c -- the host-side memory bookkeeping of contexts, multi objects, pipes and LOWLAT channels (round 6):
 *   - the in-process table of host-UMEM registrations (the HIP runtime keeps one registration per base and counts
 *     nothing, so several users of one UMEM share one counted registration);
 *   - the buffers kept for reuse while a resident LOWLAT grid runs on their device (the runtime's frees would wait for
 *     that grid).
 * Plain C over a handful of HIP runtime calls; tests/c/test_mem.c runs it against stub runtime calls on the CPU. */
#define __HIP_PLATFORM_AMD__ 1
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "xsk_gpu_internal.h"

/* Registrations of host UMEMs, shared in process (round 6).  The HIP runtime keeps one registration per base address
 * and counts nothing: a second hipHostRegister of a registered base succeeds, and the first hipHostUnregister removes
 * it for every user (tools/doublereg_probe.py, profiles/r06/doublereg_attributes.jsonl).  So when one of two contexts
 * over one UMEM -- AF_XDP sockets sharing a UMEM (XDP_SHARED_UMEM), one context per RX queue -- closed, the other went
 * on over a UMEM the runtime no longer held registered, and a registration the caller had made was removed by the
 * library's close.  Every registration the library makes goes through this table: the first user of a base
 * registers it (portable + mapped), later users of the same UMEM -- or of a part of it -- take a reference of that
 * registration, the last one unregisters.  A UMEM that overlaps a registration without lying inside it gets -EBUSY:
 * the library never makes two registrations that share a page (round 5's failures all ran on such layouts, DESIGN.md
 * §5).  A base the runtime already knows as host memory and that lies in none of the library's registrations (the
 * caller registered it) is used and never unregistered here.  The lock is held across the runtime calls, so a
 * concurrent user of the same base never sees it half registered or half released. */
#define UMEM_REG_MAX 256
static pthread_mutex_t g_reg_mu = PTHREAD_MUTEX_INITIALIZER;
static struct {
    void* base;
    uint64_t size;
    int refs;
    int external; /* registered by the caller: never unregistered here */
} g_reg[UMEM_REG_MAX];
static int g_nreg;

int xsk_gpu__umem_ref(void* base, uint64_t size, void** reg_base) {
    int rc = 0;
    *reg_base = NULL;
    const uintptr_t lo = (uintptr_t)base, hi = lo + size;
    pthread_mutex_lock(&g_reg_mu);
    for (int i = 0; i < g_nreg; i++) {
        const uintptr_t elo = (uintptr_t)g_reg[i].base, ehi = elo + g_reg[i].size;
        if (elo <= lo && hi <= ehi) { /* the same UMEM, or a part of one the library registered */
            g_reg[i].refs++;
            *reg_base = g_reg[i].base;
            goto out;
        }
        if (lo < ehi && elo < hi) { /* overlaps a registration without lying inside it */
            rc = -EBUSY;
            goto out;
        }
    }
    if (g_nreg == UMEM_REG_MAX) {
        rc = -ENOMEM;
        goto out;
    }
    /* a base the runtime already knows as host memory (it lies in none of the library's registrations): the caller
     * registered it */
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof at);
    const int external = hipPointerGetAttributes(&at, base) == hipSuccess && at.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    if (!external) {
        const hipError_t e = hipHostRegister(base, size, hipHostRegisterPortable | hipHostRegisterMapped);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            rc = e == hipErrorOutOfMemory ? -ENOMEM : -EIO;
            goto out;
        }
    }
    g_reg[g_nreg].base = base;
    g_reg[g_nreg].size = size;
    g_reg[g_nreg].refs = 1;
    g_reg[g_nreg].external = external;
    g_nreg++;
    *reg_base = base;
out:
    pthread_mutex_unlock(&g_reg_mu);
    return rc;
}

void xsk_gpu__umem_unref(void* reg_base) {
    if (!reg_base) return;
    pthread_mutex_lock(&g_reg_mu);
    for (int i = 0; i < g_nreg; i++)
        if (g_reg[i].base == reg_base) {
            if (--g_reg[i].refs == 0) {
                if (!g_reg[i].external) {
                    /* the runtime waits here for every stream of the device: resident LOWLAT grids are asked to
                     * leave once idle (their next batch relaunches them) instead of being waited out */
                    xsk_gpu__ll_yield_all(+1);
                    (void)hipHostUnregister(reg_base);
                    xsk_gpu__ll_yield_all(-1);
                }
                g_reg[i] = g_reg[--g_nreg];
            }
            break;
        }
    pthread_mutex_unlock(&g_reg_mu);
}

int xsk_gpu__umem_refs(const void* base) {
    int n = 0;
    pthread_mutex_lock(&g_reg_mu);
    for (int i = 0; i < g_nreg; i++)
        if (g_reg[i].base == base) n = g_reg[i].refs;
    pthread_mutex_unlock(&g_reg_mu);
    return n;
}

/* Buffers of contexts and LOWLAT channels (round 6). The HIP runtime's hipFree, and its hipHostFree of pinned memory a
 * kernel has used, wait for every stream of the device -- another context's resident LOWLAT grid included, which leaves
 * its stream only when it stops or has idled 50 ms (tools/fini_block.py, profiles/r06/fini_block.jsonl: 2.5 s beside a
 * busy grid). So a buffer released while any LOWLAT slot of its device is taken is kept here instead, for the next
 * allocation of the same device, kind and size; kept buffers are freed once no slot of the device is taken
 * (xsk_gpu__buf_free(d, 0, NULL, 0) at the end of every fini). Past 256 buffers or 8 GiB a release frees at once, with
 * the resident grids asked to step aside (xsk_gpu__ll_yield_all) for the runtime's wait. With the UMEM registration
 * shared (xsk_gpu__umem_ref), closing one RX queue's context beside another queue's busy LOWLAT context then waits for
 * nothing. `kind`: XSK_GPU__BUF_DEV (hipMalloc) or XSK_GPU__BUF_HOST | hipHostMalloc flags. A reused host buffer is
 * zeroed as a fresh one's pages are; device buffers carry no such promise either way. */
#define POOL_MAX 256
#define POOL_BYTES_MAX (8ull << 30) /* kept at most, over every device and kind (a STAGED mirror is the UMEM's size) */
static pthread_mutex_t g_pool_mu = PTHREAD_MUTEX_INITIALIZER;
static uint64_t g_pool_bytes;
static struct {
    void* p;
    size_t size;
    int device;
    unsigned kind;
} g_pool[POOL_MAX];
static int g_npool;

static void buf_release(unsigned kind, void* p) {
    if (kind & XSK_GPU__BUF_HOST)
        (void)hipHostFree(p);
    else
        (void)hipFree(p);
}

int xsk_gpu__buf_alloc(int device, unsigned kind, void** p, size_t size) {
    *p = NULL;
    pthread_mutex_lock(&g_pool_mu);
    for (int i = 0; i < g_npool; i++)
        if (g_pool[i].device == device && g_pool[i].kind == kind && g_pool[i].size == size) {
            *p = g_pool[i].p;
            g_pool_bytes -= size;
            g_pool[i] = g_pool[--g_npool];
            break;
        }
    pthread_mutex_unlock(&g_pool_mu);
    if (*p) {
        if (kind & XSK_GPU__BUF_HOST) memset(*p, 0, size);
        return (int)hipSuccess;
    }
    return kind & XSK_GPU__BUF_HOST ? (int)hipHostMalloc(p, size, kind & ~XSK_GPU__BUF_HOST) : (int)hipMalloc(p, size);
}

void xsk_gpu__buf_free(int device, unsigned kind, void* p, size_t size) {
    struct {
        void* p;
        unsigned kind;
    } drop[POOL_MAX + 1];
    int ndrop = 0, busy = 0;
    pthread_mutex_lock(&g_pool_mu);
    if (!xsk_gpu__ll_busy(device)) { /* no resident grid: free it, and whatever was kept for this device */
        for (int i = 0; i < g_npool;)
            if (g_pool[i].device == device) {
                drop[ndrop].p = g_pool[i].p;
                drop[ndrop++].kind = g_pool[i].kind;
                g_pool_bytes -= g_pool[i].size;
                g_pool[i] = g_pool[--g_npool];
            } else {
                i++;
            }
        if (p) {
            drop[ndrop].p = p;
            drop[ndrop++].kind = kind;
        }
    } else if (p && g_npool < POOL_MAX && g_pool_bytes + size <= POOL_BYTES_MAX) {
        g_pool_bytes += size;
        g_pool[g_npool].p = p;
        g_pool[g_npool].size = size;
        g_pool[g_npool].device = device;
        g_pool[g_npool].kind = kind;
        g_npool++;
    } else if (p) { /* the pool is full (entries or bytes): free it, the resident grids asked to step aside */
        drop[ndrop].p = p;
        drop[ndrop++].kind = kind;
        busy = 1;
    }
    pthread_mutex_unlock(&g_pool_mu);
    if (busy) xsk_gpu__ll_yield_all(+1);
    for (int i = 0; i < ndrop; i++) buf_release(drop[i].kind, drop[i].p);
    if (busy) xsk_gpu__ll_yield_all(-1);
}

int xsk_gpu__buf_kept(int device) {
    int n = 0;
    pthread_mutex_lock(&g_pool_mu);
    for (int i = 0; i < g_npool; i++) n += g_pool[i].device == device;
    pthread_mutex_unlock(&g_pool_mu);
    return n;
}
