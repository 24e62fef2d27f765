// xsk_lowlat.hip — the low-latency RX-loop channel of an XSK_GPU_MODE_LOWLAT host context.
//
// The reference hands its transform RX_BATCH_SIZE = 64 descriptors per poll() (src/lib/xsk_receive.c:196,
// :251-257; src/lib/xsk_utils.h:8).  At that size a kernel launch plus a stream synchronisation costs
// far more than the work, so this channel keeps ONE workgroup of the round kernel
// resident: it polls a doorbell in fine-grained pinned host memory, runs the round kernel's body
// (echo6_body, xsk_echo_device.h — the same code the launched kernel runs, bit for bit) over the posted
// descriptors, writes verdicts and records into mapped host memory, and publishes completion (the host
// adds the counters from the descriptors and verdicts it has anyway).
// A batch is "write descriptors, bump the doorbell, spin on the completion word": no launch, no sync.
//
// Memory ordering (AMDGPU memory model, system scope): the host stores descriptors, then the doorbell
// sequence number (x86 TSO keeps the order).  Wave 0 of the kernel polls the doorbell with relaxed
// system-scope loads (two in flight, one per copy of the word); on a new batch it issues ONE system-scope
// acquire (`buffer_inv sc0 sc1`: the CU's L1, shared by the workgroup's waves, and the L2 lines of host
// memory, so recycled UMEM frames are never read stale), waits for it, and then the workgroup meets.
// After the body every wave waits for its own stores' acknowledgements, the workgroup meets, and thread 0
// issues ONE system-scope release fence (the L2 write-back covers every wave's stores to the UMEM,
// verdicts and records: one L2 per workgroup), waits for the write-back, and stores the batch's sequence
// number to `done`.  (A fence per wave queued sixteen L2 write-backs in front of `done`.)
//
// Exit conditions every wave reaches: the host's stop word, or no batch for kIdleTicks (50 ms of the
// 100-MHz wall clock) — so a process that dies without xsk_gpu_fini() never leaves the grid running.
// The host relaunches the kernel lazily when it finds it gone (alive == 0 before posting, or the
// kernel's stream idle while a batch waits).  The exit path is Dekker-safe: the kernel clears `alive`,
// then looks at the doorbell once more and resumes if a batch slipped in.
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "xsk_echo_device.h"
#include "xsk_gpu_internal.h"
#include "xsk_hip_util.h"

using namespace xskgpu;

namespace {

constexpr uint64_t kIdleTicks = 5000000ull;  // 50 ms at 100 MHz (s_memrealtime)
constexpr int kLLTPW = 1;                    // 16 tiles = 1024 frames per doorbell, one round
constexpr int kLLSync = 0;                   // one round: write as soon as the wave has read

constexpr int kPollCopies = 2;  // doorbell words (and first-64 descriptor blocks) polled in turn

struct LowlatArgs {
    xsk_gpu__bell* bell;  // device alias of the mapped doorbell
    xsk_gpu__lldiag* diag;  // device memory
    uint8_t* umem;
    uint64_t umem_size;
    const xsk_gpu_desc* descs;  // XSK_GPU_LOWLAT_MAX slots, then a copy of the first 64 for the second poll
    uint8_t* verdicts;
    xsk_gpu_rec* recs;
    uint32_t opts;
};

__device__ __forceinline__ uint32_t ld_sys(const volatile uint32_t* p) {
    return __hip_atomic_load((uint32_t*)p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(volatile uint32_t* p, uint32_t v) {
    __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool WIRE>
__global__ __launch_bounds__(kThreads6, 1) void lowlat_kernel(LowlatArgs L) {
    __shared__ Echo6Smem<kLLTPW, WIRE, kShip6Stream> sm;
    __shared__ uint32_t s_cmd[3];  // work?, n, recs
    // the body's phase stamps land in the LDS and go to the device-memory diagnostics after `done`: a store
    // to host memory would put its PCIe acknowledgement in front of every later wait on a load (the
    // vector memory counter retires in order) -- and a volatile one waits for its own
    __shared__ unsigned long long s_trace[6];
    xsk_gpu__bell* bell = L.bell;
    uint32_t served = 0;
    uint64_t t_seen = 0, t_poll = 0;  // wave 0: diagnostics
    uint64_t n_batches = 0, n_polls = 0, n_stale = 0;
    if (threadIdx.x < 64) {  // wave 0 polls; every lane keeps the same `served`
        served = uniform(ld_sys(&bell->done));  // a previous instance's last batch (stream order: it has exited)
        st_sys(&bell->alive, 1u);
    }
    const uint32_t lane = threadIdx.x & 63u;
    // the two polls' registers live across the body: a batch is taken while the other poll is still in
    // flight, and registers the compiler reused would first have to wait for it to land
    uint64_t cA = 0, aA = 0, bA = 0, cB = 0, aB = 0, bB = 0;
    while (true) {
        if (threadIdx.x < 64) {
            // wave 0 polls: every read brings the command word AND the first 64 descriptor slots, so a
            // batch of <= 64 frames needs no second round trip for its descriptors; the host tags each
            // slot's `options` with the batch's sequence number, and a slot seen with an older tag (its
            // write not yet visible) makes the wave poll again
            uint32_t work = 0, n = 0, recs = 0, tq = 0, dl = 0;
            uint64_t t0 = wall_clock64(), tr = 0, it = 0;
            const uint64_t t_loop = t0;
            // Two polls in flight, issued half a PCIe round trip apart (relaxed system-scope loads: no
            // wait at issue; the acquire fence follows the barrier below), so the doorbell is sampled
            // every ~0.6 us instead of every round trip.
            // A descriptor slot is read with ONE 16-byte load (system-coherent: sc0 sc1), so the tag in its
            // `options` word and its addr / len come from one snapshot of the host's cache line: a slot seen
            // with the new tag has the new descriptor (the host writes the descriptor, then the tag, then
            // the doorbell; x86 keeps that order).  Two separate 8-byte reads could tear.
            // The two polls read different lines (`cmd` / `cmd_b`, slots 0-63 / their copy after the last
            // slot): a read of a line that is already being read waits for the first to return, so polls
            // of one line would sample the doorbell only once per round trip.
            const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)L.descs, (short)0, (int)((XSK_GPU_LOWLAT_MAX + kTile) * sizeof(xsk_gpu_desc)), kRsrcFlags);
            constexpr int kSysCoherent = 1 | 16;  // cache policy SC0 | SC1
            static_assert(kPollCopies == 2, "the loop below alternates two copies");
            auto issue = [&](int copy, uint64_t& c, uint64_t& d0, uint64_t& d1) {
                c = __hip_atomic_load((uint64_t*)(copy ? &bell->cmd_b : &bell->cmd), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
                const int dofs = (int)((copy ? XSK_GPU_LOWLAT_MAX : 0u) * sizeof(xsk_gpu_desc) + lane * 16u);
                const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(drs, dofs, 0, kSysCoherent);
                d0 = (uint64_t)d.x | ((uint64_t)d.y << 32);
                d1 = (uint64_t)d.z | ((uint64_t)d.w << 32);
            };
            // 0: keep polling, 1: a batch, 2: leave
            auto examine = [&](uint64_t cv, uint64_t d0, uint64_t d1) -> int {
                ++it;
                const uint64_t c = ((uint64_t)uniform((uint32_t)(cv >> 32)) << 32) | uniform((uint32_t)cv);
                tr = (wall_clock64() - t_loop) / it;  // mean sampling interval so far
                if ((uint32_t)c != served) {
                    const uint32_t nn = (uint32_t)(c >> 32) & 0xFFFFu;
                    if (nn <= (uint32_t)kTile) {
                        if (__ballot(lane < nn && (uint32_t)(d1 >> 32) != (uint32_t)c) != 0ull) {
                            ++n_stale;
                            return 0;  // not yet
                        }
                        sm.desc[lane] = u32x4{(uint32_t)d0, (uint32_t)(d0 >> 32), (uint32_t)d1, (uint32_t)(d1 >> 32)};
                        dl = 1;
                    }
                    n = nn;
                    recs = (uint32_t)(c >> 48) & 1u;
                    tq = (uint32_t)(c >> 49) & 0x7Fu;
                    served = (uint32_t)c;
                    work = 1;
                    return 1;
                }
                if (c & XSK_GPU__BELL_STOP) return 2;
                if (wall_clock64() - t0 > kIdleTicks) {
                    // leaving: clear `alive`, then look once more (the host posts, then reads `alive`)
                    __hip_atomic_store((uint32_t*)&bell->alive, 0u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
                    const uint64_t c2 = __hip_atomic_load((uint64_t*)&bell->cmd, __ATOMIC_SEQ_CST,
                                                          __HIP_MEMORY_SCOPE_SYSTEM);
                    if (uniform((uint32_t)c2) == served || (uniform((uint32_t)(c2 >> 32)) & 0x80000000u)) return 2;
                    st_sys(&bell->alive, 1u);
                    t0 = wall_clock64();
                }
                return 0;
            };
            issue(0, cA, aA, bA);
            __builtin_amdgcn_s_sleep(22);  // ~0.6 us: half a round trip
            while (true) {
                issue(1, cB, aB, bB);
                int r = examine(cA, aA, bA);  // waits for A only (B is still in flight)
                if (r) break;
                issue(0, cA, aA, bA);
                r = examine(cB, aB, bB);
                if (r) break;
            }
            // ONE system-scope acquire for the workgroup: fresh descriptors and frames.  The doorbell read it
            // follows has returned (it was examined).  The invalidation completes asynchronously and only
            // this wave's own later loads are ordered behind it, so the wave waits for it (and for the other
            // poll, still in flight: at most half a round trip) before the barrier below releases the
            // other waves' loads (MI355X_MICROARCH.md, cross-CU hand-off recipe).
            if (work) asm volatile("buffer_inv sc0 sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
            if (n > (uint32_t)XSK_GPU_LOWLAT_MAX) n = XSK_GPU_LOWLAT_MAX;  // the host never posts more
            if (lane == 0) {
                s_cmd[0] = work;
                s_cmd[1] = n;
                s_cmd[2] = recs | (tq << 8) | (dl << 16);
            }
            t_seen = wall_clock64();
            t_poll = tr;
            n_polls += it;
            ++n_batches;
        }
        // the command travels through the LDS only: an LDS-only barrier (__syncthreads() would first wait
        // for wave 0's poll still in flight)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const uint32_t work = s_cmd[0], n = s_cmd[1], recs = s_cmd[2] & 1u, tq = (s_cmd[2] >> 8) & 0xFFu;
        const uint32_t dl = s_cmd[2] >> 16;
        if (!work) break;  // workgroup-uniform
        const uint64_t t_body = wall_clock64();
        const uint64_t c_body = __builtin_amdgcn_s_memtime();
        EchoArgs a;
        a.umem = L.umem;
        a.umem_size = L.umem_size;
        a.descs = L.descs;
        a.n = n;
        a.verdicts = L.verdicts;
        a.recs = recs ? L.recs : nullptr;
        a.partials = nullptr;
        a.opts = L.opts;
        a.stats_direct = nullptr;  // the host counts from the descriptors and verdicts: no counter phase
        a.trace = s_trace;
        a.desc_in_lds = dl;
        // spread the batch over all 16 waves: tiles of ceil(n / 16) frames (a multiple of 4: one 16-lane
        // row per frame and step), so a 64-frame batch is 16 tiles of 4 frames, each wave one step
        uint32_t tl = tq ? 4u * tq : ((n + kWaves6 - 1) / kWaves6 + 3u) & ~3u;
        tl = tl < 4u ? 4u : (tl > (uint32_t)kTile ? (uint32_t)kTile : tl);
        a.tile_live = tl;
        const uint32_t ntiles = (n + tl - 1) / tl;
        if (ntiles)
            echo6_body<kShip6U, kLLTPW, kLLSync, kShip6Stream, false, false, WIRE, false, false, !WIRE && kShip6Mid,
                       kShip6D2 && !WIRE, kShip6Skm && !WIRE, true, false, true, true>(a, 0u, ntiles, ntiles, sm);
        asm volatile("" ::"v"(cA), "v"(aA), "v"(bA), "v"(cB), "v"(aB), "v"(bB));
        const uint64_t t_rel = wall_clock64();
        const uint64_t c_rel = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have reached the L2 / fabric
        __syncthreads();  // (also: sm.desc is rewritten by the next poll only after every wave is done)
        if (threadIdx.x == 0) {
            // system scope, once for the workgroup: write back the L2 lines of host memory the body wrote,
            // wait for it, then publish completion (diagnostics after it: they are not waited for)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            // the write-back must have completed before `done` leaves: ROCm 7.2 drops the fence's own
            // `s_waitcnt vmcnt(0)` after buffer_wbl2 when this wave's scoreboard is provably empty (it is:
            // the wait above), and `done` then overtook the verdicts (MI355X_MICROARCH.md, compiler hazard)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t t_end = wall_clock64();
            __hip_atomic_store((uint32_t*)&bell->done, served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // plain stores to device memory: no wait here, acknowledged long before the first poll returns
            xsk_gpu__lldiag* dg = L.diag;
            dg->trace[0] = t_poll;
            dg->trace[1] = t_body - t_seen;
            dg->trace[2] = t_rel - t_body;
            dg->trace[3] = t_end - t_rel;
            for (int k = 0; k < 5; ++k) dg->body[k] = s_trace[k];
            dg->body[5] = t_body;
            dg->clk[0] = c_rel - c_body;
            dg->clk[1] = t_rel - t_body;
            dg->polls[0] = n_batches;
            dg->polls[1] = n_polls;
            dg->polls[2] = n_stale;
        }
    }
}

}  // namespace

struct xsk_gpu__lowlat {
    int device;
    hipStream_t stream;
    xsk_gpu__bell* h_bell;
    xsk_gpu__lldiag* d_diag;
    LowlatArgs args;
    struct xsk_gpu_desc* h_descs;
    uint8_t* h_verd;
    struct xsk_gpu_rec* h_recs;
    int launched;  // a kernel instance was launched and may still run
    uint32_t seq;     // last posted batch
    uint32_t tile_q;  // frames per wave / 4 (0: ceil(n / 16)); XSK_GPU_LOWLAT_TILE (diagnostics)
    uint64_t host_ns[2];  // last batch on the host: entry -> doorbell posted, posted -> completion seen
};

// the doorbell word and its copy (the host is their only writer)
static void ll_post(xsk_gpu__bell* b, uint64_t c) {
    __atomic_store_n(&b->cmd_b, c, __ATOMIC_SEQ_CST);
    __atomic_store_n(&b->cmd, c, __ATOMIC_SEQ_CST);
}

static int ll_launch(xsk_gpu__lowlat* ll) {
    HIP_TRY(hipSetDevice(ll->device));
    // clear a stop request, keeping a batch that may already be posted in the same word
    const uint64_t c = __atomic_load_n(&ll->h_bell->cmd, __ATOMIC_SEQ_CST);
    if (c & XSK_GPU__BELL_STOP) ll_post(ll->h_bell, c & ~XSK_GPU__BELL_STOP);
    if (ll->args.opts)
        hipLaunchKernelGGL(lowlat_kernel<true>, dim3(1), dim3(kThreads6), 0, ll->stream, ll->args);
    else
        hipLaunchKernelGGL(lowlat_kernel<false>, dim3(1), dim3(kThreads6), 0, ll->stream, ll->args);
    HIP_TRY(hipGetLastError());
    ll->launched = 1;
    return 0;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

extern "C" {

void xsk_gpu__lowlat_stop(xsk_gpu__lowlat* ll) {
    if (!ll) return;
    (void)hipSetDevice(ll->device);
    if (ll->launched) {
        ll_post(ll->h_bell, (uint64_t)ll->seq | XSK_GPU__BELL_STOP);
        (void)hipStreamSynchronize(ll->stream);  // the kernel sees `stop` within one poll
        ll->launched = 0;
    }
}

static void ll_free(xsk_gpu__lowlat* ll) {
    if (!ll) return;
    xsk_gpu__lowlat_stop(ll);
    if (ll->stream) (void)hipStreamDestroy(ll->stream);
    if (ll->h_bell) (void)hipHostFree(ll->h_bell);
    if (ll->d_diag) (void)hipFree(ll->d_diag);
    if (ll->h_descs) (void)hipHostFree(ll->h_descs);
    if (ll->h_verd) (void)hipHostFree(ll->h_verd);
    if (ll->h_recs) (void)hipHostFree(ll->h_recs);
    free(ll);
}

int xsk_gpu__lowlat_start(xsk_gpu__lowlat** out, void* d_umem, uint64_t umem_size, uint32_t opts) {
    if (!out || !d_umem || (umem_size >> 48) || (opts & ~XSK_GPU_OPT_ALL)) return -EINVAL;
    *out = nullptr;
    xsk_gpu__lowlat* ll = (xsk_gpu__lowlat*)calloc(1, sizeof *ll);
    if (!ll) return -ENOMEM;
    int rc = 0;
    // the doorbell is fine-grained (polled across PCIe); the data buffers are mapped like the UMEM itself:
    // the kernel's system-scope acquire / release fences order them (selectable for measurements)
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    const char* dfe = getenv("XSK_GPU_LOWLAT_FINE");
    const unsigned dfl = (dfe && dfe[0] == '1') ? fl : (unsigned)hipHostMallocMapped;
#define LL_TRY(expr)                         \
    do {                                     \
        const hipError_t e_ = (expr);        \
        if (e_ != hipSuccess) {              \
            rc = xsk_gpu__hip_fail(e_);      \
            ll_free(ll);                     \
            return rc;                       \
        }                                    \
    } while (0)
    LL_TRY(hipGetDevice(&ll->device));
    // a non-blocking stream of its own at the highest priority: the resident kernel neither orders the
    // null stream nor shares a hardware queue with the context's launch streams
    int lo = 0, hi = 0;
    LL_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    LL_TRY(hipStreamCreateWithPriority(&ll->stream, hipStreamNonBlocking, hi));
    LL_TRY(hipHostMalloc((void**)&ll->h_bell, sizeof(xsk_gpu__bell), fl));
    // XSK_GPU_LOWLAT_MAX slots plus a copy of the first 64 (the second poll's)
    LL_TRY(hipHostMalloc((void**)&ll->h_descs, (size_t)(XSK_GPU_LOWLAT_MAX + 64u) * sizeof(struct xsk_gpu_desc), dfl));
    LL_TRY(hipHostMalloc((void**)&ll->h_verd, XSK_GPU_LOWLAT_MAX, dfl));
    LL_TRY(hipHostMalloc((void**)&ll->h_recs, (size_t)XSK_GPU_LOWLAT_MAX * sizeof(struct xsk_gpu_rec), dfl));
    memset((void*)ll->h_bell, 0, sizeof(xsk_gpu__bell));
    LL_TRY(hipMalloc((void**)&ll->d_diag, sizeof(xsk_gpu__lldiag)));
    LL_TRY(hipMemset(ll->d_diag, 0, sizeof(xsk_gpu__lldiag)));
    LowlatArgs& A = ll->args;
    LL_TRY(hipHostGetDevicePointer((void**)&A.bell, ll->h_bell, 0));
    A.diag = ll->d_diag;
    LL_TRY(hipHostGetDevicePointer((void**)&A.descs, ll->h_descs, 0));
    LL_TRY(hipHostGetDevicePointer((void**)&A.verdicts, ll->h_verd, 0));
    LL_TRY(hipHostGetDevicePointer((void**)&A.recs, ll->h_recs, 0));
#undef LL_TRY
    A.umem = (uint8_t*)d_umem;
    A.umem_size = umem_size;
    A.opts = opts;
    if (const char* e = getenv("XSK_GPU_LOWLAT_TILE")) {  // tuning: frames per wave (multiple of 4, <= 64)
        const long t = strtol(e, nullptr, 10);
        if (t >= 4 && t <= 64 && (t & 3) == 0) ll->tile_q = (uint32_t)(t / 4);
    }
    *out = ll;
    return 0;  // the kernel starts with the first batch
}

int xsk_gpu__lowlat_set_opts(xsk_gpu__lowlat* ll, uint32_t opts) {
    if (!ll || (opts & ~XSK_GPU_OPT_ALL)) return -EINVAL;
    if (opts == ll->args.opts) return 0;
    xsk_gpu__lowlat_stop(ll);  // the next batch launches the kernel of the new mode
    ll->args.opts = opts;
    return 0;
}

int xsk_gpu__lowlat_run(xsk_gpu__lowlat* ll, uint32_t n, int want_recs) {
    if (!ll || n > XSK_GPU_LOWLAT_MAX) return -EINVAL;
    xsk_gpu__bell* b = ll->h_bell;
    const double h_enter = now_s();
    int fresh = 0;  // a kernel launched by this call: it reads `done` at start and serves the new seq
    if (!ll->launched || !__atomic_load_n(&b->alive, __ATOMIC_SEQ_CST)) {
        // gone (idle exit) or never started: launch; stream order puts it behind an exiting instance
        const int rc = ll_launch(ll);
        if (rc) return rc;
        fresh = 1;
    }
    const uint32_t tq = ll->tile_q ? ll->tile_q : xsk_gpu__small_tile(ll->h_descs, n) / 4u;  // frames per wave / 4
    const uint32_t seq = ll->seq + 1u;
    // tag the slots the polling wave reads with the doorbell (the transform never reads `options`), and
    // copy them for the second poll
    const uint32_t n64 = n < 64u ? n : 64u;
    struct xsk_gpu_desc* shadow = ll->h_descs + XSK_GPU_LOWLAT_MAX;
    for (uint32_t i = 0; i < n64; i++) {
        ll->h_descs[i].options = seq;
        shadow[i] = ll->h_descs[i];
    }
    ll->seq = seq;
    // descriptors are written before these stores
    ll_post(b, (uint64_t)seq | XSK_GPU__BELL_N(n) | (want_recs ? XSK_GPU__BELL_RECS : 0ull) | XSK_GPU__BELL_TILE(tq));
    if (!fresh && !__atomic_load_n(&b->alive, __ATOMIC_SEQ_CST)) {
        // the kernel was leaving (Dekker: it re-reads seq after clearing alive, or this launch serves it)
        const int rc = ll_launch(ll);
        if (rc) return rc;
    }
    const double h_post = now_s();
    // spin on completion; past 200 us check the kernel is still there, past 2 s give up
    double t0 = 0.0, t_query = 0.0;
    for (uint32_t spin = 0;; ++spin) {
        if (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == seq) break;
        if ((spin & 1023u) == 1023u) {
            const double t = now_s();
            if (t0 == 0.0) t0 = t_query = t;
            if (t - t_query > 2e-4) {
                t_query = t;
                if (hipStreamQuery(ll->stream) == hipSuccess && __atomic_load_n(&b->done, __ATOMIC_ACQUIRE) != seq) {
                    const int rc = ll_launch(ll);  // exited without serving the batch: serve it now
                    if (rc) return rc;
                }
            }
            if (t - t0 > 2.0) return -ETIMEDOUT;
        }
        __builtin_ia32_pause();
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    const double h_done = now_s();
    ll->host_ns[0] = (uint64_t)((h_post - h_enter) * 1e9);
    ll->host_ns[1] = (uint64_t)((h_done - h_post) * 1e9);
    return 0;
}

struct xsk_gpu_desc* xsk_gpu__lowlat_descs(xsk_gpu__lowlat* ll) { return ll->h_descs; }
uint8_t* xsk_gpu__lowlat_verdicts(xsk_gpu__lowlat* ll) { return ll->h_verd; }
struct xsk_gpu_rec* xsk_gpu__lowlat_recs(xsk_gpu__lowlat* ll) { return ll->h_recs; }

// out: [0-3] phase durations, [4-8] wave 0's body stamps, [9] shader MHz, [10-11] host phases (ns);
// [12-14] poll counts of the running instance -- diagnostics for tools/echo_replay
int xsk_gpu__lowlat_trace(xsk_gpu_ctx* ctx, uint64_t out_ns[15]) {
    xsk_gpu__lowlat* ll = xsk_gpu__ctx_lowlat(ctx);
    for (int i = 0; i < 15; ++i) out_ns[i] = 0;
    if (!ll) return -EINVAL;
    // a snapshot while the kernel may run on: fields of different batches can mix (diagnostics only)
    xsk_gpu__lldiag d;
    if (hipMemcpy(&d, ll->d_diag, sizeof d, hipMemcpyDeviceToHost) != hipSuccess) return -EIO;
    for (int i = 0; i < 4; ++i) out_ns[i] = d.trace[i] * 10u;
    for (int i = 0; i < 5; ++i) out_ns[4 + i] = d.body[i] > d.body[5] ? (d.body[i] - d.body[5]) * 10u : 0u;
    out_ns[9] = d.clk[1] ? d.clk[0] * 100u / d.clk[1] : 0u;  // MHz
    out_ns[10] = ll->host_ns[0];
    out_ns[11] = ll->host_ns[1];
    for (int i = 0; i < 3; ++i) out_ns[12 + i] = d.polls[i];  // counts, not nanoseconds
    return 0;
}

void xsk_gpu__lowlat_free(xsk_gpu__lowlat* ll) { ll_free(ll); }

}  // extern "C"
