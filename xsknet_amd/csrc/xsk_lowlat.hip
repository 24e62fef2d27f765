// xsk_lowlat.hip — the low-latency RX-loop channel of an XSK_GPU_MODE_LOWLAT host context.
//
// The reference hands its transform RX_BATCH_SIZE = 64 descriptors per poll() (src/lib/xsk_receive.c:196,
// :251-257; src/lib/xsk_utils.h:8).  At that size a kernel launch plus a stream synchronisation costs
// far more than the work, so this channel keeps XSK_GPU__LL_WG workgroups of the round kernel
// resident: they poll a doorbell in fine-grained pinned host memory, run the round kernel's body
// (echo6_body, xsk_echo_device.h — the same code the launched kernel runs, bit for bit) over their slices of
// the posted descriptors, write verdicts and records into mapped host memory, and publish completion (the
// host adds the counters from the descriptors and verdicts it has anyway).  A batch of <= 64 frames (and any
// batch of <= 128 frames and <= 16 KiB) is served by workgroup 0 alone; larger ones by all XSK_GPU__LL_WG,
// because one CU caps the PCIe reads of a batch (its waves have only so many loads in flight).
// A batch is "write descriptors, bump the doorbell, spin on the completion words": no launch, no sync.
// The host side of the protocol (posting, waiting, relaunch, timeout and recovery) is
// xsk_lowlat_proto.h, unit-tested on the CPU.
//
// Memory ordering (AMDGPU memory model, system scope): the host stores descriptors, then the doorbell
// sequence number (x86 TSO keeps the order).  Wave 0 of each workgroup polls the doorbell with relaxed
// system-scope loads (two in flight, one per copy of the word); on a new batch it issues ONE system-scope
// acquire (`buffer_inv sc0 sc1`: the CU's L1, shared by the workgroup's waves, and the L2 lines of host
// memory, so recycled UMEM frames are never read stale), waits for it, and then the workgroup meets.
// After the body every wave waits for its own stores' acknowledgements, the workgroup meets, and thread 0
// issues ONE system-scope release fence (the L2 write-back covers every wave's stores to the UMEM,
// verdicts and records), waits for the write-back, and stores the batch's sequence number to its `done`.
//
// Exit conditions every wave reaches: the host's stop word, or no batch for kIdleTicks (50 ms of the 100-MHz wall
// clock) at the leader -- or, idle, its channel's yield word raised (another context is about to unregister host
// memory, which waits for every stream of the device) -- whose exit flag (device memory, tagged with the launch
// generation) the other workgroups poll — so a process that dies without xsk_gpu_fini() never leaves the grid running.
// The host relaunches the grid lazily when it finds the leader gone (alive == 0 before posting, or the kernel's stream
// idle while a batch waits); a relaunched workgroup takes its baseline from its own `done`, so no slice is served
// twice. The exit path is Dekker-safe: the leader clears `alive`, then looks at the doorbell once more and resumes if a
// batch slipped in.
#include <errno.h>
#include <stddef.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "xsk_echo_device.h"
#include "xsk_gpu_internal.h"
#include "xsk_hip_util.h"

using namespace xskgpu;

namespace {

constexpr uint64_t kIdleTicks = 5000000ull;  // 50 ms at 100 MHz (s_memrealtime)
// The leader reads its channel's yield word (xsk_gpu__ll_yield_all) in the same 16-B load as the command word, so
// looking at it costs no extra read.  XSK_LL_YIELD=0 is for the A/B of tools/ab_yield.py only: the round-5 poll (an
// 8-B load of the command word) and no yield.
#ifndef XSK_LL_YIELD
#define XSK_LL_YIELD 1
#endif
constexpr bool kYield = XSK_LL_YIELD != 0;
constexpr int kLLTPW = 1;                    // 16 tiles = 1024 frames per doorbell, one round
constexpr int kLLSync = 0;                   // one round: write as soon as the wave has read

constexpr int kPollCopies = 2;  // doorbell words (and first-64 descriptor blocks) polled in turn

// workgroups of resident grids running now, in this process (device memory; each workgroup adds one when it starts
// and takes it back when it leaves): xsk_gpu__lowlat_live, the tests' check that no grid outlives its channel
__device__ unsigned int g_ll_live;

struct LowlatArgs {
    xsk_gpu__bell* bell;  // device alias of the mapped doorbell
    xsk_gpu__lldiag* diag;  // device memory
    uint8_t* umem;
    uint64_t umem_size;
    const xsk_gpu_desc* descs;  // XSK_GPU_LOWLAT_MAX slots, then a copy of the first 64 for the second poll
    uint8_t* verdicts;
    xsk_gpu_rec* recs;
    uint32_t opts;
    uint32_t gen;  // launch generation (the leader's exit flag names it)
};

__device__ __forceinline__ uint32_t ld_sys(const volatile uint32_t* p) {
    return __hip_atomic_load((uint32_t*)p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(volatile uint32_t* p, uint32_t v) {
    __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wave 0's doorbell poll until a batch for this workgroup (or the exit).  LEADER is a template parameter, not a
// runtime test: the two polls in flight are waited for by counting (s_waitcnt vmcnt(N)), and a load issued under
// a runtime condition makes the compiler wait for every outstanding load instead -- the doorbell was then
// sampled once per round trip (~1.1 us) instead of every half round trip.
struct PollState {
    uint32_t served;
    uint64_t cA, aA, bA, cB, aB, bB;  // the two polls' registers: they stay live across the body
    uint32_t yA, yB;                  // the leader's: the yield word read with each command word
    uint64_t t_seen, t_poll, n_batches, n_polls, n_stale;
};
template <bool LEADER>
__device__ __forceinline__ void poll_doorbell(const LowlatArgs& L, u32x4* sdesc, uint32_t* s_cmd, PollState& P,
                                              uint32_t g, uint32_t lane) {
    xsk_gpu__bell* bell = L.bell;
    // wave 0 polls: the leader's every read brings the command word AND the first 64 descriptor slots,
    // so a batch of <= 64 frames needs no second round trip for its descriptors; the host tags each
    // slot's `options` with the batch's sequence number, and a slot seen with an older tag (its write
    // not yet visible) makes the wave poll again.  The other workgroups read the command word only.
    uint32_t work = 0, n = 0, recs = 0, tq = 0, dl = 0, f0 = 0;
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
    // the other workgroups read a line of their own, one poll at a time (their second "copy" is the
    // same word: the second read waits for the first)
    volatile uint64_t* const own = LEADER ? nullptr : &bell->wcmd[g - 1].cmd;
    // the leader's command word and yield word: ONE 16-B system-coherent load of the line's first 16 bytes
    const __amdgpu_buffer_rsrc_t brs =
        __builtin_amdgcn_make_buffer_rsrc((void*)bell, (short)0, (int)sizeof(xsk_gpu__bell), kRsrcFlags);
    auto issue = [&](int copy, uint64_t& c, uint64_t& d0, uint64_t& d1, uint32_t& y) {
        if (LEADER && kYield) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
                brs, copy ? (int)offsetof(xsk_gpu__bell, cmd_b) : (int)offsetof(xsk_gpu__bell, cmd), 0, kSysCoherent);
            c = (uint64_t)v.x | ((uint64_t)v.y << 32);
            y = v.z;
        } else {
            c = __hip_atomic_load((uint64_t*)(!LEADER ? own : copy ? &bell->cmd_b : &bell->cmd), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
            y = 0u;
        }
        if (LEADER) {
            const int dofs = (int)((copy ? XSK_GPU_LOWLAT_MAX : 0u) * sizeof(xsk_gpu_desc) + lane * 16u);
            const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(drs, dofs, 0, kSysCoherent);
            d0 = (uint64_t)d.x | ((uint64_t)d.y << 32);
            d1 = (uint64_t)d.z | ((uint64_t)d.w << 32);
        }
    };
    // 0: keep polling, 1: a batch for this workgroup, 2: leave
    auto examine = [&](uint64_t cv, uint64_t d0, uint64_t d1, uint32_t y) -> int {
        ++it;
        const uint64_t c = ((uint64_t)uniform((uint32_t)(cv >> 32)) << 32) | uniform((uint32_t)cv);
        tr = (wall_clock64() - t_loop) / it;  // mean sampling interval so far
        if ((uint32_t)c != P.served) {
            const uint32_t nn = (uint32_t)(c >> 32) & 0xFFFFu;
            uint32_t w = (uint32_t)(c >> 56) & 7u;
            w = w < 1u ? 1u : (w > XSK_GPU__LL_WG ? XSK_GPU__LL_WG : w);
            if (g >= w) {  // not serving this batch
                P.served = (uint32_t)c;
                return 0;
            }
            if (c & XSK_GPU__BELL_STOP) {
                // posted, then cancelled before this workgroup took it (its call timed out, e.g. while this instance
                // was still queued): retire it WITHOUT serving -- the host then knows the slice is untouched
                // (xsk_gpu__ll_unserved) and the caller's retry transforms it exactly once
                P.served = (uint32_t)c;
                if (lane == 0) {
                    st_sys(&bell->wg[g].cancel, (uint32_t)c);
                    st_sys(&bell->wg[g].done, (uint32_t)c);
                }
                return 2;
            }
            if (LEADER && w == 1u && nn <= (uint32_t)kTile) {
                if (__ballot(lane < nn && (uint32_t)(d1 >> 32) != (uint32_t)c) != 0ull) {
                    ++P.n_stale;
                    return 0;  // not yet
                }
                sdesc[lane] = u32x4{(uint32_t)d0, (uint32_t)(d0 >> 32), (uint32_t)d1, (uint32_t)(d1 >> 32)};
                dl = 1;
            }
            uint32_t f1 = 0;
            xsk_gpu__ll_slice(nn > XSK_GPU_LOWLAT_MAX ? XSK_GPU_LOWLAT_MAX : nn, w, g, &f0, &f1);
            n = f1 - f0;
            recs = (uint32_t)(c >> 48) & 1u;
            tq = (uint32_t)(c >> 49) & 0x7Fu;
            P.served = (uint32_t)c;
            work = 1;
            return 1;
        }
        if (c & XSK_GPU__BELL_STOP) return 2;
        if (!LEADER) {  // the leader's idle exit takes every workgroup of this launch with it
            if (__hip_atomic_load(&L.diag->exit_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == L.gen)
                return 2;
        } else if (wall_clock64() - t0 > kIdleTicks || (kYield && uniform(y) != 0u)) {
            // leaving -- idle, or asked to yield the device while another context unregisters host memory (the next
            // batch brings the grid back): clear `alive`, then look once more (the host posts, then reads `alive`)
            __hip_atomic_store((uint32_t*)&bell->wg[0].alive, 0u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
            const uint64_t c2 = __hip_atomic_load((uint64_t*)&bell->cmd, __ATOMIC_SEQ_CST,
                                                  __HIP_MEMORY_SCOPE_SYSTEM);
            if (uniform((uint32_t)c2) == P.served || (uniform((uint32_t)(c2 >> 32)) & 0x80000000u)) {
                __hip_atomic_store(&L.diag->exit_gen, L.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return 2;
            }
            st_sys(&bell->wg[0].alive, 1u);
            t0 = wall_clock64();
        }
        return 0;
    };
    issue(0, P.cA, P.aA, P.bA, P.yA);
    __builtin_amdgcn_s_sleep(22);  // ~0.6 us: half a round trip
    while (true) {
        issue(1, P.cB, P.aB, P.bB, P.yB);
        int r = examine(P.cA, P.aA, P.bA, P.yA);  // waits for A only (B is still in flight)
        if (r) break;
        issue(0, P.cA, P.aA, P.bA, P.yA);
        r = examine(P.cB, P.aB, P.bB, P.yB);
        if (r) break;
    }
    // ONE system-scope acquire for the workgroup: fresh descriptors and frames.  The doorbell read it
    // follows has returned (it was examined).  The invalidation completes asynchronously and only
    // this wave's own later loads are ordered behind it, so the wave waits for it (and for the other
    // poll, still in flight: at most half a round trip) before the barrier below releases the
    // other waves' loads (MI355X_MICROARCH.md, cross-CU hand-off recipe).
    if (work) asm volatile("buffer_inv sc0 sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
        s_cmd[0] = work;
        s_cmd[1] = n;
        s_cmd[2] = recs | (tq << 8) | (dl << 16);
        s_cmd[3] = f0;
    }
    P.t_seen = wall_clock64();
    P.t_poll = tr;
    P.n_polls += it;
    ++P.n_batches;
}

// XSK_GPU__LL_WG workgroups, one per CU.  Workgroup g serves slice g of a batch posted for w > g workgroups
// (xsk_gpu__ll_slice) and publishes bell->wg[g].done; workgroup 0 (the leader) also polls the first 64
// descriptor slots with the doorbell and owns `alive` and the idle exit.
template <bool WIRE>
__global__ __launch_bounds__(kThreads6, 1) void lowlat_kernel(LowlatArgs L) {
    __shared__ Echo6Smem<kLLTPW> sm;  // 64-B windows in both modes (wire: wire_header_phase64)
    __shared__ uint32_t s_cmd[4];  // work?, n, recs | tile | dl, f0
    // the body's phase stamps land in the LDS and go to the device-memory diagnostics after `done`: a store
    // to host memory would put its PCIe acknowledgement in front of every later wait on a load (the
    // vector memory counter retires in order) -- and a volatile one waits for its own
    __shared__ unsigned long long s_trace[6];
    xsk_gpu__bell* bell = L.bell;
    const uint32_t g = blockIdx.x;
    const bool leader = g == 0;
    PollState P = {};  // wave 0: `served`, the two polls' registers, diagnostics
    if (threadIdx.x == 0) atomicAdd(&g_ll_live, 1u);
    if (threadIdx.x < 64) {  // wave 0 polls; every lane keeps the same `served`
        // this workgroup's last completed batch (a previous instance's; stream order: it has exited)
        P.served = uniform(ld_sys(&bell->wg[g].done));
        if (leader) st_sys(&bell->wg[0].alive, 1u);
    }
    const uint32_t lane = threadIdx.x & 63u;
    while (true) {
        if (threadIdx.x < 64) {
            if (leader) poll_doorbell<true>(L, sm.desc, s_cmd, P, g, lane);
            else poll_doorbell<false>(L, sm.desc, s_cmd, P, g, lane);
        }
        // the command travels through the LDS only: an LDS-only barrier (__syncthreads() would first wait
        // for wave 0's poll still in flight)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const uint32_t work = s_cmd[0], n = s_cmd[1], recs = s_cmd[2] & 1u, tq = (s_cmd[2] >> 8) & 0xFFu;
        const uint32_t dl = s_cmd[2] >> 16, f0 = s_cmd[3];
        if (!work) break;  // workgroup-uniform
        const uint64_t t_body = wall_clock64();
        const uint64_t c_body = __builtin_amdgcn_s_memtime();
        EchoArgs a;
        a.umem = L.umem;
        a.umem_size = L.umem_size;
        a.descs = L.descs + f0;
        a.n = n;
        a.verdicts = L.verdicts + f0;
        a.recs = recs ? L.recs + f0 : nullptr;
        a.partials = nullptr;
        a.opts = L.opts;
        a.stats_direct = nullptr;  // the host counts from the descriptors and verdicts: no counter phase
        a.trace = s_trace;
        a.desc_in_lds = dl;
        // spread the slice over all 16 waves: tiles of ceil(n / 16) frames (a multiple of 4: one 16-lane
        // row per frame and step), so a 64-frame batch is 16 tiles of 4 frames, each wave one step
        uint32_t tl = tq ? 4u * tq : ((n + kWaves6 - 1) / kWaves6 + 3u) & ~3u;
        tl = tl < 4u ? 4u : (tl > (uint32_t)kTile ? (uint32_t)kTile : tl);
        a.tile_live = tl;
        const uint32_t ntiles = (n + tl - 1) / tl;
        if (ntiles)
            // wire mode on the reference form's 64-B windows and streams with wire_header_phase64 (the 128-B form took
            // 11.6 us per 64 x 64-B call with every option against 8.7 in reference mode, profiles/r04/wll/)
            echo6_body<kLLTPW, kLLSync, WIRE, true, true, true, false, kRefHeavy, kU, false, false, 0, true>(a, 0u,
                                                                                                          ntiles, sm);
        // the two polls' registers live across the body: a batch is taken while the other poll is still in
        // flight, and registers the compiler reused would first have to wait for it to land
        asm volatile("" ::"v"(P.cA), "v"(P.aA), "v"(P.bA), "v"(P.cB), "v"(P.aB), "v"(P.bB), "v"(P.yA), "v"(P.yB));
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
            // the wait above), and `done` then overtook the verdicts (MI355X_MICROARCH.md, compiler hazard).
            // tests/test_lowlat_isa.py checks this sequence in the built code object.
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t t_end = wall_clock64();
            __hip_atomic_store((uint32_t*)&bell->wg[g].done, P.served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (leader) {  // plain stores to device memory: no wait here, acknowledged long before the next poll
                xsk_gpu__lldiag* dg = L.diag;
                dg->trace[0] = P.t_poll;
                dg->trace[1] = t_body - P.t_seen;
                dg->trace[2] = t_rel - t_body;
                dg->trace[3] = t_end - t_rel;
                for (int k = 0; k < 5; ++k) dg->body[k] = s_trace[k];
                dg->body[5] = t_body;
                dg->clk[0] = c_rel - c_body;
                dg->clk[1] = t_rel - t_body;
                dg->polls[0] = P.n_batches;
                dg->polls[1] = P.n_polls;
                dg->polls[2] = P.n_stale;
            }
        }
    }
    if (threadIdx.x == 0) atomicSub(&g_ll_live, 1u);
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
    xsk_gpu__ll_state st;  // protocol state (xsk_lowlat_proto.h)
    uint32_t tile_q;       // frames per wave / 4 (0: from the slice's bytes); xsk_gpu__lowlat_tune
    uint32_t groups;       // serving workgroups (0: xsk_gpu__ll_groups); xsk_gpu__lowlat_tune
    uint64_t host_ns[2];   // last batch on the host: entry -> doorbell posted, posted -> completion seen
    double h_enter, h_post; // the batch in flight: entry, doorbell posted
    uint32_t width;        // workgroups a launch starts (0: XSK_GPU__LL_WG); xsk_gpu__lowlat_test_width
    xsk_gpu__lowlat* next; // the live channels (xsk_gpu__ll_yield_all)
    int listed;
};

static int ll_launch(void* u) {
    xsk_gpu__lowlat* ll = (xsk_gpu__lowlat*)u;
    HIP_TRY(hipSetDevice(ll->device));
    // clear a stop request, keeping a batch that may already be posted in the same word
    const uint64_t c = __atomic_load_n(&ll->h_bell->cmd, __ATOMIC_SEQ_CST);
    if (c & XSK_GPU__BELL_STOP) xsk_gpu__ll_post(ll->h_bell, c & ~XSK_GPU__BELL_STOP);
    ll->args.gen++;
    const dim3 grid(ll->width ? ll->width : XSK_GPU__LL_WG);
    if (ll->args.opts)
        hipLaunchKernelGGL(lowlat_kernel<true>, grid, dim3(kThreads6), 0, ll->stream, ll->args);
    else
        hipLaunchKernelGGL(lowlat_kernel<false>, grid, dim3(kThreads6), 0, ll->stream, ll->args);
    HIP_TRY(hipGetLastError());
    return 0;
}
static int ll_stream_idle(void* u) { return hipStreamQuery(((xsk_gpu__lowlat*)u)->stream) == hipSuccess; }
static double ll_now(void*) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
static void ll_relax(void*) { __builtin_ia32_pause(); }

static xsk_gpu__ll_ops ll_ops(xsk_gpu__lowlat* ll) {
    xsk_gpu__ll_ops o;
    o.u = ll;
    o.launch = ll_launch;
    o.stream_idle = ll_stream_idle;
    o.now = ll_now;
    o.relax = ll_relax;
    return o;
}

extern "C" {

void xsk_gpu__lowlat_stop(xsk_gpu__lowlat* ll) {
    if (!ll) return;
    (void)hipSetDevice(ll->device);
    const xsk_gpu__ll_ops o = ll_ops(ll);
    (void)xsk_gpu__ll_stop(&ll->st, &o, -1.0);  // every workgroup sees `stop` within one poll
}

int xsk_gpu__lowlat_broken(xsk_gpu__lowlat* ll) { return ll && ll->st.broken; }

int xsk_gpu__lowlat_last_late(const xsk_gpu__lowlat* ll) { return ll && ll->st.last_late; }

int xsk_gpu__lowlat_recover(xsk_gpu__lowlat* ll) {
    if (!ll || !ll->st.broken) return 1;
    (void)hipSetDevice(ll->device);
    if (!ll_stream_idle(ll)) return 0;
    xsk_gpu__ll_retire(&ll->st);  // the stopped instance's batch is never served by a relaunch
    ll->st.broken = 0;
    ll->st.launched = 0;
    return 1;
}

// The live channels of the process and the yield requests in force (xsk_gpu__ll_yield_all): a channel's yield words
// hold the count, set when the channel starts and whenever the count changes.
static pthread_mutex_t g_yield_mu = PTHREAD_MUTEX_INITIALIZER;
static xsk_gpu__lowlat* g_chans;
static uint32_t g_yield_req;

static void set_yield(xsk_gpu__lowlat* ll, uint32_t v) {
    __atomic_store_n(&ll->h_bell->yield, v, __ATOMIC_SEQ_CST);
    __atomic_store_n(&ll->h_bell->yield_b, v, __ATOMIC_SEQ_CST);
}

// the channel's pinned host buffers: fine-grained (coherent) and mapped, so no GPU cache ever holds a copy
constexpr unsigned kHostFlags = hipHostMallocMapped | hipHostMallocCoherent;
constexpr size_t kDescBytes = (size_t)(XSK_GPU_LOWLAT_MAX + 64u) * sizeof(struct xsk_gpu_desc);
constexpr size_t kRecBytes = (size_t)XSK_GPU_LOWLAT_MAX * sizeof(struct xsk_gpu_rec);

static void ll_free(xsk_gpu__lowlat* ll) {
    if (!ll) return;
    if (ll->listed) {  // no yield request writes to this channel's bell from here on
        pthread_mutex_lock(&g_yield_mu);
        for (xsk_gpu__lowlat** p = &g_chans; *p; p = &(*p)->next)
            if (*p == ll) {
                *p = ll->next;
                break;
            }
        pthread_mutex_unlock(&g_yield_mu);
        ll->listed = 0;
    }
    xsk_gpu__lowlat_stop(ll);
    if (ll->stream) (void)hipStreamDestroy(ll->stream);
    // kept for the next channel while another resident grid runs on the device (xsk_gpu__buf_free: the runtime's
    // free would wait for that grid)
    const int d = ll->device;
    const unsigned kh = XSK_GPU__BUF_HOST | kHostFlags;
    if (ll->h_bell) xsk_gpu__buf_free(d, kh, (void*)ll->h_bell, sizeof(xsk_gpu__bell));
    if (ll->d_diag) xsk_gpu__buf_free(d, XSK_GPU__BUF_DEV, ll->d_diag, sizeof(xsk_gpu__lldiag));
    if (ll->h_descs) xsk_gpu__buf_free(d, kh, ll->h_descs, kDescBytes);
    if (ll->h_verd) xsk_gpu__buf_free(d, kh, ll->h_verd, XSK_GPU_LOWLAT_MAX);
    if (ll->h_recs) xsk_gpu__buf_free(d, kh, ll->h_recs, kRecBytes);
    free(ll);
}

extern "C" void xsk_gpu__ll_yield_all(int delta) {
    pthread_mutex_lock(&g_yield_mu);
    g_yield_req += (uint32_t)delta;
    for (xsk_gpu__lowlat* c = g_chans; c; c = c->next) set_yield(c, g_yield_req);
    pthread_mutex_unlock(&g_yield_mu);
}

int xsk_gpu__lowlat_start(xsk_gpu__lowlat** out, void* d_umem, uint64_t umem_size, uint32_t opts) {
    if (!out || !d_umem || (umem_size >> 48) || (opts & ~XSK_GPU_OPT_ALL)) return -EINVAL;
    *out = nullptr;
    xsk_gpu__lowlat* ll = (xsk_gpu__lowlat*)calloc(1, sizeof *ll);
    if (!ll) return -ENOMEM;
    int rc = 0;
    // every buffer of the channel is fine-grained: the doorbell and the descriptor slots are polled across PCIe, and the
    // verdicts and records the host copies out once `done` is seen are stored past the GPU's L2, so their visibility
    // rests on the stores' own acknowledgements (the wave waits for them before `done`) and not on the L2 write-back
    // of the release (a late completion once returned exact verdicts with wrong records while these two
    // were coarse-grained; tests/test_gpu_staged.py::test_lowlat_late_completion_deterministic)
    const unsigned fl = XSK_GPU__BUF_HOST | kHostFlags;
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
    LL_TRY((hipError_t)xsk_gpu__buf_alloc(ll->device, fl, (void**)&ll->h_bell, sizeof(xsk_gpu__bell)));
    // XSK_GPU_LOWLAT_MAX slots plus a copy of the first 64 (the second poll's); fine-grained like the doorbell: every
    // batch rewrites them, so no GPU cache should ever hold a copy (round 5: once in ~1 G frames a whole 256-frame slice
    // came back DROP -- profiles/r05/rxpipe_pages.jsonl -- and a slice served from stale descriptors would do exactly
    // that; not seen again in 0.9 G frames either way, profiles/r05/lowlat_slice_recheck.jsonl)
    LL_TRY((hipError_t)xsk_gpu__buf_alloc(ll->device, fl, (void**)&ll->h_descs, kDescBytes));
    LL_TRY((hipError_t)xsk_gpu__buf_alloc(ll->device, fl, (void**)&ll->h_verd, XSK_GPU_LOWLAT_MAX));
    LL_TRY((hipError_t)xsk_gpu__buf_alloc(ll->device, fl, (void**)&ll->h_recs, kRecBytes));
    memset((void*)ll->h_bell, 0, sizeof(xsk_gpu__bell));
    // the descriptor slots too: the leader takes a polled slot as this batch's when its `options` tag equals the
    // batch's seq, and a recycled allocation may still hold an earlier channel's slots tagged 1, 2, 3, ... -- the seqs
    // this channel starts with.  A poll that read such a slot before the host's new one landed took the old channel's
    // descriptors for its own (seen once the pipelined loop made channels come and go: wrong verdicts, frames
    // untouched).  Zeroed, a slot's tag is never a posted seq (seqs start at 1).
    memset((void*)ll->h_descs, 0, (size_t)(XSK_GPU_LOWLAT_MAX + 64u) * sizeof(struct xsk_gpu_desc));
    LL_TRY((hipError_t)xsk_gpu__buf_alloc(ll->device, XSK_GPU__BUF_DEV, (void**)&ll->d_diag,
                                          sizeof(xsk_gpu__lldiag)));
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
    A.gen = 0;
    pthread_mutex_lock(&g_yield_mu);  // a live channel from here on: its yield words follow the requests
    set_yield(ll, g_yield_req);
    ll->next = g_chans;
    g_chans = ll;
    ll->listed = 1;
    pthread_mutex_unlock(&g_yield_mu);
    ll->st.bell = ll->h_bell;
    ll->st.timeout_s = 2.0;
    ll->st.quiesce_s = 1.0;
    ll->st.recheck_s = 2e-4;
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

int xsk_gpu__lowlat_post(xsk_gpu__lowlat* ll, uint32_t n, int want_recs, uint32_t* groups) {
    if (groups) *groups = 0;
    if (!ll || n > XSK_GPU_LOWLAT_MAX) return -EINVAL;
    if (ll->st.inflight) return -EBUSY;
    ll->h_enter = ll_now(nullptr);
    if (ll->st.broken && !ll_stream_idle(ll)) return -EBUSY;  // before touching the slots it may still read
    const uint32_t w = ll->groups ? (ll->groups < n ? ll->groups : (n ? n : 1u)) : xsk_gpu__ll_groups(ll->h_descs, n);
    uint32_t f0 = 0, f1 = 0;
    xsk_gpu__ll_slice(n, w, 0, &f0, &f1);
    const uint32_t tq = ll->tile_q ? ll->tile_q : xsk_gpu__small_tile(ll->h_descs, f1 - f0) / 4u;  // per wave / 4
    // tag the slots the leader's poll reads with the doorbell's seq (the transform never reads `options`),
    // and copy them for the second poll
    const uint32_t seq = ll->st.seq + 1u;
    const uint32_t n64 = n < 64u ? n : 64u;
    struct xsk_gpu_desc* shadow = ll->h_descs + XSK_GPU_LOWLAT_MAX;
    for (uint32_t i = 0; i < n64; i++) {
        ll->h_descs[i].options = seq;
        shadow[i] = ll->h_descs[i];
    }
    const xsk_gpu__ll_ops o = ll_ops(ll);
    ll->h_post = ll_now(nullptr);
    if (groups) *groups = w;
    return xsk_gpu__ll_begin(&ll->st, &o,
                             XSK_GPU__BELL_N(n) | (want_recs ? XSK_GPU__BELL_RECS : 0ull) | XSK_GPU__BELL_TILE(tq), w);
}

int xsk_gpu__lowlat_wait(xsk_gpu__lowlat* ll, uint32_t* unserved) {
    if (unserved) *unserved = 0;
    if (!ll) return -EINVAL;
    const xsk_gpu__ll_ops o = ll_ops(ll);
    const int rc = xsk_gpu__ll_wait(&ll->st, &o, unserved);
    if (rc) return rc;
    const double h_done = ll_now(nullptr);
    ll->host_ns[0] = (uint64_t)((ll->h_post - ll->h_enter) * 1e9);
    ll->host_ns[1] = (uint64_t)((h_done - ll->h_post) * 1e9);
    return 0;
}

int xsk_gpu__lowlat_ready(const xsk_gpu__lowlat* ll) { return ll && xsk_gpu__ll_ready(&ll->st); }

int xsk_gpu__lowlat_run(xsk_gpu__lowlat* ll, uint32_t n, int want_recs, uint32_t* groups, uint32_t* unserved) {
    if (unserved) *unserved = 0;
    const int rc = xsk_gpu__lowlat_post(ll, n, want_recs, groups);
    if (rc) return rc;
    return xsk_gpu__lowlat_wait(ll, unserved);
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

int xsk_gpu__lowlat_tune(xsk_gpu_ctx* ctx, uint32_t tile_frames, uint32_t groups, uint32_t timeout_us) {
    xsk_gpu__lowlat* ll = xsk_gpu__ctx_lowlat(ctx);
    if (!ll || (tile_frames && (tile_frames < 4 || tile_frames > 64 || (tile_frames & 3))) || groups > XSK_GPU__LL_WG)
        return -EINVAL;
    ll->tile_q = tile_frames / 4u;
    ll->groups = groups;
    ll->st.timeout_s = timeout_us ? 1e-6 * (double)timeout_us : 2.0;
    return 0;
}

int xsk_gpu__lowlat_test_width(xsk_gpu_ctx* ctx, uint32_t wgs) {
    xsk_gpu__lowlat* ll = xsk_gpu__ctx_lowlat(ctx);
    if (!ll || wgs > XSK_GPU__LL_WG) return -EINVAL;
    xsk_gpu__lowlat_stop(ll);  // the next batch launches a grid of the new width
    ll->width = wgs;
    return 0;
}

void xsk_gpu__lowlat_free(xsk_gpu__lowlat* ll) { ll_free(ll); }

int xsk_gpu__lowlat_live(int device, uint32_t* out) {
    if (!out) return -EINVAL;
    *out = 0;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (hipSetDevice(device) != hipSuccess) return -ENODEV;
    // its own non-blocking stream: the null stream could wait behind a resident grid
    hipStream_t st = nullptr;
    int rc = 0;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
        hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(g_ll_live), sizeof *out, 0, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        rc = -EIO;
    if (st) (void)hipStreamDestroy(st);
    if (prev >= 0) (void)hipSetDevice(prev);
    return rc;
}

}  // extern "C"
