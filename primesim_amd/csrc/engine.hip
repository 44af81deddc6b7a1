// engine.hip — MI355X (gfx950) uncore timing engine: the hot path of
//   UncoreManager::uncore_access -> System::access   (reference uncore_manager.cpp:82,
//   system.cpp:144) for sys_type = DIRECTORY (mesi_directory, system.cpp:372-482).
//
// Execution model.  The reference is a strictly sequential fold over requests:
// every request's timing depends on the link-queue, directory and cache state
// left by all earlier requests, so one uncore instance is
// executed by ONE wavefront, in canonical order, bit-exactly.  The 64 lanes
// parallelise the inner loops of each step instead of the requests:
//   * set probes       lane w holds way w: tag/prog/state match by ballot,
//                      first-invalid-way by ballot, LRU by a wave argmin
//                      (lowest way wins ties, cache.cpp:167-179);
//   * sharer sets      lane k holds bitmap word k; ascending iteration by
//                      ballot + ctz (std::set<int> order, system.cpp:607);
//   * link queues      the Graphite history tree is a sorted ring of <=100
//                      free intervals, lane s%64 holding slots s and s+64;
//                      the tree search becomes one predicate + ballot, and
//                      insert/remove become one register shift (shuffles);
//   * routes           XY(Z) routes are computed arithmetically, so the next
//                      hop's link record is loaded while this hop is timed.
// Throughput comes from running many independent replicas (one wavefront
// each) side by side on the 256 CUs; a replica's state is laid out SoA in
// HBM as described in geometry.h.
//
// All floating point (the M/G/1 fallback, queue_model_m_g_1.cpp:26-35) is
// IEEE double in the reference's operation order; this file is compiled with
// -ffp-contract=off so no FMA contraction changes a rounding.

#ifndef __HIPCC_RTC__        // hipRTC (jit.cpp) supplies the runtime and <stdint.h> itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#if defined(__HIPCC_RTC__) || defined(PU_JIT_OFFLINE)
#include "primeuncore.h"      // the same file, registered (hipRTC) or written (offline) under this name by jit.cpp
#else
#include "../../include/primeuncore.h"
#endif
#include "geometry.h"

namespace {

// Compile-time configuration (jit.cpp): built with -DPU_JIT_GEO='"file"', a file
// written by pu_config_geo_source (`__device__ constexpr Geo kJitGeo = {...};`
// and `#define PU_JIT_NL <levels>`), only the kernels of that one
// configuration are emitted and they read their geometry from the constant,
// so every configuration value folds into the code.
#ifdef PU_JIT_GEO
#include PU_JIT_GEO
#endif
// Tool builds only (tools/build_exp.sh: profiling, experiments): the
// ahead-of-time kernels on one configuration's constant geometry.
#if defined(PU_FIXED_GEO) && !defined(PU_JIT_GEO)
#include PU_FIXED_GEO
#define PU_AOT_GEO(g) (&kJitGeo)
#else
#define PU_AOT_GEO(g) (g)
#endif


// Compiled configuration, throughput kernel: the replica-layout offsets reach
// the code as opaque scalars (every other geometry value stays a constant).
// Folded into the address arithmetic they cost the 96-VGPR kernel 17 VGPRs
// spilled to scratch (opaque: 4; the latency kernel, with registers to spare,
// keeps them folded): +4.6% on the C4 headline against the ahead-of-time
// kernel, same box (profiles/r3o_ab_opq.txt).
template <bool LH, int NL, class T>
__device__ __forceinline__ T off_v(T c) {
#ifdef PU_JIT_GEO
    if constexpr (!LH && NL == 1) {   // (measured on the one-level engine; deeper hierarchies keep them folded)
        // two 32-bit moves: a 64-bit SALU move takes only a 32-bit literal
        uint32_t lo, hi;
        asm("s_mov_b32 %0, %1" : "=s"(lo) : "s"((uint32_t)(uint64_t)c));
        asm("s_mov_b32 %0, %1" : "=s"(hi) : "s"((uint32_t)((uint64_t)c >> 32)));
        return (T)(((uint64_t)hi << 32) | lo);
    }
#endif
    return c;
}
#define OFF(x) off_v<LH, NL>(x)
constexpr uint32_t ST_I = 0, ST_S = 1, ST_E = 2, ST_M = 3, ST_V = 4, ST_B = 5;

// Lane within the wavefront (latency-mode workgroups hold two waves).
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63u); }

__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    uint32_t lo = rl32((uint32_t)v, l);
    uint32_t hi = rl32((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
// lane l of v becomes x (x wave-uniform)
__device__ __forceinline__ uint32_t wl32(uint32_t v, uint32_t x, int l) { return lane_id() == l ? x : v; }
__device__ __forceinline__ uint64_t wl64(uint64_t v, uint64_t x, int l) { return lane_id() == l ? x : v; }
// A tree hop's results into lane l of the window's per-hop registers: one
// v_writelane_b32 per dword (a lane compare and a select per dword in
// wl32/wl64; clang has no writelane builtin here).  The lane select goes
// through M0, saved and restored as ring_dma does (an SGPR lane select and
// SGPR data would take the constant bus twice); s_nop 3 covers a
// VALU-written lane select (4 wait states on CDNA).
__device__ __forceinline__ void wl_hop(uint32_t& a, uint32_t xa, uint32_t& b, uint32_t xb, uint64_t& c, uint64_t xc,
                                       uint64_t& d, uint64_t xd, int l) {
    uint32_t c0 = (uint32_t)c, c1 = (uint32_t)(c >> 32), d0 = (uint32_t)d, d1 = (uint32_t)(d >> 32);
    uint32_t keep;
    asm("s_mov_b32 %6, m0\n\t"
        "s_mov_b32 m0, %13\n\t"
        "s_nop 3\n\t"
        "v_writelane_b32 %0, %7, m0\n\t"
        "v_writelane_b32 %1, %8, m0\n\t"
        "v_writelane_b32 %2, %9, m0\n\t"
        "v_writelane_b32 %3, %10, m0\n\t"
        "v_writelane_b32 %4, %11, m0\n\t"
        "v_writelane_b32 %5, %12, m0\n\t"
        "s_mov_b32 m0, %6"
        : "+v"(a), "+v"(b), "+v"(c0), "+v"(c1), "+v"(d0), "+v"(d1), "=&s"(keep)
        : "s"(xa), "s"(xb), "s"((uint32_t)xc), "s"((uint32_t)(xc >> 32)), "s"((uint32_t)xd),
          "s"((uint32_t)(xd >> 32)), "s"(l));
    c = ((uint64_t)c1 << 32) | c0;
    d = ((uint64_t)d1 << 32) | d0;
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t uni32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    uint32_t lo = uni32((uint32_t)v), hi = uni32((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void atomic_add_u64(uint64_t* p, uint64_t v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Req {
    uint64_t addr;
    int32_t prog;
    int32_t type;
};

// A set of one cache, as held by the wave: uniform set coordinates plus the
// lane's own way (lanes >= nways hold an invalid, never-LRU way).  Sets of
// more than 64 ways are held one 64-way chunk at a time: lane w holds way
// w0 + w (w0 = 0 for every narrower set).
struct SetView {
    uint64_t line0;   // global line index of way 0
    uint64_t set;
    uint64_t tag;     // tag of the probed address
    uint64_t mtag;    // per lane
    int32_t mid;
    uint32_t mst;
    int64_t mts;
    uint32_t w0;      // first way of the chunk held
};

// Sets wider than 64 ways (walked in 64-way chunks, way order) are compiled
// into configuration-specific kernels only (jit.cpp: the geometry is a
// constant, so narrower configurations carry none of that code); pu_create
// refuses them for the ahead-of-time kernels.
#if defined(PU_JIT_GEO) || defined(PU_FIXED_GEO)
constexpr bool kWideSets = true;
#else
constexpr bool kWideSets = false;
#endif

// A queue's ring as held by the wave, in logical order: lane l holds the
// live intervals l and l+64 counted from the ring cursor (physical slots
// (head + l) & 127 and (head + 64 + l) & 127), so the search's hit mask needs no
// rotation and an edit's index ranges no wrap against the cursor.
struct RingView {
    uint64_t lf, ls, hf, hs;
};

// A queue's state as held by a lane (hdr_state): the ring cursor, the M/G/1
// moments (queue_model_m_g_1.cpp: _num_arrivals as an exact double, the
// service-time sum and sum of squares), the newest finish time, the first
// free-interval start; sum1 is the packed header's count of p1 visits.
struct QState {
    uint32_t head, count;
    double n;           // _num_arrivals, held as an exact double (< 2^53)
    double sum, sum_sq;
    uint64_t newest;
    uint64_t f0;
    double sum1;        // packed header: visits with packet length p1 (an exact double)
};

#define AS1 __attribute__((address_space(1)))
#ifndef PU_RING_PF
#define PU_RING_PF 3   // staged rings in flight per wave (6 KB LDS: 5 waves/SIMD fit the CU's 160 KB)
#endif
// The throughput kernels' own count.  The compiled one-level configuration
// runs 7 waves per SIMD with 1 staged ring: 3,376 B of LDS per wave = three
// 1,280-B units, so all 28 waves of a CU reside.  6 waves with 2 rings (five
// units, 25 per CU) was +4.0% on the C4 headline against 5 waves with 3 rings
// (profiles/r5j_ab_ens.txt); at 6 waves 1 ring equals 2 (r5s_ab_ens_waves7.txt);
// 7 waves, once the sharer bit below stopped spilling, +4.3% on the driver's
// 20-step window over 6 (r5w_ab_driver.txt), same box.
#ifndef PU_RING_PF_TP
#if defined(PU_JIT_GEO) && PU_JIT_NL == 1
#define PU_RING_PF_TP 1
#else
#define PU_RING_PF_TP PU_RING_PF
#endif
#endif
template <bool LH>
constexpr int ring_pf() { return LH ? PU_RING_PF : PU_RING_PF_TP; }
// Waves per SIMD the kernel is compiled for (the register budget: 5 waves =
// 96 VGPRs).  The one-level engine fits 96 with a 5-VGPR spill (once the
// pool/page-table state moved to LDS) and runs 2.9% faster at 5 resident
// waves than at 4 (120 VGPRs, no spill; same-box A/B); the deeper hierarchies
// would spill ~120 VGPRs at 128, so they keep the compiler's choice.
#ifndef PU_WAVES_1LEVEL
#if defined(PU_JIT_GEO)
#define PU_WAVES_1LEVEL 7   // compiled configuration: 72 VGPRs, one 4-B spill (jit.cpp's options)
#else
#define PU_WAVES_1LEVEL 5
#endif
#endif
// Deeper hierarchies (NL > 1), compiled configuration: 4 waves per SIMD (128
// VGPRs, no spill at C3, where the compiler's own choice was 150 VGPRs = 3
// waves): C3 +20% (448.1 / 449.4 vs 373.4 / 373.2 M/s; 5 waves, 31 VGPRs
// spilled, +13%; profiles/r6e_ab_c3.txt, same box).  The ahead-of-time
// kernels keep the compiler's choice.
#ifndef PU_WAVES_DEEP
#if defined(PU_JIT_GEO)
#define PU_WAVES_DEEP 4
#else
#define PU_WAVES_DEEP 1
#endif
#endif
#define PU_MIN_WAVES(NL) ((NL) == 1 ? PU_WAVES_1LEVEL : PU_WAVES_DEEP)
// native vectors (not classes), so loads/stores through global-address-space
// pointers need no conversion: slot = {first, second}, header = 10 dwords
typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));

// Per-wave statistics in LDS (one workgroup = one wave = one replica); lane 0
// adds with ds_add_u64 (no return, no wait) and the kernel flushes once.  A
// transmit adds its six network sums at once (lanes 0-5); the router, link and
// inject delay totals are derived from them at the flush (Network::transmit's
// per-packet terms are linear in them, network.cpp:146-156).
// The compiled configuration of a configuration without verbose_report
// (Geo.cnt_sum) also keeps the per-level {ins, miss, evict, wb} sums here
// (SN_CNT0 + 4 * level + k; levels 0-3, PU_CNT_DIR, PU_CNT_TLB) instead of
// one device-scope atomic per event on a per-cache counter: those atomics
// bypass the XCD's L2 to the memory side (4.55 per access at C4,
// TCC_EA0_WRREQ_ATOMIC_DRAM_32B) and sit in the wave's in-order vector
// memory queue.  Only the verbose report lists caches one by one
// (system.cpp:1020-1069); the ahead-of-time kernels keep per-cache counters.
#if defined(PU_JIT_GEO)
constexpr bool kCntSum = kJitGeo.cnt_sum != 0;
#else
constexpr bool kCntSum = false;
#endif
enum StatId {
    SN_ACC, SN_DIST, SN_TOTAL, SN_PLEN, SN_FLITS, SN_MG1, SN_DRAM, SN_BUSCONT,
    SN_LOCKDOWN, SN_BUSACC, SN_REQS, SN_BCAST, SN_ROWHIT, SN_ROWEMPTY, SN_ROWCONF, SN_BANKWAIT, SN_CNT0
};
constexpr int SN_COUNT = SN_CNT0 + (kCntSum ? 24 : 0);
constexpr uint32_t SN_NET_LANES = 0x3F;   // SN_ACC .. SN_MG1
static __shared__ unsigned long long lds_stat[SN_COUNT];
// kCntSum: caches this launch already marked alive (System::init_caches'
// lazy creation, system.cpp:172-207), one bit per cache of every level, so
// the alive word in HBM is stored on first touch only (when all levels'
// caches fit 4,096 bits).
#ifndef PU_ALIVE_LDS
#define PU_ALIVE_LDS 1
#endif
#if defined(PU_JIT_GEO)
constexpr int alive_base(int l) { return l <= 0 ? 0 : alive_base(l - 1) + kJitGeo.lv[l - 1].ncaches; }
constexpr bool kAliveLds = kCntSum && PU_ALIVE_LDS && alive_base(PU_JIT_NL) <= 4096;
constexpr int kAliveWords = kAliveLds ? (alive_base(PU_JIT_NL) + 31) / 32 : 1;
#else
constexpr int alive_base(int) { return 0; }
constexpr bool kAliveLds = false;
constexpr int kAliveWords = 1;
#endif
static __shared__ uint32_t lds_alive[kAliveWords];
static __shared__ unsigned long long lds_err;
// The message loop's state (uncore_kernel), lane 0 its writer.
struct LoopCtl {
    int64_t msg_shift;     // PU_KF_CLOSED: core shift at the open message's start
    uint64_t dead_tags;    // PU_KF_MSGHALT: receive threads that have exited
    uint64_t deadline;     // s_memrealtime at which a time-sliced launch stops
    uint64_t done;         // requests processed in this launch
    int32_t D;             // prime.cpp's running `delay` of the open message
    int32_t halted, halted0, skip;
    uint32_t flags;
    int32_t last_d;        // latency kernels: the last request's delay (0: none ran), for the resident fast answer
    uint64_t cur;          // index of the request being simulated
    uint64_t limit_at;     // first request that raised a PU_ERRF_LIMITS bit (UINT64_MAX: none)
};
static __shared__ LoopCtl lds_ctl;
// Engine state that only the sharer pool and the page table touch: in LDS, so
// it holds no scalar registers across the request loop (every lane reads and
// writes the same wave-uniform value).
struct EngShared {
    int32_t pool_top;    // sharer-bitmap pool stack (RunState.pool_top)
    int32_t stop;        // replica must stop (engine limit)
    uint64_t page_next;  // RunState.page_next
    uint64_t last_addr;  // RunState.last_addr
};
static __shared__ EngShared lds_eng;

// LDS updates by a fixed set of lanes, with the exec mask narrowed inside
// the asm: written as `if (lane_id() == k)`, the lane compares are loop
// invariants the compiler hoists and then spills (a v_readlane pair and a
// wait state at every use).  LDS operations of a wave complete in order, so
// the compiler's own lgkmcnt waits stay correct (at worst conservative).
// s_and_b64 writes SCC, which the compiler may hold live across the asm: it
// is declared clobbered.
__device__ __forceinline__ void lds_add_u64_lanes(uint32_t lds_byte_addr, uint64_t v, uint32_t lanes) {
    uint64_t keep;
    asm volatile("s_mov_b64 %0, exec\n\t"
                 "s_and_b64 exec, exec, %3\n\t"
                 "ds_add_u64 %1, %2\n\t"
                 "s_mov_b64 exec, %0"
                 : "=&s"(keep) : "v"(lds_byte_addr), "v"(v), "s"((uint64_t)lanes) : "memory", "scc");
}
__device__ __forceinline__ void lds_or_u64_lane0(uint32_t lds_byte_addr, uint64_t v) {
    uint64_t keep;
    asm volatile("s_mov_b64 %0, exec\n\t"
                 "s_and_b64 exec, exec, 1\n\t"
                 "ds_or_b64 %1, %2\n\t"
                 "s_mov_b64 exec, %0"
                 : "=&s"(keep) : "v"(lds_byte_addr), "v"(v) : "memory", "scc");
}
// Device-scope atomic add by lane 0 (the per-cache counters), the same way.
// Vector memory operations retire in issue order, so the compiler's vmcnt
// waits (and the staging waits) stay correct with this one unseen: at worst they
// wait for it too.
__device__ __forceinline__ void gatomic_add_u64_lane0(uint64_t* p, uint64_t v) {
    uint64_t keep;
    asm volatile("s_mov_b64 %0, exec\n\t"
                 "s_and_b64 exec, exec, 1\n\t"
                 "global_atomic_add_x2 %1, %2, off\n\t"
                 "s_mov_b64 exec, %0"
                 : "=&s"(keep) : "v"(p), "v"(v) : "memory", "scc");
}
// lane L of v becomes the wave-uniform x (v_writelane_b32 with a constant lane)
template <int L>
__device__ __forceinline__ uint32_t wlane(uint32_t v, uint32_t x) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(uni32(x)), "i"(L));
    return v;
}
__device__ __forceinline__ uint32_t lds_u32addr(const void* p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}
__device__ __forceinline__ void stat_add(int k, uint64_t v) {
    lds_add_u64_lanes(lds_u32addr(&lds_stat[k]), v, 1u);
}
__device__ __forceinline__ void err_or(uint64_t f) {
    lds_or_u64_lane0(lds_u32addr(&lds_err), f);
    // rare: remember where the first engine-limit / undefined-state bit came
    // from, so a host caller can still trust every request before it
    if (f & PU_ERRF_LIMITS) {
        const uint64_t cur = lds_ctl.cur;
        if (lane_id() == 0 && cur < lds_ctl.limit_at) lds_ctl.limit_at = cur;
    }
}

// Region cycle counters, compiled in only with -DPU_PROF (the profiling build,
// libprimeuncore_prof.so; tools/prof_regions.py).  Regions are inclusive.
enum ProfId {
    PF_LOOP, PF_REQ, PF_NET, PF_NSETUP, PF_NHOPS, PF_NTREE, PF_NWAIT, PF_NWB, PF_SETL0, PF_SETLN, PF_HOME_LD,
    PF_HOME, PF_DOWN, PF_WINDOWS, PF_TREEHOPS, PF_DEMAND, PF_T_LDS, PF_T_SEARCH, PF_T_DECIDE, PF_T_EDIT,
    PF_T_STORE, PF_T_REFILL, PF_NPRE, PF_NPOST, PF_MG1RUN, PF_MG1LANES, PF_MG1HITS, PF_MAINTAIL,
    PF_MG1PRESENT, PF_MG1STORED, PF_MG1BATCH, PF_T_UPD, PF_COUNT
};
#ifdef PU_PROF
static __shared__ unsigned long long lds_prof[PF_COUNT];
}  // namespace
// (outside the anonymous namespace: a compiled-configuration module exports
// them by name, jit.cpp's jit_prof_read)
__device__ unsigned long long g_prof[PF_COUNT];
// per-replica (block) wall-clock stamps of the last launch and summed durations
#define PU_PROF_BLOCKS 4096
__device__ unsigned long long g_blk_t0[PU_PROF_BLOCKS], g_blk_t1[PU_PROF_BLOCKS], g_blk_dur[PU_PROF_BLOCKS];
namespace {
#define PROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PROF_ADD(id, t0) \
    do { if (lane_id() == 0) atomicAdd(&lds_prof[id], (unsigned long long)(__builtin_amdgcn_s_memtime() - (t0))); } while (0)
// n is evaluated by the whole wave (it may be a ballot), then lane 0 adds it
#define PROF_CNT(id, n) \
    do { const unsigned long long pf_n_ = (unsigned long long)(n); \
         if (lane_id() == 0) atomicAdd(&lds_prof[id], pf_n_); } while (0)
#else
#define PROF_T(v)
#define PROF_ADD(id, t0) do { } while (0)
#define PROF_CNT(id, n) do { } while (0)
#endif

// Wave-uniform context of the queue/network code (all values in SGPRs).
// Narrow on purpose: it stays live across the whole transmit, and SGPRs are the
// engine's scarcest resource (each one spilled costs a v_writelane/v_readlane).
// Delays are < 2^31 (checked at pu_create); the magics are < 2^32 for w >= 2
// (a 1-node mesh never routes).
struct NetCtx {
    AS1 char* qhdr;            // the replica's queue headers (packed: 32 B each; wide: {a, b} of every queue, then c)
    AS1 char* qring;           // ... and rings
    uint32_t router, link_delay, inject;
    uint32_t hdr_c;            // wide headers: byte offset of the c pieces (nqueues x 32)
    uint32_t p0, p1;           // packed headers: the two packet lengths (n counts all visits, n1 those of p1)
    int header_flits, data_width, w, net_type;
    uint32_t w_magic, w2_magic;
    int w2, blk_len, plen_blk;
};

__device__ __forceinline__ AS1 v2u64* q_ring(const NetCtx& c, int q) {
    return reinterpret_cast<AS1 v2u64*>(c.qring) + (size_t)q * PU_QRING;
}
__device__ __forceinline__ AS1 v4u32* q_hdr_ab(const NetCtx& c, int q) {
    return reinterpret_cast<AS1 v4u32*>(c.qhdr + (uint64_t)q * PU_HDR_AB);
}
__device__ __forceinline__ AS1 v4u32* q_hdr_c(const NetCtx& c, int q) {
    return reinterpret_cast<AS1 v4u32*>(c.qhdr + c.hdr_c + (uint64_t)q * PU_HDR_C);
}

// Load the `cnt` live slots of ring q starting at `head` in logical order
// (lane l holds intervals l and l+64); dead intervals are not fetched and
// read as 0.
__device__ __forceinline__ void ring_load(const NetCtx& c, int q, uint32_t head, uint32_t cnt, RingView& v) {
    const AS1 v2u64* R = q_ring(c, q);
    const uint32_t ln = (uint32_t)lane_id();
    v = RingView{0, 0, 0, 0};
    if (ln < cnt) {
        v2u64 a = R[(head + ln) & (PU_QRING - 1)];
        v.lf = a.x;
        v.ls = a.y;
    }
    if (ln + 64 < cnt) {
        v2u64 b = R[(head + 64 + ln) & (PU_QRING - 1)];
        v.hf = b.x;
        v.hs = b.y;
    }
    // settle the loads here: otherwise hipcc carries them as pending into code
    // shared with the LDS-staged path and drains every staging DMA there
    asm volatile("" : "+v"(v.lf), "+v"(v.ls), "+v"(v.hf), "+v"(v.hs));
}

// IEEE double division a / b, correctly rounded, as hipcc's own lowering does
// it (v_rcp_f64, two Newton steps, one residual correction) minus its
// range-scaling and special-case steps (v_div_scale/v_div_fixup): every
// M/G/1 operand is a positive normal double far from overflow and underflow
// (counts, cycle sums and their ratios), where those steps are the identity,
// so the result is the same correctly rounded quotient.  The refined
// reciprocal of a shared divisor is computed once.
// PU_DIV_NR1: one Newton step instead of two before the residual correction
// (an A/B knob; tools/probe/rcp_probe.hip measures whether gfx950's v_rcp_f64
// is accurate enough for it to stay correctly rounded).
__device__ __forceinline__ double rcp_nr(double b) {
    double y = __builtin_amdgcn_rcp(b);
#ifndef PU_DIV_NR1
    y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
#endif
    return __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
}
__device__ __forceinline__ double div_nr(double a, double b, double y) {
    const double q = a * y;
    return __builtin_fma(__builtin_fma(-b, q, a), y, q);
}

// M/G/1 (queue_model_m_g_1.cpp:16-42), reference operation order.
__device__ __forceinline__ uint64_t mg1_wait(const QState& s) {
    if (s.n == 0.0) return 0;
    const double nd = s.n;
    const double rn = rcp_nr(nd);
    double mean = div_nr(s.sum, nd, rn);
    double var = div_nr(s.sum_sq, nd, rn) - mean * mean;
    double mu = div_nr(1.0, mean, rcp_nr(mean));
    const double newest = (double)s.newest;
    double lambda = div_nr(nd, newest, rcp_nr(newest));
    if (lambda >= mu) lambda = 0.999 * mu;
    const double mu2 = mu * mu;
    double inv = div_nr(1.0, mu2, rcp_nr(mu2));
    double num = 0.5 * mu;
    num = num * lambda;
    num = num * (inv + var);
    const double den = mu - lambda;
    double w = div_nr(num, den, rcp_nr(den));
    return (uint64_t)ceil(w);
}

// Whole-wave rotates (DPP): lane i receives lane (i+1)&63 / (i-1)&63.
__device__ __forceinline__ uint32_t dpp_next(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x134, 0xF, 0xF, false);   // wave_rol:1
}
__device__ __forceinline__ uint32_t dpp_prev(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x13C, 0xF, 0xF, false);   // wave_ror:1
}
// The 128-slot ring moved by one slot: slot i receives slot i+1 (NEXT) or
// i-1 (PREV); lane 63 / lane 0 cross between the low and high halves.
template <bool NEXT>
__device__ __forceinline__ void ring_shift(uint64_t lo, uint64_t hi, uint64_t& olo, uint64_t& ohi) {
    const bool cross = NEXT ? lane_id() == 63 : lane_id() == 0;
    const uint32_t a0 = NEXT ? dpp_next((uint32_t)lo) : dpp_prev((uint32_t)lo);
    const uint32_t a1 = NEXT ? dpp_next((uint32_t)(lo >> 32)) : dpp_prev((uint32_t)(lo >> 32));
    const uint32_t b0 = NEXT ? dpp_next((uint32_t)hi) : dpp_prev((uint32_t)hi);
    const uint32_t b1 = NEXT ? dpp_next((uint32_t)(hi >> 32)) : dpp_prev((uint32_t)(hi >> 32));
    olo = cross ? (((uint64_t)b1 << 32) | b0) : (((uint64_t)a1 << 32) | a0);
    ohi = cross ? (((uint64_t)a1 << 32) | a0) : (((uint64_t)b1 << 32) | b0);
}

// Inclusive prefix sum of a u64 over the wave (lane 0 first): rows of 16 by
// row_shr 1/2/4/8, then row_bcast 15/31 across rows.  Lanes a DPP step
// cannot source from add 0 (the builtin's `old` operand).
template <int CTRL, int RM>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, RM, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, RM, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}
// The same scan on 32 bits: one v_add_u32 with a DPP source per step
// (bound_ctrl: lanes without a source add 0).  Exact when the 64 terms sum
// below 2^32 (the caller checks every term < 2^26).
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp_u32z(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, true);
}
__device__ __forceinline__ uint32_t scan_incl_u32(uint32_t v) {
    v += dpp_u32z<0x111, 0xF>(v);
    v += dpp_u32z<0x112, 0xF>(v);
    v += dpp_u32z<0x114, 0xF>(v);
    v += dpp_u32z<0x118, 0xF>(v);
    v += dpp_u32z<0x142, 0xA>(v);
    v += dpp_u32z<0x143, 0xC>(v);
    return v;
}
__device__ __forceinline__ uint64_t scan_incl_u64(uint64_t v) {
    v += dpp_u64<0x111, 0xF>(v);   // row_shr:1
    v += dpp_u64<0x112, 0xF>(v);   // row_shr:2
    v += dpp_u64<0x114, 0xF>(v);   // row_shr:4
    v += dpp_u64<0x118, 0xF>(v);   // row_shr:8
    v += dpp_u64<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3
    v += dpp_u64<0x143, 0xC>(v);   // row_bcast:31 -> rows 2, 3
    return v;
}

// Cache::lru (cache.cpp:167-179): the way with the smallest timestamp, lowest
// way on ties, over lanes 0..nways-1 (other lanes pass INT64_MAX / way 64).
// Up to 16 ways the butterfly stays inside a DPP row (quad_perm xor 1, xor 2,
// row_half_mirror, row_mirror: a few cycles per step); wider sets fall back to
// cross-row shuffles.  The (ts, way) minimum is order-independent.
template <int CTRL>
__device__ __forceinline__ void lru_step_dpp(int64_t& bt, int& bw) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)bt, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)bt >> 32), CTRL, 0xF, 0xF,
                                                              false);
    const int ow = __builtin_amdgcn_update_dpp(0, bw, CTRL, 0xF, 0xF, false);
    const int64_t ot = (int64_t)(((uint64_t)hi << 32) | lo);
    if (ot < bt || (ot == bt && ow < bw)) {
        bt = ot;
        bw = ow;
    }
}
__device__ __forceinline__ int lru_way(int64_t bt, int bw, uint64_t nways) {
    if (nways <= 16) {
        lru_step_dpp<0xB1>(bt, bw);      // quad_perm [1,0,3,2]
        lru_step_dpp<0x4E>(bt, bw);      // quad_perm [2,3,0,1]
        lru_step_dpp<0x141>(bt, bw);     // row_half_mirror
        if (nways > 8) lru_step_dpp<0x140>(bt, bw);   // row_mirror
        return (int)__builtin_amdgcn_readfirstlane(bw);
    }
    for (int o = 32; o >= 1; o >>= 1) {
        int64_t ot = (int64_t)shfl64((uint64_t)bt, lane_id() ^ o);
        int ow = __shfl(bw, lane_id() ^ o, 64);
        if (ot < bt || (ot == bt && ow < bw)) {
            bt = ot;
            bw = ow;
        }
    }
    return (int)__builtin_amdgcn_readfirstlane(bw);
}

// Cache::addrParse's set index (cache.cpp:145-152): a mask when the set count
// is a power of two (a runtime-uniform branch), the general modulo otherwise.
__device__ __forceinline__ uint64_t set_index(uint64_t addr, int offbits, uint64_t nsets) {
    const uint64_t x = addr >> offbits;
    return (nsets & (nsets - 1)) == 0 ? (x & (nsets - 1)) : x % nsets;
}

// LDS staging ring for predicted tree hops: ring_pf<LH>() full link rings per wave
// (one wave per workgroup), filled by global_load_lds_dwordx4 and consumed in
// hop order behind a counted vmcnt (loads, stores and LDS-DMA retire in issue
// order, MI355X_MICROARCH.md §waitcnt; hipcc would drain everything instead).
static __shared__ v2u64 lds_ring[PU_RING_PF][PU_QRING];        // latency kernel (LH)
static __shared__ v2u64 lds_ring_tp[PU_RING_PF_TP][PU_QRING];  // throughput kernels
template <bool LH>
__device__ __forceinline__ v2u64* ring_slot(int slot) {
    if constexpr (LH) return lds_ring[slot];
    else return lds_ring_tp[slot];
}

// computeQueueDelay's outcome for interval [f, s] if the search stops there
// (queue_model_history_tree.cpp:74-106): op 1 second<-t, 2 first<-t+d+p,
// 3 remove, 4 split; returns the delay d.
__device__ __forceinline__ uint64_t tree_case(uint64_t f, uint64_t s, uint64_t t, uint64_t p, uint64_t minp,
                                              uint32_t& op) {
    const uint64_t tp = t + p;
    const bool ge = t >= f;
    const bool fit_after = s - tp >= minp;
    const uint32_t op_ge = (t - f >= minp) ? (fit_after ? 4u : 1u) : (fit_after ? 2u : 3u);
    const uint32_t op_lt = (s - (f + p) >= minp) ? 2u : 3u;
    op = ge ? op_ge : op_lt;
    return ge ? 0 : f - t;
}

// Tree branch of QueueModelHistoryTree::computeQueueDelay
// (queue_model_history_tree.cpp:64-112) on the full ring, branch-light: every
// lane evaluates the search predicate and the outcome for its two intervals
// (the view is in logical order, RingView), the leftmost hit is picked with
// one 128-bit scan, and the edit is one range move (DPP rotate) plus at most
// two overridden fields.  head/cnt are the post-prune values and are updated;
// edited slots are written back.  The ring side that moves is the shorter one
// (a prefix move shifts `head`): only the logical order is observable.
// `slot` >= 0: the view is also staged in LDS slot `slot` (ring_dma, logical
// order), and the range move reads each lane's new intervals from there, at
// its logical index +-1 (two ds_read_b128, no cross-lane moves); -1: the view
// came from HBM (ring_load) and the move is a DPP rotate of the registers.
template <bool LH>
__device__ __forceinline__ uint64_t tree_op(const NetCtx& c, int q, const RingView& v, uint32_t& head,
                                            uint32_t& cnt, uint64_t t, uint64_t p, uint64_t minp, uint64_t& err,
                                            uint64_t& f0n, uint64_t& f1n, int slot) {
    const int ln = lane_id();
    PROF_T(p_s);
    const uint64_t tp = t + p;
    const uint32_t head0 = head;
    const uint32_t jl = (uint32_t)ln, jh = (uint32_t)ln + 64;   // logical indices of the lane's intervals
    const bool pl = jl < cnt && ((v.lf <= t && tp <= v.ls) || (t < v.lf && v.ls - v.lf >= p));
    const bool ph = jh < cnt && ((v.hf <= t && tp <= v.hs) || (t < v.hf && v.hs - v.hf >= p));
    const uint64_t rlo = ballot(pl), rhi = ballot(ph);
    uint32_t k;
    if (rlo) k = (uint32_t)__builtin_ctzll(rlo);
    else if (rhi) k = 64 + (uint32_t)__builtin_ctzll(rhi);
    else {                        // search returned NULL: an assert in the reference
        err |= PU_ERRF_QUEUE;
        k = 0;
    }
    PROF_ADD(PF_T_SEARCH, p_s);
    PROF_T(p_d);
    // the outcome for the found interval only, on the scalar unit
    uint64_t sf, ss;
    if (k >= 64) {              // uniform: no selects between the halves
        sf = rl64(v.hf, (int)(k - 64));
        ss = rl64(v.hs, (int)(k - 64));
    } else {
        sf = rl64(v.lf, (int)k);
        ss = rl64(v.ls, (int)k);
    }
    uint32_t op;
    const uint64_t d = tree_case(sf, ss, t, p, minp, op);
    // the edit as: slots whose logical index is in [r0, r0+rlen) take their
    // NEXT/PREV neighbour; then first<-fv at logical fi, second<-t at si
    uint32_t r0 = 0, rlen = 0, fi = 0xFFFFFFFFu, si = 0xFFFFFFFFu;
    bool next = true;
    const uint64_t fv = op == 2 ? tp + d : tp;
    if (op == 1) {
        si = k;
    } else if (op == 2) {
        fi = k;
    } else if (op == 3) {
        if (k == 0) {
            head = (head + 1) & (PU_QRING - 1);
        } else if (k < cnt - 1 - k) {             // move [0, k) up one, head+1
            r0 = 1; rlen = k; next = false;
            head = (head + 1) & (PU_QRING - 1);
        } else {                                  // move (k, cnt) down one
            r0 = k; rlen = cnt - 1 - k; next = true;
        }
        cnt = cnt - 1;
    } else {
        if (2 * k + 1 < cnt) {                    // [0, k] down one, head-1; node k-1 = [f, t], k = [t+p, s]
            r0 = PU_QRING - 1; rlen = k + 1; next = true;
            si = (k - 1) & (PU_QRING - 1); fi = k;
            head = (head + PU_QRING - 1) & (PU_QRING - 1);
        } else {                                  // (k, cnt) up one; node k = [f, t], k+1 = [t+p, s]
            r0 = k + 1; rlen = cnt - k; next = false;
            si = k; fi = k + 1;
        }
        cnt = cnt + 1;
    }
    PROF_ADD(PF_T_DECIDE, p_d);
    PROF_T(p_e);
    uint64_t lf = v.lf, ls = v.ls, hf = v.hf, hs = v.hs;
    bool wl = false, wh = false;
    if (rlen) {
        wl = ((jl - r0) & (PU_QRING - 1)) < rlen;
        wh = ((jh - r0) & (PU_QRING - 1)) < rlen;
        if (slot >= 0) {
            // lanes outside the range read their own (unchanged, or dead and
            // never written back) slot: no select afterwards
            const v2u64* L = ring_slot<LH>(slot);
            const uint32_t dn = next ? 1u : PU_QRING - 1;
            const v2u64 a = L[wl ? (jl + dn) & (PU_QRING - 1) : jl];
            const v2u64 b = L[wh ? (jh + dn) & (PU_QRING - 1) : jh];
            lf = a.x;
            ls = a.y;
            hf = b.x;
            hs = b.y;
        } else {
            uint64_t nlf, nls, nhf, nhs;
            if (next) {
                ring_shift<true>(v.lf, v.hf, nlf, nhf);
                ring_shift<true>(v.ls, v.hs, nls, nhs);
            } else {
                ring_shift<false>(v.lf, v.hf, nlf, nhf);
                ring_shift<false>(v.ls, v.hs, nls, nhs);
            }
            lf = wl ? nlf : lf;
            ls = wl ? nls : ls;
            hf = wh ? nhf : hf;
            hs = wh ? nhs : hs;
        }
    }
    lf = jl == fi ? fv : lf;
    hf = jh == fi ? fv : hf;
    ls = jl == si ? t : ls;
    hs = jh == si ? t : hs;
    wl = wl || jl == fi || jl == si;
    wh = wh || jh == fi || jh == si;
    PROF_ADD(PF_T_EDIT, p_e);
    PROF_T(p_w);
    AS1 v2u64* R = q_ring(c, q);
    if (wl) R[(head0 + jl) & (PU_QRING - 1)] = v2u64{lf, ls};
    if (wh) R[(head0 + jh) & (PU_QRING - 1)] = v2u64{hf, hs};
    // the header's copies of the first two interval starts: the new cursor is
    // the old logical index (head - head0) & 127 (0, 1 or 127)
    // (0, 1 or 127: a uniform branch, no selects between the halves)
    const uint32_t s0 = (head - head0) & (PU_QRING - 1);
    if (s0 == PU_QRING - 1) {
        f0n = rl64(hf, 63);
        f1n = rl64(lf, 0);
    } else {
        f0n = rl64(lf, (int)s0);
        f1n = rl64(lf, (int)s0 + 1);
    }
    PROF_ADD(PF_T_STORE, p_w);
    return d;
}

// ---- SGPR lane-mask helpers (the latency kernel's window loop) ---------------
// lane bit of m set ? b : a: one v_cndmask with the mask as its SGPR selector
// (a predicate held as a wave mask never goes through a VGPR boolean)
__device__ __forceinline__ uint32_t selm32(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    m = uni64(m);   // wave-uniform; a mask the compiler knows as a constant still goes in an SGPR pair
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
__device__ __forceinline__ uint64_t selm64(uint64_t m, uint64_t a, uint64_t b) {
    const uint32_t lo = selm32(m, (uint32_t)a, (uint32_t)b), hi = selm32(m, (uint32_t)(a >> 32), (uint32_t)(b >> 32));
    return ((uint64_t)hi << 32) | lo;
}
// ---- queue headers ---------------------------------------------------------
// The engine's header (PU_HDR_BYTES = 32 per queue, two 16-B pieces):
//   a = {n | head, n1 | count}   b = {newest, f0}
// n (all visits) and n1 (visits with packet length p1) are exact doubles; the
// ring cursor rides in their low 7 mantissa bits, which are 0 for integers
// below 2^45.  The engine sends only two packet lengths over a link (0-byte
// messages: header_flits = p0; blocks: plen_blk = p1, network.cpp:104) and
// one over a bus (bus_latency), so the M/G/1 moments of
// queue_model_m_g_1.cpp:45-55 follow from the counts:
//   Σs = p0·n + (p1 - p0)·n1,  Σs² = p0²·n + (p1² - p0²)·n1
// — the same doubles the reference accumulates (each partial sum is an
// integer below 2^53, so every addition is exact, and each fma's exact result
// is representable; a moment reaching 2^53 or n reaching 2^45 sets
// PU_ERRF_QUEUE, an engine limit past ~10^13 visits of one link).  The first
// interval start f0 (the M/G/1 test) is in b: one 32-B read-modify-write per
// visit, four neighbouring hops of a route per 128-B line (round 4's 48-B
// header read a second line of c pieces per four hops).
// The unit hooks (any packet length: unit_queue_kernel, unit_network_kernel)
// keep the wide header (WIDE, PU_HDR_WIDE_BYTES = 48: {a, b} of every queue,
// then c of every queue): a = {n, Σs}, b = {Σs², newest} as doubles,
// c = {head, count, f0}.
//
// Latency mode (LH): a launch with at most one replica per CU keeps every
// queue header of its replica in the CU's LDS for the whole launch (copied in
// at the start, back at the end), so the header round trip of each route
// window becomes an LDS read: PU_LDS_Q queues, a 32-B slot {a, b} each, plus
// one 8-B M/G/1 cache word per queue (lds_qcache).
//
// The M/G/1 cache: the queue delay of an M/G/1 visit depends only on the
// moments the link holds before the visit (queue_model_m_g_1.cpp:16-42), and
// those change only when the link is visited.  In latency mode a second wave
// of the workgroup (mg1_helper) recomputes the wait of every link a route
// window just updated, on another SIMD, and stores it as
// wait | (n ^ wait) << 32 (n < 2^32, waits < 2^32 - 1; larger ones
// are not cached); the simulating wave uses it when the high half xor the
// wait equals its header's n and computes the wait itself otherwise.  The tag
// is n itself, not a residue, so a slot the helper skipped (it fell more than
// PU_HQ ids behind) can never match a later visit; folding the wait into it
// makes a read of the slot torn against the helper's write (old wait, new tag
// or the reverse) fail the check unless both waits are equal.  The main wave
// writes piece a (which holds n) after b; the helper reads a, then b, then a
// again and stores only when both reads of a are bit-identical (n grows at
// every visit, so a read of a torn against the main wave's write, or a b newer
// than a, shows as a mismatch, and a wait computed from such a mix carries a
// tag no later visit has): a stored wait was computed from exactly the
// moments its tag names.
#define PU_LDS_Q 3400u                     // queues of the LDS header image (a 32x32 mesh has 1,984)
#define PU_LDS_SLOT 2u                     // 16-B pieces per LDS header slot
#define PU_MG1_CACHE_NONE 0xFFFFFFFFFFFFFFFFull
#define PU_MG1_WAIT_BITS 32
#define AS3 __attribute__((address_space(3)))
static __shared__ v4u32 lds_qhdr[PU_LDS_Q * PU_LDS_SLOT];
static __shared__ uint64_t lds_qcache[PU_LDS_Q];
// queue ids whose header the main wave just wrote back, for the helper
#define PU_HQ 256u
static __shared__ uint16_t lds_hq[PU_HQ];
static __shared__ uint32_t lds_hq_head;    // ids pushed so far (main writes)
static __shared__ uint32_t lds_main_done;  // the main wave left its request loop

constexpr uint32_t PU_HDR_CUR = 0x7Fu;              // ring cursor bits in the low mantissa bits
constexpr double PU_TWO53 = 9007199254740992.0, PU_TWO45 = 35184372088832.0;
__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ double dbl_of(uint32_t lo, uint32_t hi) { return __longlong_as_double((long long)u64of(lo, hi)); }

// Header write-back of queue q by the calling lane(s).  Packed: b = {newest,
// f0} then a = {n|head, n1|count} (one aligned 32-B piece pair).  Wide: a =
// {n, Σs} and b = {Σs², newest} (every visit changes them), c = {head, count,
// f0} only when the visit changed the free-interval ring.
template <bool LH, bool WIDE>
__device__ __forceinline__ void q_store_hdr(const NetCtx& c, int q, const QState& st, bool ring_changed = true) {
    if constexpr (WIDE) {
        uint64_t sb = (uint64_t)__double_as_longlong(st.sum), qb = (uint64_t)__double_as_longlong(st.sum_sq);
        const uint64_t nb = (uint64_t)__double_as_longlong(st.n);
        const v4u32 a = v4u32{(uint32_t)nb, (uint32_t)(nb >> 32), (uint32_t)sb, (uint32_t)(sb >> 32)};
        const v4u32 b = v4u32{(uint32_t)qb, (uint32_t)(qb >> 32), (uint32_t)st.newest, (uint32_t)(st.newest >> 32)};
        const v4u32 cc = v4u32{st.head, st.count, (uint32_t)st.f0, (uint32_t)(st.f0 >> 32)};
        AS1 v4u32* H = q_hdr_ab(c, q);
        H[0] = a;
        H[1] = b;
        if (ring_changed) *q_hdr_c(c, q) = cc;
    } else {
        const uint64_t w0 = (uint64_t)__double_as_longlong(st.n), w1 = (uint64_t)__double_as_longlong(st.sum1);
        const v4u32 a = v4u32{(uint32_t)w0 | st.head, (uint32_t)(w0 >> 32), (uint32_t)w1 | st.count,
                              (uint32_t)(w1 >> 32)};
        const v4u32 b = v4u32{(uint32_t)st.newest, (uint32_t)(st.newest >> 32), (uint32_t)st.f0,
                              (uint32_t)(st.f0 >> 32)};
        if constexpr (LH) {
            // b first, a (with n) last: see the M/G/1 cache above
            volatile AS3 v4u32* H = (volatile AS3 v4u32*)&lds_qhdr[(size_t)q * PU_LDS_SLOT];
            H[1] = b;
            H[0] = a;
        } else {
            AS1 v4u32* H = reinterpret_cast<AS1 v4u32*>(c.qhdr + (uint64_t)q * PU_HDR_BYTES);
            H[0] = a;
            H[1] = b;
        }
    }
}

// M/G/1 update (queue_model_m_g_1.cpp:45-55) and header write-back (lane 0).
template <bool LH, bool WIDE>
__device__ __forceinline__ void q_finish(const NetCtx& c, int q, QState& st, uint64_t t, uint64_t p, uint64_t d) {
    if constexpr (WIDE) {
        st.sum_sq = st.sum_sq + (double)p * (double)p;
        st.sum = st.sum + (double)p;
        st.n = st.n + 1.0;
    } else {
        st.n = st.n + 1.0;
        if (p != c.p0) st.sum1 = st.sum1 + 1.0;
    }
    uint64_t fin = t + d + p;
    st.newest = fin > st.newest ? fin : st.newest;
    if (lane_id() == 0) q_store_hdr<LH, WIDE>(c, q, st);
}

// One computeQueueDelay on a uniform header (bus queues, unit tests).
template <bool LH, bool WIDE>
__device__ __forceinline__ uint64_t q_step(const NetCtx& c, int q, QState& st, uint64_t t, uint64_t p, uint64_t minp,
                                           uint64_t& mg1, uint64_t& err) {
    uint64_t d;
    if (st.f0 > t + p) {             // older than the tracked history: M/G/1 (history_tree.cpp:58-63)
        d = mg1_wait(st);
        mg1++;
    } else {
        RingView v;
        ring_load(c, q, st.head, st.count, v);
        uint64_t f1;
        d = tree_op<LH>(c, q, v, st.head, st.count, t, p, minp, err, st.f0, f1, -1);
        if (st.count >= PU_QMAX) {   // the next call's prune (history_tree.cpp:49-55), done now
            st.head = (st.head + 1) & (PU_QRING - 1);
            st.count--;
            st.f0 = f1;
        }
    }
    if constexpr (!WIDE)
        if (p != c.p0 && p != c.p1) err |= PU_ERRF_QUEUE;   // a length the packed header cannot count
    q_finish<LH, WIDE>(c, q, st, t, p, d);
    return d;
}

// The queue state a header holds.  Packed: the moments from the counts
// (exact, see above; a moment at 2^53 or more sets PU_ERRF_QUEUE through
// `err`).  Wide: as stored.
template <bool WIDE>
__device__ __forceinline__ QState hdr_state(const NetCtx& ctx, v4u32 a, v4u32 b, v4u32 c, uint64_t& err) {
    QState st;
    if constexpr (WIDE) {
        st.n = __longlong_as_double((long long)u64of(a.x, a.y));
        st.sum = __longlong_as_double((long long)u64of(a.z, a.w));
        st.sum_sq = __longlong_as_double((long long)u64of(b.x, b.y));
        st.newest = u64of(b.z, b.w);
        st.head = c.x;
        st.count = c.y;
        st.f0 = u64of(c.z, c.w);
        st.sum1 = 0.0;
    } else {
        st.head = a.x & PU_HDR_CUR;
        st.count = a.z & PU_HDR_CUR;
        st.n = dbl_of(a.x & ~PU_HDR_CUR, a.y);
        st.sum1 = dbl_of(a.z & ~PU_HDR_CUR, a.w);
        st.newest = u64of(b.x, b.y);
        st.f0 = u64of(b.z, b.w);
        const double p0 = (double)ctx.p0, p1 = (double)ctx.p1;
        st.sum = __builtin_fma(p1 - p0, st.sum1, p0 * st.n);
        st.sum_sq = __builtin_fma(p1 * p1 - p0 * p0, st.sum1, (p0 * p0) * st.n);
        if (st.sum_sq >= PU_TWO53 || st.n >= PU_TWO45) err |= PU_ERRF_QUEUE;
    }
    return st;
}
__device__ __forceinline__ v4u32 uni4(v4u32 v) { return v4u32{uni32(v.x), uni32(v.y), uni32(v.z), uni32(v.w)}; }
template <bool LH, bool WIDE>
__device__ __forceinline__ void hdr_load(const NetCtx& c, int q, v4u32& a, v4u32& b, v4u32& cc) {
    if constexpr (WIDE) {
        const AS1 v4u32* H = q_hdr_ab(c, q);
        a = H[0];
        b = H[1];
        cc = *q_hdr_c(c, q);
    } else if constexpr (LH) {
        const AS3 v4u32* H = (const AS3 v4u32*)&lds_qhdr[(size_t)q * PU_LDS_SLOT];
        a = H[0];
        b = H[1];
        cc = v4u32{0u, 0u, 0u, 0u};
    } else {
        const AS1 v4u32* H = reinterpret_cast<const AS1 v4u32*>(c.qhdr + (uint64_t)q * PU_HDR_BYTES);
        a = H[0];
        b = H[1];
        cc = v4u32{0u, 0u, 0u, 0u};
    }
}

// A whole queue op loading its own state (bus queues, unit tests).
template <bool LH, bool WIDE>
__device__ __forceinline__ uint64_t q_op(const NetCtx& c, int q, uint64_t t, uint64_t p, uint64_t minp, uint64_t& mg1,
                                         uint64_t& err) {
    v4u32 a, b, cc;
    hdr_load<LH, WIDE>(c, q, a, b, cc);
    QState st = hdr_state<WIDE>(c, uni4(a), uni4(b), uni4(cc), err);
    return q_step<LH, WIDE>(c, q, st, t, p, minp, mg1, err);
}

// n / d for n < 2^16 as a multiply-high by m = ceil(2^32 / d) (exact there:
// n * (m*d - 2^32) < 2^32); uniform operands stay on the scalar unit.
__device__ __forceinline__ uint32_t div_magic(uint32_t n, uint32_t m) { return (uint32_t)(((uint64_t)n * m) >> 32); }
__device__ __forceinline__ void net_coords(const NetCtx& c, int id, int& x, int& y, int& z) {
    const uint32_t w = (uint32_t)c.w;
    if (c.net_type == 1) {
        const uint32_t zq = div_magic((uint32_t)id, c.w2_magic);
        const uint32_t rem = (uint32_t)id - zq * (uint32_t)c.w2;
        const uint32_t yq = div_magic(rem, c.w_magic);
        x = (int)(rem - yq * w);
        y = (int)yq;
        z = (int)zq;
    } else {
        const uint32_t yq = div_magic((uint32_t)id, c.w_magic);
        x = (int)((uint32_t)id - yq * w);
        y = (int)yq;
        z = 0;
    }
}
// Network::getLink (network.cpp:213-307), one record per undirected edge: the
// link of hop h of the X-then-Y-then-Z route from (sx,sy,sz) to (rx,ry,rz),
// computed branch-free across lanes (hops of one route take different ranges):
// hop h < hx moves along x at (sy, sz), then along y at (rx, sz), then along z
// at (rx, ry); a = the coordinate (or coordinate - 1 moving down).  The record
// index is ours, not getLink's numbering (only the edge -> record bijection is
// observable): the edges of one row (x), column (y) or pillar (z) are
// consecutive, so the hops of a route segment are consecutive records and two
// neighbouring hops share a 128-B line of headers (a visit reads half a line
// instead of a whole one) and the LDS image's slots of a window spread over the
// banks.  2-D: x (sy*(w-1) + a), y (w(w-1) + rx*(w-1) + a); 3-D: x, y, z blocks
// of w^2(w-1) each, (sz*w + sy), (sz*w + rx), (ry*w + rx) rows of w-1.
__device__ __forceinline__ int net_route_link(const NetCtx& c, int h, int sx, int sy, int sz, int rx, int ry, int rz,
                                              int hx, int hy) {
    const int w = c.w, w1 = c.w - 1;
    const bool e = rx > sx, n = ry > sy, u = rz > sz;   // wave-uniform
    const bool inx = h < hx, iny = h < hx + hy;
    const int hy_ = h - hx, hz_ = h - hx - hy;
    const int ax = e ? sx + h : sx - h - 1;
    const int ay = n ? sy + hy_ : sy - hy_ - 1;
    if (c.net_type != 1) return inx ? sy * w1 + ax : (w + rx) * w1 + ay;
    const int az = u ? sz + hz_ : sz - hz_ - 1;
    const int blk = w * w * w1;
    return inx ? (sz * w + sy) * w1 + ax : iny ? blk + (sz * w + rx) * w1 + ay : 2 * blk + (ry * w + rx) * w1 + az;
}


// Stage ring q (live slots [head, head+cnt)) into LDS slot `slot` in logical
// order; dead positions read the last live slot instead (a line the live
// part reads anyway) and are never used.
template <bool LH>
__device__ __forceinline__ void ring_dma(const NetCtx& c, int q, uint32_t head, uint32_t cnt, int slot) {
    const int ln = lane_id();
    const AS1 v2u64* R = q_ring(c, q);
    // logical order (RingView): LDS position l <- interval l from the cursor
    // (dead positions re-read the last live slot: min instead of a compare and select)
    const uint32_t last = cnt - 1;
    const AS1 v2u64* ga = R + ((head + __builtin_elementwise_min((uint32_t)ln, last)) & (PU_QRING - 1));
    const AS1 v2u64* gb = R + ((head + __builtin_elementwise_min((uint32_t)ln + 64, last)) & (PU_QRING - 1));
    const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) v2u64*)ring_slot<LH>(slot);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(la), hi = lo + 64 * sizeof(v2u64);
    unsigned keep;
    // lgkmcnt(0): the slot's previous ds_reads have returned before it is refilled
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(ga), "v"(gb), "s"(lo), "s"(hi)
        : "memory");
}
template <bool LH>
__device__ __forceinline__ void ring_from_lds(int slot, RingView& v) {
    const int ln = lane_id();
    const v2u64* r = ring_slot<LH>(slot);
    const v2u64 a = r[ln], b = r[ln + 64];
    v = RingView{a.x, a.y, b.x, b.y};
}

// LDS-DMA of one 16-B (X4) or 4-B (X1) piece per active lane to lds + 16*lane
// (X4) / 4*lane (X1).  lgkmcnt(0) first: earlier ds_reads of the target are done.
template <bool X4>
__device__ __forceinline__ void lds_dma(const AS1 char* src, uint32_t lds_base) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(lds_base);
    unsigned keep;
    if (X4)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(lo) : "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(lo) : "memory");
}
template <class T>
__device__ __forceinline__ uint32_t lds_addr(T* p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)p;
}

// The request's home directory set, staged before the request transmit (lane
// w = way w: bytes 0-15 and the two dwords of the sharer word).  Up to 32 ways.
static __shared__ v4u32 lds_dir_a[32];
static __shared__ uint32_t lds_dir_w[2][32];

// Network::transmit (network.cpp:97-160).  Inlined (a call would wait for every
// outstanding store at entry and reload a spilled register at exit); every
// argument is made wave-uniform so the hop loop runs on SGPRs and scalar
// branches.  The protocol code reaches it from four sites only.
// Lane h prefetches hop h's link header and the two interval starts at its
// ring head; only hops taking the tree branch fetch their full ring.
template <bool LH, int NL, bool WIDE>
__device__ __forceinline__ uint64_t net_transmit(const Geo* __restrict__ g, char* base_in, int src, int dst, int len,
                                                 uint64_t timer, uint32_t& hq_head) {
    PROF_T(p_pre);
    NetCtx c;
    AS1 char* base = (AS1 char*)(char*)uni64((uint64_t)base_in);
    c.qhdr = base + OFF(g->off_qhdr);
    c.qring = base + OFF(g->off_qring);
    c.hdr_c = (uint32_t)g->nqueues * PU_HDR_AB;
    c.p0 = (uint32_t)g->header_flits;     // packed headers: 0-byte messages ...
    c.p1 = (uint32_t)g->plen_blk;         // ... and blocks
    c.router = (uint32_t)g->router_delay;
    c.link_delay = (uint32_t)g->link_delay;
    c.inject = (uint32_t)g->inject_delay;
    c.header_flits = g->header_flits;
    c.data_width = g->data_width;
    c.w = g->net_width;
    c.net_type = g->net_type;
    c.w_magic = (uint32_t)g->w_magic;
    c.w2_magic = (uint32_t)g->w2_magic;
    c.w2 = g->w2;
    c.blk_len = g->blk_len;
    c.plen_blk = g->plen_blk;
    src = (int)uni32((uint32_t)src);
    dst = (int)uni32((uint32_t)dst);
    len = (int)uni32((uint32_t)len);
    timer = uni64(timer);
    if (src == dst) return 0;
    const int ln = lane_id();
    // network.cpp:104 packet length; the engine only sends 0-byte and block
    // messages (the packed header counts those two lengths; the unit hook's
    // wide header takes any)
    int plen;
    uint64_t err = 0;
    if constexpr (WIDE) {
        plen = len == 0 ? c.header_flits
             : len == c.blk_len ? c.plen_blk
             : c.header_flits + (int)ceil((double)len / (double)c.data_width);
    } else {
        plen = len == 0 ? c.header_flits : c.plen_blk;
        if (len != 0 && len != c.blk_len) err |= PU_ERRF_QUEUE;
    }
    int sx, sy, sz, rx, ry, rz;
    net_coords(c, src, sx, sy, sz);
    net_coords(c, dst, rx, ry, rz);
    const int hx = abs(rx - sx), hy = abs(ry - sy), hz = abs(rz - sz);
    const int hops = hx + hy + hz;
    uint64_t t = timer + c.inject;
    uint64_t mg1 = 0;
    PROF_ADD(PF_NPRE, p_pre);
    for (int b0 = 0; b0 < hops; b0 += 64) {
        PROF_T(p_setup);
        PROF_CNT(PF_WINDOWS, 1);
        // ---- prefetch the window: lane h = hop b0+h loads its link's header
        // (32 B: visit counts, ring cursor, newest finish, the first interval start)
        const int h = b0 + ln;
        const int nh = hops - b0 < 64 ? hops - b0 : 64;
        // Every lane loads: a lane past the route takes the route's last hop,
        // the same address as that hop's own lane (no extra line, no
        // exec-masked branch, no zeroed registers); such lanes are masked
        // wherever a hop's results are used (ln < nh), and their copy of a
        // real header raises no error that hop does not raise itself.
        const int rq = net_route_link(c, h < hops ? h : hops - 1, sx, sy, sz, rx, ry, rz, hx, hy);
        v4u32 ha, hb, hc;
        hdr_load<LH, WIDE>(c, rq, ha, hb, hc);
        uint64_t vcache = PU_MG1_CACHE_NONE;
        if constexpr (LH) vcache = lds_qcache[rq];
        // Everything about hop h that does not depend on its arrival time is
        // computed by lane h here, once per window: the front interval (the
        // prune of a full history was applied when it filled), the M/G/1 wait
        // from the pre-update moments (queue_model_m_g_1.cpp:16-42) and the
        // moment updates of q_finish.  The route's links are distinct, so no
        // hop sees another hop's update.
        const QState hs = hdr_state<WIDE>(c, ha, hb, hc, err);
        uint32_t vhead = hs.head, vcnt = hs.count;
        uint64_t vf0 = hs.f0;
        const uint64_t vfront = vf0;    // the tree's minimum: the M/G/1 test
        // hop h's queue delay if it takes M/G/1: the helper's cached wait when
        // its tag is this header's n, else computed here (latency mode), or
        // computed here (throughput mode)
        uint64_t vd = 0;
        [[maybe_unused]] bool need = ln < nh;
        if constexpr (LH) {
            const uint64_t wmask = (1ull << PU_MG1_WAIT_BITS) - 1;
            const bool hit = need && (vcache & wmask) != wmask && hs.n < 4294967296.0 &&
                             ((uint32_t)(vcache >> PU_MG1_WAIT_BITS) ^ (uint32_t)vcache) == (uint32_t)hs.n;
            if (hit) vd = vcache & wmask;
            need = need && !hit;
            if (ballot(need)) {
                PROF_T(p_mg1);
                const uint64_t w = mg1_wait(hs);
                if (need) vd = w;
                PROF_ADD(PF_MG1RUN, p_mg1);
            }
        } else {
            // every lane: a lane past the route holds a copy of the route's last
            // hop, and its wait only reaches lanes above the route in the
            // inclusive scan below (no mask, no select)
            PROF_T(p_mg1);
            vd = mg1_wait(hs);
            PROF_ADD(PF_MG1RUN, p_mg1);
        }
        PROF_CNT(PF_MG1LANES, (uint64_t)nh);
        PROF_CNT(PF_MG1HITS, (uint64_t)__builtin_popcountll(ballot(ln < nh && !need)));
        PROF_CNT(PF_MG1PRESENT, (uint64_t)__builtin_popcountll(ballot(ln < nh && vcache != PU_MG1_CACHE_NONE)));
        uint64_t vfin = 0;              // t + d + p of hop h
        // Hop j arrives no earlier than LB_j = t + (j+1)*router + j*link_delay
        // (queue delays are >= 0).  A hop whose front free interval starts by
        // LB_j + p cannot take the M/G/1 branch, so its full ring is certainly
        // needed: stage those rings now, ring_pf<LH>() ahead, in hop order.
        // (every lane computes; the mask drops the lanes past the route)
        const uint64_t nhm = nh >= 64 ? ~0ull : ((1ull << nh) - 1);
        const uint64_t lb = t + (uint64_t)(ln + 1) * c.router + (uint64_t)ln * c.link_delay;
        const uint64_t M = ballot(vfront <= lb + (uint64_t)plen) & nhm;
        uint64_t mi = M, mc = M;        // issue / consume cursors over the predicted hops
        int issued = 0, consumed = 0;
        constexpr int RPF = ring_pf<LH>();
        while (mi && issued < RPF) {
            const int jj = (int)__builtin_ctzll(mi);
            mi &= mi - 1;
            ring_dma<LH>(c, (int)rl32((uint32_t)rq, jj), rl32(vhead, jj), rl32(vcnt, jj), issued % RPF);
            issued++;
        }
        PROF_ADD(PF_NSETUP, p_setup);
        PROF_T(p_hops);
        // ---- the arrival-time recurrence t_j = t + (j+1)*router + sum_{i<j}(d_i
        // + link_delay), lane-parallel: assume every remaining hop takes M/G/1
        // (its delay is then known), get all arrival times with one wave
        // prefix scan, and find the first hop whose front interval starts by
        // its arrival + p — the first tree hop.  Hops before it are final; the
        // tree hop is done by the wave.  Its delay d replaces the assumed
        // M/G/1 wait, which moves every later arrival by the same d - wait:
        // both kernels carry that as one uniform shift `sh` (mod 2^64, like
        // the sums): one scan per window.  (Round 3 measured the throughput
        // kernel 2.5% slower with the scan kept live across the tree
        // operation at 96 VGPRs and had it rescan after each tree hop; with
        // the 32-B headers that kernel spills no VGPR, and the shift is +0.5%
        // on the C4 headline, same box: profiles/r5c_ab_ens.txt.)
        uint64_t S = 0, A0 = 0, sh = 0;
        const uint64_t t0 = t;
        {
            // lanes past the route add their copies' terms above it: an
            // inclusive scan never carries them down
            const uint64_t e = vd + c.link_delay + c.router;
            S = ballot(e >= (1ull << 26)) == 0 ? (uint64_t)scan_incl_u32((uint32_t)e) : scan_incl_u64(e);
            A0 = t + c.router + (S - e);
        }
        int js = 0;
        {
            // the window's live hops and the M/G/1 hops' finish times as wave
            // masks (one v_cndmask per dword), the staging slots as wrapping
            // counters and a three-way DMA wait instead of a modulo and an
            // eight-way ladder: one simulation alone +1.6% open loop, +3.4%
            // closed loop (same-box A/B, profiles/r4d_ab_single.txt; a tree
            // operation on wave masks, tree_op's predicates combined on the
            // scalar unit, ran 9% slower closed loop: more scalar
            // instructions than it saved)
            int islot = issued % RPF, cslot = 0;
            while (js < nh) {
                const uint64_t live = nhm & (~0ull << js);
                const uint64_t A = A0 + sh;
                const uint64_t cand = ballot(vfront <= A + (uint64_t)plen) & live;
                const int jt = cand ? (int)__builtin_ctzll(cand) : nh;
                // hops [js, jt) took M/G/1: their finish times
                const uint64_t fm = jt >= 64 ? live : live & ((1ull << jt) - 1);
                vfin = selm64(fm, vfin, A + vd + (uint64_t)plen);
                mg1 += (uint64_t)(jt - js);
                if (jt == nh) {                               // the rest of the window is M/G/1
                    t = t0 + rl64(S, nh - 1) + sh;
                    break;
                }
                PROF_T(p_tree);
                PROF_CNT(PF_TREEHOPS, 1);
                PROF_T(p_pick);
                const uint64_t tj = rl64(A, jt);
                const int q = (int)rl32((uint32_t)rq, jt);
                uint32_t head = rl32(vhead, jt), cnt = rl32(vcnt, jt);
                uint64_t f0n, f1n, d;
                RingView v;
                const bool staged = mc && jt == (int)__builtin_ctzll(mc);
                int tslot = -1;
                if (staged) {
                    // predicted: its ring is (being) staged in LDS slot cslot
                    mc &= mc - 1;
                    PROF_T(p_wait);
                    const int newer = issued - consumed - 1;  // rings issued after this one, < RPF
                    static_assert(RPF <= 3, "the three-way wait covers at most 2 newer staged rings");
                    if (newer <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    else if (newer == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                    PROF_ADD(PF_NWAIT, p_wait);
                    ring_from_lds<LH>(cslot, v);
                    tslot = cslot;
                    cslot = cslot == RPF - 1 ? 0 : cslot + 1;
                    consumed++;
                } else {                            // not predicted (arrival pushed past the front)
                    PROF_CNT(PF_DEMAND, 1);
                    ring_load(c, q, head, cnt, v);
                }
#ifdef PU_PROF
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the ring's LDS read, in this region
#endif
                PROF_ADD(PF_T_LDS, p_pick);         // hop pick, DMA wait (NWAIT), ring from LDS
                d = tree_op<LH>(c, q, v, head, cnt, tj, (uint64_t)plen, c.link_delay, err, f0n, f1n, tslot);
                PROF_T(p_upd);
                if (cnt >= PU_QMAX) {               // the next call's prune (history_tree.cpp:49-55), done now
                    head = (head + 1) & (PU_QRING - 1);
                    cnt--;
                    f0n = f1n;
                }
                if (staged && mi) {                 // keep PF rings in flight
                    PROF_T(p_r);
                    const int jj = (int)__builtin_ctzll(mi);
                    mi &= mi - 1;
                    ring_dma<LH>(c, (int)rl32((uint32_t)rq, jj), rl32(vhead, jj), rl32(vcnt, jj), islot);
                    islot = islot == RPF - 1 ? 0 : islot + 1;
                    issued++;
                    PROF_ADD(PF_T_REFILL, p_r);
                }
                sh += d - rl64(vd, jt);
                // (hop jt's assumed wait vd is not read again: later M/G/1 finish
                // times and shifts use the lanes after it)
                wl_hop(vhead, head, vcnt, cnt, vf0, f0n, vfin, tj + d + (uint64_t)plen, jt);
                t = tj + d + c.link_delay;
                js = jt + 1;
                PROF_ADD(PF_T_UPD, p_upd);          // prune, refill (T_REFILL), hop results into the window
                PROF_ADD(PF_NTREE, p_tree);
            }
        }
        PROF_ADD(PF_NHOPS, p_hops);
        PROF_T(p_wb);
        // ---- header write-back, one hop per lane (queue_model_m_g_1.cpp:45-55)
        if (ln < nh) {
            QState st = hs;
            st.head = vhead;
            st.count = vcnt;
            st.f0 = vf0;
            if constexpr (WIDE) {
                st.sum_sq = st.sum_sq + (double)plen * (double)plen;
                st.sum = st.sum + (double)plen;
                st.n = st.n + 1.0;
            } else {
                st.n = st.n + 1.0;
                if (plen != (int)c.p0) st.sum1 = st.sum1 + 1.0;
            }
            st.newest = vfin > st.newest ? vfin : st.newest;
            q_store_hdr<LH, WIDE>(c, rq, st, vhead != hs.head || vcnt != hs.count || vf0 != hs.f0);
            if constexpr (LH) lds_hq[(hq_head + (uint32_t)ln) & (PU_HQ - 1)] = (uint16_t)rq;
        }
        if constexpr (LH) {   // publish the window's links to the helper, after their ids
            hq_head += (uint32_t)nh;
            asm volatile("" ::: "memory");
            if (ln == 0) *(volatile AS3 uint32_t*)&lds_hq_head = hq_head;
        }
        // No drain here: every staged ring was waited for when its hop consumed
        // it (predicted hops are a subset of the tree hops), and the header
        // stores' acknowledgements overlap the next window's loads (a wave's
        // vector memory operations are processed in order, so those loads
        // see the stores).
        PROF_ADD(PF_NWB, p_wb);
    }
    PROF_T(p_post);
    t += c.router;
    t += (uint64_t)(plen - 1);
    const uint64_t dist = (uint64_t)hops;
    {   // the six network sums in one ds_add_u64, lane k adding sum k (written
        // into the lanes by v_writelane: no lane compares)
        const uint64_t tot = t - timer, fl = dist * (uint64_t)plen;
        uint32_t lo = 0, hi = 0;
        lo = wlane<SN_ACC>(lo, 1u);
        lo = wlane<SN_DIST>(lo, (uint32_t)dist);
        lo = wlane<SN_TOTAL>(lo, (uint32_t)tot);
        hi = wlane<SN_TOTAL>(hi, (uint32_t)(tot >> 32));
        lo = wlane<SN_PLEN>(lo, (uint32_t)plen);
        lo = wlane<SN_FLITS>(lo, (uint32_t)fl);
        // mg1 <= hops < 2^9 (at most 65,536 nodes): no high word; flits =
        // hops x plen has none either while the packed header's two packet
        // lengths stay below 2^23 (a constant test in a compiled configuration)
        if (WIDE || (c.p0 | c.p1) >= (1u << 23)) hi = wlane<SN_FLITS>(hi, (uint32_t)(fl >> 32));
        lo = wlane<SN_MG1>(lo, (uint32_t)mg1);
        lds_add_u64_lanes(lds_u32addr(&lds_stat[0]) + 8u * (uint32_t)ln, ((uint64_t)hi << 32) | lo, SN_NET_LANES);
    }
    // err is per lane (a hop's header state): every bit here is
    // PU_ERRF_QUEUE, reported if any lane raised it (err_or stores lane 0's)
    if (ballot(err != 0)) err_or(PU_ERRF_QUEUE);
    PROF_ADD(PF_NPOST, p_post);
    return t - timer;
}

// Latency mode, the workgroup's second wave: recompute the M/G/1 wait of every
// link the simulating wave publishes (lds_hq), from the moments in the LDS
// header image, and store it in the link's cache slot tagged with n.  Reads
// piece a (n), then b, then a again (the main wave writes a after b and c)
// and stores only when the two reads of a agree.
// Returns once the main wave has left its loop and every id is processed.
// Latency mode, the helper wave while it has no M/G/1 work (one simulation
// alone +3.4% open loop, +0.4% closed loop, same-box A/B,
// profiles/r4e_ab_single.txt): pull the lines
// the simulating wave will load for its next PU_PF_AHEAD requests toward this
// CU (its vector L1 and the XCD's L2): the request record, the requesting
// core's L1 set (tags/state and timestamps) and the home directory set.  Only
// loads (into a scratch LDS area, by LDS-DMA: no register of this wave waits
// for them, and the simulating wave's own vmcnt never sees them); the
// simulating wave reads everything again itself, so a prefetch can only be
// early, never wrong.  `cur` (lds_ctl.cur) is read as a hint and clamped.
#ifndef PU_PF_AHEAD
#define PU_PF_AHEAD 4
#endif
static __shared__ uint32_t lds_pf_junk[64];
__device__ __forceinline__ void pf_requests(const Geo* __restrict__ g, const char* base, const pu_req* reqs,
                                            uint64_t first, uint32_t n) {
    const int ln = lane_id();
    const uint32_t j = (uint32_t)ln >> 3, k = (uint32_t)ln & 7u;
    const bool mine = j < n;
    uint64_t addr = 0;
    int core = 0;
    if (mine) {
        const pu_req q = reqs[first + j];
        addr = q.addr;
        core = q.core;
    }
    const char* p = nullptr;
    if (mine && (uint32_t)core < (uint32_t)g->num_cores) {
        const LevelGeo& L = g->lv[0];
        const uint64_t set = set_index(addr, L.offbits, L.nsets);
        const uint64_t line0 = ((uint64_t)(uint32_t)core * L.nsets + set) * L.nways;
        if (k == 0) p = (const char*)(reqs + first + j);
        else if (k <= 2) {
            if ((k - 1) * 64 < L.nways * sizeof(LineMeta)) p = base + L.off_meta + line0 * sizeof(LineMeta) + (k - 1) * 64;
        } else if (k == 3) p = base + L.off_ts + line0 * 8;
        else if (g->sys_type == 0 && k <= 6 && (k - 4) * 64 < g->dir.nways * sizeof(DirLine)) {
            const DirGeo& D = g->dir;
            int hb = (int)((addr >> g->home_offbits) & (((uint64_t)1 << g->home_mask_bits) - 1));
            if (hb >= g->N) hb &= (1 << (g->home_mask_bits - 1)) - 1;    // System::allocHomeId
            const uint64_t ds = set_index(addr, D.offbits, D.nsets);
            const uint64_t dl0 = ((uint64_t)(uint32_t)hb * D.csets + (ds >> D.cset_shift)) * D.nways;
            p = base + D.off_line + dl0 * sizeof(DirLine) + (k - 4) * 64;
        }
    }
    if (p) lds_dma<false>((const AS1 char*)p, lds_addr(&lds_pf_junk[0]));
}

__device__ void mg1_helper(const Geo* __restrict__ g, const char* base, const pu_req* reqs, uint64_t b, uint64_t end) {
    // no prefetch where the L1 probe is not on the request's own address
    const bool pf_on = !g->tlb_enable;
    uint64_t pf = b;                              // first request not yet prefetched

    const int ln = lane_id();
    uint32_t tail = 0;
    for (;;) {
        const uint32_t head = uni32(*(volatile AS3 uint32_t*)&lds_hq_head);
        if (head == tail) {
            if (uni32(*(volatile AS3 uint32_t*)&lds_main_done)) {
                if (uni32(*(volatile AS3 uint32_t*)&lds_hq_head) == tail) break;
                continue;
            }
            if (pf_on) {
                const uint64_t cur = uni64(*(volatile AS3 uint64_t*)&lds_ctl.cur);
                if (cur >= b && cur < end) {
                    const uint64_t lim = end - cur > PU_PF_AHEAD ? cur + 1 + PU_PF_AHEAD : end;
                    if (pf <= cur) pf = cur + 1;
                    if (pf < lim) {
                        pf_requests(g, base, reqs, pf, (uint32_t)(lim - pf));
                        pf = lim;
                        continue;
                    }
                }
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        if (head - tail > PU_HQ) tail = head - PU_HQ;     // fell behind: those links just miss the cache
        const uint32_t n = head - tail < 64u ? head - tail : 64u;
        if ((uint32_t)ln < n) {
            const uint32_t q = lds_hq[(tail + (uint32_t)ln) & (PU_HQ - 1)];
            volatile AS3 v4u32* H = (volatile AS3 v4u32*)&lds_qhdr[(size_t)q * PU_LDS_SLOT];
            const v4u32 a = H[0];
            asm volatile("" ::: "memory");
            const v4u32 b = H[1];
            asm volatile("" ::: "memory");
            const v4u32 a2 = H[0];
            NetCtx hc;                      // the helper only sees link queues: 0-byte and block packets
            hc.p0 = (uint32_t)g->header_flits;
            hc.p1 = (uint32_t)g->plen_blk;
            uint64_t herr = 0;
            const QState st = hdr_state<false>(hc, a, b, v4u32{0u, 0u, 0u, 0u}, herr);
            const uint64_t w = mg1_wait(st);
            const uint64_t wmask = (1ull << PU_MG1_WAIT_BITS) - 1;
            const bool same = a.x == a2.x && a.y == a2.y && a.z == a2.z && a.w == a2.w;
            const bool st_ok = same && !herr && w < wmask && st.n < 4294967296.0;
            if (st_ok)
                *(volatile AS3 uint64_t*)&lds_qcache[q] = w | ((uint64_t)((uint32_t)st.n ^ (uint32_t)w) << PU_MG1_WAIT_BITS);
#ifdef PU_PROF
            const uint64_t nst = __builtin_popcountll(ballot(st_ok));
            if (ln == 0) atomicAdd(&lds_prof[PF_MG1STORED], (unsigned long long)nst);
#endif
        }
        PROF_CNT(PF_MG1BATCH, 1);
        tail += n;
    }
}

template <int NL, bool LH = false, bool WIDE = false>
struct Engine {
    const Geo* __restrict__ g;
    char* base;
    int ln;

    // reference System scratch for the requesting core (delay[core], hit_flag[core])
    int dly;
    bool hit;
    uint32_t hq_head;   // latency mode: links published to the M/G/1 helper so far

    __device__ __forceinline__ void init_shared(int32_t pool_top, uint64_t page_next, uint64_t last_addr) const {
        lds_eng.pool_top = pool_top;
        lds_eng.stop = 0;
        lds_eng.page_next = page_next;
        lds_eng.last_addr = last_addr;
    }


    template <class T>
    __device__ __forceinline__ T* at(uint64_t off) const {
        return reinterpret_cast<T*>(base + off);
    }

    // ------------------------------------------------------------ network
    __device__ __forceinline__ NetCtx net_ctx() const {
        NetCtx c;
        c.qhdr = (AS1 char*)base + OFF(g->off_qhdr);
        c.qring = (AS1 char*)base + OFF(g->off_qring);
        c.hdr_c = (uint32_t)g->nqueues * PU_HDR_AB;
        c.p0 = c.p1 = (uint32_t)g->bus_latency;   // packed headers: a bus queue sees one packet length
        c.router = (uint32_t)g->router_delay;
        c.link_delay = (uint32_t)g->link_delay;
        c.inject = (uint32_t)g->inject_delay;
        c.header_flits = g->header_flits;
        c.data_width = g->data_width;
        c.w = g->net_width;
        c.net_type = g->net_type;
        return c;
    }
    __device__ __forceinline__ uint64_t transmit(int src, int dst, int len, uint64_t timer) {
        PROF_T(p0);
        uint64_t d = net_transmit<LH, NL, WIDE>(g, base, src, dst, len, timer, hq_head);
        PROF_ADD(PF_NET, p0);
        return d;
    }

    // ------------------------------------------------------------ sets
    __device__ __forceinline__ void set_load(SetView& v, const LineMeta* meta, const int64_t* ts,
                                             uint64_t nsets, uint64_t nways, int offbits, int idxbits,
                                             uint64_t cache_index, uint64_t addr) const {
        v.set = set_index(addr, offbits, nsets);
        v.tag = addr >> (offbits + idxbits);
        // 32-bit index math: a level holds fewer than 2^32 lines (pu_create checks)
        v.line0 = (uint64_t)(((uint32_t)cache_index * (uint32_t)nsets + (uint32_t)v.set) * (uint32_t)nways);
        set_chunk(v, meta, ts, nways, 0);
    }
    // lane w <- way w0 + w of the set
    __device__ __forceinline__ void set_chunk(SetView& v, const LineMeta* meta, const int64_t* ts, uint64_t nways,
                                              uint32_t w0) const {
        v.w0 = w0;
        const uint64_t w = (uint64_t)w0 + (uint64_t)ln;
        if (w < nways) {
            LineMeta m = meta[v.line0 + w];
            v.mtag = m.tag;
            v.mid = m.id;
            v.mst = m.state;
            v.mts = ts[v.line0 + w];
        } else {
            v.mtag = 0;
            v.mid = 0;
            v.mst = ST_I;
            v.mts = INT64_MAX;
        }
    }
    static __device__ __forceinline__ bool wide(uint64_t nways) { return kWideSets && nways > 64; }
    // the lane holding `way` (a way of the chunk held)
    static __device__ __forceinline__ int wl(const SetView& v, int way) { return way - (int)v.w0; }
    // Cache::accessLine (cache.cpp:184-202): the first matching way
    __device__ __forceinline__ int set_find(SetView& v, const LineMeta* meta, const int64_t* ts, uint64_t nways,
                                            int prog) const {
        if (!wide(nways)) {
            uint64_t m = ballot((uint64_t)ln < nways && v.mst != ST_I && v.mid == prog && v.mtag == v.tag);
            return m ? (int)__builtin_ctzll(m) : -1;
        }
        for (uint32_t c = 0;; c += 64) {
            if (c != v.w0) set_chunk(v, meta, ts, nways, c);
            const uint64_t m =
                ballot((uint64_t)c + (uint64_t)ln < nways && v.mst != ST_I && v.mid == prog && v.mtag == v.tag);
            if (m) return (int)c + (int)__builtin_ctzll(m);
            if ((uint64_t)c + 64 >= nways) return -1;
        }
    }
    // Cache::replaceLine (cache.cpp:204-235): first invalid way, else LRU
    // (strictly smaller timestamp, lowest way on ties).  Sets tag/id only.
    __device__ __forceinline__ int set_replace(SetView& v, LineMeta* meta, const int64_t* ts, uint64_t nways,
                                               int offbits, int idxbits, int prog, uint32_t* old_state,
                                               uint64_t* old_addr, int* old_prog) const {
        int way = -1;
        bool invalid = false;
        if (!wide(nways)) {
            const uint64_t inv = ballot((uint64_t)ln < nways && v.mst == ST_I);
            if (inv) {
                invalid = true;
                way = (int)__builtin_ctzll(inv);
            } else {
                way = lru_way(v.mts, (uint64_t)ln < nways ? ln : 64, nways);
            }
        } else {
            // first invalid way over the chunks, else the (timestamp, way)
            // minimum over them: a later chunk wins only when strictly older
            int64_t best = INT64_MAX;
            for (uint32_t c = 0; (uint64_t)c < nways && !invalid; c += 64) {
                if (c != v.w0) set_chunk(v, meta, ts, nways, c);
                const bool mine = (uint64_t)c + (uint64_t)ln < nways;
                const uint64_t inv = ballot(mine && v.mst == ST_I);
                if (inv) {
                    invalid = true;
                    way = (int)c + (int)__builtin_ctzll(inv);
                } else {
                    const int lw = lru_way(v.mts, mine ? ln : 64, 64);
                    const int64_t t = (int64_t)rl64((uint64_t)v.mts, lw);
                    if (way < 0 || t < best) {
                        best = t;
                        way = (int)c + lw;
                    }
                }
            }
            if ((uint32_t)way - v.w0 >= 64u) set_chunk(v, meta, ts, nways, (uint32_t)way & ~63u);
        }
        const int wlane = wl(v, way);
        if (invalid) {
            *old_state = ST_I;
            *old_addr = 0;
            *old_prog = 0;
        } else {
            *old_state = rl32(v.mst, wlane);
            *old_addr = (v.set << offbits) | (rl64(v.mtag, wlane) << (offbits + idxbits));
            *old_prog = (int)rl32((uint32_t)v.mid, wlane);
        }
        if (ln == wlane) {
            v.mtag = v.tag;
            v.mid = prog;
            meta[v.line0 + (uint64_t)way] = LineMeta{v.tag, prog, v.mst};
        }
        return way;
    }
    __device__ __forceinline__ void set_state(SetView& v, LineMeta* meta, int way, uint32_t st) const {
        if (ln == wl(v, way)) {
            v.mst = st;
            meta[v.line0 + (uint64_t)way].state = st;
        }
    }
    __device__ __forceinline__ void set_ts(SetView& v, int64_t* ts, int way, int64_t t) const {
        if (ln == wl(v, way)) {
            v.mts = t;
            ts[v.line0 + (uint64_t)way] = t;
        }
    }

    // ------------------------------------------------------------ per-cache bookkeeping
    __device__ __forceinline__ void mark_alive(int l, int cid) const {
        // System::init_caches (system.cpp:172-207) creates the cache and its
        // ancestors on first touch; only the existence bit is observable.
        for (int k = l; k < NL; k++) {
            if constexpr (kAliveLds) {
                const uint32_t bit = (uint32_t)(alive_base(k) + cid), m = 1u << (bit & 31);
                const uint32_t w = uni32(lds_alive[bit >> 5]);
                if (!(w & m)) {                 // first touch in this launch
                    if (ln == (cid & 63)) at<uint32_t>(OFF(g->lv[k].off_alive))[cid] = 1u;
                    if (ln == 0) lds_alive[bit >> 5] = w | m;
                }
            } else {
                if (ln == (cid & 63)) at<uint32_t>(OFF(g->lv[k].off_alive))[cid] = 1u;
            }
            if (k + 1 < NL) cid = cid * g->lv[k].share / g->lv[k + 1].share;
        }
    }
    // one {ins, miss, evict, wb} event of cache cid at level K (0-3,
    // PU_CNT_DIR, PU_CNT_TLB): a per-level LDS sum (kCntSum) or the cache's
    // own counter
    template <int K>
    __device__ __forceinline__ void count(uint64_t off_cnt, int cid, int which) const {
        if constexpr (kCntSum) stat_add(SN_CNT0 + 4 * K + which, 1);
        else gatomic_add_u64_lane0(at<uint64_t>(off_cnt) + (size_t)cid * 4 + which, 1ull);
    }

    // Dram::access (dram.cpp:43-47) at cycle t for line address addr: the
    // reference's fixed latency, or with the opt-in bank model (Geo.dram_banks
    // > 0, pu_dram_cfg; no reference counterpart) one open-page bank access.
    // The bank record is read by every lane (one broadcast line) and written
    // by lane 0; its delay only depends on wave-uniform values.
    __device__ __forceinline__ int dram(uint64_t addr, int64_t t) {
        stat_add(SN_DRAM, 1);
        if (g->dram_banks == 0) return g->dram_access_time;
        const uint64_t row = uni64(addr) >> g->dram_row_shift;
        const uint64_t bank = row & (uint64_t)(g->dram_banks - 1);
        const uint64_t page = (row >> g->dram_bank_shift) + 1;   // + 1: 0 means closed
        t = (int64_t)uni64((uint64_t)t);
        DramBank* B = at<DramBank>(OFF(g->off_dram)) + bank;
        const int64_t ready = (int64_t)uni64((uint64_t)B->ready);
        const uint64_t open = uni64(B->open);
        const int64_t start = ready > t ? ready : t;
        int64_t act;
        if (open == page) {
            act = 0;
            stat_add(SN_ROWHIT, 1);
        } else if (open == 0) {
            act = g->dram_t_rcd;
            stat_add(SN_ROWEMPTY, 1);
        } else {
            act = (int64_t)g->dram_t_rp + g->dram_t_rcd;
            stat_add(SN_ROWCONF, 1);
        }
        if (ln == 0) *B = DramBank{start + act + g->dram_t_burst, page};
        stat_add(SN_BANKWAIT, (uint64_t)(start - t));
        return (int)(start - t + act) + g->dram_access_time;
    }

    // ------------------------------------------------------------ downward propagation
    // System::share / System::inval (system.cpp:488-555); LV is the level of `cid`.
    template <int LV, bool INVAL>
    __device__ __forceinline__ int down(int cid, const Req& r) {
        PROF_T(p0);
        int d = down_impl<LV, INVAL>(cid, r);
        PROF_ADD(PF_DOWN, p0);
        return d;
    }
    template <int LV, bool INVAL>
    __device__ __forceinline__ int down_impl(int cid, const Req& r) {
        const LevelGeo& L = g->lv[LV];
        uint32_t alive_v = ln == (cid & 63) ? at<uint32_t>(OFF(L.off_alive))[cid] : 0u;
        SetView v;
        set_load(v, at<LineMeta>(OFF(L.off_meta)), at<int64_t>(OFF(L.off_ts)), L.nsets, L.nways, L.offbits, L.idxbits,
                 (uint64_t)cid, r.addr);
        if (!rl32(alive_v, cid & 63)) return 0;   // cache never created: NULL in the reference
        stat_add(SN_LOCKDOWN, 1);
        int d = L.access_time;
        int way = set_find(v, at<LineMeta>(OFF(L.off_meta)), at<int64_t>(OFF(L.off_ts)), L.nways, r.prog);
        if (way >= 0) {
            uint32_t st = rl32(v.mst, wl(v, way));
            if (INVAL || st == ST_M || st == ST_E) {
                set_state(v, at<LineMeta>(OFF(L.off_meta)), way, INVAL ? ST_I : ST_S);
                d += children<LV, INVAL>(cid, r);
            }
        }
        return d;
    }
    // share_children / inval_children (system.cpp:514-572): max over children.
    template <int LV, bool INVAL>
    __device__ __forceinline__ int children(int cid, const Req& r) {
        if constexpr (LV == 0) {
            return 0;
        } else {
            const int nc = g->lv[LV].nchildren;
            int mx = 0;
            for (int k = 0; k < nc; k++) {
                int d = down<LV - 1, INVAL>(cid * nc + k, r);
                mx = d > mx ? d : mx;
            }
            return mx;
        }
    }

    // ------------------------------------------------------------ sharer sets
    // Line::sharer_set (a std::set<int>, cache.h:86): up to 4 ids inline in
    // `sh`, ascending, 16 bits each (12 bits each in the stored DirLine word;
    // above 4096 LLC nodes, DirGeo.sh_wide: 3 ids of 16 bits); one more sharer
    // moves the set to a full-map bitmap from the replica's pool, read 64 words
    // at a time (lane k holds word base + k).
    // the line's 10-bit program field: the id itself, or the escape for ids
    // outside [0, 1023) (their full value goes to the side array)
    static __device__ __forceinline__ uint32_t prog10(int prog) {
        return (uint32_t)prog < PU_DIR_PROG_ESC ? (uint32_t)prog : PU_DIR_PROG_ESC;
    }
    __device__ __forceinline__ uint64_t dir_word(uint32_t nsh, uint64_t sh, uint32_t st, uint32_t p10) const {
        const uint64_t s = nsh == PU_SH_POOL || g->dir.sh_wide
                               ? (sh & 0xFFFFFFFFFFFFull)
                               : (sh & 0xFFFull) | ((sh >> 4) & 0xFFF000ull) | ((sh >> 8) & 0xFFF000000ull) |
                                     ((sh >> 12) & 0xFFF000000000ull);
        return s | ((uint64_t)(nsh == PU_SH_POOL ? 7u : nsh) << 48) | ((uint64_t)st << 51) | ((uint64_t)p10 << 54);
    }
    static __device__ __forceinline__ uint32_t dir_state(uint64_t w) { return (uint32_t)(w >> 51) & 7u; }
    __device__ __forceinline__ void dir_sharers(uint64_t w, uint32_t& nsh, uint64_t& sh) const {
        const uint32_t n = (uint32_t)(w >> 48) & 7u;
        const uint64_t s = w & 0xFFFFFFFFFFFFull;
        nsh = n == 7u ? PU_SH_POOL : n;
        sh = n == 7u || g->dir.sh_wide
                 ? s
                 : (s & 0xFFFull) | ((s & 0xFFF000ull) << 4) | ((s & 0xFFF000000ull) << 8) |
                       ((s & 0xFFF000000000ull) << 12);
    }
    __device__ __forceinline__ uint64_t* pool_of(uint64_t idx) const {
        return at<uint64_t>(OFF(g->dir.off_pool)) + idx * (uint64_t)g->dir.nwords;
    }
    // bitmap words base .. base+63 of pool entry idx, lane k holding word base + k
    __device__ __forceinline__ uint64_t pool_word(uint64_t idx, int base = 0) const {
        return base + ln < g->dir.nwords ? pool_of(idx)[base + ln] : 0ull;
    }
    __device__ __forceinline__ void pool_release(uint32_t nsh, uint64_t sh) {
        if (nsh != PU_SH_POOL) return;
        const int32_t pt = (int32_t)uni32((uint32_t)lds_eng.pool_top);
        if (ln == 0) at<int32_t>(OFF(g->dir.off_pool_free))[pt] = (int32_t)sh;
        lds_eng.pool_top = pt + 1;
    }
    __device__ __forceinline__ bool pool_alloc(uint64_t* idx) {
        const int32_t pt = (int32_t)uni32((uint32_t)lds_eng.pool_top);
        if (pt <= 0) {
            err_or(PU_ERRF_POOL);
            lds_eng.stop = 1;
            return false;
        }
        lds_eng.pool_top = pt - 1;
        uint32_t v = ln == 0 ? (uint32_t)at<int32_t>(OFF(g->dir.off_pool_free))[pt - 1] : 0u;
        *idx = rl32(v, 0);
        return true;
    }
    __device__ __forceinline__ int first_sharer(uint32_t nsh, uint64_t sh) {
        if (nsh == PU_SH_POOL) {
            for (int base = 0; base < g->dir.nwords; base += 64) {
                uint64_t w = pool_word(sh, base);
                uint64_t m = ballot(w != 0);
                if (m) {
                    int k = (int)__builtin_ctzll(m);
                    return (base + k) * 64 + (int)__builtin_ctzll(rl64(w, k));
                }
            }
        } else if (nsh > 0) {
            return (int)(sh & 0xFFFF);
        }
        err_or(PU_ERRF_EMPTY_SHARER);     // *sharer_set.begin() on an empty set
        return 0;
    }
    __device__ __forceinline__ int count_sharers(uint32_t nsh, uint64_t sh) const {
        if (nsh != PU_SH_POOL) return (int)nsh;
        int c = 0;
        for (int base = 0; base < g->dir.nwords; base += 64) c += __builtin_popcountll(pool_word(sh, base));
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
        return (int)uni32((uint32_t)c);
    }
    // sharer_set.insert(cid)
    __device__ __forceinline__ void add_sharer(uint32_t& nsh, uint64_t& sh, int cid) {
        if (nsh == PU_SH_POOL) {
            if (ln == ((cid >> 6) & 63)) {
                uint64_t* P = pool_of(sh) + (cid >> 6);
                *P = *P | (1ull << (cid & 63));
            }
            return;
        }
        int below = 0;
        bool present = false;
        for (uint32_t i = 0; i < nsh; i++) {
            int id = (int)((sh >> (16 * i)) & 0xFFFF);
            present |= id == cid;
            below += id < cid;
        }
        if (present) return;
        if (nsh < (uint32_t)g->dir.sh_cap) {
            uint64_t low = below == 0 ? 0ull : ((1ull << (16 * below)) - 1);
            sh = (sh & low) | ((uint64_t)cid << (16 * below)) | ((sh & ~low) << 16);
            nsh++;
            return;
        }
        uint64_t idx;
        if (!pool_alloc(&idx)) return;
        // cid through an opaque move: its lane bit is built here, not hoisted
        // to where cid is first known and held in VGPRs across the probes (at
        // 7 waves per SIMD two 8-B scratch spills per access: fabric traffic
        // 1.30x, and 7 waves only +1.2%; profiles/r5u_traffic.json, r5t_ab_driver.txt)
        int c;
        asm volatile("s_mov_b32 %0, %1" : "=s"(c) : "s"(cid));
        for (int base = 0; base < g->dir.nwords; base += 64) {
            uint64_t w = 0;
            for (uint32_t i = 0; i < nsh; i++) {
                int id = (int)((sh >> (16 * i)) & 0xFFFF);
                if ((id >> 6) == base + ln) w |= 1ull << (id & 63);
            }
            if ((c >> 6) == base + ln) w |= 1ull << (c & 63);
            if (base + ln < g->dir.nwords) pool_of(idx)[base + ln] = w;
        }
        nsh = PU_SH_POOL;
        sh = idx;
    }

    // ------------------------------------------------------------ probes from home
    // Every message exchange a home slice starts with other caches has the
    // same shape: for each target p in order, home -> p, share/inval down p's
    // hierarchy, p -> home (reply_len bytes), t_p = pipe + those delays, the
    // result the max over targets, pipe += header_flits per target
    // (system.cpp:605-633, 660-671, 687-705, 766-795, 820-831, 846-866).  The
    // single owner (first_sharer) of an M/E line is a one-target probe.  One
    // loop serves all of them, so the two transmits below are the only ones
    // the home code inlines.
    enum ProbeMode { PR_NONE, PR_ONE, PR_INLINE, PR_POOL, PR_ALL };
    // Returns the home's delay after the probe.  The owner case accumulates
    // into `delay` directly (delay += ...; timer + delay), a sharer set adds
    // the max over targets (initialised to 0) of times relative to
    // timer + delay: the two differ once an int wraps, so both are kept.
    __device__ __forceinline__ int probe(int mode, int one, uint32_t nsh, uint64_t sh, bool inval, int reply_len, int home,
                         const Req& r, int64_t timer, int delay) {
        constexpr int last = NL - 1;
        const bool single = mode == PR_ONE;
        const int64_t base_t = single ? timer : timer + delay;
        int pipe = single ? delay : 0, mx = 0;
        int pbase = 0;                                            // bitmap words pbase .. pbase+63
        uint64_t rem = mode == PR_POOL ? pool_word(sh) : 0ull;   // lane k: bitmap word pbase + k
        uint32_t k = 0;
        while (true) {
            int p;
            if (mode == PR_ONE) {
                if (k) break;
                p = one;
            } else if (mode == PR_INLINE) {
                if (k >= nsh) break;
                p = (int)((sh >> (16 * k)) & 0xFFFF);
            } else if (mode == PR_POOL) {
                uint64_t m = ballot(rem != 0);
                while (!m && pbase + 64 < g->dir.nwords) {         // next 64 words (> 4096 LLC nodes)
                    pbase += 64;
                    rem = pool_word(sh, pbase);
                    m = ballot(rem != 0);
                }
                if (!m) break;
                const int w = (int)__builtin_ctzll(m);
                p = (pbase + w) * 64 + (int)__builtin_ctzll(rl64(rem, w));
                if (ln == w) rem &= rem - 1;
            } else if (mode == PR_ALL) {
                if ((int)k >= g->num_cores) break;
                p = (int)k;
            } else {
                break;
            }
            k++;
            int t = pipe;
            // home -> p, share/inval below p, p -> home: one transmit site
#pragma clang loop unroll(disable)
            for (int back = 0; back < 2; back++) {
                t += (int)transmit(back ? p : home, back ? home : p, back ? reply_len : 0, (uint64_t)(base_t + t));
                if (!back) t += inval ? down<last, true>(p, r) : down<last, false>(p, r);
            }
            if (single) return t;
            mx = t > mx ? t : mx;
            pipe += g->header_flits;
        }
        return delay + mx;
    }

    // ------------------------------------------------------------ home slice
    // accessSharedCache (system.cpp:734-893) / accessDirectoryCache (577-731).
    // The home line is read once (lane w: way w, 24 B) and written once at the
    // end: nothing reached from here touches directory lines.  Every branch
    // that messages other caches does so first, at timer + access_time, so
    // the branch only chooses the probe; `probe` runs it.
    // Stage the home set of `addr` into LDS (lane w = way w) before the request
    // transmit; 0 when the set is too wide to stage.  The caller tells
    // access_home whether the transmit ran hops (2: it did not).
    __device__ __forceinline__ int dir_stage(int home, uint64_t addr, bool no_hops) const {
        const DirGeo& D = g->dir;
        if (D.nways > 32) return 0;
        const uint64_t set = set_index(addr, D.offbits, D.nsets);
        const uint64_t line0 = (uint64_t)(((uint32_t)home * (uint32_t)D.csets + (uint32_t)(set >> D.cset_shift)) * (uint32_t)D.nways);
        if ((uint64_t)ln < D.nways) {
            const AS1 char* lp = (const AS1 char*)(const char*)(at<DirLine>(OFF(D.off_line)) + line0 + (uint64_t)ln);
            lds_dma<true>(lp, lds_addr(&lds_dir_a[0]));
            lds_dma<false>(lp + 16, lds_addr(&lds_dir_w[0][0]));
            lds_dma<false>(lp + 20, lds_addr(&lds_dir_w[1][0]));
        }
        return no_hops ? 2 : 1;
    }
    __device__ __forceinline__ int access_home(int cid, int home, const Req& r, int64_t timer, uint32_t* out_state, int staged = 0) {
        PROF_T(p0);
        int d = access_home_impl(cid, home, r, timer, out_state, staged);
        PROF_ADD(PF_HOME, p0);
        return d;
    }
    __device__ __forceinline__ int access_home_impl(int cid, int home, const Req& r, int64_t timer, uint32_t* out_state,
                                    int staged) {
        PROF_T(p_ld);
        const DirGeo& D = g->dir;
        const bool shared = g->shared_llc != 0;
        constexpr int last = NL - 1;
        const int blk = (int)g->lv[last].block;
        DirLine* lines = at<DirLine>(OFF(D.off_line));
        // home_stat[home] = 1 (read by the verbose report only)
        if (!kCntSum && ln == (home & 63)) at<uint32_t>(OFF(D.off_alive))[home] = 1u;
        const uint64_t set = set_index(r.addr, D.offbits, D.nsets);
        const uint64_t tag = r.addr >> (D.offbits + D.idxbits);
        const uint64_t line0 = (uint64_t)(((uint32_t)home * (uint32_t)D.csets + (uint32_t)(set >> D.cset_shift)) * (uint32_t)D.nways);
        bool mine = (uint64_t)ln < D.nways;
        uint32_t dw0 = 0;        // sets wider than 64 ways: lane w holds way dw0 + w
        DirLine m;
        if (staged == 1) {
            // staged before a transmit that ran hops.  With headers in HBM that
            // transmit waited for its first header load, and vector memory
            // returns in issue order, so the staging DMA has landed (the
            // vmcnt(8) only bounds it).  With headers in LDS (latency mode) an
            // M/G/1-only transmit issues no vector memory operation at all:
            // wait for the DMA itself.
            if constexpr (LH) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else if (staged == 2) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (mine && staged) {
            const v4u32 a = lds_dir_a[ln];
            m.tag = u64of(a.x, a.y);
            m.ts = (int64_t)u64of(a.z, a.w);
            m.w = u64of(lds_dir_w[0][ln], lds_dir_w[1][ln]);
        } else if (mine) {
            m = lines[line0 + (uint64_t)ln];
        } else {
            m.tag = 0; m.ts = INT64_MAX; m.w = 0;
        }
        uint32_t m_state = dir_state(m.w);
        // program ids: the 10-bit field decides unless either side is escaped;
        // the side array is read only then (ids >= 1023 or negative)
        const uint32_t want10 = prog10(r.prog), m_p10 = (uint32_t)(m.w >> 54);
        int32_t* side = at<int32_t>(OFF(D.off_prog));
        int32_t m_prog = (int32_t)m_p10;
        if (want10 == PU_DIR_PROG_ESC || ballot(mine && m_p10 == PU_DIR_PROG_ESC)) {
            if (mine && m_p10 == PU_DIR_PROG_ESC) m_prog = side[line0 + (uint64_t)ln];
        }
        // ways c..c+63 of a wide set (never staged: dir_stage takes <= 32 ways)
        auto dir_chunk = [&](uint32_t c) {
            dw0 = c;
            mine = (uint64_t)c + (uint64_t)ln < D.nways;
            if (mine) {
                m = lines[line0 + (uint64_t)c + (uint64_t)ln];
            } else {
                m.tag = 0; m.ts = INT64_MAX; m.w = 0;
            }
            m_state = dir_state(m.w);
            const uint32_t p10 = (uint32_t)(m.w >> 54);
            m_prog = (int32_t)p10;
            if (mine && p10 == PU_DIR_PROG_ESC) m_prog = side[line0 + (uint64_t)c + (uint64_t)ln];
        };
        uint64_t hm = ballot(mine && m_state != ST_I && m_prog == r.prog && m.tag == tag);
        int way = hm ? (int)__builtin_ctzll(hm) : -1;
        if (wide(D.nways) && !hm) {
            for (uint32_t c = 64; (uint64_t)c < D.nways; c += 64) {
                dir_chunk(c);
                hm = ballot(mine && m_state != ST_I && m_prog == r.prog && m.tag == tag);
                if (hm) {
                    way = (int)c + (int)__builtin_ctzll(hm);
                    break;
                }
            }
        }
        PROF_ADD(PF_HOME_LD, p_ld);
        count<PU_CNT_DIR>(OFF(D.off_cnt), home, 0);
        int delay = D.access_time;
        uint32_t st, nsh;
        uint64_t sh;
        // the probe this transition makes, and what follows it
        int pmode = PR_NONE, pone = 0, preply = 0;
        bool pinval = true;
        uint32_t psh_n = 0;
        uint64_t psh = 0;
        Req pr = r;
        int extra_dram = 0;      // dram() after the probe: 1 = counted only, 2 = counted and timed
        bool release_set = false, miss_fill = false;
        if (way < 0 && r.type != PU_WB) {
            // replaceLine (cache.cpp:204-235): first invalid way, else LRU
            uint32_t old_st = ST_I;
            uint64_t old_addr = 0;
            int old_prog = 0;
            bool inv = false;
            if (!wide(D.nways)) {
                const uint64_t im = ballot(mine && m_state == ST_I);
                inv = im != 0;
                if (inv) {
                    way = (int)__builtin_ctzll(im);
                } else {
                    way = lru_way(m.ts, mine ? ln : 64, D.nways);
                }
            } else {
                // first invalid way over the chunks, else the (timestamp, way)
                // minimum (a later chunk wins only when strictly older)
                int64_t best = INT64_MAX;
                for (uint32_t c = 0; (uint64_t)c < D.nways && !inv; c += 64) {
                    if (c != dw0) dir_chunk(c);
                    const uint64_t im = ballot(mine && m_state == ST_I);
                    if (im) {
                        inv = true;
                        way = (int)c + (int)__builtin_ctzll(im);
                    } else {
                        const int lw = lru_way(m.ts, mine ? ln : 64, 64);
                        const int64_t t = (int64_t)rl64((uint64_t)m.ts, lw);
                        if (way < 0 || t < best) {
                            best = t;
                            way = (int)c + lw;
                        }
                    }
                }
                if ((uint32_t)way - dw0 >= 64u) dir_chunk((uint32_t)way & ~63u);
            }
            const int wlane = way - (int)dw0;
            const uint64_t ww = rl64(m.w, wlane);
            if (!inv) {
                old_st = dir_state(ww);
                old_addr = (set << D.offbits) | (rl64(m.tag, wlane) << (D.offbits + D.idxbits));
                old_prog = (int)rl32((uint32_t)m_prog, wlane);
            }
            dir_sharers(ww, nsh, sh);
            if (old_st != ST_I) {
                count<PU_CNT_DIR>(OFF(D.off_cnt), home, 2);
                pr = Req{old_addr, old_prog, PU_RD};
                if (old_st == ST_M || old_st == ST_E) {
                    pmode = PR_ONE;
                    pone = first_sharer(nsh, sh);
                    preply = (!shared || old_st == ST_M) ? blk : 0;
                    extra_dram = 1;
                } else if (old_st == ST_S) {
                    pmode = nsh == PU_SH_POOL ? PR_POOL : PR_INLINE;
                } else if (old_st == ST_B) {
                    pmode = PR_ALL;
                }
            }
            st = r.type == PU_WR ? ST_M : ST_E;
            count<PU_CNT_DIR>(OFF(D.off_cnt), home, 1);
            release_set = true;
            miss_fill = true;
        } else if (way < 0) {
            err_or(PU_ERRF_WB_MISS);         // WB missed at home: NULL deref in the reference (Q13)
            *out_state = ST_I;
            return delay;
        } else {
            const uint64_t ww = rl64(m.w, way - (int)dw0);
            st = dir_state(ww);
            dir_sharers(ww, nsh, sh);
            if (r.type == PU_WR) {
                if (st == ST_M || st == ST_E) {
                    pmode = PR_ONE;
                    pone = first_sharer(nsh, sh);
                    preply = blk;
                } else if (st == ST_S) {
                    pmode = nsh == PU_SH_POOL ? PR_POOL : PR_INLINE;
                    if (!shared) extra_dram = 2;
                } else if (st == ST_B) {
                    pmode = PR_ALL;
                    if (!shared) extra_dram = 2;
                }
                st = ST_M;
                release_set = true;
            } else if (r.type == PU_RD) {
                if (st == ST_M || st == ST_E) {
                    pmode = PR_ONE;
                    pone = first_sharer(nsh, sh);
                    preply = blk;
                    pinval = false;                  // share, not inval (system.cpp:660-671)
                    st = ST_S;
                } else if (st == ST_S) {
                    if (!shared) delay += dram(r.addr, timer + delay);
                    if (g->protocol_type == 1 && count_sharers(nsh, sh) >= g->max_num_sharers) st = ST_B;
                } else if (st == ST_B) {
                    if (!shared) delay += dram(r.addr, timer + delay);
                } else if (st == ST_V) {
                    st = ST_E;
                }
            } else {
                st = shared ? ST_V : ST_I;
                pool_release(nsh, sh);
                nsh = 0;
                sh = 0;
                dram(r.addr, timer + delay);
            }
        }
        if (pmode != PR_NONE) {
            if (pmode == PR_ALL) stat_add(SN_BCAST, 1);
            psh_n = nsh;
            psh = sh;
            delay = probe(pmode, pone, psh_n, psh, pinval, preply, home, pr, timer, delay);
        }
        if (extra_dram == 1) dram(pr.addr, timer + delay);   // the evicted owner's write-back
        if (extra_dram == 2) delay += dram(r.addr, timer + delay);
        if (release_set) {                   // sharer_set.clear(); insert(cache_id)
            pool_release(nsh, sh);
            nsh = 1;
            sh = (uint64_t)cid;
            if (miss_fill) delay += dram(r.addr, timer + delay);

        } else if (r.type == PU_RD) {
            add_sharer(nsh, sh, cid);
        }
        *out_state = st == ST_B ? ST_S : st;
        if (ln == way - (int)dw0) {
            // home slices stamp the arrival time (Q4)
            lines[line0 + (uint64_t)way] = DirLine{tag, timer, dir_word(nsh, sh, st, want10)};
            if (want10 == PU_DIR_PROG_ESC) side[line0 + (uint64_t)way] = r.prog;
        }
        return delay;
    }

    __device__ __forceinline__ int home_of(uint64_t addr) const {
        // System::allocHomeId (system.cpp:921-936)
        int hb = (int)((addr >> g->home_offbits) & (((uint64_t)1 << g->home_mask_bits) - 1));
        if (hb < g->N) return hb;
        return hb & ((1 << (g->home_mask_bits - 1)) - 1);
    }

    // ------------------------------------------------------------ directory MESI walk
    // System::mesi_directory (system.cpp:372-482); LV is the level of `cid`.
    // Each level calls its parent from one place, and the last level runs its
    // home transactions (write-back, request/reply, or the S->M upgrade) from
    // one loop, so the transmit and home-slice code is inlined once.
    template <int LV>
    __device__ __forceinline__ uint32_t mesi(int cid, const Req& r, int64_t timer) {
        const LevelGeo& L = g->lv[LV];
        constexpr bool kLast = LV == NL - 1;
        LineMeta* meta = at<LineMeta>(OFF(L.off_meta));
        int64_t* tsa = at<int64_t>(OFF(L.off_ts));
        SetView v;
        PROF_T(p_set);
        set_load(v, meta, tsa, L.nsets, L.nways, L.offbits, L.idxbits, (uint64_t)cid, r.addr);
        mark_alive(LV, cid);
        if (L.has_bus) {              // Bus::access (bus.cpp:55-61)
            stat_add(SN_BUSACC, 1);
            uint64_t bl = (uint64_t)g->bus_latency, mg1 = 0, err = 0;
            int db = (int)q_op<LH, WIDE>(net_ctx(), L.bus_q0 + cid, (uint64_t)(timer + dly), bl, bl, mg1, err);
            stat_add(SN_MG1, mg1);
            if (err) err_or(err);
            stat_add(SN_BUSCONT, (uint64_t)(int64_t)db);
            dly += db;
        }
        if (!hit) count<LV>(OFF(L.off_cnt), cid, 0);
        dly += L.access_time;
        int way = set_find(v, meta, tsa, L.nways, r.prog);
        PROF_ADD(LV == 0 ? PF_SETL0 : PF_SETLN, p_set);
        bool is_miss = false, call_parent = false;
        int64_t ptimer = 0;
        uint32_t ret = ST_M;
        // home transactions of the last level: [0] write-back of the victim
        // (delays discarded, Q3), [1] the request (or the S->M upgrade)
        bool tx_wb = false, tx_req = false;
        int wb_home = 0, req_reply = 0;
        Req wb_req = r;
        if (way >= 0) {                                      // hit
            set_ts(v, tsa, way, timer + dly);
            hit = true;
            const uint32_t st = rl32(v.mst, wl(v, way));
            if (r.type == PU_WR) {
                if constexpr (!kLast) {
                    if (st != ST_M) {
                        set_state(v, meta, way, ST_I);
                        call_parent = true;
                        ptimer = timer + dly;
                    }
                } else {
                    if (st == ST_S) {
                        tx_req = true;
                        req_reply = 0;
                    }
                }
                ret = ST_M;
            } else {
                if (st != ST_S) dly += children<LV, false>(cid, r);
                return ST_S;
            }
        } else {                                             // miss
            is_miss = true;
            uint32_t old_st;
            uint64_t old_addr;
            int old_prog;
            way = set_replace(v, meta, tsa, L.nways, L.offbits, L.idxbits, r.prog, &old_st, &old_addr, &old_prog);
            if (old_st != ST_I) {
                count<LV>(OFF(L.off_cnt), cid, 2);
                Req o{old_addr, old_prog, PU_RD};
                dly += children<LV, true>(cid, o);
                if (old_st == ST_M || old_st == ST_E) {
                    count<LV>(OFF(L.off_cnt), cid, 3);
                    if constexpr (kLast) {
                        tx_wb = true;
                        wb_home = home_of(old_addr);
                        wb_req = Req{old_addr, old_prog, PU_WB};
                    }
                }
            }
            set_ts(v, tsa, way, timer + dly);
            if constexpr (!kLast) {
                call_parent = true;
                ptimer = timer;                               // `timer`, not timer+delay (Q2)
            } else {
                tx_req = true;
                req_reply = (int)L.block;
            }
        }
        if constexpr (!kLast) {
            if (call_parent) {
                const int parent = cid * L.share / g->lv[LV + 1].share;
                const uint32_t ns = mesi<LV + 1>(parent, r, ptimer);
                set_state(v, meta, way, ns);
                if (is_miss) ret = ns;
            }
        } else {
            // legs: 0 the write-back to its home (delays discarded, Q3), 1 the
            // request to its home, 2 the reply; one transmit site and one home
            // access site serve all of them
            const int req_home = home_of(r.addr);
            int leg = tx_wb ? 0 : (tx_req ? 1 : 3);
            while (leg < 3) {
                const bool wb = leg == 0;
                const int home = wb ? wb_home : req_home;
                const int src = leg == 2 ? home : cid, dst = leg == 2 ? cid : home;
                const int len = wb ? (int)L.block : (leg == 1 ? 0 : req_reply);
                // the request's home set is fetched while the request travels
                // (nothing on the way writes directory lines; the write-back's
                // home access, which may, is done)
                const int staged = leg == 1 ? dir_stage(home, r.addr, src == dst) : 0;
                const int d1 = (int)transmit(src, dst, len, (uint64_t)(timer + dly));
                if (!wb) dly += d1;
                if (leg == 2) break;
                uint32_t hs;
                const int d2 = access_home(cid, home, wb ? wb_req : r, timer + dly, &hs, staged);
                if (!wb) {
                    dly += d2;
                    if (is_miss) ret = hs;
                }
                leg = wb ? (tx_req ? 1 : 3) : 2;
            }
            set_state(v, meta, way, is_miss ? ret : ST_M);
        }
        if (is_miss) count<LV>(OFF(L.off_cnt), cid, 1);
        return ret;
    }

    // ------------------------------------------------------------ snoopy bus MESI walk
    // System::mesi_bus (system.cpp:224-368); LV is the level of `cid`.  The
    // share/inval of children is done for its state changes only: mesi_bus
    // never adds those delays.  Evict/write-back counters are not kept on this
    // path (Q17).
    //
    // Snoop of the other last-level caches for r's line, ascending cache id
    // (system.cpp:264-276, 311-329, 335-354).  Lane k probes cache base+k's set
    // (first matching way, like Cache::accessLine), 64 caches per round trip;
    // holders are then handled in order.  mode 0: write hit in S — every holder
    // -> I, inval below; 1: write miss — holder inval below, -> I, stop at the
    // first M/E holder; 2: read miss — share below, -> S, stop at the first
    // M/E holder.  Returns whether any cache held the line.  (The reference
    // also creates every cache it snoops; a never-created cache holds no line
    // and mesi_bus discards the delays where that would show, so the engine
    // does not mark them.)
    __device__ __forceinline__ bool snoop(int cid, const Req& r, int mode) {
        constexpr int last = NL - 1;
        const LevelGeo& L = g->lv[last];
        LineMeta* meta = at<LineMeta>(OFF(L.off_meta));
        const uint64_t set = set_index(r.addr, L.offbits, L.nsets);
        const uint64_t tag = r.addr >> (L.offbits + L.idxbits);
        bool any = false;
        for (int base = 0; base < L.ncaches; base += 64) {
            const int c = base + ln;
            int myway = -1;
            uint32_t myst = ST_I;
            if (c < L.ncaches && c != cid) {
                const LineMeta* sp = meta + ((uint64_t)c * L.nsets + set) * L.nways;
                for (uint64_t w = L.nways; w-- > 0;) {      // lowest matching way wins
                    const LineMeta m = sp[w];
                    if (m.state != ST_I && m.id == r.prog && m.tag == tag) {
                        myway = (int)w;
                        myst = m.state;
                    }
                }
            }
            uint64_t hits = ballot(myway >= 0);
            while (hits) {
                const int k = (int)__builtin_ctzll(hits);
                hits &= hits - 1;
                const int i = base + k;
                const int way = (int)rl32((uint32_t)myway, k);
                const uint32_t st = rl32(myst, k);
                any = true;
                if (mode == 2) children<last, false>(i, r);
                else children<last, true>(i, r);
                if (ln == 0) meta[((uint64_t)i * L.nsets + set) * L.nways + (uint64_t)way].state = mode == 2 ? ST_S : ST_I;
                if (mode != 0 && (st == ST_M || st == ST_E)) return any;
            }
        }
        return any;
    }

    template <int LV>
    __device__ __forceinline__ uint32_t mesi_bus(int cid, const Req& r, int64_t timer) {
        const LevelGeo& L = g->lv[LV];
        constexpr bool kLast = LV == NL - 1;
        LineMeta* meta = at<LineMeta>(OFF(L.off_meta));
        int64_t* tsa = at<int64_t>(OFF(L.off_ts));
        SetView v;
        set_load(v, meta, tsa, L.nsets, L.nways, L.offbits, L.idxbits, (uint64_t)cid, r.addr);
        mark_alive(LV, cid);
        if (L.has_bus) {              // Bus::access (bus.cpp:55-61)
            stat_add(SN_BUSACC, 1);
            uint64_t bl = (uint64_t)g->bus_latency, mg1 = 0, err = 0;
            int db = (int)q_op<LH, WIDE>(net_ctx(), L.bus_q0 + cid, (uint64_t)(timer + dly), bl, bl, mg1, err);
            stat_add(SN_MG1, mg1);
            if (err) err_or(err);
            stat_add(SN_BUSCONT, (uint64_t)(int64_t)db);
            dly += db;
        }
        dly += L.access_time;
        if (!hit) count<LV>(OFF(L.off_cnt), cid, 0);
        int way = set_find(v, meta, tsa, L.nways, r.prog);
        bool is_miss = false, call_parent = false;
        int snoop_mode = -1;
        uint32_t ret = ST_M;
        if (way >= 0) {                                      // hit
            set_ts(v, tsa, way, timer + dly);
            hit = true;
            const uint32_t st = rl32(v.mst, wl(v, way));
            if (r.type != PU_WR) {
                if (st != ST_S) children<LV, false>(cid, r);   // share_children, delay discarded
                return ST_S;
            }
            if constexpr (!kLast) {
                if (st != ST_M) {
                    set_state(v, meta, way, ST_I);
                    call_parent = true;
                }
            } else {
                if (st == ST_S) snoop_mode = 0;
            }
        } else {                                             // miss
            is_miss = true;
            uint32_t old_st;
            uint64_t old_addr;
            int old_prog;
            way = set_replace(v, meta, tsa, L.nways, L.offbits, L.idxbits, r.prog, &old_st, &old_addr, &old_prog);
            if (old_st != ST_I) {
                Req o{old_addr, old_prog, PU_RD};
                children<LV, true>(cid, o);                  // inval_children, delay discarded
            }
            set_ts(v, tsa, way, timer + dly);
            if constexpr (!kLast) call_parent = true;
            else snoop_mode = r.type == PU_WR ? 1 : 2;
        }
        if constexpr (!kLast) {
            if (call_parent) {
                const int parent = cid * L.share / g->lv[LV + 1].share;
                const uint32_t ns = mesi_bus<LV + 1>(parent, r, timer + dly);   // timer + delay here
                set_state(v, meta, way, ns);
                if (is_miss) ret = ns;
            }
        } else {
            bool shared_line = false;
            if (snoop_mode >= 0) shared_line = snoop(cid, r, snoop_mode);
            if (is_miss) {
                ret = r.type == PU_WR ? ST_M : (shared_line ? ST_S : ST_E);
                set_state(v, meta, way, ret);
                dly += dram(r.addr, timer + dly);
            } else {
                set_state(v, meta, way, ST_M);
            }
        }
        if (is_miss) {
            count<LV>(OFF(L.off_cnt), cid, 1);
            return ret;
        }
        children<LV, true>(cid, r);                          // write hit: inval_children, discarded
        return ST_M;
    }

    // ------------------------------------------------------------ TLB + page table
    // PageTable::translate (page_table.cpp:56-72): physical pages are numbered
    // by first touch of (prog, vpage) in processing order.  Open addressing,
    // linear probing, no deletion: lane k reads slot h+k, so one round trip
    // covers 64 probe positions; the key is present iff it appears before the
    // first empty slot.
    __device__ __forceinline__ uint64_t page_translate(int prog, uint64_t vpage) {
        const TlbGeo& T = g->tlb;
        PageEnt* tab = at<PageEnt>(OFF(T.off_pages));
        const uint64_t mask = T.pages_cap - 1;
        uint64_t x = vpage * 0x9E3779B97F4A7C15ull ^ ((uint64_t)(uint32_t)prog * 0xC2B2AE3D27D4EB4Full);
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        uint64_t h = x & mask;
        for (uint64_t done = 0; done < T.pages_cap; done += 64) {
            const uint64_t slot = (h + (uint64_t)ln) & mask;
            const PageEnt e = tab[slot];
            const bool used = e.used != 0;
            const uint64_t mm = ballot(used && e.vpage == vpage && e.prog == prog);
            const uint64_t me = ballot(!used);
            const int fe = me ? (int)__builtin_ctzll(me) : 64;
            if (mm && (int)__builtin_ctzll(mm) < fe) return rl64(e.ppage, (int)__builtin_ctzll(mm));
            if (me) {
                const uint64_t pp = uni64(lds_eng.page_next);
                if (pp * 4 >= T.pages_cap * 3) {              // keep probes short; engine limit
                    err_or(PU_ERRF_PAGES);
                    lds_eng.stop = 1;
                }
                lds_eng.page_next = pp + 1;
                if (ln == fe) tab[slot] = PageEnt{vpage, prog, 1u, pp, 0ull};
                return pp;
            }
            h = (h + 64) & mask;
        }
        err_or(PU_ERRF_PAGES);
        lds_eng.stop = 1;
        return 0;
    }

    // System::tlb_translate (system.cpp:897-918): private TLB per core; the
    // request's address becomes physical (ppage << log2(page) | offset).
    __device__ __forceinline__ int tlb_translate(int core, Req& r, int64_t timer) {
        const TlbGeo& T = g->tlb;
        LineMeta* meta = at<LineMeta>(OFF(T.off_meta));
        int64_t* tsa = at<int64_t>(OFF(T.off_ts));
        uint64_t* ppa = at<uint64_t>(OFF(T.off_ppage));
        SetView v;
        set_load(v, meta, tsa, T.nsets, T.nways, T.offbits, T.idxbits, (uint64_t)core, r.addr);
        const uint64_t mypp = !wide(T.nways) && (uint64_t)ln < T.nways ? ppa[v.line0 + (uint64_t)ln] : 0ull;
        count<PU_CNT_TLB>(OFF(T.off_cnt), core, 0);
        int d = T.access_time;
        int way = set_find(v, meta, tsa, T.nways, r.prog);
        uint64_t ppage;
        if (way < 0) {
            uint32_t old_st;
            uint64_t old_addr;
            int old_prog;
            way = set_replace(v, meta, tsa, T.nways, T.offbits, T.idxbits, r.prog, &old_st, &old_addr, &old_prog);
            if (old_st != ST_I) count<PU_CNT_TLB>(OFF(T.off_cnt), core, 2);
            count<PU_CNT_TLB>(OFF(T.off_cnt), core, 1);
            set_state(v, meta, way, ST_V);
            ppage = page_translate(r.prog, r.addr >> T.offbits);
            if (ln == wl(v, way)) ppa[v.line0 + (uint64_t)way] = ppage;
            d += T.page_miss_delay;
        } else if (wide(T.nways)) {
            ppage = uni64(ppa[v.line0 + (uint64_t)way]);
        } else {
            ppage = rl64(mypp, way);
        }
        set_ts(v, tsa, way, timer);
        r.addr = (ppage << T.offbits) | (r.addr % T.page_size);
        return d;
    }

    // System::access (system.cpp:144-168).
    __device__ __forceinline__ int access(int core, const Req& r_in, int64_t timer) {
        if (core < 0 || core >= g->num_cores) {
            err_or(PU_ERRF_CORE_RANGE);
            return -1;
        }
        stat_add(SN_REQS, 1);
        hit = false;
        dly = 0;
        Req r = r_in;
        if (g->tlb_enable) {
            dly = tlb_translate(core, r, timer);
            lds_eng.last_addr = r.addr;
        }
        if (g->sys_type == 0) mesi<0>(core, r, timer + dly);
        else mesi_bus<0>(core, r, timer + dly);
        return dly;
    }

    __device__ __forceinline__ void flush_stats() {
        EngineStats* S = at<EngineStats>(OFF(g->off_stats));
        if constexpr (kCntSum) {   // lane k: per-level sum k
            const uint64_t v = ln < SN_COUNT - SN_CNT0 ? lds_stat[SN_CNT0 + ln] : 0ull;
            if (v) atomic_add_u64(&S->lvl_cnt[0][0] + ln, v);
        }
        if (ln != 0) return;
        // Network::transmit's per-packet router term (hops+1)*router, inject
        // term and link remainder total - router - (plen-1) - inject, summed
        // (mod 2^64, as the per-packet sums are)
        const uint64_t acc = lds_stat[SN_ACC], dist = lds_stat[SN_DIST], tot = lds_stat[SN_TOTAL];
        const uint64_t rt = (dist + acc) * (uint64_t)(uint32_t)g->router_delay;
        const uint64_t inj = acc * (uint64_t)(uint32_t)g->inject_delay;
        atomic_add_u64(&S->net_accesses, acc);
        atomic_add_u64(&S->net_distance, dist);
        atomic_add_u64(&S->net_total_delay, tot);
        atomic_add_u64(&S->net_router_delay, rt);
        atomic_add_u64(&S->net_link_delay, tot - rt - (lds_stat[SN_PLEN] - acc) - inj);
        atomic_add_u64(&S->net_inject_delay, inj);
        atomic_add_u64(&S->dram_accesses, lds_stat[SN_DRAM]);
        atomic_add_u64(&S->total_bus_contention, lds_stat[SN_BUSCONT]);
        atomic_add_u64(reinterpret_cast<uint64_t*>(&S->total_num_broadcast), lds_stat[SN_BCAST]);
        atomic_add_u64(&S->link_flits, lds_stat[SN_FLITS]);
        atomic_add_u64(&S->mg1_calls, lds_stat[SN_MG1]);
        atomic_add_u64(&S->lockdown_calls, lds_stat[SN_LOCKDOWN]);
        atomic_add_u64(&S->bus_accesses, lds_stat[SN_BUSACC]);
        atomic_add_u64(&S->requests, lds_stat[SN_REQS]);
        atomic_add_u64(&S->dram_row_hits, lds_stat[SN_ROWHIT]);
        atomic_add_u64(&S->dram_row_empty, lds_stat[SN_ROWEMPTY]);
        atomic_add_u64(&S->dram_row_conflicts, lds_stat[SN_ROWCONF]);
        atomic_add_u64(&S->dram_bank_wait, lds_stat[SN_BANKWAIT]);
        __hip_atomic_fetch_or(&S->error_flags, (uint64_t)lds_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};

__device__ __forceinline__ void stats_init() {
    const int ln = lane_id();
    if (ln < SN_COUNT) lds_stat[ln] = 0;
    if constexpr (kAliveLds)
        for (int i = ln; i < kAliveWords; i += 64) lds_alive[i] = 0u;
#ifdef PU_PROF
    if (ln < PF_COUNT) lds_prof[ln] = 0;
#endif
    if (ln == 0) lds_err = 0;
    __syncthreads();
}

// A replica-pool wave's own state (uncore_body), in LDS: lane 0 writes it.
struct PoolCtl {
    int32_t nrep;
    int32_t r;            // the replica the wave holds, -1 = none
};
static __shared__ PoolCtl lds_pool;
// The replica a pool wave runs next: `cur` if it holds one, else the next
// unstarted replica (sched[0], one device-scope atomic by lane 0); -1 once
// every replica has been taken.
__device__ __forceinline__ int pool_next(uint32_t* sched, int cur) {
    if (cur >= 0) return cur;
    uint32_t t = 0;
    if (lane_id() == 0) t = __hip_atomic_fetch_add(&sched[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int r = (int)rl32(t, 0);
    return r < (int)uni32((uint32_t)lds_pool.nrep) ? r : -1;
}

// Latency mode: the replica's packed queue headers (32 B each, the same
// layout in HBM and in the LDS image) into / out of the LDS image, and the
// M/G/1 cache words set empty.  Thread t of the two-wave workgroup copies
// pieces t, t + 128, ...
__device__ __forceinline__ void hdr_image_in(const char* qhdr, uint32_t nqueues, uint32_t t) {
    const AS1 v4u32* gh = (const AS1 v4u32*)(AS1 char*)qhdr;
    for (uint32_t k = t; k < nqueues * PU_LDS_SLOT; k += 128) lds_qhdr[k] = gh[k];
    for (uint32_t k = t; k < nqueues; k += 128) lds_qcache[k] = PU_MG1_CACHE_NONE;
}
__device__ __forceinline__ void hdr_image_out(char* qhdr, uint32_t nqueues, uint32_t t) {
    AS1 v4u32* gh = (AS1 v4u32*)(AS1 char*)qhdr;
    for (uint32_t k = t; k < nqueues * PU_LDS_SLOT; k += 128) gh[k] = lds_qhdr[k];
}

// A 16-B request record (pu_req16, primeuncore.h): a = addr_dmem; b = timer
// (bits 0-39) | core (40-55) | prog_id (56-61) | mem_type (62) | batch_start
// (63); tag 0.  pu_pack_req16 refuses what does not fit, so this is exact.
__device__ __forceinline__ pu_req req_unpack16(v2u64 w) {
    pu_req q;
    q.addr = w.x;
    q.timer = (int64_t)(w.y & ((1ull << 40) - 1));
    q.core = (int32_t)((w.y >> 40) & 0xFFFFu);
    q.prog_id = (int32_t)((w.y >> 56) & 63u);
    q.mem_type = (uint8_t)((w.y >> 62) & 1u);
    q.batch_start = (uint8_t)(w.y >> 63);
    q.tag = 0;
    q._pad1 = 0;
    return q;
}

// One replica's message loop (prime.cpp:120-137): reqs[b .. end) in order, D
// restarting at each batch_start; d = access(core, req, timer + D); D += d - 1.
// e.base is the replica's arena.  Time-sliced launches (deadline != MAX) stop
// before the first request that would begin at or after `deadline`
// (s_memrealtime, 100 MHz); a replica only ever stops between requests, so
// its stream continues exactly in the next launch.  The index of the first
// request not processed goes to *pos_out (if given); returns whether the
// range is done.
template <int NL, bool SLICED, bool LH>
__device__ __forceinline__ bool replica_steps(Engine<NL, LH>& e, const pu_req* __restrict__ reqs,
                                              int32_t* __restrict__ delays, uint64_t b, uint64_t end,
                                              uint64_t* __restrict__ pos_out);
// The message loop's state from the replica's RunState (lane 0 into lds_ctl,
// lds_eng), counters zeroed: the start of a launch's work on one replica.
template <int NL, bool LH>
__device__ __forceinline__ void replica_begin(Engine<NL, LH>& e, uint64_t deadline, uint32_t flags) {
    e.hq_head = 0;
    stats_init();
    e.dly = 0;
    e.hit = false;
    // The message loop's own state lives in LDS (lane 0 writes, every lane reads
    // it back wave-uniform): nothing of it stays in registers across the
    // inlined access(), whose register budget is tight (5 waves/SIMD).
    RunState* rs = e.template at<RunState>(OFF(e.g->off_run));
    if (e.ln == 0) {
        const int32_t h0 = rs->halted;
        lds_ctl.D = rs->batch_delay;
        lds_ctl.halted0 = h0;
        lds_ctl.halted = (flags & PU_KF_NOHALT) ? 0 : h0;
        lds_ctl.skip = rs->skip_msg;
        lds_ctl.flags = flags;
        lds_ctl.msg_shift = rs->msg_shift;
        lds_ctl.dead_tags = rs->dead_tags;
        lds_ctl.deadline = deadline;
        lds_ctl.done = 0;
        lds_ctl.cur = 0;
        lds_ctl.limit_at = UINT64_MAX;
    }
    __builtin_amdgcn_wave_barrier();
    e.init_shared((int32_t)rl32(e.ln == 0 ? (uint32_t)rs->pool_top : 0u, 0), rl64(e.ln == 0 ? rs->page_next : 0ull, 0),
                  rl64(e.ln == 0 ? rs->last_addr : 0ull, 0));
}

template <int NL, bool SLICED, bool LH>
__device__ __forceinline__ bool replica_loop(Engine<NL, LH>& e, const pu_req* __restrict__ reqs,
                                             int32_t* __restrict__ delays, uint64_t b, uint64_t end,
                                             uint64_t* __restrict__ pos_out, uint64_t deadline, uint32_t flags) {
    replica_begin<NL, LH>(e, deadline, flags);
    return replica_steps<NL, SLICED, LH>(e, reqs, delays, b, end, pos_out);
}

// The requests [b, end) through prime.cpp's message loop on the state in
// lds_ctl / lds_eng (replica_begin).
template <int NL, bool SLICED, bool LH>
__device__ __forceinline__ bool replica_steps(Engine<NL, LH>& e, const pu_req* __restrict__ reqs,
                                              int32_t* __restrict__ delays, uint64_t b, uint64_t end,
                                              uint64_t* __restrict__ pos_out) {
    uint64_t i = b;
    for (; i < end; i++) {
        // the slice's clock, every fourth request (a slice still ends between
        // requests, at most three requests later)
        if (SLICED && (i & 3) == 0 && __builtin_amdgcn_s_memrealtime() >= uni64(lds_ctl.deadline)) break;
        if (uni32((uint32_t)lds_ctl.halted)) break;   // the rest is zero-filled below
        PROF_T(p_loop);
        const uint32_t fl = uni32(lds_ctl.flags);
        const pu_req q = (fl & PU_KF_REQ16) ? req_unpack16(reinterpret_cast<const v2u64*>(reqs)[i]) : reqs[i];
        const bool core_ok = q.core >= 0 && q.core < e.g->num_cores;
        if (e.ln == 0) lds_ctl.cur = i;
        if (q.batch_start && e.ln == 0) {
            lds_ctl.D = 0;
            lds_ctl.skip = (fl & PU_KF_MSGHALT) ? (int32_t)((lds_ctl.dead_tags >> (q.tag & 63)) & 1) : 0;
            if ((fl & PU_KF_CLOSED) && core_ok)
                lds_ctl.msg_shift = e.template at<int64_t>(OFF(e.g->off_core_shift))[q.core];
        }
        __builtin_amdgcn_wave_barrier();
        if (uni32((uint32_t)lds_ctl.skip)) {     // PU_KF_MSGHALT: this message's receive thread has exited
            if (e.ln == 0) {
                delays[i] = 0;
                if constexpr (LH) lds_ctl.last_d = 0;
            }
            continue;
        }
        PROF_ADD(PF_REQ, p_loop);
        const int64_t shift = (fl & PU_KF_CLOSED) ? (int64_t)uni64((uint64_t)lds_ctl.msg_shift) : 0;
        const int64_t t = q.timer + shift + (int32_t)uni32((uint32_t)lds_ctl.D);
        Req r{q.addr, q.prog_id, (int32_t)q.mem_type};
        int d = e.access(q.core, r, t);
        if (e.ln == 0) {
            const int32_t D = lds_ctl.D + d - 1;
            lds_ctl.D = D;
            lds_ctl.done++;
            delays[i] = d;
            if constexpr (LH) lds_ctl.last_d = d;
            if (core_ok) {
                e.template at<int64_t>(OFF(e.g->off_completion))[q.core] = t + d;
                if (lds_ctl.flags & PU_KF_CLOSED)
                    e.template at<int64_t>(OFF(e.g->off_core_shift))[q.core] = lds_ctl.msg_shift + D;
            }
            if (D < 0) {                         // prime.cpp:130-134
                err_or(PU_ERRF_NEG_DELAY);
                if (lds_ctl.flags & PU_KF_MSGHALT) {
                    lds_ctl.skip = 1;
                    lds_ctl.dead_tags |= 1ull << (q.tag & 63);
                } else if (!(lds_ctl.flags & PU_KF_NOHALT)) {
                    lds_ctl.halted = 1;
                }
            }
            if (lds_eng.stop) {                  // engine limit hit: cannot continue exactly
                lds_ctl.halted = 1;
                lds_ctl.skip = 0;
            }
        }
        __builtin_amdgcn_wave_barrier();
        PROF_ADD(PF_LOOP, p_loop);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no staging DMA outlives the loop
    if (i < end && uni32((uint32_t)lds_ctl.halted)) {
        // the reference's handler thread has exited (prime.cpp:130-134):
        // nothing more is simulated; the rest of the range reads 0, written
        // by the whole wave at once
        for (uint64_t k = i + (uint64_t)e.ln; k < end; k += 64) delays[k] = 0;
        i = end;
    }
    if (pos_out && e.ln == 0) *pos_out = i;
    return i >= end;
}

// The replica's run state back to HBM and its counters flushed, after
// replica_loop (and, in latency mode, after the header image went back).
template <int NL, bool LH>
__device__ __forceinline__ void replica_close(Engine<NL, LH>& e) {
    RunState* rs = e.template at<RunState>(OFF(e.g->off_run));
    if (e.ln == 0) {
        rs->batch_delay = lds_ctl.D;
        rs->halted = (lds_ctl.flags & PU_KF_NOHALT) ? (lds_ctl.halted0 | lds_ctl.halted) : lds_ctl.halted;
        rs->skip_msg = lds_ctl.skip;
        rs->msg_shift = lds_ctl.msg_shift;
        rs->dead_tags = lds_ctl.dead_tags;
        rs->limit_at = lds_ctl.limit_at;
        rs->processed += lds_ctl.done;
        rs->pool_top = lds_eng.pool_top;
        rs->page_next = lds_eng.page_next;
        rs->last_addr = lds_eng.last_addr;
    }
    __syncthreads();
    e.flush_stats();
#ifdef PU_PROF
    if (e.ln < PF_COUNT) atomicAdd(&g_prof[e.ln], lds_prof[e.ln]);
#endif
}

// One replica on this wave: replica `rep` runs requests [pos[ix] or off[ix],
// off[ix+1]) (replica_loop) and its state goes back (replica_close); in
// latency mode with the queue-header image in LDS around the loop (the
// workgroup's helper wave runs mg1_helper meanwhile, uncore_body).  Returns
// whether the range is done.
template <int NL, int MODE, bool LH>
__device__ __forceinline__ bool replica_run(Engine<NL, LH>& e, char* __restrict__ arena, int rep, int ix,
                                            const pu_req* __restrict__ reqs, const uint64_t* __restrict__ off,
                                            int32_t* __restrict__ delays, uint64_t* __restrict__ pos,
                                            uint64_t deadline, uint32_t flags) {
    constexpr bool SLICED = MODE >= 1;
    // (pointer arithmetic on the kernel argument: the compiler keeps it a
    // global-memory pointer, so the engine's accesses stay global_*, not flat_*)
    e.base = arena + (size_t)rep * OFF(e.g->replica_bytes);
    if constexpr (LH) {
        // Latency mode: a two-wave workgroup; the helper wave (the second,
        // uncore_body) copies the other half of the queue-header image.  The
        // simulating wave copies slots lane, lane + 128, ... of the replica's
        // queue headers into the LDS image (pieces a, b, c; d = no cached
        // wait) before [1].
        hdr_image_in(e.base + OFF(e.g->off_qhdr), (uint32_t)e.g->nqueues, (uint32_t)e.ln);
        if (e.ln == 0) {
            lds_hq_head = 0;
            lds_main_done = 0;
        }
    }
#ifdef PU_PROF
    const uint64_t blk_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const uint64_t b = pos ? pos[ix] : off[ix], end = off[ix + 1];
    const bool done = replica_loop<NL, SLICED, LH>(e, reqs, delays, b, end, pos ? pos + ix : nullptr, deadline, flags);
    if constexpr (LH) {                                   // the headers back
        if (e.ln == 0) *(volatile AS3 uint32_t*)&lds_main_done = 1u;
        __syncthreads();                                  // [2] the helper has stopped writing the image
        hdr_image_out(e.base + OFF(e.g->off_qhdr), (uint32_t)e.g->nqueues, (uint32_t)e.ln);
    }
    replica_close<NL, LH>(e);
#ifdef PU_PROF
    if (e.ln == 0 && blockIdx.x < PU_PROF_BLOCKS) {
        const uint64_t blk_t1 = __builtin_amdgcn_s_memrealtime();
        g_blk_t0[blockIdx.x] = blk_t0;
        g_blk_t1[blockIdx.x] = blk_t1;
        g_blk_dur[blockIdx.x] += blk_t1 - blk_t0;
    }
#endif
    return done;
}


// Resident mode (MODE 3, latency kernels only; geometry.h PuMailbox): one
// two-wave workgroup stays on the GPU for replica `rep` and serves the host's
// commands — a lone uncore_access (uncore_manager.cpp:82-85, prime.cpp:129)
// or a short host batch — without a launch per call.  Across commands it
// keeps in its CU what a launch would reload and write back: the queue-header
// image (LDS), the message loop's run state (lds_ctl / lds_eng) and the
// counter sums (lds_stat, lds_err), which go back to HBM (replica_close) once,
// when the kernel leaves; the host stops it before anything reads them
// (uncore.cpp resident_quiesce).  Each command runs replica_steps over its
// requests with exactly the per-launch transitions of replica_begin /
// replica_close (the halted flag under PU_KF_NOHALT, the engine-limit stop,
// the first limit position), so results are the launch path's.  A one-request
// command travels inside the command line itself; longer ones are copied from
// the mailbox's request area into device memory.  Delays go straight into the
// host buffer; `ack` follows a system-scope release.  The kernel leaves on a
// STOP command or after `idle_ticks` (s_memrealtime, 100 MHz) without one: a
// persistent kernel that always drains by itself.
struct ResCtl {
    uint64_t seq;      // the last command taken
    uint64_t n;        // its requests
    uint64_t err;      // the replica's error flags in HBM when the kernel started
    uint32_t flags, cmd;
    int32_t halted;    // RunState.halted between commands
};
static __shared__ ResCtl lds_res;

// (relaxed: a system-scope load reads the host's value without invalidating
// the caches at every poll; the acquire fence follows once the value changed)
__device__ __forceinline__ uint64_t sys_load_u64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int NL>
__device__ __forceinline__ void resident_body(const Geo* __restrict__ g, char* __restrict__ arena, int rep,
                                              pu_req* __restrict__ stage, PuMailbox* mb, uint64_t idle_ticks,
                                              uint64_t cap) {
    constexpr bool LH = true;                 // (OFF)
    Engine<NL, LH> e;
    e.g = g;
    e.ln = lane_id();
    const bool helper = __builtin_amdgcn_readfirstlane(threadIdx.x) >= 64;
    e.base = arena + (size_t)rep * OFF(g->replica_bytes);
    char* hb = e.base + OFF(g->off_qhdr);
    const uint32_t nq = (uint32_t)g->nqueues;
    const AS1 v4u32* hline = (const AS1 v4u32*)(AS1 char*)(char*)&mb->h;
    const AS1 v4u32* hreq = (const AS1 v4u32*)(AS1 char*)(char*)(mb + 1);
    int32_t* hdelay = reinterpret_cast<int32_t*>(reinterpret_cast<pu_req*>(mb + 1) + cap);
    AS1 v4u32* dst = (AS1 v4u32*)(AS1 char*)(char*)stage;
    hdr_image_in(hb, nq, threadIdx.x);        // threads 0..127: pieces t, t + 128, ...
    if (helper) {
        __syncthreads();                      // [S] replica_begin's stats_init
    } else {
        replica_begin<NL, LH>(e, UINT64_MAX, 0u);   // run state and counters, once per kernel   [S]
        if (e.ln == 0) {
            lds_res.seq = sys_load_u64(&mb->d.ack);   // the host sets ack = seq before the launch
            lds_res.err = e.template at<EngineStats>(OFF(g->off_stats))->error_flags;
            lds_res.halted = lds_ctl.halted0;
        }
    }
    for (;;) {
        uint64_t tk0 = 0;
        if (!helper) {
            // lane 0 polls the host's command word; the other lanes wait with it
            const uint64_t last = uni64(lds_res.seq);
            const uint64_t t_idle = __builtin_amdgcn_s_memrealtime() + idle_ticks;
            uint64_t sq = last;
            for (;;) {
                if (e.ln == 0) sq = sys_load_u64(&mb->h.seq);
                sq = rl64(sq, 0);
                if (sq != last || __builtin_amdgcn_s_memrealtime() >= t_idle) break;
                __builtin_amdgcn_s_sleep(2);
            }
            tk0 = __builtin_amdgcn_s_memrealtime();
            if (sq != last) {
                // the whole command line in one round trip (written before seq):
                // lane 0 {seq, n | flags | cmd}, lanes 1-2 the inline request
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                v4u32 w = v4u32{0u, 0u, 0u, 0u};
                if (e.ln < 3) w = *(const volatile AS1 v4u32*)&hline[e.ln];
                const uint32_t n = rl32(w.z, 0), fc = rl32(w.w, 0);
                if (fc >> 16 == PU_RES_RUN && n == 1 && (e.ln == 1 || e.ln == 2)) dst[e.ln - 1] = w;
                if (e.ln == 0) {
                    lds_res.n = n;
                    lds_res.flags = fc & 0xFFFFu;
                    lds_res.cmd = fc >> 16;
                    lds_res.seq = sq;
                }
            } else if (e.ln == 0) {
                lds_res.cmd = PU_RES_STOP;            // idle: leave
            }
        }
        __syncthreads();                              // [A] the command is in LDS
        if (uni32(lds_res.cmd) != PU_RES_RUN) break;
        const uint64_t n = min(uni64(lds_res.n), cap);
        if (helper) {
            __syncthreads();                          // [B] the command's state is set
            mg1_helper(g, e.base, stage, 0, n);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no prefetch DMA outlives the command
            continue;                                 // to [A]: the main wave has left its loop
        }
        if (n > 1) {   // the requests: mailbox -> device staging, 16 B per lane and step, 4 steps in flight
            const uint64_t pieces = 2 * n;
            for (uint64_t k = (uint64_t)e.ln; k < pieces; k += 256) {
                v4u32 a0 = v4u32{0u, 0u, 0u, 0u}, a1 = a0, a2 = a0, a3 = a0;
                a0 = hreq[k];
                if (k + 64 < pieces) a1 = hreq[k + 64];
                if (k + 128 < pieces) a2 = hreq[k + 128];
                if (k + 192 < pieces) a3 = hreq[k + 192];
                dst[k] = a0;
                if (k + 64 < pieces) dst[k + 64] = a1;
                if (k + 128 < pieces) dst[k + 128] = a2;
                if (k + 192 < pieces) dst[k + 192] = a3;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t tk1 = __builtin_amdgcn_s_memrealtime();
        // replica_begin's per-launch transitions, on the state kept in LDS
        const uint32_t fl = uni32(lds_res.flags);
        if (e.ln == 0) {
            const int32_t h0 = lds_res.halted;
            lds_ctl.halted0 = h0;
            lds_ctl.halted = (fl & PU_KF_NOHALT) ? 0 : h0;
            lds_ctl.flags = fl;
            lds_ctl.cur = 0;
            lds_ctl.limit_at = UINT64_MAX;
            lds_ctl.last_d = 0;
            lds_eng.stop = 0;
            lds_hq_head = 0;
            lds_main_done = 0;
        }
        const uint64_t err0 = uni64(lds_err);
        e.dly = 0;
        e.hit = false;
        e.hq_head = 0;
        __syncthreads();                              // [B]
        replica_steps<NL, false, LH>(e, stage, hdelay, 0, n, nullptr);
        const uint64_t tk2 = __builtin_amdgcn_s_memrealtime();
        if (e.ln == 0) {
            *(volatile AS3 uint32_t*)&lds_main_done = 1u;
            // replica_close's halted rule
            lds_res.halted = (fl & PU_KF_NOHALT) ? (lds_ctl.halted0 | lds_ctl.halted) : lds_ctl.halted;
        }
        // The fast answer: a one-request command that raised no error bit, on a
        // configuration without TLB translation, needs nothing but its delay,
        // which travels with the command's seq in one 8-B store (atomic to the
        // host; the host already holds the error flags): no release fence, no
        // other mailbox store.  Everything else takes the full answer below.
        if (n == 1 && uni64(lds_err) == err0 && !g->tlb_enable) {
            if (e.ln == 0)
                __hip_atomic_store(&mb->d.fast, (uint64_t)(uint32_t)uni64(lds_res.seq) |
                                                    ((uint64_t)(uint32_t)lds_ctl.last_d << 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            continue;
        }
        if (e.ln == 0) {
            volatile PuResDev* Dv = &mb->d;
            Dv->err = lds_res.err | lds_err;
            Dv->last_addr = lds_eng.last_addr;
            Dv->phase[0] = (uint32_t)(tk1 - tk0);
            Dv->phase[1] = (uint32_t)(tk2 - tk1);
            Dv->phase[2] = 0u;
            Dv->phase[3] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - tk2);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the delays and the mailbox visible
        if (e.ln == 0) __hip_atomic_store(&mb->d.ack, uni64(lds_res.seq), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // leave: the headers, the run state and the counters back to HBM
    hdr_image_out(hb, nq, threadIdx.x);
    if (helper) {
        __syncthreads();                              // replica_close's barrier
        return;
    }
    if (e.ln == 0) {
        lds_ctl.flags = 0u;                           // replica_close writes lds_ctl.halted as the run state's
        lds_ctl.halted = lds_res.halted;
    }
    replica_close<NL, LH>(e);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (e.ln == 0) __hip_atomic_store(&mb->d.exited, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One workgroup (= one wavefront) per replica.  Replica replica0 + blockIdx.x
// processes reqs[off[blockIdx.x] .. off[blockIdx.x+1]) in order (replica_loop).
//
// Time-sliced launches (pos != nullptr): replica r starts at pos[r] instead of
// off[r], stops before the first request that would begin after
// `budget_ticks` of the s_memrealtime clock (100 MHz) have passed since the
// wave started, and writes its next position back to pos[r]; the slice keeps
// every wave busy instead of waiting for the slowest replica of a fixed-size
// step.
//
// Replica pool (sched != nullptr; time-sliced throughput launches of more
// replicas than the device keeps resident, pu_run_device_pool): the grid is
// one wave per resident slot.  Slot w continues the replica it held when the
// previous launch ended (sched[PU_POOL_SLOT0 + w] = replica + 1; 0 = none);
// once that replica's range is done (its end reached, or stopped by the
// prime.cpp:130-134 rule) the wave takes the next unstarted replica from the
// queue (sched[0], one device-scope atomic by lane 0) and continues within
// the same slice, so no wave idles while replicas remain.  nrep = replicas.
// Each slot adds its wave's lifetime in s_memrealtime ticks to a counter
// (the host's busy-time accounting).
// MODE: 0 fixed ranges, 1 time-sliced, 2 replica pool (time-sliced), 3
// resident (latency kernels: reqs = device staging, off = the host mailbox,
// budget_ticks = idle ticks, nrep = staging capacity; resident_body); each a
// separate instantiation, so the pool's bookkeeping costs the others nothing
// and profiles list the launch kinds apart.
template <int NL, int MODE, bool LH>
__device__ __forceinline__ void uncore_body(const Geo* __restrict__ g, char* __restrict__ arena, int replica0,
                                            const pu_req* __restrict__ reqs, const uint64_t* __restrict__ off,
                                            int32_t* __restrict__ delays, uint64_t* __restrict__ pos,
                                            uint64_t budget_ticks, uint32_t flags, uint32_t* __restrict__ sched,
                                            int nrep) {
  if constexpr (MODE == 3) {
    static_assert(LH, "resident mode runs the latency kernel");
    resident_body<NL>(g, arena, replica0, const_cast<pu_req*>(reqs),
                      reinterpret_cast<PuMailbox*>(const_cast<uint64_t*>(off)), budget_ticks, (uint64_t)nrep);
    (void)delays; (void)pos; (void)flags; (void)sched;
  } else {
    constexpr bool SLICED = MODE >= 1;
    constexpr bool pool = MODE == 2 && !LH;
    if constexpr (!SLICED) {
        pos = nullptr;
        budget_ticks = 0;
    }
    if constexpr (!pool) sched = nullptr;
    const uint64_t wave_t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t deadline = budget_ticks ? wave_t0 + budget_ticks : UINT64_MAX;
    Engine<NL, LH> e;
    e.g = g;
    e.ln = lane_id();
    if constexpr (LH) {
        // the workgroup's second wave is the M/G/1 helper (the test is
        // wave-uniform: readfirstlane tells the compiler so, and everything
        // the simulating wave does after it stays uniform)
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 64) {
            char* rb = arena + (size_t)(replica0 + (int)blockIdx.x) * OFF(g->replica_bytes);
            char* hb = rb + OFF(g->off_qhdr);
            hdr_image_in(hb, (uint32_t)g->nqueues, threadIdx.x);
            __syncthreads();                              // [1] the image is in (stats_init's barrier)
            const uint64_t rb0 = pos ? pos[blockIdx.x] : off[blockIdx.x];
            mg1_helper(g, rb, reqs, rb0, off[blockIdx.x + 1]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no prefetch DMA outlives the wave
            __syncthreads();                              // [2] the main wave left its loop
            hdr_image_out(hb, (uint32_t)g->nqueues, threadIdx.x);
            __syncthreads();                              // [3] before the stats flush
            return;
        }
    }
    if constexpr (!pool) {
        replica_run<NL, MODE, LH>(e, arena, replica0 + (int)blockIdx.x, (int)blockIdx.x, reqs, off, delays, pos,
                                  deadline, flags);
    } else {
        // The replica pool: the wave's own state (the pool arguments, its
        // replica) stays in LDS across the inlined engine, whose register
        // budget is tight, and the one replica_run call site below serves
        // every replica the wave takes.
        if (e.ln == 0) {
            lds_pool.nrep = nrep;
            lds_pool.r = (int32_t)sched[PU_POOL_SLOT0 + blockIdx.x] - 1;
        }
        __builtin_amdgcn_wave_barrier();
        int r = pool_next(sched, (int)uni32((uint32_t)lds_pool.r));
        while (r >= 0) {
            if (e.ln == 0) lds_pool.r = r;
            // off[] and pos[] are indexed by replica in a pool
            if (!replica_run<NL, MODE, LH>(e, arena, r, r, reqs, off, delays, pos, deadline, flags)) break;
            r = pool_next(sched, -1);                     // its range is done: take the next
            if (r < 0 && e.ln == 0) lds_pool.r = -1;
        }
        if (e.ln == 0) {
            sched[PU_POOL_SLOT0 + blockIdx.x] = (uint32_t)(lds_pool.r + 1);
            reinterpret_cast<uint64_t*>(sched + PU_POOL_BUSY0(gridDim.x))[blockIdx.x] +=
                __builtin_amdgcn_s_memrealtime() - wave_t0;
        }
    }
  }
}

#ifndef PU_JIT_GEO
template <int NL, int MODE, bool LH = false>
__global__ __launch_bounds__(LH ? 128 : 64) __attribute__((amdgpu_waves_per_eu(LH ? 1 : PU_MIN_WAVES(NL)))) void uncore_kernel(
    const Geo* __restrict__ g, char* __restrict__ arena, int replica0, const pu_req* __restrict__ reqs,
    const uint64_t* __restrict__ off, int32_t* __restrict__ delays, uint64_t* __restrict__ pos, uint64_t budget_ticks,
    uint32_t flags, uint32_t* __restrict__ sched, int nrep) {
    uncore_body<NL, MODE, LH>(PU_AOT_GEO(g), arena, replica0, reqs, off, delays, pos, budget_ticks, flags, sched,
                                nrep);
}
#else
}  // namespace
// Compile-time configuration (jit.cpp): the four launch shapes of this one
// configuration, unmangled so the host finds them by name in the code object.
#define PU_JIT_KERNEL(NAME, S, H)                                                                                  \
    extern "C" __global__ __launch_bounds__(H ? 128 : 64) __attribute__((amdgpu_waves_per_eu(H ? 1 : PU_MIN_WAVES(PU_JIT_NL)))) \
    void NAME(const Geo* __restrict__ g, char* __restrict__ arena, int replica0, const pu_req* __restrict__ reqs,     \
              const uint64_t* __restrict__ off, int32_t* __restrict__ delays, uint64_t* __restrict__ pos,            \
              uint64_t budget_ticks, uint32_t flags, uint32_t* __restrict__ sched, int nrep) {                       \
        uncore_body<PU_JIT_NL, S, H>(&kJitGeo, arena, replica0, reqs, off, delays, pos, budget_ticks, flags, sched,  \
                                     nrep);                                                                          \
    }
// PU_JIT_PART 0: the throughput kernels (one wave per replica), 1: the
// latency kernels (headers in LDS + the M/G/1 helper); jit.cpp compiles each
// part with its own options.  Undefined: all five (offline tools).
#if !defined(PU_JIT_PART) || PU_JIT_PART == 0
PU_JIT_KERNEL(pu_jit_uncore_s0_h0, 0, false)
PU_JIT_KERNEL(pu_jit_uncore_s1_h0, 1, false)
PU_JIT_KERNEL(pu_jit_uncore_s2_h0, 2, false)
#endif
#if !defined(PU_JIT_PART) || PU_JIT_PART == 1
PU_JIT_KERNEL(pu_jit_uncore_s0_h1, 0, true)
PU_JIT_KERNEL(pu_jit_uncore_s1_h1, 1, true)
PU_JIT_KERNEL(pu_jit_uncore_s3_h1, 3, true)
#endif
namespace {
#endif

#ifndef PU_JIT_GEO
// Queue records start as the single free interval [0, UINT64_MAX]
// (QueueModelHistoryTree ctor, queue_model_history_tree.cpp:28).
// Packed headers (the engine): n = n1 = 0.0, head 0, count 1, newest 0, f0 0;
// wide headers (the unit hooks): n, Σs, Σs², newest 0, then head 0, count 1, f0 0.
__global__ void init_queues_kernel(char* arena, uint64_t replica_bytes, uint64_t off_qhdr, uint64_t off_qring,
                                   int nqueues, int nreplicas, int wide) {
    uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t total = (uint64_t)nqueues * (uint64_t)nreplicas;
    if (id >= total) return;
    uint64_t r = id / (uint64_t)nqueues, q = id % (uint64_t)nqueues;
    char* base = arena + r * replica_bytes;
    if (wide) {
        uint64_t* ab = reinterpret_cast<uint64_t*>(base + off_qhdr + q * PU_HDR_AB);
        for (int i = 0; i < 4; i++) ab[i] = 0;   // n, sum, sum_sq, newest
        uint32_t* cc = reinterpret_cast<uint32_t*>(base + off_qhdr + (uint64_t)nqueues * PU_HDR_AB + q * PU_HDR_C);
        cc[0] = 0;   // head
        cc[1] = 1;   // count
        cc[2] = 0;   // f0
        cc[3] = 0;
    } else {
        uint64_t* h = reinterpret_cast<uint64_t*>(base + off_qhdr + q * PU_HDR_BYTES);
        h[0] = 0;                 // n = 0.0 | head 0
        h[1] = 1;                 // n1 = 0.0 | count 1
        h[2] = 0;                 // newest
        h[3] = 0;                 // f0
    }
    QueueSlot* ring = reinterpret_cast<QueueSlot*>(base + off_qring) + q * PU_QRING;
    ring[0] = QueueSlot{0ull, UINT64_MAX};
}

// ---- unit-test hooks: the queue model / the network alone, one wavefront
__global__ __launch_bounds__(64) void unit_queue_kernel(const Geo* __restrict__ g, char* base, uint64_t minp,
                                                        const uint64_t* __restrict__ t,
                                                        const uint64_t* __restrict__ p, uint64_t n,
                                                        uint64_t* __restrict__ out, uint64_t* __restrict__ mg1) {
    Engine<1, false, true> e;   // wide headers: any packet length
    e.g = g;
    e.ln = lane_id();
    e.base = base;
    e.init_shared(0, 0, 0);
    const NetCtx c = e.net_ctx();
    uint64_t calls = 0, err = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t d = q_op<false, true>(c, 0, t[i], p[i], minp, calls, err);
        if (e.ln == 0) out[i] = d;
    }
    if (e.ln == 0) *mg1 = calls;
}

__global__ __launch_bounds__(64) void unit_network_kernel(const Geo* __restrict__ g, char* base,
                                                          const int32_t* __restrict__ src,
                                                          const int32_t* __restrict__ dst,
                                                          const int32_t* __restrict__ len,
                                                          const uint64_t* __restrict__ timer, uint64_t n,
                                                          uint64_t* __restrict__ out) {
    Engine<1, false, true> e;   // wide headers: any packet length
    e.g = g;
    e.ln = lane_id();
    e.base = base;
    stats_init();
    e.init_shared(0, 0, 0);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t d = e.transmit(src[i], dst[i], len[i], timer[i]);
        if (e.ln == 0) out[i] = d;
    }
    __syncthreads();
    e.flush_stats();
#ifdef PU_PROF
    if (e.ln < PF_COUNT) atomicAdd(&g_prof[e.ln], lds_prof[e.ln]);
#endif
}

// M/G/1 wait (mg1_wait, queue_model_m_g_1.cpp:16-42) of many queue states at
// once, one state per lane: the arithmetic fuzz of tests/test_gpu_mg1.py.  n is
// the reference's UInt64 _num_arrivals, held by the engine as an exact double
// (n < 2^53, checked by the caller).
__global__ __launch_bounds__(256) void unit_mg1_kernel(const uint64_t* __restrict__ n, const double* __restrict__ sum,
                                                       const double* __restrict__ sum_sq,
                                                       const uint64_t* __restrict__ newest, uint64_t cnt,
                                                       uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    QState s;
    s.head = 0;
    s.count = 0;
    s.n = (double)n[i];
    s.sum = sum[i];
    s.sum_sq = sum_sq[i];
    s.newest = newest[i];
    s.f0 = 0;
    out[i] = mg1_wait(s);
}

// Sharer-bitmap pool: free stack [0, P) and RunState.pool_top = P per replica.
__global__ void init_pool_kernel(char* arena, uint64_t replica_bytes, uint64_t off_pool_free, uint64_t off_run,
                                 int pool_entries, int nreplicas) {
    uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t total = (uint64_t)pool_entries * (uint64_t)nreplicas;
    if (id >= total) return;
    uint64_t r = id / (uint64_t)pool_entries, k = id % (uint64_t)pool_entries;
    char* base = arena + r * replica_bytes;
    reinterpret_cast<int32_t*>(base + off_pool_free)[k] = (int32_t)k;
    if (k == 0) reinterpret_cast<RunState*>(base + off_run)->pool_top = pool_entries;
}

#endif  // !PU_JIT_GEO
}  // namespace

#if !defined(__HIPCC_RTC__) && !defined(PU_JIT_OFFLINE)   // the library's host side
extern "C" int pu_engine_init_pool(char* arena, uint64_t replica_bytes, uint64_t off_pool_free, uint64_t off_run,
                                   int pool_entries, int nreplicas, hipStream_t stream) {
    uint64_t total = (uint64_t)pool_entries * (uint64_t)nreplicas;
    if (total == 0) return 0;
    unsigned blocks = (unsigned)((total + 255) / 256);
    hipLaunchKernelGGL(init_pool_kernel, dim3(blocks), dim3(256), 0, stream, arena, replica_bytes, off_pool_free,
                       off_run, pool_entries, nreplicas);
    return hipGetLastError() == hipSuccess ? 0 : PU_EIO;
}

extern "C" int pu_engine_unit_queue(const Geo* d_geo, char* base, uint64_t minp, const uint64_t* t,
                                    const uint64_t* p, uint64_t n, uint64_t* out, uint64_t* mg1, hipStream_t s) {
    hipLaunchKernelGGL(unit_queue_kernel, dim3(1), dim3(64), 0, s, d_geo, base, minp, t, p, n, out, mg1);
    return hipGetLastError() == hipSuccess ? 0 : PU_EIO;
}

extern "C" int pu_engine_unit_mg1(const uint64_t* n, const double* sum, const double* sum_sq, const uint64_t* newest,
                                  uint64_t cnt, uint64_t* out, hipStream_t s) {
    if (cnt == 0) return 0;
    hipLaunchKernelGGL(unit_mg1_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, n, sum, sum_sq, newest,
                       cnt, out);
    return hipGetLastError() == hipSuccess ? 0 : PU_EIO;
}

extern "C" int pu_engine_unit_network(const Geo* d_geo, char* base, const int32_t* src, const int32_t* dst,
                                      const int32_t* len, const uint64_t* timer, uint64_t n, uint64_t* out,
                                      hipStream_t s) {
    hipLaunchKernelGGL(unit_network_kernel, dim3(1), dim3(64), 0, s, d_geo, base, src, dst, len, timer, n, out);
    return hipGetLastError() == hipSuccess ? 0 : PU_EIO;
}

// ---------------------------------------------------------------- launchers
extern "C" int pu_engine_launch(const Geo* d_geo, int num_levels, char* arena, int replica0, int nblocks,
                                const pu_req* reqs, const uint64_t* off, int32_t* delays, uint64_t* pos,
                                uint64_t budget_ticks, uint32_t flags, int lds_headers, uint32_t* sched, int nrep,
                                hipStream_t stream) {
    dim3 grid((unsigned)nblocks), block(lds_headers ? 128 : 64);   // latency mode: + the M/G/1 helper wave
#define PU_LAUNCH3(L, S, H)                                                                                        \
    hipLaunchKernelGGL((uncore_kernel<L, S, H>), grid, block, 0, stream, d_geo, arena, replica0, reqs, off, delays,   \
                       pos, budget_ticks, flags, sched, nrep)
#define PU_LAUNCH(L)                                                                                              \
    if (sched) PU_LAUNCH3(L, 2, false);                                                                            \
    else if (pos) { if (lds_headers) PU_LAUNCH3(L, 1, true); else PU_LAUNCH3(L, 1, false); }                      \
    else { if (lds_headers) PU_LAUNCH3(L, 0, true); else PU_LAUNCH3(L, 0, false); }
    switch (num_levels) {
        case 1: PU_LAUNCH(1); break;
        case 2: PU_LAUNCH(2); break;
        case 3: PU_LAUNCH(3); break;
        case 4: PU_LAUNCH(4); break;
#undef PU_LAUNCH
#undef PU_LAUNCH3
        default: return PU_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? 0 : PU_EIO;
}

// Replicas (one-wave workgroups) of the throughput kernel of launch mode
// `mode` (1 time-sliced, 2 replica pool) resident per CU at once by
// hipOccupancy (VGPRs and the LDS ring staging bound it), and the kernel's
// static LDS bytes (uncore.cpp applies the device's LDS granularity).  A
// launch of more replicas runs the rest only after resident ones finish.
template <int NL>
static hipError_t occ_of(int mode, int* n, int* lds) {
    hipFuncAttributes a{};
    hipError_t e;
    if (mode == 2) {
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(n, uncore_kernel<NL, 2>, 64, 0);
        if (e == hipSuccess) e = hipFuncGetAttributes(&a, (const void*)uncore_kernel<NL, 2>);
    } else {
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(n, uncore_kernel<NL, 1>, 64, 0);
        if (e == hipSuccess) e = hipFuncGetAttributes(&a, (const void*)uncore_kernel<NL, 1>);
    }
    *lds = (int)a.sharedSizeBytes;
    return e;
}
extern "C" int pu_engine_occupancy(int num_levels, int mode, int* blocks_per_cu, int* lds_bytes) {
    int n = 0, lds = 0;
    hipError_t e;
    switch (num_levels) {
        case 1: e = occ_of<1>(mode, &n, &lds); break;
        case 2: e = occ_of<2>(mode, &n, &lds); break;
        case 3: e = occ_of<3>(mode, &n, &lds); break;
        case 4: e = occ_of<4>(mode, &n, &lds); break;
        default: return PU_EINVAL;
    }
    *blocks_per_cu = n;
    *lds_bytes = lds;
    return e == hipSuccess ? 0 : PU_EIO;
}

// Queue headers of one replica that fit the latency-mode LDS image.
extern "C" int pu_engine_lds_header_queues(void) { return (int)PU_LDS_Q; }

extern "C" int pu_engine_init_queues(char* arena, uint64_t replica_bytes, uint64_t off_qhdr, uint64_t off_qring,
                                     int nqueues, int nreplicas, int wide, hipStream_t stream) {
    uint64_t total = (uint64_t)nqueues * (uint64_t)nreplicas;
    if (total == 0) return 0;
    unsigned blocks = (unsigned)((total + 255) / 256);
    hipLaunchKernelGGL(init_queues_kernel, dim3(blocks), dim3(256), 0, stream, arena, replica_bytes, off_qhdr,
                       off_qring, nqueues, nreplicas, wide);
    return hipGetLastError() == hipSuccess ? 0 : PU_EIO;
}

#ifdef PU_PROF
// Profiling build only: read (and optionally clear) the region counters.
extern "C" int pu_engine_prof_read(unsigned long long* out, int n, int reset) {
    if (n > PF_COUNT) n = PF_COUNT;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (n > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * n) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[PF_COUNT] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return -1;
        static unsigned long long zb[PU_PROF_BLOCKS];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_blk_dur), zb, sizeof(zb)) != hipSuccess) return -1;
    }
    return n;
}
// Per-block stamps (s_memrealtime, 100 MHz) of the last launch and summed durations.
extern "C" int pu_engine_prof_blocks(unsigned long long* t0, unsigned long long* t1, unsigned long long* dur, int n) {
    if (n > PU_PROF_BLOCKS) n = PU_PROF_BLOCKS;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    size_t b = sizeof(unsigned long long) * (size_t)n;
    if (hipMemcpyFromSymbol(t0, HIP_SYMBOL(g_blk_t0), b) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(t1, HIP_SYMBOL(g_blk_t1), b) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(dur, HIP_SYMBOL(g_blk_dur), b) != hipSuccess) return -1;
    return n;
}
#endif
#endif  // !__HIPCC_RTC__ && !PU_JIT_OFFLINE
