// uncore.cpp — the C ABI of include/primeuncore.h: engine lifetime, replica
// layout, the thread->core map, the batch paths that launch the HIP engine,
// statistics and the report text.
//
// Replaces, for the hot path only:
//   UncoreManager::init/allocCore/deallocCore/getCoreId/uncore_access/report
//                                   (reference src/uncore_manager.cpp:46-98)
//   System::init/report             (reference src/system.cpp:47-141, 956-1111)
//   ThreadSched                     (reference src/thread_sched.cpp:44-118)
// There is no CPU fallback: without a HIP device pu_create fails (PU_ENODEV).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <ctime>
#include <cstddef>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "../../include/primeuncore.h"
#include "common.h"
#include "geometry.h"
#include "geo_emit.h"
#include "jit.h"

extern "C" int pu_engine_launch(const Geo* d_geo, int num_levels, char* arena, int replica0, int nblocks,
                                const pu_req* reqs, const uint64_t* off, int32_t* delays, uint64_t* pos,
                                uint64_t budget_ticks, uint32_t flags, int lds_headers, uint32_t* sched, int nrep,
                                hipStream_t stream);
extern "C" int pu_engine_lds_header_queues(void);
extern "C" int pu_engine_init_pool(char* arena, uint64_t replica_bytes, uint64_t off_pool_free, uint64_t off_run,
                                   int pool_entries, int nreplicas, hipStream_t stream);
extern "C" int pu_engine_unit_queue(const Geo* d_geo, char* base, uint64_t minp, const uint64_t* t,
                                    const uint64_t* p, uint64_t n, uint64_t* out, uint64_t* mg1, hipStream_t s);
extern "C" int pu_engine_unit_mg1(const uint64_t* n, const double* sum, const double* sum_sq, const uint64_t* newest,
                                  uint64_t cnt, uint64_t* out, hipStream_t s);
extern "C" int pu_engine_unit_network(const Geo* d_geo, char* base, const int32_t* src, const int32_t* dst,
                                      const int32_t* len, const uint64_t* timer, uint64_t n, uint64_t* out,
                                      hipStream_t s);
extern "C" int pu_engine_init_queues(char* arena, uint64_t replica_bytes, uint64_t off_qhdr, uint64_t off_qring,
                                     int nqueues, int nreplicas, int wide, hipStream_t stream);
extern "C" int pu_engine_occupancy(int num_levels, int mode, int* blocks_per_cu, int* lds_bytes);

namespace pu {

static thread_local std::string g_err;

int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

}  // namespace pu

namespace {

int ilog2(uint64_t x) { return (int)std::log2((double)x); }

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

struct Layout {
    uint64_t cur = 0;
    uint64_t take(uint64_t bytes, uint64_t align = 256) {
        cur = align_up(cur, align);
        uint64_t o = cur;
        cur += bytes;
        return o;
    }
};

// Validates the configuration (every condition under which the reference
// is undefined or this engine does not implement the branch) and computes the
// replica layout.
int build_geo(const pu_sim_cfg* c, Geo* g, uint64_t pool_cap = 0) {
    std::memset(g, 0, sizeof(*g));
    const pu_sys_cfg& y = c->sys;
    if (y.num_levels < 1 || y.num_levels > PU_MAX_LEVELS) return pu::set_error(PU_EINVAL, "num_levels must be 1..4");
    if (y.num_cores < 1) return pu::set_error(PU_EINVAL, "num_cores must be >= 1");
    if (y.sys_type != 0 && y.sys_type != 1) return pu::set_error(PU_EINVAL, "sys_type must be 0 (directory) or 1 (bus)");
    const bool bus_sys = y.sys_type == 1;
    g->num_cores = y.num_cores;
    g->num_levels = y.num_levels;
    g->sys_type = y.sys_type;
    g->protocol_type = y.protocol_type;
    g->max_num_sharers = y.max_num_sharers;
    g->shared_llc = y.shared_llc;
    g->tlb_enable = y.tlb_enable;
    g->dram_access_time = y.dram_access_time;
    g->bus_latency = y.bus_latency;
    g->cnt_sum = y.verbose_report ? 0 : 1;   // per-level sums suffice unless the report lists every cache
    Layout lay;
    int nbus = 0;
    for (int l = 0; l < y.num_levels; l++) {
        const pu_cache_cfg& cc = y.cache[l];
        LevelGeo& L = g->lv[l];
        if (cc.share < 1 || cc.block_size < 1 || cc.num_ways < 1) return pu::set_error(PU_EINVAL, "bad cache geometry");
        if (cc.num_ways > PU_MAX_WAYS_WIDE) return pu::set_error(PU_ENOTSUP, "at most 4096 ways per set");
        L.nsets = cc.size / (cc.block_size * cc.num_ways);
        if (L.nsets < 1) return pu::set_error(PU_EINVAL, "cache has no sets");
        L.nways = cc.num_ways;
        L.block = cc.block_size;
        L.offbits = ilog2(cc.block_size);
        L.idxbits = ilog2(L.nsets);
        if (L.offbits + L.idxbits >= 64) return pu::set_error(PU_EINVAL, "cache geometry exceeds 64-bit addresses");
        L.access_time = cc.access_time;
        L.share = cc.share;
        L.ncaches = (int)std::ceil((double)y.num_cores / cc.share);
        L.nchildren = l == 0 ? 0 : cc.share / y.cache[l - 1].share;
        L.has_bus = cc.share > 1 ? 1 : 0;
        if (l > 0 && cc.share % y.cache[l - 1].share != 0) return pu::set_error(PU_EINVAL, "cache shares must nest");
        if (L.has_bus) {
            if (y.bus_latency < 1) return pu::set_error(PU_EINVAL, "bus_latency must be >= 1 for shared levels");
            L.bus_q0 = nbus;   // fixed up below (after the link count is known)
            nbus += L.ncaches;
        }
    }
    if (y.cache[0].share != 1)
        return pu::set_error(PU_ENOTSUP, "L1 share must be 1 (System::access passes cache[0][core_id], system.cpp:161)");
    const int N = g->lv[y.num_levels - 1].ncaches;
    g->N = N;
    const pu_cache_cfg& dc = y.directory_cache;
    if (dc.size == 0) return pu::set_error(PU_EINVAL, "a directory is required (system.cpp:1052)");
    if (dc.num_ways < 1 || dc.block_size < 1) return pu::set_error(PU_EINVAL, "bad directory geometry");
    if (dc.num_ways > PU_MAX_WAYS_WIDE) return pu::set_error(PU_ENOTSUP, "at most 4096 directory ways");
    DirGeo& D = g->dir;
    D.nsets = dc.size / (dc.block_size * dc.num_ways);
    if (D.nsets < 1) return pu::set_error(PU_EINVAL, "directory has no sets");
    D.nways = dc.num_ways;
    D.block = dc.block_size;
    D.offbits = ilog2(dc.block_size);
    D.idxbits = ilog2(D.nsets);
    D.access_time = dc.access_time;
    D.nwords = (N + 63) / 64;
    if (D.nwords > PU_MAX_NWORDS) return pu::set_error(PU_ENOTSUP, "at most 65536 LLC nodes");
    D.sh_wide = N > 4096 ? 1 : 0;         // inline sharer ids: 4 x 12 bits, or 3 x 16 bits
    D.sh_cap = D.sh_wide ? 3 : PU_SH_INLINE;
    if (y.protocol_type == 1 && N != y.num_cores)
        return pu::set_error(PU_EINVAL, "limited-pointer broadcast needs one LLC per core (system.cpp:623)");
    if (!bus_sys && y.network.link_delay < 1) return pu::set_error(PU_EINVAL, "link_delay must be >= 1");
    if (y.network.data_width < 1) return pu::set_error(PU_EINVAL, "data_width must be >= 1");
    if (y.network.router_delay >= (1ull << 31) || y.network.link_delay >= (1ull << 31) ||
        y.network.inject_delay >= (1ull << 31))
        return pu::set_error(PU_ENOTSUP, "router/link/inject delays must be < 2^31 cycles");
    g->home_offbits = ilog2(dc.block_size);
    g->home_mask_bits = (int)std::ceil(std::log2((double)N));
    {
        // Reachable directory sets (DirGeo): with a = addr >> offbits, the raw
        // home is a mod 2^hb (folded to raw mod 2^(hb-1) when >= N) and the set
        // is a mod nsets, so a home only sees sets congruent to it modulo
        // G = gcd(nsets, 2^hb), or 2^(hb-1) when folding can occur.
        int lg = 0;
        const int hb = g->home_mask_bits;
        if (D.offbits == g->home_offbits && hb > 0) {
            int v2 = 0;
            while (v2 < 63 && ((D.nsets >> v2) & 1) == 0) v2++;
            lg = std::min(v2, hb);
            if ((uint64_t)N < (1ull << hb)) lg = std::min(lg, hb - 1);
        }
        D.cset_shift = lg;
        D.csets = D.nsets >> lg;
    }
    g->net_type = y.network.net_type;
    g->net_width = g->net_type == 1 ? (int)std::ceil(std::cbrt((double)N)) : (int)std::ceil(std::sqrt((double)N));
    g->header_flits = y.network.header_flits;
    g->data_width = y.network.data_width;
    g->router_delay = y.network.router_delay;
    g->link_delay = y.network.link_delay;
    g->inject_delay = y.network.inject_delay;
    const int w = g->net_width;
    pu_set_net_magic(w, g->header_flits, g->data_width, (int)g->lv[y.num_levels - 1].block, &g->w_magic,
                     &g->w2_magic, &g->w2, &g->blk_len, &g->plen_blk);
    // the bus system never transmits (mesi_bus has no network), so it keeps no link queues
    g->nlinks = bus_sys ? 0 : (w > 1 ? (w - 1) * w * (g->net_type == 1 ? 3 * w : 2) : 0);
    g->nqueues = g->nlinks + nbus;
    if (y.tlb_enable) {
        const pu_cache_cfg& tc = y.tlb_cache;
        TlbGeo& T = g->tlb;
        if (tc.size == 0 || tc.num_ways < 1 || tc.block_size < 1) return pu::set_error(PU_EINVAL, "tlb_enable needs a TLB");
        if (tc.num_ways > PU_MAX_WAYS_WIDE) return pu::set_error(PU_ENOTSUP, "at most 4096 TLB ways");
        if (y.page_size < 1) return pu::set_error(PU_EINVAL, "page_size must be >= 1");
        T.nsets = tc.size / (tc.block_size * tc.num_ways);
        if (T.nsets < 1) return pu::set_error(PU_EINVAL, "TLB has no sets");
        T.nways = tc.num_ways;
        T.page_size = (uint64_t)y.page_size;
        T.offbits = ilog2((uint64_t)y.page_size);     // Cache::init for TLB_CACHE (cache.cpp:66-69)
        T.idxbits = ilog2(T.nsets);
        T.access_time = tc.access_time;
        T.page_miss_delay = y.page_miss_delay;
        uint64_t cap = 1ull << 22;     // 3.1 M distinct pages (12 GiB at 4 KB) before PU_ERRF_PAGES
        if (const char* e = std::getenv("PRIMEUNCORE_PAGE_ENTRIES")) cap = std::strtoull(e, nullptr, 10);
        uint64_t p2 = 64;
        while (p2 < cap && p2 < (1ull << 32)) p2 <<= 1;
        T.pages_cap = p2;
    }
    for (int l = 0; l < y.num_levels; l++)
        if (g->lv[l].has_bus) g->lv[l].bus_q0 += g->nlinks;
    const pu_dram_cfg& dm = y.dram;   // opt-in bank model (pu_dram_cfg); 0 banks = the reference's Dram
    if (dm.banks < 0 || dm.banks > (1 << 20) || (dm.banks & (dm.banks - 1)) != 0)
        return pu::set_error(PU_EINVAL, "dram banks must be 0 or a power of two <= 2^20");
    if (dm.banks > 0) {
        if (dm.row_bytes < 64 || (dm.row_bytes & (dm.row_bytes - 1)) != 0 || dm.row_bytes > (1ull << 40))
            return pu::set_error(PU_EINVAL, "dram row_bytes must be a power of two in [64, 2^40]");
        if (dm.t_rcd < 0 || dm.t_rp < 0 || dm.t_burst < 0 || dm.t_rcd >= (1 << 24) || dm.t_rp >= (1 << 24) ||
            dm.t_burst >= (1 << 24))
            return pu::set_error(PU_EINVAL, "dram timings must be in [0, 2^24) cycles");
        g->dram_banks = dm.banks;
        g->dram_bank_shift = ilog2((uint64_t)dm.banks);
        g->dram_row_shift = ilog2(dm.row_bytes);
        g->dram_t_rcd = dm.t_rcd;
        g->dram_t_rp = dm.t_rp;
        g->dram_t_burst = dm.t_burst;
    }

    // ---- layout
    for (int l = 0; l < y.num_levels; l++) {
        LevelGeo& L = g->lv[l];
        uint64_t lines = (uint64_t)L.ncaches * L.nsets * L.nways;
        if (lines >= (1ull << 32)) return pu::set_error(PU_ENOTSUP, "at most 2^32 lines per cache level");
        L.off_meta = lay.take(lines * sizeof(LineMeta));
        L.off_ts = lay.take(lines * sizeof(int64_t));
        L.off_alive = lay.take((uint64_t)L.ncaches * 4);
        L.off_cnt = lay.take((uint64_t)L.ncaches * 32);
    }
    // the bus system has no directory lines (its report still prints the
    // directory block, from counters that stay 0)
    uint64_t dlines = bus_sys ? 0 : (uint64_t)N * D.csets * D.nways;
    if (dlines >= (1ull << 32)) return pu::set_error(PU_ENOTSUP, "at most 2^32 directory lines");
    D.off_line = lay.take(dlines * sizeof(DirLine));
    D.off_prog = lay.take(dlines * sizeof(int32_t));
    // sharer sets of more than 4 LLCs live in pool bitmaps: one entry per
    // directory line (a line holds at most one, so the pool cannot run out)
    // unless that exceeds 2 GiB of bitmaps; then as many as fit, and running
    // out stops the replica with PU_ERRF_POOL rather than diverge.
    // PRIMEUNCORE_POOL_ENTRIES overrides (tests)
    uint64_t pool = 0;
    if (!bus_sys) {
        const uint64_t cap = (2ull << 30) / ((uint64_t)D.nwords * 8);
        pool = std::max<uint64_t>(std::min(dlines, cap), 64);
    }
    if (pool_cap && !bus_sys) pool = std::max<uint64_t>(std::min(pool, pool_cap), 64);
    if (const char* e = std::getenv("PRIMEUNCORE_POOL_ENTRIES"); e && !bus_sys) pool = std::strtoull(e, nullptr, 10);
    if (pool > (1ull << 30)) pool = 1ull << 30;
    D.pool_entries = (int32_t)pool;
    D.off_pool = lay.take(pool * (uint64_t)D.nwords * 8);
    D.off_pool_free = lay.take(pool * 4);
    D.off_alive = lay.take((uint64_t)N * 4);
    D.off_cnt = lay.take((uint64_t)N * 32);
    if (y.tlb_enable) {
        TlbGeo& T = g->tlb;
        const uint64_t tl = (uint64_t)y.num_cores * T.nsets * T.nways;
        if (tl >= (1ull << 32)) return pu::set_error(PU_ENOTSUP, "at most 2^32 TLB entries");
        T.off_meta = lay.take(tl * sizeof(LineMeta));
        T.off_ts = lay.take(tl * sizeof(int64_t));
        T.off_ppage = lay.take(tl * sizeof(uint64_t));
        T.off_cnt = lay.take((uint64_t)y.num_cores * 32);
        T.off_pages = lay.take(T.pages_cap * sizeof(PageEnt));
    }
    g->off_qhdr = lay.take((uint64_t)g->nqueues * PU_HDR_BYTES);
    g->off_qring = lay.take((uint64_t)g->nqueues * PU_QRING * sizeof(QueueSlot));
    g->off_stats = lay.take(sizeof(EngineStats));
    g->off_completion = lay.take((uint64_t)y.num_cores * 8);
    g->off_run = lay.take(sizeof(RunState));
    g->off_core_shift = lay.take((uint64_t)y.num_cores * 8);
    g->off_dram = lay.take((uint64_t)g->dram_banks * sizeof(DramBank));
    g->replica_bytes = align_up(lay.cur, 4096);
    return 0;
}

}  // namespace

struct pu_handle {
    pu_sim_cfg cfg;
    Geo geo;
    Geo* d_geo = nullptr;
    char* arena = nullptr;
    int R = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0.0;
    struct timespec sim_start{}, sim_finish{};   // UncoreManager::sim_start_time / sim_finish_time
    uint32_t replay_flags = 0;   // PU_KF_CLOSED under PU_REPLAY_CLOSED
    uint32_t dev_req_flags = 0;  // PU_KF_REQ16 under PU_REQ_FMT_16 (the device-run entry points)
    int cus = 0;                 // compute units of the device (latency-mode launches)
    bool lds_headers_ok = false; // the replica's queue headers fit one CU's LDS
    bool lds_headers_short = false;   // latency mode for short host batches too
    pu::JitKernels jit;          // the engine compiled for this configuration (jit.cpp), if available
    bool jit_throughput = false; // throughput launches (headers in HBM) also run the compiled configuration
                                 // (the default; PRIMEUNCORE_JIT_THROUGHPUT=0 keeps them ahead-of-time)
    // ThreadSched (thread_sched.cpp): the shared one, and per-replica copies
    // made on first use of a per-replica call (pu_*_core_replica: the server's
    // sessions); the shared calls update both
    pu::Sched sched;
    std::vector<std::unique_ptr<pu::Sched>> rsched;
    pu::Sched& sched_of(int r) { return rsched[(size_t)r] ? *rsched[(size_t)r] : sched; }
    // staging for host-buffer batches: one device block [offsets | requests]
    // filled by one copy from a pinned host twin, and pinned landing slots for
    // the delays and the replica's error flags
    pu_req* d_reqs = nullptr;
    int32_t* d_delays = nullptr;
    uint64_t* d_off = nullptr;
    uint8_t* h_in = nullptr;     // pinned: [offsets (64 B) | reqs[cap]]
    int32_t* h_delays = nullptr; // pinned: delays[cap]
    uint64_t* h_tail = nullptr;  // pinned: error flags, RunState
    size_t stage_cap = 0;
    // Resident mode (engine.hip resident_body; geometry.h PuMailbox): one
    // latency-mode workgroup serving pu_access / short host batches of one
    // replica through a mailbox in host-coherent pinned memory
    struct Resident {
        int mode = 1;               // PRIMEUNCORE_RESIDENT (0 off) / pu_set_resident
        bool running = false;       // a resident kernel was launched and not yet joined
        int replica = -1;
        uint64_t seq = 0;           // commands posted
        uint64_t acked = 0;         // commands completed
        PuMailbox* mb = nullptr;    // host address
        void* mb_dev = nullptr;     // the same memory, as the device sees it
        pu_req* stage = nullptr;    // device staging of a command's requests
        hipStream_t stream = nullptr;
        hipEvent_t after = nullptr; // orders the kernel after the handle's stream
        uint64_t idle_ticks = 5000000;   // 50 ms of s_memrealtime (100 MHz)
        uint64_t commands = 0, launches = 0;
        uint64_t phase_ticks[4] = {0, 0, 0, 0};   // summed kernel-side phases (PuResDev.phase, full answers)
        uint64_t err = 0;                         // the replica's error flags as of the last full answer
        uint64_t fast = 0;                        // commands answered by the fast word
        uint64_t call_ns = 0;                     // summed host-side post-to-ack time
    } res;
    std::mutex mu;
};

#define HIP_TRY(expr, code)                                                                   \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) return pu::set_error(code, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

namespace {

// the widest set of the configuration (cache levels, directory slices, TLBs)
uint64_t max_ways(const Geo& g) {
    uint64_t w = g.sys_type == 0 ? g.dir.nways : 0;
    for (int l = 0; l < g.num_levels; l++) w = g.lv[l].nways > w ? g.lv[l].nways : w;
    if (g.tlb_enable) w = g.tlb.nways > w ? g.tlb.nways : w;
    return w;
}

int reset_state(pu_handle* h) {
    HIP_TRY(hipMemsetAsync(h->arena, 0, h->geo.replica_bytes * (size_t)h->R, h->stream), PU_EIO);
    // completion cycles start at -1 ("no request yet")
    HIP_TRY(hipMemset2DAsync(h->arena + h->geo.off_completion, h->geo.replica_bytes, 0xFF,
                             (size_t)h->geo.num_cores * 8, (size_t)h->R, h->stream), PU_EIO);
    int rc = pu_engine_init_queues(h->arena, h->geo.replica_bytes, h->geo.off_qhdr, h->geo.off_qring,
                                   h->geo.nqueues, h->R, 0, h->stream);
    if (rc) return pu::set_error(rc, "queue init launch failed");
    rc = pu_engine_init_pool(h->arena, h->geo.replica_bytes, h->geo.dir.off_pool_free, h->geo.off_run,
                             h->geo.dir.pool_entries, h->R, h->stream);
    if (rc) return pu::set_error(rc, "pool init launch failed");
    HIP_TRY(hipStreamSynchronize(h->stream), PU_EIO);
    return 0;
}

constexpr size_t kOffBytes = 64;   // offsets, padded so the requests start on a cache line
constexpr size_t kTailBytes = 8 + sizeof(RunState);
constexpr size_t kShortBatch = 16384;   // host batches below this skip the LDS header image

int resident_stop(pu_handle* h);
void resident_free(pu_handle* h);

void free_stage(pu_handle* h) {
    if (h->d_off) (void)hipFree(h->d_off);   // d_reqs lives in the same block
    if (h->d_delays) (void)hipFree(h->d_delays);
    if (h->h_in) (void)hipHostFree(h->h_in);
    if (h->h_delays) (void)hipHostFree(h->h_delays);
    if (h->h_tail) (void)hipHostFree(h->h_tail);
    h->d_off = nullptr;
    h->d_reqs = nullptr;
    h->d_delays = nullptr;
    h->h_in = nullptr;
    h->h_delays = nullptr;
    h->h_tail = nullptr;
    h->stage_cap = 0;
}

int ensure_stage(pu_handle* h, size_t n) {
    if (n <= h->stage_cap && h->d_off) return 0;
    size_t cap = n < 4096 ? 4096 : n;
    int rc = resident_stop(h);   // hipFree may wait for the whole device
    if (rc) return rc;
    free_stage(h);
    const size_t in_bytes = kOffBytes + cap * sizeof(pu_req);
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, in_bytes), PU_ENOMEM);
    h->d_off = (uint64_t*)p;
    h->d_reqs = (pu_req*)((uint8_t*)p + kOffBytes);
    HIP_TRY(hipMalloc(&h->d_delays, cap * sizeof(int32_t)), PU_ENOMEM);
    HIP_TRY(hipHostMalloc((void**)&h->h_in, in_bytes, hipHostMallocDefault), PU_ENOMEM);
    HIP_TRY(hipHostMalloc((void**)&h->h_delays, cap * sizeof(int32_t), hipHostMallocDefault), PU_ENOMEM);
    HIP_TRY(hipHostMalloc((void**)&h->h_tail, kTailBytes, hipHostMallocDefault), PU_ENOMEM);
    h->stage_cap = cap;
    return 0;
}

// Wait for a short synchronous launch by polling: a blocking wait lets the
// host thread sleep and it wakes well after the kernel ends (the
// per-request API pays that on every call). Long launches fall back to the
// blocking wait after a few milliseconds of polling.
int wait_stream(hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return 0;
        if (e != hipErrorNotReady) return pu::set_error(PU_EIO, std::string("hipStreamQuery: ") + hipGetErrorString(e));
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    }
    HIP_TRY(hipStreamSynchronize(s), PU_EIO);
    return 0;
}

// ---- resident mode (the caller holds h->mu) ----
constexpr size_t kResCap = 16384;   // requests per command (= the short-batch bound)

size_t res_bytes() { return sizeof(PuMailbox) + kResCap * (sizeof(pu_req) + sizeof(int32_t)); }

// Join the resident kernel: a STOP command unless it already left (idle), then
// wait for its stream.  Its headers are back in HBM afterwards.
int resident_stop(pu_handle* h) {
    auto& R = h->res;
    if (!R.running) return 0;
    volatile PuMailbox* mb = R.mb;
    if (!mb->d.exited) {
        mb->h.flags_cmd = PU_RES_STOP << 16;
        mb->h.n = 0;
        std::atomic_thread_fence(std::memory_order_release);
        mb->h.seq = ++R.seq;
    }
    R.running = false;
    HIP_TRY(hipStreamSynchronize(R.stream), PU_EIO);
    // (commands answered by the fast word leave d.ack behind: R.acked knows them)
    R.acked = std::max<uint64_t>(R.acked, (uint64_t)mb->d.ack);
    R.seq = R.acked;   // a STOP is never acked; the next kernel starts from the last completed command
    return 0;
}

// Every handle with a resident kernel, joined at process exit through the
// mailbox alone (the kernel leaves by itself within the idle time anyway).
std::mutex g_res_mu;
std::vector<pu_handle*> g_res_handles;
void resident_atexit() {
    std::lock_guard<std::mutex> lk(g_res_mu);
    for (pu_handle* h : g_res_handles) {
        auto& R = h->res;
        if (!R.running || !R.mb) continue;
        volatile PuMailbox* mb = R.mb;
        mb->h.flags_cmd = PU_RES_STOP << 16;
        std::atomic_thread_fence(std::memory_order_release);
        mb->h.seq = ++R.seq;
        const auto t0 = std::chrono::steady_clock::now();
        while (!mb->d.exited && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) {}
    }
}

bool resident_eligible(const pu_handle* h, size_t n) {
    return h->res.mode && h->jit.ok && h->jit.f[3][1] && h->lds_headers_ok && n <= kResCap;
}

// A resident kernel for `replica` is running (started or restarted here).
int resident_ensure(pu_handle* h, int replica) {
    auto& R = h->res;
    if (R.running && R.replica == replica && !((volatile PuMailbox*)R.mb)->d.exited) return 0;
    int rc = resident_stop(h);
    if (rc) return rc;
    if (!R.mb) {
        void* p = nullptr;
        HIP_TRY(hipHostMalloc(&p, res_bytes(), hipHostMallocCoherent | hipHostMallocMapped), PU_ENOMEM);
        std::memset(p, 0, res_bytes());
        R.mb = (PuMailbox*)p;
        HIP_TRY(hipHostGetDevicePointer(&R.mb_dev, p, 0), PU_EIO);
        HIP_TRY(hipMalloc(&R.stage, kResCap * sizeof(pu_req)), PU_ENOMEM);
        HIP_TRY(hipStreamCreateWithFlags(&R.stream, hipStreamNonBlocking), PU_EIO);
        HIP_TRY(hipEventCreateWithFlags(&R.after, hipEventDisableTiming), PU_EIO);
        std::lock_guard<std::mutex> lk(g_res_mu);
        if (g_res_handles.empty()) std::atexit(resident_atexit);
        g_res_handles.push_back(h);
    }
    {   // the error flags this kernel starts from (fast answers do not carry them; full answers do)
        uint64_t e0 = 0;
        HIP_TRY(hipMemcpyAsync(&e0, h->arena + (size_t)replica * h->geo.replica_bytes + h->geo.off_stats +
                                        offsetof(EngineStats, error_flags), 8, hipMemcpyDeviceToHost, h->stream),
                PU_EIO);
        HIP_TRY(hipStreamSynchronize(h->stream), PU_EIO);
        R.err = e0;
    }
    volatile PuMailbox* mb = R.mb;
    mb->d.exited = 0;
    mb->d.ack = R.acked;   // the kernel waits for seq != ack: a posted, unacked command runs first
    mb->h.seq = R.seq;
    std::atomic_thread_fence(std::memory_order_release);
    // after everything already queued on the handle's stream (the header image it copies in)
    HIP_TRY(hipEventRecord(R.after, h->stream), PU_EIO);
    HIP_TRY(hipStreamWaitEvent(R.stream, R.after, 0), PU_EIO);
    if (pu::jit_launch_resident(h->jit, R.stream, h->d_geo, h->arena, replica, R.stage, R.mb_dev, R.idle_ticks,
                                (int)kResCap) != 0)
        return pu::set_error(PU_EIO, "resident kernel launch failed");
    R.running = true;
    R.replica = replica;
    R.launches++;
    return 0;
}

// One command: the requests through the resident kernel; delays, error flags
// and (TLB) the last translated address come back through the mailbox.
int resident_run(pu_handle* h, int replica, const pu_req* reqs, size_t n, uint32_t flags, int32_t* delay_out,
                 uint64_t* err_out, uint64_t* last_addr) {
    auto& R = h->res;
    int rc = resident_ensure(h, replica);
    if (rc) return rc;
    volatile PuMailbox* mb = R.mb;
    const auto t0 = std::chrono::steady_clock::now();
    static_assert(sizeof(pu_req) == sizeof(PuResHost::req0), "a request fits the command line");
    if (n == 1) std::memcpy((void*)mb->h.req0, reqs, sizeof(pu_req));   // travels with the command
    else std::memcpy(R.mb + 1, reqs, n * sizeof(pu_req));
    mb->h.n = (uint32_t)n;
    mb->h.flags_cmd = (flags & 0xFFFFu) | (PU_RES_RUN << 16);
    std::atomic_thread_fence(std::memory_order_release);
    const uint64_t seq = ++R.seq;
    mb->h.seq = seq;
    // a one-request command may come back as the fast word {seq, delay}
    bool fast = false;
    for (uint64_t spin = 1;; spin++) {
        if (n == 1) {
            const uint64_t f = mb->d.fast;
            if ((uint32_t)f == (uint32_t)seq) {
                fast = true;
                if (delay_out) delay_out[0] = (int32_t)(uint32_t)(f >> 32);
                break;
            }
        }
        if (mb->d.ack == seq) break;
        if ((spin & 1023) == 0) {
            if (mb->d.exited && mb->d.ack != seq) {
                // it left (idle) just before the command arrived: a new kernel takes it
                R.running = false;
                HIP_TRY(hipStreamSynchronize(R.stream), PU_EIO);
                R.acked = std::max<uint64_t>(R.acked, (uint64_t)mb->d.ack);
                rc = resident_ensure(h, replica);
                if (rc) return rc;
                continue;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
                R.mode = 0;   // never again on this handle
                return pu::set_error(PU_EIO, "resident kernel did not answer within 60 s");
            }
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    R.acked = seq;
    R.commands++;
    if (fast) {
        R.fast++;
        *err_out = R.err;      // no new error bit (else the kernel answers in full)
    } else {
        for (int k = 0; k < 4; k++) R.phase_ticks[k] += mb->d.phase[k];
        if (delay_out)
            std::memcpy(delay_out, (const int32_t*)((const pu_req*)(R.mb + 1) + kResCap), n * sizeof(int32_t));
        R.err = mb->d.err;
        *err_out = R.err;
        if (last_addr) *last_addr = mb->d.last_addr;
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    h->last_ms = ms;
    R.call_ns += (uint64_t)(ms * 1e6);
    return 0;
}

void resident_free(pu_handle* h) {
    auto& R = h->res;
    (void)resident_stop(h);
    {
        std::lock_guard<std::mutex> lk(g_res_mu);
        for (size_t i = 0; i < g_res_handles.size(); i++)
            if (g_res_handles[i] == h) {
                g_res_handles.erase(g_res_handles.begin() + (long)i);
                break;
            }
    }
    if (R.stage) (void)hipFree(R.stage);
    if (R.mb) (void)hipHostFree(R.mb);
    if (R.after) (void)hipEventDestroy(R.after);
    if (R.stream) (void)hipStreamDestroy(R.stream);
    R.stage = nullptr;
    R.mb = nullptr;
    R.after = nullptr;
    R.stream = nullptr;
}

int launch(pu_handle* h, int replica0, int nblocks, const pu_req* d_reqs, const uint64_t* d_off, int32_t* d_delay,
           hipStream_t s, uint64_t* d_pos = nullptr, uint64_t budget_ticks = 0, uint32_t extra_flags = 0,
           bool short_launch = false, bool use_replay_mode = true, uint32_t* d_sched = nullptr) {
    int rrc = resident_stop(h);   // a launch reads the queue headers from HBM
    if (rrc) return rrc;
    HIP_TRY(hipEventRecord(h->ev0, s), PU_EIO);
    // latency mode: with at most one replica per CU each wave keeps its queue
    // headers in the CU's LDS for the launch (engine.hip, LH). Copying the
    // image in and out costs ~17 us a launch, more than a short host batch
    // (a lone uncore_access, one MEM_REQUESTS message) wins back, so those
    // run with the headers in HBM (tools/latency_bench.py)
    // (a replica-pool launch is always a throughput launch)
    // (16-B request records: throughput kernels only, the latency helper reads pu_req)
    const int lh = h->lds_headers_ok && nblocks <= h->cus && !short_launch && !d_sched &&
                   !(extra_flags & PU_KF_REQ16) ? 1 : 0;
    const uint32_t flags = (extra_flags & PU_KF_NOHALT) || !use_replay_mode ? extra_flags
                                                                          : (h->replay_flags | extra_flags);
    // latency launches run the compiled configuration (one simulation alone +23%
    // over the ahead-of-time kernel, profiles/r3i_ab_jit_single.txt); throughput
    // launches too (+4.6% at C4 with the replica-layout offsets kept opaque,
    // profiles/r3o_ab_opq.txt) unless PRIMEUNCORE_JIT_THROUGHPUT=0
    const bool use_jit = h->jit.ok && (lh != 0 || h->jit_throughput);
    int rc = use_jit ? pu::jit_launch(h->jit, d_pos != nullptr, lh != 0, nblocks, s, h->d_geo, h->arena, replica0,
                                        d_reqs, d_off, d_delay, d_pos, budget_ticks, flags, d_sched, h->R)
                       : pu_engine_launch(h->d_geo, h->geo.num_levels, h->arena, replica0, nblocks, d_reqs, d_off,
                                          d_delay, d_pos, budget_ticks, flags, lh, d_sched, h->R, s);
    if (rc) return pu::set_error(rc, "engine launch failed");
    HIP_TRY(hipEventRecord(h->ev1, s), PU_EIO);
    return 0;
}

// Gathers EngineStats.error_flags of replicas [0, n) (one strided copy).
int gather_error_flags(pu_handle* h, uint64_t* out, size_t n) {
    if (n == 0) return 0;
    int rrc = resident_stop(h);
    if (rrc) return rrc;
    const Geo& g = h->geo;
    HIP_TRY(hipStreamSynchronize(h->stream), PU_EIO);
    HIP_TRY(hipMemcpy2D(out, sizeof(uint64_t), h->arena + g.off_stats + offsetof(EngineStats, error_flags),
                        g.replica_bytes, sizeof(uint64_t), n, hipMemcpyDeviceToHost), PU_EIO);
    return 0;
}

// PU_ESTATE with a message when `flags` holds an engine-limit or undefined-
// state bit (everything but the reference's own negative-delay stop).
int limit_error(uint64_t flags, int replica) {
    const uint64_t bad = flags & PU_ERRF_LIMITS;
    if (!bad) return 0;
    std::string m = "replica " + std::to_string(replica) + " stopped:";
    if (bad & PU_ERRF_POOL) m += " sharer-bitmap pool exhausted (PRIMEUNCORE_POOL_ENTRIES);";
    if (bad & PU_ERRF_PAGES) m += " page table full (PRIMEUNCORE_PAGE_ENTRIES);";
    if (bad & PU_ERRF_PROG) m += " prog_id outside the packed directory line's range;";
    if (bad & PU_ERRF_WB_MISS) m += " write-back missed at its home (reference NULL dereference, Q13);";
    if (bad & PU_ERRF_EMPTY_SHARER) m += " owner lookup on an empty sharer set;";
    if (bad & PU_ERRF_QUEUE) m += " queue-model precondition violated;";
    return pu::set_error(PU_ESTATE, m);
}

// Copies replica r's engine-side counters.
int resident_quiesce(pu_handle* h) {   // (unlocked callers) the engine state in HBM is current
    std::lock_guard<std::mutex> lk(h->mu);
    return resident_stop(h);
}

int read_replica(pu_handle* h, int r, EngineStats* es, std::vector<uint64_t> cnt[PU_MAX_LEVELS + 2],
                 std::vector<uint32_t> alive[PU_MAX_LEVELS + 2]) {
    int qrc = resident_quiesce(h);
    if (qrc) return qrc;
    const Geo& g = h->geo;
    char* base = h->arena + (size_t)r * g.replica_bytes;
    HIP_TRY(hipStreamSynchronize(h->stream), PU_EIO);
    HIP_TRY(hipMemcpy(es, base + g.off_stats, sizeof(EngineStats), hipMemcpyDeviceToHost), PU_EIO);
    // [num_levels + 1]: per-core TLB counters (ins, miss, evict, wb)
    cnt[g.num_levels + 1].assign(g.tlb_enable ? (size_t)g.num_cores * 4 : 0, 0);
    if (g.tlb_enable)
        HIP_TRY(hipMemcpy(cnt[g.num_levels + 1].data(), base + g.tlb.off_cnt, (size_t)g.num_cores * 32,
                          hipMemcpyDeviceToHost), PU_EIO);
    for (int l = 0; l <= g.num_levels; l++) {
        bool dir = l == g.num_levels;
        size_t nc = dir ? (size_t)g.N : (size_t)g.lv[l].ncaches;
        cnt[l].resize(nc * 4);
        alive[l].resize(nc);
        uint64_t oc = dir ? g.dir.off_cnt : g.lv[l].off_cnt;
        uint64_t oa = dir ? g.dir.off_alive : g.lv[l].off_alive;
        HIP_TRY(hipMemcpy(cnt[l].data(), base + oc, nc * 32, hipMemcpyDeviceToHost), PU_EIO);
        HIP_TRY(hipMemcpy(alive[l].data(), base + oa, nc * 4, hipMemcpyDeviceToHost), PU_EIO);
    }
    return 0;
}

// The page table of replica r (empty unless tlb_enable).
int read_pages(pu_handle* h, int r, std::vector<PageEnt>* out) {
    const Geo& g = h->geo;
    out->clear();
    if (!g.tlb_enable) return 0;
    out->resize(g.tlb.pages_cap);
    char* base = h->arena + (size_t)r * g.replica_bytes;
    HIP_TRY(hipMemcpy(out->data(), base + g.tlb.off_pages, g.tlb.pages_cap * sizeof(PageEnt), hipMemcpyDeviceToHost),
            PU_EIO);
    return 0;
}

// Cache::report (cache.cpp:430-441)
void cache_report(std::ostream& o, uint64_t size, uint64_t ways, const uint64_t* c) {
    o << "=================================================================\n";
    o << "Simulation results for " << size << " Bytes " << ways << "-way set associative cache model:\n";
    o << "The total # of memory instructions: " << c[0] << std::endl;
    o << "The # of cache-missed instructions: " << c[1] << std::endl;
    o << "The # of evicted instructions: " << c[2] << std::endl;
    o << "The # of writeback instructions: " << c[3] << std::endl;
    o << "The cache miss rate: " << 100 * (double)c[1] / (double)c[0] << "%" << std::endl;
    o << "=================================================================\n\n";
}

}  // namespace

extern "C" {

const char* pu_last_error(void) { return pu::g_err.c_str(); }
#ifndef PU_SRC_HASH
#define PU_SRC_HASH "unknown"
#endif
// The source hash (tools/src_hash.py over primesim_amd/csrc and include/) the
// library was built from: tests and smoke() compare it with the checkout.
const char* pu_version(void) { return "primeuncore 0.2 (gfx950) src " PU_SRC_HASH; }

int pu_set_replay_mode(pu_handle* h, int mode) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    if (mode != PU_REPLAY_OPEN && mode != PU_REPLAY_CLOSED) return pu::set_error(PU_EINVAL, "unknown replay mode");
    std::lock_guard<std::mutex> lk(h->mu);
    h->replay_flags = mode == PU_REPLAY_CLOSED ? PU_KF_CLOSED : 0u;
    return 0;
}

int pu_error_flags(pu_handle* h, uint64_t* out, size_t n) {
    if (!h || (!out && n)) return pu::set_error(PU_EINVAL, "bad arguments");
    if (n > (size_t)h->R) return pu::set_error(PU_ERANGE, "more replicas than the handle holds");
    std::lock_guard<std::mutex> lk(h->mu);
    return gather_error_flags(h, out, n);
}

int pu_config_jit_warm(const pu_sim_cfg* cfg) {
    if (!cfg) return pu::set_error(PU_EINVAL, "bad arguments");
    Geo geo;
    if (build_geo(cfg, &geo) != 0) return PU_EINVAL;
    return pu::jit_warm(geo, nullptr);
}

int pu_set_resident(pu_handle* h, int mode) {
    if (!h || mode < -1 || mode > 1) return pu::set_error(PU_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    const int prev = h->res.mode;
    if (mode == 0) {
        int rc = resident_stop(h);
        if (rc) return rc;
    }
    if (mode >= 0) h->res.mode = mode;
    return prev;
}

int pu_resident_info(pu_handle* h, uint64_t* out, size_t n) {
    if (!h || (!out && n)) return pu::set_error(PU_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    const auto& R = h->res;
    const bool live = R.running && R.mb && !((volatile PuMailbox*)R.mb)->d.exited;
    const uint64_t v[10] = {live ? 1u : 0u, R.commands, R.launches, resident_eligible(h, 1) ? 1u : 0u,
                            R.phase_ticks[0], R.phase_ticks[1], R.phase_ticks[2], R.phase_ticks[3], R.call_ns,
                            R.fast};
    for (size_t k = 0; k < n && k < 10; k++) out[k] = v[k];
    return (int)(n < 10 ? n : 10);
}

int pu_compiled_config(const pu_handle* h) { return h && h->jit.ok ? (h->jit_throughput ? 2 : 1) : 0; }
int pu_compiled_compiler(const pu_handle* h) {
    if (!h || !h->jit.ok) return 0;
    int off = 0;
    for (int part = 0; part < pu::kJitParts; part++) off += h->jit.cc[part] == pu::kJitOffline;
    return off == pu::kJitParts ? 2 : off == 0 ? 1 : 3;   // 3: the parts came from different compilers
}

const char* pu_jit_source_tag(void) {
    static const std::string tag = pu::jit_source_tag();
    return tag.c_str();
}

int pu_jit_prof_read(unsigned long long* out, int n, int reset) {
    if (n < 0 || (n > 0 && !out)) return pu::set_error(PU_EINVAL, "bad arguments");
    return pu::jit_prof_read(out, n, reset);
}

long pu_config_geo_source(const pu_sim_cfg* cfg, char* buf, size_t cap) {
    if (!cfg) return pu::set_error(PU_EINVAL, "bad arguments");
    Geo geo;
    if (build_geo(cfg, &geo) != 0) return PU_EINVAL;
    const std::string s = pu::geo_cxx(geo);
    if (buf && cap) {
        const size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (long)s.size();
}

int pu_limit_positions(pu_handle* h, uint64_t* out, size_t n) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    return pu::limit_positions(h, out, n);
}

pu_handle* pu_create(const pu_sim_cfg* cfg, int num_replicas, int device) {
    if (!cfg || num_replicas < 1) {
        pu::set_error(PU_EINVAL, "bad arguments");
        return nullptr;
    }
    Geo geo;
    if (build_geo(cfg, &geo) != 0) return nullptr;
    pu::jit_note_gpu();   // this process starts no compiler from here on
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
        pu::set_error(PU_ENODEV, "no HIP device available (the engine has no CPU fallback)");
        return nullptr;
    }
    pu_handle* h = new pu_handle();
    h->cfg = *cfg;
    h->geo = geo;
    h->R = num_replicas;
    h->device = device;
    auto fail = [&](const std::string& m) -> pu_handle* {
        pu::set_error(PU_ENOMEM, m);
        pu_destroy(h);
        return nullptr;
    };
    if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice failed");
    if (hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) h->cus = 0;
    {
        // "0" turns latency mode off, "2" uses it for short host batches too (A/B runs, tests)
        const char* e = std::getenv("PRIMEUNCORE_LDS_HEADERS");
        h->lds_headers_ok = geo.nqueues <= pu_engine_lds_header_queues() && !(e && e[0] == '0');
        h->lds_headers_short = e && e[0] == '2';
        // resident mode for pu_access / short host batches (on unless "0")
        const char* r = std::getenv("PRIMEUNCORE_RESIDENT");
        h->res.mode = r && r[0] == '0' ? 0 : 1;
        const char* idle = std::getenv("PRIMEUNCORE_RESIDENT_IDLE_MS");
        if (idle && std::atof(idle) > 0) h->res.idle_ticks = (uint64_t)(std::atof(idle) * 1e5);
    }
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) return fail("stream create failed");
    if (hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) return fail("event create failed");
    if (hipMalloc(&h->d_geo, sizeof(Geo)) != hipSuccess) return fail("hipMalloc(geo) failed");
    {
        // The exact sharer pool (one bitmap per directory line, up to 2 GiB) is
        // usually a small share of a replica, but a config whose homes see every
        // set can make it dominate.  When the replicas asked for would not fit
        // the device with it, shrink the pool to what fits rather than fail:
        // running out then stops a replica loudly (PU_ERRF_POOL), never silently.
        size_t free_b = 0, total_b = 0;
        const uint64_t pool_b = (uint64_t)geo.dir.pool_entries * ((uint64_t)geo.dir.nwords * 8 + 4);
        if (pool_b && hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
            geo.replica_bytes * (uint64_t)num_replicas > (uint64_t)(free_b * 0.95)) {
            const uint64_t rest = geo.replica_bytes - pool_b;
            const uint64_t per = (uint64_t)(free_b * 0.95) / (uint64_t)num_replicas;
            if (per > rest + 64 * ((uint64_t)geo.dir.nwords * 8 + 4)) {
                const uint64_t entries = (per - rest) / ((uint64_t)geo.dir.nwords * 8 + 4);
                Geo g2;
                if (build_geo(cfg, &g2, entries) == 0 && g2.replica_bytes < geo.replica_bytes) {
                    std::fprintf(stderr,
                                 "[primeuncore] sharer-bitmap pool reduced from %d to %d entries per replica so %d "
                                 "replicas fit the device (%.1f -> %.1f MiB each); exhausting it stops a replica "
                                 "with PU_ERRF_POOL\n",
                                 geo.dir.pool_entries, g2.dir.pool_entries, num_replicas,
                                 geo.replica_bytes / 1048576.0, g2.replica_bytes / 1048576.0);
                    geo = g2;
                    h->geo = geo;
                }
            }
        }
    }
    if (hipMemcpy(h->d_geo, &geo, sizeof(Geo), hipMemcpyHostToDevice) != hipSuccess) return fail("geo upload failed");
    size_t bytes = geo.replica_bytes * (size_t)num_replicas;
    if (hipMalloc(&h->arena, bytes) != hipSuccess) {
        h->arena = nullptr;
        return fail("hipMalloc of " + std::to_string(bytes) + " bytes for the replica arena failed");
    }
    if (pu::jit_load(geo, &h->jit, true) != 0) return fail(pu::g_err);
    if (!h->jit.ok && max_ways(geo) > PU_MAX_WAYS)
        return fail("sets of more than 64 ways run only in the compiled configuration (hipRTC, jit.cpp), which is "
                    "unavailable (PRIMEUNCORE_JIT=0 or the compile failed)");
    if (h->jit.ok) {
        const char* e = std::getenv("PRIMEUNCORE_JIT_THROUGHPUT");
        h->jit_throughput = max_ways(geo) > PU_MAX_WAYS || !(e && *e && std::atoi(e) == 0);
    }
    h->sched.stat.assign((size_t)cfg->sys.num_cores, 0);
    h->rsched.resize((size_t)num_replicas);
    if (reset_state(h) != 0) {
        std::string m = pu::g_err;
        pu_destroy(h);
        pu::set_error(PU_EIO, m);
        return nullptr;
    }
    return h;
}

void pu_destroy(pu_handle* h) {
    if (!h) return;
    resident_free(h);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->arena) (void)hipFree(h->arena);
    if (h->d_geo) (void)hipFree(h->d_geo);
    pu::jit_unload(&h->jit);
    free_stage(h);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int pu_reset(pu_handle* h) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = resident_stop(h);
    if (rc) return rc;
    return reset_state(h);
}

int pu_num_replicas(const pu_handle* h) { return h ? h->R : 0; }
uint64_t pu_replica_bytes(const pu_handle* h) { return h ? h->geo.replica_bytes : 0; }
uint64_t pu_replica_pool_bytes(const pu_handle* h) {
    return h ? (uint64_t)h->geo.dir.pool_entries * ((uint64_t)h->geo.dir.nwords * 8 + 4) : 0;
}

extern "C++" {   // inside the C-ABI block: these helpers keep C++ linkage
namespace pu {
// The device's target name ("gfx950" from "gfx950:sramecc+:xnack-").
std::string device_target(int device) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return "";
    const std::string a = p.gcnArchName;
    return a.substr(0, a.find(':'));
}
// gfx950 hands LDS to workgroups in 1,280-B units out of a CU's 160 KB
// (measured: tools/probe/residency.hip, profiles/r5a_residency.json — one-wave
// workgroups of 6,144 / 7,152 / 8,192 / 16,384 / 32,768 B reside 25 / 21 /
// 18 / 9 / 4 per CU, hipOccupancy says 26 / 22 / 20 / 10 / 5).  A time-sliced
// launch whose grid exceeds the resident waves takes two slices: round 4's
// six-wave kernel (7,152 B: 22 by hipOccupancy, 21 resident) ran at half rate.
// Other targets are not measured: their residency is hipOccupancy's alone.
constexpr int kLdsGranule = 1280;
int lds_limited_per_cu(int lds_bytes, int lds_per_cu, int granule) {
    if (lds_bytes <= 0 || lds_per_cu <= 0 || granule <= 0) return 1 << 30;
    const int unit = (lds_bytes + granule - 1) / granule * granule;
    return lds_per_cu / unit;
}
}  // namespace pu
}  // extern "C++"

int pu_resident_replicas(const pu_handle* h) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    int cus = 0, lds_cu = 0, per_cu = 1 << 30;
    HIP_TRY(hipSetDevice(h->device), PU_ENODEV);
    // a device that reports no per-CU LDS (0, or a per-block figure below one
    // workgroup's) keeps hipOccupancy's count rather than resolving to 0 slots
    if (hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, h->device) != hipSuccess)
        lds_cu = 0;
    const int granule = pu::device_target(h->device) == "gfx950" ? pu::kLdsGranule : 0;
    // both throughput launch kinds (time-sliced, replica pool: separate
    // instantiations, each its own registers and LDS), one wave per replica
    for (int mode = 1; mode <= 2; mode++) {
        int n = 0, lds = 0;
        int rc = h->jit.ok && h->jit_throughput ? pu::jit_occupancy(h->jit, mode, &n, &lds)
                                                : pu_engine_occupancy(h->geo.num_levels, mode, &n, &lds);
        if (rc) return pu::set_error(rc, "occupancy query failed");
        const int by_lds = pu::lds_limited_per_cu(lds, lds_cu, granule);
        if (by_lds > 0) n = std::min(n, by_lds);
        per_cu = std::min(per_cu, n);
    }
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device), PU_EIO);
    return per_cu * cus;
}

int pu_alloc_core(pu_handle* h, int prog_id, int thread_id) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    for (auto& r : h->rsched)
        if (r) r->alloc(prog_id, thread_id);
    return h->sched.alloc(prog_id, thread_id);
}

int pu_get_core_id(pu_handle* h, int prog_id, int thread_id) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    for (auto& r : h->rsched)
        if (r) r->get(prog_id, thread_id);
    return h->sched.get(prog_id, thread_id);   // operator[]: inserts 0 like the reference
}

int pu_dealloc_core(pu_handle* h, int prog_id, int thread_id) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    for (auto& r : h->rsched)
        if (r) r->dealloc(prog_id, thread_id);
    return h->sched.dealloc(prog_id, thread_id);
}

namespace {
pu::Sched* replica_sched(pu_handle* h, int replica) {
    if (replica < 0 || replica >= h->R) return nullptr;
    auto& r = h->rsched[(size_t)replica];
    if (!r) r.reset(new pu::Sched(h->sched));
    return r.get();
}
}  // namespace

int pu_alloc_core_replica(pu_handle* h, int replica, int prog_id, int thread_id) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    pu::Sched* s = replica_sched(h, replica);
    if (!s) return pu::set_error(PU_ERANGE, "replica out of range");
    return s->alloc(prog_id, thread_id);
}

int pu_dealloc_core_replica(pu_handle* h, int replica, int prog_id, int thread_id) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    pu::Sched* s = replica_sched(h, replica);
    if (!s) return pu::set_error(PU_ERANGE, "replica out of range");
    return s->dealloc(prog_id, thread_id);
}

int pu_get_core_id_replica(pu_handle* h, int replica, int prog_id, int thread_id) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    pu::Sched* s = replica_sched(h, replica);
    if (!s) return pu::set_error(PU_ERANGE, "replica out of range");
    return s->get(prog_id, thread_id);
}

namespace {
int access_batch(pu_handle* h, int replica, const pu_req* reqs, size_t n, int32_t* delay_out, uint32_t extra,
                 uint64_t* last_addr = nullptr) {
    if (!h || (!reqs && n)) return pu::set_error(PU_EINVAL, "bad arguments");
    if (replica < 0 || replica >= h->R) return pu::set_error(PU_ERANGE, "replica out of range");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> lk(h->mu);
    if (resident_eligible(h, n)) {
        // no launch: the resident kernel (headers already in its CU's LDS)
        const uint32_t flags = (extra & PU_KF_NOHALT) ? extra : (h->replay_flags | extra);
        uint64_t err = 0;
        int rrc = resident_run(h, replica, reqs, n, flags, delay_out, &err, last_addr);
        if (rrc) return rrc;
        return limit_error(err, replica);
    }
    int rc = ensure_stage(h, n);
    if (rc) return rc;
    // one host-to-device copy of [offsets | requests] from pinned memory
    const uint64_t off[2] = {0, (uint64_t)n};
    std::memcpy(h->h_in, off, kOffBytes);
    std::memcpy(h->h_in + kOffBytes, reqs, n * sizeof(pu_req));
    HIP_TRY(hipMemcpyAsync(h->d_off, h->h_in, kOffBytes + n * sizeof(pu_req), hipMemcpyHostToDevice, h->stream),
            PU_EIO);
    rc = launch(h, replica, 1, h->d_reqs, h->d_off, h->d_delays, h->stream, nullptr, 0, extra,
                n < kShortBatch && !h->lds_headers_short);
    if (rc) return rc;
    if (delay_out)
        HIP_TRY(hipMemcpyAsync(h->h_delays, h->d_delays, n * sizeof(int32_t), hipMemcpyDeviceToHost, h->stream),
                PU_EIO);
    char* rbase = h->arena + (size_t)replica * h->geo.replica_bytes;
    HIP_TRY(hipMemcpyAsync(h->h_tail, rbase + h->geo.off_stats + offsetof(EngineStats, error_flags), 8,
                           hipMemcpyDeviceToHost, h->stream), PU_EIO);
    if (last_addr)
        HIP_TRY(hipMemcpyAsync(h->h_tail + 1, rbase + h->geo.off_run, sizeof(RunState), hipMemcpyDeviceToHost,
                               h->stream), PU_EIO);
    rc = wait_stream(h->stream);
    if (rc) return rc;
    if (delay_out) std::memcpy(delay_out, h->h_delays, n * sizeof(int32_t));
    if (last_addr) {
        RunState rs;
        std::memcpy(&rs, h->h_tail + 1, sizeof(rs));
        *last_addr = rs.last_addr;
    }
    float ms = 0;
    if (hipEventElapsedTime(&ms, h->ev0, h->ev1) == hipSuccess) h->last_ms = ms;
    // an engine limit stopped the replica where the reference would continue:
    // the delays after that request are not the reference's, say so
    return limit_error(h->h_tail[0], replica);
}
}  // namespace

int pu_access_batch(pu_handle* h, int replica, const pu_req* reqs, size_t n, int32_t* delay_out) {
    return access_batch(h, replica, reqs, n, delay_out, 0);
}

int pu_access(pu_handle* h, int core_id, int prog_id, int mem_type, uint64_t* addr, int64_t timer) {
    int32_t d = 0;
    int rc = pu_access_status(h, core_id, prog_id, mem_type, addr, timer, &d);
    return rc ? rc : d;
}

int pu_access_status(pu_handle* h, int core_id, int prog_id, int mem_type, uint64_t* addr, int64_t timer,
                     int32_t* delay_out) {
    if (!h || !addr || !delay_out) return pu::set_error(PU_EINVAL, "bad arguments");
    if (core_id >= h->cfg.sys.num_cores) {              // System::access, system.cpp:147-150
        *delay_out = -1;
        return 0;
    }
    pu_req r;
    std::memset(&r, 0, sizeof(r));
    r.addr = *addr;
    r.timer = timer;
    r.core = core_id;
    r.prog_id = prog_id;
    r.mem_type = (uint8_t)mem_type;
    r.batch_start = 1;   // a lone request: running delay 0, `timer` used as given
    int32_t d = 0;
    // UncoreManager::uncore_access has no prime.cpp halt rule (PU_KF_NOHALT); a
    // closed-loop shift would move the caller's timer, so it is never applied here
    // with the TLB on, InsMem::addr_dmem comes back as the physical address (system.cpp:916)
    int rc = access_batch(h, 0, &r, 1, &d, PU_KF_NOHALT, h->geo.tlb_enable ? addr : nullptr);
    if (rc) return rc;
    *delay_out = d;
    return 0;
}

int pu_run_device(pu_handle* h, const pu_req* d_reqs, const uint64_t* d_off, int32_t* d_delay, void* hip_stream) {
    if (!h || !d_reqs || !d_off || !d_delay) return pu::set_error(PU_EINVAL, "bad arguments");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
    std::lock_guard<std::mutex> lk(h->mu);
    return launch(h, 0, h->R, d_reqs, d_off, d_delay, s, nullptr, 0, h->dev_req_flags);
}

int pu_set_device_req_format(pu_handle* h, int fmt) {
    if (!h || (fmt != PU_REQ_FMT_32 && fmt != PU_REQ_FMT_16)) return pu::set_error(PU_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    h->dev_req_flags = fmt == PU_REQ_FMT_16 ? PU_KF_REQ16 : 0u;
    return 0;
}

int pu_pack_req16(const pu_req* in, size_t n, pu_req16* out) {
    if (n && (!in || !out)) return pu::set_error(PU_EINVAL, "bad arguments");
    for (size_t i = 0; i < n; i++) {
        const pu_req& q = in[i];
        if (q.timer < 0 || q.timer >= (int64_t)1 << 40 || q.core < 0 || q.core >= 1 << 16 || q.prog_id < 0 ||
            q.prog_id >= 64 || q.mem_type > 1 || q.batch_start > 1 || q.tag != 0)
            return pu::set_error(PU_ERANGE, "request " + std::to_string(i) + " does not fit pu_req16");
        out[i].a = q.addr;
        out[i].b = (uint64_t)q.timer | (uint64_t)(uint32_t)q.core << 40 | (uint64_t)(uint32_t)q.prog_id << 56 |
                   (uint64_t)q.mem_type << 62 | (uint64_t)q.batch_start << 63;
    }
    return 0;
}

}  // extern "C"

int pu::limit_positions(pu_handle* h, uint64_t* out, size_t n) {
    if (!h || (!out && n)) return pu::set_error(PU_EINVAL, "bad arguments");
    if (n > (size_t)h->R) return pu::set_error(PU_ERANGE, "more replicas than the handle holds");
    if (n == 0) return 0;
    int rrc = resident_stop(h);
    if (rrc) return rrc;
    const Geo& g = h->geo;
    HIP_TRY(hipStreamSynchronize(h->stream), PU_EIO);
    HIP_TRY(hipMemcpy2D(out, sizeof(uint64_t), h->arena + g.off_run + offsetof(RunState, limit_at), g.replica_bytes,
                        sizeof(uint64_t), n, hipMemcpyDeviceToHost), PU_EIO);
    return 0;
}

int pu::run_device_flags(pu_handle* h, const pu_req* d_reqs, const uint64_t* d_off, int32_t* d_delay,
                         uint32_t extra_flags, bool use_replay_mode) {
    if (!h || !d_reqs || !d_off || !d_delay) return pu::set_error(PU_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(h->mu);
    return launch(h, 0, h->R, d_reqs, d_off, d_delay, h->stream, nullptr, 0, extra_flags, false, use_replay_mode);
}

extern "C" {

int pu_run_device_sliced(pu_handle* h, const pu_req* d_reqs, const uint64_t* d_off, int32_t* d_delay,
                         uint64_t* d_pos, uint64_t budget_us, void* hip_stream) {
    if (!h || !d_reqs || !d_off || !d_delay || !d_pos) return pu::set_error(PU_EINVAL, "bad arguments");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
    std::lock_guard<std::mutex> lk(h->mu);
    return launch(h, 0, h->R, d_reqs, d_off, d_delay, s, d_pos, budget_us * 100,   // s_memrealtime: 100 MHz
                  h->dev_req_flags);
}

int pu_pool_slots(pu_handle* h) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    const int res = pu_resident_replicas(h);
    if (res < 0) return res;
    return res < h->R ? res : h->R;
}

long pu_pool_words(int slots) { return slots < 1 ? pu::set_error(PU_EINVAL, "slots < 1") : (long)PU_POOL_WORDS(slots); }

int pu_run_device_pool(pu_handle* h, const pu_req* d_reqs, const uint64_t* d_off, int32_t* d_delay,
                       uint64_t* d_pos, uint32_t* d_sched, int slots, uint64_t budget_us, void* hip_stream) {
    if (!h || !d_reqs || !d_off || !d_delay || !d_pos || !d_sched || budget_us == 0)
        return pu::set_error(PU_EINVAL, "bad arguments (the pool needs a time slice: budget_us > 0)");
    const int most = pu_pool_slots(h);
    if (most < 0) return most;
    if (slots < 1 || slots > most)
        return pu::set_error(PU_ERANGE, "slots must be 1.." + std::to_string(most) + " (pu_pool_slots)");
    hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
    std::lock_guard<std::mutex> lk(h->mu);
    return launch(h, 0, slots, d_reqs, d_off, d_delay, s, d_pos, budget_us * 100, h->dev_req_flags, false, true,
                  d_sched);
}

int pu_synchronize(pu_handle* h) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    int qrc = resident_quiesce(h);   // a device-wide wait would otherwise last until the resident kernel idles out
    if (qrc) return qrc;
    HIP_TRY(hipDeviceSynchronize(), PU_EIO);
    float ms = 0;
    if (hipEventElapsedTime(&ms, h->ev0, h->ev1) == hipSuccess) h->last_ms = ms;
    return 0;
}

double pu_last_kernel_ms(pu_handle* h) { return h ? h->last_ms : 0.0; }

void pu_sim_start_time(pu_handle* h) {
    if (h) clock_gettime(CLOCK_REALTIME, &h->sim_start);
}
void pu_sim_finish_time(pu_handle* h) {
    if (h) clock_gettime(CLOCK_REALTIME, &h->sim_finish);
}

int pu_core_completion(pu_handle* h, int replica, int64_t* out, size_t n) {
    if (!h || !out) return pu::set_error(PU_EINVAL, "bad arguments");
    if (replica < 0 || replica >= h->R) return pu::set_error(PU_ERANGE, "replica out of range");
    size_t k = n < (size_t)h->geo.num_cores ? n : (size_t)h->geo.num_cores;
    int qrc = resident_quiesce(h);
    if (qrc) return qrc;
    std::vector<int64_t> tmp((size_t)h->geo.num_cores);
    char* base = h->arena + (size_t)replica * h->geo.replica_bytes;
    HIP_TRY(hipStreamSynchronize(h->stream), PU_EIO);
    HIP_TRY(hipMemcpy(tmp.data(), base + h->geo.off_completion, tmp.size() * 8, hipMemcpyDeviceToHost), PU_EIO);
    for (size_t i = 0; i < k; i++) out[i] = tmp[i];
    return 0;
}

int pu_stats_get(pu_handle* h, int replica, pu_stats* out) {
    if (!h || !out) return pu::set_error(PU_EINVAL, "bad arguments");
    if (replica < 0 || replica >= h->R) return pu::set_error(PU_ERANGE, "replica out of range");
    EngineStats es;
    std::vector<uint64_t> cnt[PU_MAX_LEVELS + 2];
    std::vector<uint32_t> alive[PU_MAX_LEVELS + 2];
    int rc = read_replica(h, replica, &es, cnt, alive);
    if (rc) return rc;
    std::memset(out, 0, sizeof(*out));
    out->net_accesses = es.net_accesses;
    out->net_distance = es.net_distance;
    out->net_total_delay = es.net_total_delay;
    out->net_router_delay = es.net_router_delay;
    out->net_link_delay = es.net_link_delay;
    out->net_inject_delay = es.net_inject_delay;
    out->dram_accesses = es.dram_accesses;
    out->total_bus_contention = es.total_bus_contention;
    out->total_num_broadcast = es.total_num_broadcast;
    out->num_levels = h->geo.num_levels;
    for (int l = 0; l <= h->geo.num_levels; l++) {
        const uint64_t* ls = es.lvl_cnt[l == h->geo.num_levels ? PU_CNT_DIR : l];
        pu_level_stats a{ls[0], ls[1], ls[2], ls[3]};
        for (size_t i = 0; i < alive[l].size(); i++) {
            a.ins += cnt[l][i * 4 + 0];
            a.miss += cnt[l][i * 4 + 1];
            a.evict += cnt[l][i * 4 + 2];
            a.wb += cnt[l][i * 4 + 3];
        }
        if (l == h->geo.num_levels) out->directory = a;
        else out->level[l] = a;
    }
    {
        const auto& tc = cnt[h->geo.num_levels + 1];
        const uint64_t* ls = es.lvl_cnt[PU_CNT_TLB];
        pu_level_stats t{ls[0], ls[1], ls[2], ls[3]};
        for (size_t i = 0; i + 3 < tc.size(); i += 4) {
            t.ins += tc[i];
            t.miss += tc[i + 1];
            t.evict += tc[i + 2];
            t.wb += tc[i + 3];
        }
        out->tlb = t;
    }
    out->link_flits = es.link_flits;
    out->mg1_calls = es.mg1_calls;
    out->lockdown_calls = es.lockdown_calls;
    out->bus_accesses = es.bus_accesses;
    out->requests = es.requests;
    out->error_flags = es.error_flags;
    out->dram_row_hits = es.dram_row_hits;
    out->dram_row_empty = es.dram_row_empty;
    out->dram_row_conflicts = es.dram_row_conflicts;
    out->dram_bank_wait = es.dram_bank_wait;
    return 0;
}

// UncoreManager::report (uncore_manager.cpp:87-98) -> ThreadSched::report
// (thread_sched.cpp:105-116) -> System::report (system.cpp:956-1111) with
// Network::report (network.cpp:310-323) and Dram::report (dram.cpp:50-55).
long pu_report(pu_handle* h, int replica, int include_time, char* buf, size_t cap) {
    if (!h) return pu::set_error(PU_EINVAL, "null handle");
    if (replica < 0 || replica >= h->R) return pu::set_error(PU_ERANGE, "replica out of range");
    EngineStats es;
    std::vector<uint64_t> cnt[PU_MAX_LEVELS + 2];
    std::vector<uint32_t> alive[PU_MAX_LEVELS + 2];
    int rc = read_replica(h, replica, &es, cnt, alive);
    if (rc) return rc;
    const Geo& g = h->geo;
    const pu_sys_cfg& y = h->cfg.sys;
    std::ostringstream o;
    o << "*********************************************************\n";
    o << "*                   PriME Simulator                     *\n";
    o << "*********************************************************\n\n";
    if (include_time) {                  // uncore_manager.cpp:92-93
        double sim_time = (double)(h->sim_finish.tv_sec - h->sim_start.tv_sec) +
                          (double)(h->sim_finish.tv_nsec - h->sim_start.tv_nsec) / 1000000000.0;
        o << "Total computation time: " << sim_time << " seconds\n";
    }
    o << std::endl;
    o << "Core Allocation:\n";
    for (const auto& kv : h->sched_of(replica).map)
        o << "(proc ID: " << kv.first.first << " ,thread ID: " << kv.first.second << ") => "
          << "core ID: " << kv.second << std::endl;
    o << std::endl;
    // Network::report
    double avg_delay = (double)es.net_total_delay / es.net_accesses;
    o << "Network Stat:\n";
    o << "# of accesses: " << es.net_accesses << std::endl;
    o << "Total network communication distance: " << es.net_distance << std::endl;
    o << "Total network delay: " << es.net_total_delay << std::endl;
    o << "Total router delay: " << es.net_router_delay << std::endl;
    o << "Total link delay: " << es.net_link_delay << std::endl;
    o << "Total inject delay: " << es.net_inject_delay << std::endl;
    o << "Total contention delay: " << es.net_link_delay - es.net_distance * y.network.link_delay << std::endl;
    o << "Average network delay: " << avg_delay << std::endl << std::endl;
    // Dram::report
    o << "DRAM Statistics:\n";
    o << "Total # of DRAM accesses: " << es.dram_accesses << std::endl;
    if (g.dram_banks > 0) {   // opt-in bank model (pu_dram_cfg): lines the reference never prints
        o << "DRAM banks: " << g.dram_banks << ", row bytes: " << y.dram.row_bytes << std::endl;
        o << "Row buffer hits: " << es.dram_row_hits << std::endl;
        o << "Row buffer misses (bank closed): " << es.dram_row_empty << std::endl;
        o << "Row buffer conflicts: " << es.dram_row_conflicts << std::endl;
        o << "Total bank wait cycles: " << es.dram_bank_wait << std::endl;
    }
    o << std::endl << "Simulation result for cache system: \n\n";
    if (y.verbose_report) {
        o << "Home Occupation:\n";
        const int w = g.net_width;
        if (g.net_type == 1) {
            o << "Allocated home locations in 3D coordinates:" << std::endl;
            for (int i = 0; i < g.N; i++)
                if (alive[g.num_levels][(size_t)i])
                    o << "(" << (i % (w * w)) % w << ", " << (i % (w * w)) / w << ", " << i / (w * w) << ")\n";
        } else {
            o << "Allocated home locations in 2D coordinates:" << std::endl;
            for (int i = 0; i < g.N; i++)
                if (alive[g.num_levels][(size_t)i]) o << "(" << i % w << ", " << i / w << ")\n";
        }
        o << std::endl;
    }
    o << std::endl;
    if (g.tlb_enable) {
        // system.cpp:990-1014 ("replaced" is never accumulated, Q16)
        const auto& tc = cnt[g.num_levels + 1];
        uint64_t ins = es.lvl_cnt[PU_CNT_TLB][0], miss = es.lvl_cnt[PU_CNT_TLB][1];
        for (size_t i = 0; i + 3 < tc.size(); i += 4) {
            ins += tc[i];
            miss += tc[i + 1];
        }
        double miss_rate = (double)miss / (double)ins;
        o << "TLB Cache" << "===========================================================\n";
        o << "Simulation results for " << y.tlb_cache.size << " Bytes " << y.tlb_cache.num_ways
          << "-way set associative cache model:\n";
        o << "The total # of TLB access instructions: " << ins << std::endl;
        o << "The # of cache-missed instructions: " << miss << std::endl;
        o << "The # of replaced instructions: " << 0 << std::endl;
        o << "The cache miss rate: " << 100 * miss_rate << "%" << std::endl;
        o << "=================================================================\n\n";
        if (y.verbose_report) {
            // PageTable::report (page_table.cpp:79-87): std::map order of (prog, vpage)
            std::vector<PageEnt> tab;
            int prc = read_pages(h, replica, &tab);
            if (prc) return prc;
            std::vector<std::pair<std::pair<int, uint64_t>, uint64_t>> pages;
            for (const PageEnt& e : tab)
                if (e.used) pages.push_back({{e.prog, e.vpage}, e.ppage});
            std::sort(pages.begin(), pages.end());
            o << "Page translation:\n";
            o << "Total # of pages: " << pages.size() << std::endl;
            for (const auto& kv : pages)
                o << std::dec << "(proc ID: " << kv.first.first << " ,vpage Num: " << std::hex << kv.first.second
                  << ") => " << "ppage Num: " << kv.second << std::dec << std::endl;
        }
    }
    o << std::endl;
    o << "Total delay caused by bus contention: " << es.total_bus_contention << " cycles\n";
    o << "Total # of broadcast: " << (int)es.total_num_broadcast << "\n\n";
    for (int i = 0; i < g.num_levels; i++) {
        // per-level sums (compiled configuration, Geo.cnt_sum) + per-cache
        // counters of caches that exist (a counted cache always does)
        uint64_t ins = es.lvl_cnt[i][0], miss = es.lvl_cnt[i][1], evict = es.lvl_cnt[i][2], wb = es.lvl_cnt[i][3];
        for (size_t j = 0; j < alive[i].size(); j++) {
            if (!alive[i][j]) continue;
            ins += cnt[i][j * 4 + 0];
            miss += cnt[i][j * 4 + 1];
            evict += cnt[i][j * 4 + 2];
            wb += cnt[i][j * 4 + 3];
        }
        double miss_rate = (double)miss / (double)ins;
        o << "LEVEL" << i << "===========================================================\n";
        o << "Simulation results for " << y.cache[i].size << " Bytes " << y.cache[i].num_ways
          << "-way set associative cache model:\n";
        o << "The total # of memory instructions: " << ins << std::endl;
        o << "The # of cache-missed instructions: " << miss << std::endl;
        o << "The # of evicted instructions: " << evict << std::endl;
        o << "The # of writeback instructions: " << wb << std::endl;
        o << "The cache miss rate: " << 100 * miss_rate << "%" << std::endl;
        o << "=================================================================\n\n";
    }
    {
        const auto& dc = cnt[g.num_levels];
        const auto& da = alive[g.num_levels];
        uint64_t ins = es.lvl_cnt[PU_CNT_DIR][0], miss = es.lvl_cnt[PU_CNT_DIR][1], evict = es.lvl_cnt[PU_CNT_DIR][2];
        for (size_t j = 0; j < da.size(); j++) {
            if (!da[j]) continue;
            ins += dc[j * 4 + 0];
            miss += dc[j * 4 + 1];
            evict += dc[j * 4 + 2];
        }
        double miss_rate = (double)miss / (double)ins;
        o << "Directory Cache" << "===========================================================\n";
        o << "Simulation results for " << y.directory_cache.size << " Bytes " << y.directory_cache.num_ways
          << "-way set associative cache model:\n";
        o << "The total # of memory instructions: " << ins << std::endl;
        o << "The # of cache-missed instructions: " << miss << std::endl;
        o << "The # of replaced instructions: " << evict << std::endl;
        o << "The cache miss rate: " << 100 * miss_rate << "%" << std::endl;
        o << "=================================================================\n\n";
    }
    if (y.verbose_report) {
        o << "Statistics for each cache with non-zero accesses: \n\n";
        for (int i = 0; i < g.num_levels; i++) {
            o << "LEVEL" << i << "*****************************************************\n\n";
            for (size_t j = 0; j < alive[i].size(); j++) {
                if (alive[i][j] && cnt[i][j * 4] > 0) {
                    o << "The " << j << "th cache:\n";
                    cache_report(o, y.cache[i].size, y.cache[i].num_ways, &cnt[i][j * 4]);
                }
            }
            o << "************************************************************\n\n";
        }
        o << "****************************************************" << std::endl;
        o << "Statistics for each directory caches with non-zero accesses" << std::endl;
        const auto& dc = cnt[g.num_levels];
        const auto& da = alive[g.num_levels];
        for (size_t j = 0; j < da.size(); j++) {
            if (da[j] && dc[j * 4] > 0) {
                o << "Report for directory cache " << j << std::endl;
                cache_report(o, y.directory_cache.size, y.directory_cache.num_ways, &dc[j * 4]);
            }
        }
        if (g.tlb_enable) {
            o << "****************************************************" << std::endl;
            o << "Statistics for each TLB cache with non-zero accesses" << std::endl;
            const auto& tc = cnt[g.num_levels + 1];
            for (int j = 0; j < g.num_cores; j++) {
                if (tc[(size_t)j * 4] > 0) {
                    o << "Report for tlb cache " << j << std::endl;
                    cache_report(o, y.tlb_cache.size, y.tlb_cache.num_ways, &tc[(size_t)j * 4]);
                }
            }
        }
    }
    std::string s = o.str();
    if (buf && cap) {
        size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (long)s.size();
}

}  // extern "C"

// ---------------------------------------------------------------- unit hooks
namespace {

// RAII bag of device buffers for the unit hooks.
struct DevBufs {
    std::vector<void*> ptrs;
    ~DevBufs() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <class T>
    T* up(const T* host, size_t n) {
        void* d = nullptr;
        if (hipMalloc(&d, n * sizeof(T) + 8) != hipSuccess) return nullptr;
        ptrs.push_back(d);
        if (host && n && hipMemcpy(d, host, n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return (T*)d;
    }
};

int unit_prepare(int device) {
    pu::jit_note_gpu();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev)
        return pu::set_error(PU_ENODEV, "no HIP device available");
    HIP_TRY(hipSetDevice(device), PU_ENODEV);
    return 0;
}

}  // namespace

extern "C" {

int pu_unit_queue_run(uint64_t min_proc, const uint64_t* t, const uint64_t* p, size_t n, uint64_t* delay_out,
                      uint64_t* mg1_calls, int device) {
    if ((!t || !p || !delay_out) && n) return pu::set_error(PU_EINVAL, "bad arguments");
    int rc = unit_prepare(device);
    if (rc) return rc;
    Geo g;
    std::memset(&g, 0, sizeof(g));
    g.off_qhdr = 0;
    g.off_qring = 256;
    g.nqueues = 1;
    g.replica_bytes = 256 + PU_QRING * sizeof(QueueSlot);
    DevBufs b;
    Geo* dg = b.up(&g, 1);
    char* base = b.up<char>(nullptr, g.replica_bytes);
    uint64_t* dt = b.up(t, n);
    uint64_t* dp = b.up(p, n);
    uint64_t* dout = b.up<uint64_t>(nullptr, n);
    uint64_t* dmg = b.up<uint64_t>(nullptr, 1);
    if (!dg || !base || !dt || !dp || !dout || !dmg) return pu::set_error(PU_ENOMEM, "unit buffers");
    HIP_TRY(hipMemset(base, 0, g.replica_bytes), PU_EIO);
    rc = pu_engine_init_queues(base, g.replica_bytes, g.off_qhdr, g.off_qring, 1, 1, 1, nullptr);   // wide header
    if (rc) return pu::set_error(rc, "queue init failed");
    rc = pu_engine_unit_queue(dg, base, min_proc, dt, dp, n, dout, dmg, nullptr);
    if (rc) return pu::set_error(rc, "unit queue launch failed");
    HIP_TRY(hipDeviceSynchronize(), PU_EIO);
    if (n) HIP_TRY(hipMemcpy(delay_out, dout, n * 8, hipMemcpyDeviceToHost), PU_EIO);
    if (mg1_calls) HIP_TRY(hipMemcpy(mg1_calls, dmg, 8, hipMemcpyDeviceToHost), PU_EIO);
    return 0;
}

int pu_unit_mg1_run(const uint64_t* num_arrivals, const double* sum, const double* sum_sq, const uint64_t* newest,
                    size_t n, uint64_t* wait_out, int device) {
    if ((!num_arrivals || !sum || !sum_sq || !newest || !wait_out) && n) return pu::set_error(PU_EINVAL, "bad arguments");
    for (size_t i = 0; i < n; i++)
        if (num_arrivals[i] >= (1ull << 53))   // the engine holds the count as an exact double
            return pu::set_error(PU_ERANGE, "num_arrivals >= 2^53");
    int rc = unit_prepare(device);
    if (rc) return rc;
    DevBufs b;
    uint64_t* dn = b.up(num_arrivals, n);
    double* ds = b.up(sum, n);
    double* dq = b.up(sum_sq, n);
    uint64_t* dw = b.up(newest, n);
    uint64_t* dout = b.up<uint64_t>(nullptr, n);
    if (n && (!dn || !ds || !dq || !dw || !dout)) return pu::set_error(PU_ENOMEM, "unit buffers");
    rc = pu_engine_unit_mg1(dn, ds, dq, dw, n, dout, nullptr);
    if (rc) return pu::set_error(rc, "unit M/G/1 launch failed");
    HIP_TRY(hipDeviceSynchronize(), PU_EIO);
    if (n) HIP_TRY(hipMemcpy(wait_out, dout, n * 8, hipMemcpyDeviceToHost), PU_EIO);
    return 0;
}

int pu_unit_network_run(int num_nodes, int net_type, int data_width, int header_flits, uint64_t router_delay,
                        uint64_t link_delay, uint64_t inject_delay, const int32_t* src, const int32_t* dst,
                        const int32_t* len, const uint64_t* timer, size_t n, uint64_t* delay_out, pu_stats* st,
                        int device) {
    if ((!src || !dst || !len || !timer || !delay_out) && n) return pu::set_error(PU_EINVAL, "bad arguments");
    if (num_nodes < 1 || data_width < 1 || link_delay < 1) return pu::set_error(PU_EINVAL, "bad network");
    for (size_t i = 0; i < n; i++)
        if (src[i] < 0 || src[i] >= num_nodes || dst[i] < 0 || dst[i] >= num_nodes)
            return pu::set_error(PU_ERANGE, "node id out of range");
    int rc = unit_prepare(device);
    if (rc) return rc;
    Geo g;
    std::memset(&g, 0, sizeof(g));
    g.N = num_nodes;
    g.net_type = net_type;
    g.net_width = net_type == 1 ? (int)std::ceil(std::cbrt((double)num_nodes)) : (int)std::ceil(std::sqrt((double)num_nodes));
    g.header_flits = header_flits;
    g.data_width = data_width;
    g.router_delay = router_delay;
    g.link_delay = link_delay;
    g.inject_delay = inject_delay;
    const int w = g.net_width;
    pu_set_net_magic(w, header_flits, data_width, -1, &g.w_magic, &g.w2_magic, &g.w2, &g.blk_len, &g.plen_blk);
    g.nlinks = w > 1 ? (w - 1) * w * (net_type == 1 ? 3 * w : 2) : 0;
    g.nqueues = g.nlinks;
    Layout lay;
    g.off_qhdr = lay.take((uint64_t)g.nqueues * PU_HDR_WIDE_BYTES);   // the unit hook's wide headers
    g.off_qring = lay.take((uint64_t)g.nqueues * PU_QRING * sizeof(QueueSlot));
    g.off_stats = lay.take(sizeof(EngineStats));
    g.replica_bytes = align_up(lay.cur, 4096);
    DevBufs b;
    Geo* dg = b.up(&g, 1);
    char* base = b.up<char>(nullptr, g.replica_bytes);
    int32_t* ds = b.up(src, n);
    int32_t* dd = b.up(dst, n);
    int32_t* dl = b.up(len, n);
    uint64_t* dt = b.up(timer, n);
    uint64_t* dout = b.up<uint64_t>(nullptr, n);
    if (!dg || !base || !ds || !dd || !dl || !dt || !dout) return pu::set_error(PU_ENOMEM, "unit buffers");
    HIP_TRY(hipMemset(base, 0, g.replica_bytes), PU_EIO);
    rc = pu_engine_init_queues(base, g.replica_bytes, g.off_qhdr, g.off_qring, g.nqueues, 1, 1, nullptr);
    if (rc) return pu::set_error(rc, "queue init failed");
    rc = pu_engine_unit_network(dg, base, ds, dd, dl, dt, n, dout, nullptr);
    if (rc) return pu::set_error(rc, "unit network launch failed");
    HIP_TRY(hipDeviceSynchronize(), PU_EIO);
    if (n) HIP_TRY(hipMemcpy(delay_out, dout, n * 8, hipMemcpyDeviceToHost), PU_EIO);
    if (st) {
        EngineStats es;
        HIP_TRY(hipMemcpy(&es, base + g.off_stats, sizeof(es), hipMemcpyDeviceToHost), PU_EIO);
        std::memset(st, 0, sizeof(*st));
        st->net_accesses = es.net_accesses;
        st->net_distance = es.net_distance;
        st->net_total_delay = es.net_total_delay;
        st->net_router_delay = es.net_router_delay;
        st->net_link_delay = es.net_link_delay;
        st->net_inject_delay = es.net_inject_delay;
        st->link_flits = es.link_flits;
        st->mg1_calls = es.mg1_calls;
        st->error_flags = es.error_flags;
    }
    return 0;
}

}  // extern "C"
