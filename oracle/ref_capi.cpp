// ref_capi.cpp — TEST INFRASTRUCTURE ONLY (oracle/). Never linked into the
// product.  A thin C API over the *reference's own* uncore classes, compiled
// in place from /root/reference/src by oracle/Makefile into
// oracle/_ref/libprime_ref.so.  It replays a request stream exactly as the
// reference's single-threaded msgHandler loop does (reference
// src/prime.cpp:120-137) and produces the golden vectors the parity tests
// pin the CPU restatement (oracle/cpu_ref.cpp) and the HIP engine against.
//
// Extra counters the reference does not print are taken with -Wl,--wrap on
// cross-translation-unit member functions; wrapping leaves
// the reference's results bit-identical (the wrappers only count and forward).

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "system.h"        // reference src/system.h
#include "thread_sched.h"  // reference src/thread_sched.h
#include "xml_parser.h"    // reference src/xml_parser.h
#include "network.h"       // reference src/network.h
#include "queue_model.h"   // reference src/Graphite/queue_model.h
#include "queue_model_m_g_1.h"   // reference src/Graphite/queue_model_m_g_1.h

#include "../include/primeuncore.h"

// ---------------------------------------------------------------- counters
static uint64_t g_link_visits, g_link_flits, g_mg1_calls, g_lockdown_calls,
    g_bus_accesses, g_transmits, g_dram_accesses;

// (oracle/Makefile also links this shim without the wraps, REF_NOWRAP:
// _ref/libprime_ref_nowrap.so, the plain reference timed as bench.py's CPU
// baseline; its extra counters read 0)
#ifndef REF_NOWRAP
extern "C" {
uint64_t __real__ZN4Link6accessEmi(void* self, uint64_t timer, int packet_len);
uint64_t __wrap__ZN4Link6accessEmi(void* self, uint64_t timer, int packet_len) {
    g_link_visits++;
    g_link_flits += (uint64_t)packet_len;
    return __real__ZN4Link6accessEmi(self, timer, packet_len);
}
uint64_t __real__ZN13QueueModelMG117computeQueueDelayEmmi(void* self, uint64_t t, uint64_t s, int r);
uint64_t __wrap__ZN13QueueModelMG117computeQueueDelayEmmi(void* self, uint64_t t, uint64_t s, int r) {
    g_mg1_calls++;
    return __real__ZN13QueueModelMG117computeQueueDelayEmmi(self, t, s, r);
}
void __real__ZN5Cache8lockDownEP6InsMem(void* self, void* ins);
void __wrap__ZN5Cache8lockDownEP6InsMem(void* self, void* ins) {
    g_lockdown_calls++;
    __real__ZN5Cache8lockDownEP6InsMem(self, ins);
}
uint64_t __real__ZN3Bus6accessEm(void* self, uint64_t timer);
uint64_t __wrap__ZN3Bus6accessEm(void* self, uint64_t timer) {
    g_bus_accesses++;
    return __real__ZN3Bus6accessEm(self, timer);
}
uint64_t __real__ZN7Network8transmitEiiim(void* self, int s, int r, int len, uint64_t timer);
uint64_t __wrap__ZN7Network8transmitEiiim(void* self, int s, int r, int len, uint64_t timer) {
    g_transmits++;
    return __real__ZN7Network8transmitEiiim(self, s, r, len, timer);
}
int __real__ZN4Dram6accessEP6InsMem(void* self, void* ins);
int __wrap__ZN4Dram6accessEP6InsMem(void* self, void* ins) {
    g_dram_accesses++;
    return __real__ZN4Dram6accessEP6InsMem(self, ins);
}
}
#endif

static void reset_counters() {
    g_link_visits = g_link_flits = g_mg1_calls = g_lockdown_calls = 0;
    g_bus_accesses = g_transmits = g_dram_accesses = 0;
}

// ---------------------------------------------------------------- instance
struct RefInstance {
    XmlParser parser;
    System sys;
    ThreadSched sched;
    int num_cores = 0;
    int batch_delay = 0;   // prime.cpp's running `delay` of the open message, kept across calls
    bool halted = false;   // prime.cpp:130-134: the handler thread exits on a negative delay
    std::vector<int64_t> completion;
    int mode = 0;                      // 1 closed loop, 2 no halt (as oracle/cpu_ref.h)
    std::vector<int64_t> core_shift;   // closed loop: the core's summed batch delays (core_manager.cpp:265)
    int64_t msg_shift = 0;
    bool skip_msg = false;             // mode 4: the open message went negative, its rest is skipped
    uint64_t dead_tags = 0;            // mode 4: receive threads (pu_req.tag & 63) that returned
};

static std::string slurp(const char* path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

extern "C" {

void* ref_create(const char* xml_path, int* err) {
    RefInstance* r = new RefInstance();
    if (!r->parser.parse(xml_path)) {
        if (err) *err = -1;
        delete r;
        return nullptr;
    }
    XmlSim* sim = r->parser.getXmlSim();
    r->sys.init(&sim->sys);                 // UncoreManager::init, uncore_manager.cpp:46-50
    r->sched.init(r->sys.getCoreCount());
    r->num_cores = r->sys.getCoreCount();
    r->completion.assign((size_t)r->num_cores, -1);
    r->core_shift.assign((size_t)r->num_cores, 0);
    reset_counters();
    if (err) *err = 0;
    return r;
}

// Dump the parsed XmlSim so the product's XML loader can be checked field by
// field against the reference parser.
int ref_get_config(void* h, pu_sim_cfg* out) {
    RefInstance* r = (RefInstance*)h;
    XmlSim* s = r->parser.getXmlSim();
    std::memset(out, 0, sizeof(*out));
    out->max_msg_size = s->max_msg_size;
    out->num_recv_threads = s->num_recv_threads;
    out->thread_sync_interval = s->thread_sync_interval;
    out->proc_sync_interval = s->proc_sync_interval;
    out->syscall_cost = s->syscall_cost;
    pu_sys_cfg& y = out->sys;
    XmlSys& x = s->sys;
    y.sys_type = x.sys_type; y.protocol_type = x.protocol_type;
    y.max_num_sharers = x.max_num_sharers; y.page_size = x.page_size;
    y.tlb_enable = x.tlb_enable; y.shared_llc = x.shared_llc;
    y.verbose_report = x.verbose_report; y.dram_access_time = x.dram_access_time;
    y.cpi_nonmem = x.cpi_nonmem; y.num_levels = x.num_levels; y.num_cores = x.num_cores;
    y.freq = x.freq; y.bus_latency = x.bus_latency; y.page_miss_delay = x.page_miss_delay;
    y.network.data_width = x.network.data_width; y.network.header_flits = x.network.header_flits;
    y.network.net_type = x.network.net_type; y.network.router_delay = x.network.router_delay;
    y.network.link_delay = x.network.link_delay; y.network.inject_delay = x.network.inject_delay;
    auto cc = [](pu_cache_cfg& d, const XmlCache& c) {
        d.level = c.level; d.share = c.share; d.access_time = c.access_time;
        d.size = c.size; d.block_size = c.block_size; d.num_ways = c.num_ways;
    };
    cc(y.directory_cache, x.directory_cache);
    cc(y.tlb_cache, x.tlb_cache);
    for (int i = 0; i < x.num_levels && i < PU_MAX_LEVELS; i++) cc(y.cache[i], x.cache[i]);
    return 0;
}

int ref_alloc_core(void* h, int prog, int thread) {
    return ((RefInstance*)h)->sched.allocCore(prog, thread);
}

int ref_get_core_id(void* h, int prog, int thread) {
    return ((RefInstance*)h)->sched.getCoreId(prog, thread);
}

// The per-message loop of prime.cpp:120-137, one call per request.
// Returns 0, or the index+1 of the first request whose batch delay went
// negative (prime.cpp:130 would kill the handler thread there).
long ref_run(void* h, const pu_req* reqs, size_t n, int32_t* delays) {
    RefInstance* r = (RefInstance*)h;
    const bool closed = (r->mode & 1) != 0, keep_halt = (r->mode & 2) == 0;
    if (r->halted && keep_halt) {
        if (delays) std::fill_n(delays, n, 0);
        return n ? -1 : 0;
    }
    // 4: one receive thread of several (the server): a negative running delay
    // skips the rest of its message and that thread (tag) never receives again;
    // 8: a caller of uncore_access that only abandons the message
    const bool msghalt = (r->mode & 12) != 0, thread_dies = (r->mode & 4) != 0;
    int delay = r->batch_delay;   // prime.cpp:113 `delay` is an int
    InsMem ins;
    std::memset(&ins, 0, sizeof(ins));
    for (size_t i = 0; i < n; i++) {
        const pu_req& q = reqs[i];
        const bool core_ok = q.core >= 0 && q.core < r->num_cores;
        if (q.batch_start) {
            delay = 0;
            // MSGHALT: a receive thread that returned never receives again
            // (prime.cpp:133 returns from msgHandler; its tag = pu_req.tag)
            r->skip_msg = msghalt && ((r->dead_tags >> (q.tag & 63)) & 1);
            if (closed && core_ok) r->msg_shift = r->core_shift[(size_t)q.core];
        }
        if (r->skip_msg) {          // MSGHALT: this message's handler thread has returned
            if (delays) delays[i] = 0;
            continue;
        }
        ins.prog_id = q.prog_id;
        ins.mem_type = (char)q.mem_type;
        ins.addr_dmem = q.addr;
        int64_t t = q.timer + (closed ? r->msg_shift : 0) + delay;
        int d = r->sys.access(q.core, &ins, t);
        if (delays) delays[i] = d;
        delay += d - 1;
        if (core_ok) {
            r->completion[(size_t)q.core] = t + d;
            if (closed) r->core_shift[(size_t)q.core] = r->msg_shift + delay;
        }
        if (delay < 0 && msghalt) {
            if (thread_dies) r->dead_tags |= 1ull << (q.tag & 63);
            r->skip_msg = true;
            continue;
        }
        if (delay < 0 && keep_halt) {
            r->batch_delay = delay;
            r->halted = true;
            if (delays) std::fill(delays + i + 1, delays + n, 0);
            return (long)i + 1;
        }
    }
    r->batch_delay = delay;
    return 0;
}

int ref_set_mode(void* h, int mode) {
    ((RefInstance*)h)->mode = mode;
    return 0;
}

int ref_completion(void* h, int64_t* out, size_t n) {
    RefInstance* r = (RefInstance*)h;
    for (size_t i = 0; i < n && i < r->completion.size(); i++) out[i] = r->completion[i];
    return 0;
}

// UncoreManager::report (uncore_manager.cpp:87-98) minus the wall-clock line.
long ref_report(void* h, const char* tmp_path, char* buf, size_t cap) {
    RefInstance* r = (RefInstance*)h;
    {
        std::ofstream out(tmp_path);
        out << "*********************************************************\n";
        out << "*                   PriME Simulator                     *\n";
        out << "*********************************************************\n\n";
        out << std::endl;
        r->sched.report(&out);
        r->sys.report(&out);
    }
    std::string s = slurp(tmp_path);
    std::remove(tmp_path);
    if (buf && cap) {
        size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (long)s.size();
}

void ref_counters(uint64_t out[7]) {
    out[0] = g_link_visits; out[1] = g_link_flits; out[2] = g_mg1_calls;
    out[3] = g_lockdown_calls; out[4] = g_bus_accesses; out[5] = g_transmits;
    out[6] = g_dram_accesses;
}

void ref_destroy(void* h) { delete (RefInstance*)h; }

// ---- unit goldens: the Graphite history-tree queue model on its own
// (QueueModel::create("history_tree", min_proc), queue_model.cpp:15-35).
int ref_queue_run(uint64_t min_proc, const uint64_t* t, const uint64_t* p, size_t n,
                  uint64_t* delay_out) {
    QueueModel* q = QueueModel::create("history_tree", min_proc);
    uint64_t before = g_mg1_calls;
    for (size_t i = 0; i < n; i++) delay_out[i] = q->computeQueueDelay(t[i], p[i]);
    (void)before;
    delete q;
    return 0;
}

// ---- unit: the reference's QueueModelMG1::computeQueueDelay (queue_model_m_g_1.cpp:16-42)
// on given states.  Its four state members are private (queue_model_m_g_1.h:16-19);
// a layout twin of that standard-layout class sets them on a constructed object.
struct MG1Twin {
    volatile double sigma_sq;   // _sigma_service_time_square
    volatile double sigma;      // _sigma_service_time
    UInt64 n;                   // _num_arrivals
    UInt64 newest;              // _newest_arrival_time
};
static_assert(sizeof(MG1Twin) == sizeof(QueueModelMG1), "QueueModelMG1 layout (queue_model_m_g_1.h:16-19)");

int ref_mg1_batch(const uint64_t* n, const double* sum, const double* sum_sq, const uint64_t* newest, size_t cnt,
                  uint64_t* out) {
    QueueModelMG1 q;
    MG1Twin* t = reinterpret_cast<MG1Twin*>(&q);
    for (size_t i = 0; i < cnt; i++) {
        t->sigma_sq = sum_sq[i];
        t->sigma = sum[i];
        t->n = n[i];
        t->newest = newest[i];
        out[i] = q.computeQueueDelay(0, 1);
    }
    return 0;
}

// ---- unit goldens: Network::transmit sequences (network.cpp:97-160) and the
// Network::report text (network.cpp:310-323).
long ref_network_run(int num_nodes, int net_type, int data_width, int header_flits,
                     uint64_t router_delay, uint64_t link_delay, uint64_t inject_delay,
                     const int32_t* src, const int32_t* dst, const int32_t* len,
                     const uint64_t* timer, size_t n, uint64_t* delay_out,
                     const char* tmp_path, char* buf, size_t cap) {
    XmlNetwork xn;
    xn.net_type = net_type; xn.data_width = data_width; xn.header_flits = header_flits;
    xn.router_delay = router_delay; xn.link_delay = link_delay; xn.inject_delay = inject_delay;
    Network* net = new Network();
    net->init(num_nodes, &xn);
    for (size_t i = 0; i < n; i++) delay_out[i] = net->transmit(src[i], dst[i], len[i], timer[i]);
    {
        std::ofstream out(tmp_path);
        net->report(&out);
    }
    delete net;
    std::string s = slurp(tmp_path);
    std::remove(tmp_path);
    if (buf && cap) {
        size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (long)s.size();
}

}  // extern "C"
