// primeuncore.hpp — header-only C++ mirror of the reference's UncoreManager
// (reference src/uncore_manager.h:51-68) over the C ABI in primeuncore.h.
//
// A maintainer swaps `UncoreManager uncore_manager;` (reference prime.h:63) for
// `pu::UncoreManager uncore_manager;` and keeps the call sites; the per-message
// loop of prime.cpp:120-137 can instead hand the whole message to
// access_message() (one engine launch per message).  See INTEGRATION.md.
#pragma once

#include <cstdint>
#include <cstring>
#include <ostream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "primeuncore.h"

namespace pu {

// prime.cpp:130-134: the message's running delay went negative at `index`;
// the reference's handler thread prints an error and returns without a reply.
struct NegativeDelay : std::runtime_error {
    size_t index;
    int delay;
    NegativeDelay(size_t i, int d)
        : std::runtime_error("negative delay at request " + std::to_string(i) + ": " + std::to_string(d)),
          index(i), delay(d) {}
};

// The fields of the reference InsMem (cache.h:92-99) that System::access reads.
struct InsMem {
    char mem_type;       // 0 read, 1 write
    int prog_id;
    int thread_id;
    int rec_thread_id;
    uint64_t addr_dmem;  // updated in place like System::access (system.cpp:916)
};

class UncoreManager {
   public:
    UncoreManager() = default;
    UncoreManager(const UncoreManager&) = delete;
    UncoreManager& operator=(const UncoreManager&) = delete;
    ~UncoreManager() { pu_destroy(h_); }

    // The reference's config structs (XmlSim / XmlSys / XmlCache / XmlNetwork,
    // reference src/xml_parser.h:43-100) copied field by field into the C ABI's
    // pu_sim_cfg.  A template over the struct, so this header includes no
    // reference header: any type with those member names converts (prime.cpp's
    // XmlSim from XmlParser::getXmlSim, xml_parser.cpp:121).  XmlSys::cache
    // points to num_levels XmlCache entries (xml_parser.cpp:605-681).
    template <class XmlSimT>
    static pu_sim_cfg config_from(const XmlSimT& xs) {
        if (xs.sys.num_levels < 1 || xs.sys.num_levels > PU_MAX_LEVELS)
            throw std::runtime_error("XmlSim: num_levels " + std::to_string(xs.sys.num_levels) +
                                     " outside 1.." + std::to_string(PU_MAX_LEVELS));
        pu_sim_cfg c;
        std::memset(&c, 0, sizeof c);
        c.max_msg_size = xs.max_msg_size;
        c.num_recv_threads = xs.num_recv_threads;
        c.thread_sync_interval = xs.thread_sync_interval;
        c.proc_sync_interval = xs.proc_sync_interval;
        c.syscall_cost = xs.syscall_cost;
        const auto& y = xs.sys;
        pu_sys_cfg& s = c.sys;
        s.sys_type = y.sys_type;
        s.protocol_type = y.protocol_type;
        s.max_num_sharers = y.max_num_sharers;
        s.page_size = y.page_size;
        s.tlb_enable = y.tlb_enable;
        s.shared_llc = y.shared_llc;
        s.verbose_report = y.verbose_report;
        s.dram_access_time = y.dram_access_time;
        s.cpi_nonmem = y.cpi_nonmem;
        s.num_levels = y.num_levels;
        s.num_cores = y.num_cores;
        s.freq = y.freq;
        s.bus_latency = y.bus_latency;
        s.page_miss_delay = y.page_miss_delay;
        s.network.data_width = y.network.data_width;
        s.network.header_flits = y.network.header_flits;
        s.network.net_type = y.network.net_type;
        s.network.router_delay = y.network.router_delay;
        s.network.link_delay = y.network.link_delay;
        s.network.inject_delay = y.network.inject_delay;
        copy_cache(s.directory_cache, y.directory_cache);
        copy_cache(s.tlb_cache, y.tlb_cache);
        for (int l = 0; l < y.num_levels; l++) copy_cache(s.cache[l], y.cache[l]);
        return c;   // s.dram stays 0: the reference's fixed-latency Dram
    }

    // UncoreManager::init(XmlSim*) (uncore_manager.h:54, uncore_manager.cpp:46-50):
    // prime.cpp's `uncore_manager.init(xml_sim);` (prime.cpp:198) compiles
    // unchanged.  Not selected for pu_sim_cfg (the overload below).
    template <class XmlSimT,
              typename std::enable_if<!std::is_same<typename std::remove_cv<XmlSimT>::type, pu_sim_cfg>::value,
                                      int>::type = 0>
    void init(XmlSimT* xml_sim, int replicas = 1, int device = 0) {
        if (!xml_sim) throw std::runtime_error("UncoreManager::init: null XmlSim");
        const pu_sim_cfg c = config_from(*xml_sim);
        init(&c, replicas, device);
    }

    // UncoreManager::init (uncore_manager.cpp:46-50); `replicas` independent uncores.
    void init(const pu_sim_cfg* cfg, int replicas = 1, int device = 0) {
        h_ = pu_create(cfg, replicas, device);
        if (!h_) throw std::runtime_error(std::string("pu_create: ") + pu_last_error());
        num_cores_ = cfg->sys.num_cores;
    }
    // XmlParser::parse (xml_parser.cpp:684) + init.
    void init_from_xml(const char* path, int replicas = 1, int device = 0) {
        pu_sim_cfg cfg;
        if (pu_config_load_xml(path, &cfg) != 0) throw std::runtime_error(pu_last_error());
        init(&cfg, replicas, device);
    }

    // UncoreManager::getSimStartTime / getSimFinishTime (uncore_manager.cpp:52-60).
    void getSimStartTime() { pu_sim_start_time(h_); }
    void getSimFinishTime() { pu_sim_finish_time(h_); }

    int allocCore(int prog_id, int thread_id) { return pu_alloc_core(h_, prog_id, thread_id); }
    int deallocCore(int prog_id, int thread_id) { return pu_dealloc_core(h_, prog_id, thread_id); }
    int getCoreId(int prog_id, int thread_id) { return pu_get_core_id(h_, prog_id, thread_id); }

    // UncoreManager::uncore_access (uncore_manager.cpp:82-85): -1 if core_id >=
    // num_cores; a negative value when the reference's int wraps; throws on an
    // engine error (pu_access_status's out-of-band status).
    // A template over the request struct: the reference's own InsMem (cache.h:92-99)
    // works unchanged at prime.cpp:129, and so does pu::InsMem.
    template <class InsMemT>
    int uncore_access(int core_id, InsMemT* ins, int64_t timer) {
        uint64_t a = ins->addr_dmem;
        int32_t d = 0;
        if (pu_access_status(h_, core_id, ins->prog_id, ins->mem_type, &a, timer, &d) != 0)
            throw std::runtime_error(pu_last_error());   // status out of band: every int delay is a delay
        ins->addr_dmem = a;
        return d;
    }

    // One MEM_REQUESTS message (prime.cpp:120-137): returns the `delay` prime.cpp
    // sends back (sum of (d_i - 1)).  Throws NegativeDelay where prime.cpp's
    // handler would exit (the replica then stops, as that handler does), and
    // runtime_error on engine errors (PU_ESTATE: an engine limit).
    int access_message(int core_id, int prog_id, const bool* mem_type, const uint64_t* addr,
                       const int64_t* timer, size_t n, int replica = 0) {
        static_assert(sizeof(bool) == sizeof(char), "MsgMem bool is one byte");
        reqs_.resize(n);
        delays_.resize(n);
        for (size_t i = 0; i < n; i++) {
            pu_req& r = reqs_[i];
            r = pu_req{};
            r.addr = addr[i];
            r.timer = timer[i];
            r.core = core_id;
            r.prog_id = prog_id;
            r.mem_type = mem_type[i] ? PU_WR : PU_RD;
            r.batch_start = i == 0;
        }
        if (pu_access_batch(h_, replica, reqs_.data(), n, delays_.data()) != 0)
            throw std::runtime_error(pu_last_error());
        int delay = 0;
        for (size_t i = 0; i < n; i++) {
            delay += delays_[i] - 1;
            if (delay < 0) throw NegativeDelay(i, delay);   // later delays were never computed
        }
        return delay;
    }

    // Same, reading the reference's MsgMem wire records (common.h:49-59: bool mem_type;
    // int mem_size; uint64_t addr_dmem; int64_t timer — 24 bytes) directly, e.g.
    // access_msgmem(core_id, MPI_SOURCE, &msg_mem[index_prev][1], msg_len - 1).
    int access_msgmem(int core_id, int prog_id, const void* records, size_t n, int replica = 0) {
        const unsigned char* p = static_cast<const unsigned char*>(records);
        types_.resize(n);
        addrs_.resize(n);
        timers_.resize(n);
        for (size_t i = 0; i < n; i++, p += 24) {
            types_[i] = p[0] != 0;
            std::memcpy(&addrs_[i], p + 8, 8);
            std::memcpy(&timers_[i], p + 16, 8);
        }
        return access_message(core_id, prog_id, reinterpret_cast<const bool*>(types_.data()), addrs_.data(),
                              timers_.data(), n, replica);
    }

    // UncoreManager::report (uncore_manager.cpp:87-98).
    void report(std::ostream* out, int replica = 0) {
        long n = pu_report(h_, replica, 1, nullptr, 0);
        if (n < 0) throw std::runtime_error(pu_last_error());
        std::string buf((size_t)n + 1, '\0');
        pu_report(h_, replica, 1, &buf[0], buf.size());
        buf.resize((size_t)n);
        *out << buf;
    }

    pu_handle* handle() { return h_; }

   private:
    template <class XmlCacheT>
    static void copy_cache(pu_cache_cfg& d, const XmlCacheT& x) {
        d.level = x.level;
        d.share = x.share;
        d.access_time = x.access_time;
        d.size = x.size;
        d.block_size = x.block_size;
        d.num_ways = x.num_ways;
    }

    pu_handle* h_ = nullptr;
    int num_cores_ = 0;
    std::vector<pu_req> reqs_;
    std::vector<int32_t> delays_;
    std::vector<char> types_;
    std::vector<uint64_t> addrs_;
    std::vector<int64_t> timers_;
};

}  // namespace pu
