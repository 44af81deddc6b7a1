// xmlsim_check — TEST ONLY (tests/test_xmlsim_init.py, CPU, this container).
//
// Built against the reference's own xml_parser.h / xml_parser.cpp (compiled in
// place by oracle/Makefile `ref`; never copied) and include/primeuncore.hpp:
//   * prime.cpp's call sites compile unchanged against pu::UncoreManager:
//     `uncore_manager.init(xml_sim);` (prime.cpp:198) with the reference XmlSim,
//     `uncore_manager.uncore_access(core_id, &ins_mem, timer)` (prime.cpp:129)
//     with the reference InsMem (cache.h:92-99);
//   * for every XML given, XmlParser::parse + getXmlSim (xml_parser.cpp:684,121)
//     converted by pu::UncoreManager::config_from equals pu_config_load_xml's
//     pu_sim_cfg field for field.
// Prints "OK <path>" or the first differing field per file; exit 1 on a mismatch.
#include <cstdio>
#include <cstring>

#include "xml_parser.h"   // reference src/xml_parser.h (-I /root/reference/src)
#include "primeuncore.hpp"

#include "cache.h"        // reference src/cache.h: its InsMem (cache.h:92-99)

// prime.cpp's uses of the global uncore_manager, verbatim in shape (compiled,
// never called here: it would need a GPU).
void prime_call_sites(pu::UncoreManager& uncore_manager, XmlSim* xml_sim, int core_id, int64_t timer) {
    uncore_manager.init(xml_sim);                                   // prime.cpp:198
    InsMem ins_mem;
    ins_mem.mem_type = 0;
    ins_mem.prog_id = 1;
    ins_mem.addr_dmem = 0;
    int delay = 0;
    delay += uncore_manager.uncore_access(core_id, &ins_mem, timer + delay) - 1;   // prime.cpp:129
    (void)uncore_manager.allocCore(1, 0);                          // prime.cpp:93
    (void)uncore_manager.getCoreId(1, 0);                          // prime.cpp:124
    (void)uncore_manager.deallocCore(1, 0);                        // prime.cpp:112
    uncore_manager.getSimStartTime();                               // prime.cpp:207
    uncore_manager.getSimFinishTime();                              // prime.cpp:232
    std::ofstream result("/dev/null");
    uncore_manager.report(&result);                                 // prime.cpp:233
}

static int bad = 0;
#define EQ(f)                                                                                      \
    do {                                                                                           \
        if (!(a.f == b.f)) {                                                                       \
            std::printf("MISMATCH %s %s: XmlParser %g, pu_config_load_xml %g\n", path, #f,         \
                        (double)a.f, (double)b.f);                                                 \
            bad = 1;                                                                               \
        }                                                                                          \
    } while (0)

static void cmp_cache(const char* path, const char* what, const pu_cache_cfg& a, const pu_cache_cfg& b) {
    (void)what;
    EQ(level); EQ(share); EQ(access_time); EQ(size); EQ(block_size); EQ(num_ways);
}

int main(int argc, char** argv) {
    for (int i = 1; i < argc; i++) {
        const char* path = argv[i];
        XmlParser p;
        if (!p.parse(path)) {
            std::printf("PARSEFAIL %s\n", path);
            bad = 1;
            continue;
        }
        XmlSim* xs = p.getXmlSim();
        const pu_sim_cfg a = pu::UncoreManager::config_from(*xs);
        pu_sim_cfg b;
        if (pu_config_load_xml(path, &b) != 0) {
            std::printf("LOADFAIL %s: %s\n", path, pu_last_error());
            bad = 1;
            continue;
        }
        const int before = bad;
        EQ(max_msg_size); EQ(num_recv_threads); EQ(thread_sync_interval); EQ(proc_sync_interval); EQ(syscall_cost);
        EQ(sys.sys_type); EQ(sys.protocol_type); EQ(sys.max_num_sharers); EQ(sys.page_size); EQ(sys.tlb_enable);
        EQ(sys.shared_llc); EQ(sys.verbose_report); EQ(sys.dram_access_time); EQ(sys.cpi_nonmem);
        EQ(sys.num_levels); EQ(sys.num_cores); EQ(sys.freq); EQ(sys.bus_latency); EQ(sys.page_miss_delay);
        EQ(sys.network.data_width); EQ(sys.network.header_flits); EQ(sys.network.net_type);
        EQ(sys.network.router_delay); EQ(sys.network.link_delay); EQ(sys.network.inject_delay);
        cmp_cache(path, "directory", a.sys.directory_cache, b.sys.directory_cache);
        cmp_cache(path, "tlb", a.sys.tlb_cache, b.sys.tlb_cache);
        for (int l = 0; l < a.sys.num_levels; l++) cmp_cache(path, "cache", a.sys.cache[l], b.sys.cache[l]);
        if (bad == before) std::printf("OK %s\n", path);
    }
    return bad;
}
