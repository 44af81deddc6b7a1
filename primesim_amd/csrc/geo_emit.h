// geo_emit.h — host only: a Geo (geometry.h) written out as C++ source, a
// constexpr aggregate the engine can be compiled against (engine.hip
// PU_JIT_GEO): every configuration value the kernel reads becomes a
// compile-time constant.  Field order is geometry.h's (C++20 designated
// initializers: the compiler checks every name and the order).
#pragma once

#include <cstdint>
#include <sstream>
#include <string>

#include "geometry.h"

namespace pu {

namespace geo_emit_detail {
inline void f(std::ostringstream& o, const char* name, int64_t v) { o << "." << name << " = " << v << "LL, "; }
inline void u(std::ostringstream& o, const char* name, uint64_t v) { o << "." << name << " = " << v << "ULL, "; }
}  // namespace geo_emit_detail

inline std::string geo_cxx(const Geo& g, const char* var = "kJitGeo") {
    using namespace geo_emit_detail;
    std::ostringstream o;
    o << "#define PU_JIT_NL " << g.num_levels << "\n";
    o << "__device__ constexpr Geo " << var << " = {";
#define I32(x) f(o, #x, (int64_t)g.x)
#define U64(x) u(o, #x, (uint64_t)g.x)
    I32(num_cores); I32(num_levels); I32(sys_type); I32(protocol_type);
    I32(max_num_sharers); I32(shared_llc); I32(tlb_enable); I32(dram_access_time);
    I32(bus_latency); I32(N); I32(net_type); I32(net_width);
    I32(header_flits); I32(data_width); I32(nlinks); I32(nqueues);
    I32(home_offbits); I32(home_mask_bits);
    I32(blk_len); I32(plen_blk);
    U64(w_magic); U64(w2_magic);
    I32(w2); I32(cnt_sum);
    U64(router_delay); U64(link_delay); U64(inject_delay);
#undef I32
#undef U64
    o << ".lv = {";
    for (int l = 0; l < 4; l++) {
        const LevelGeo& L = g.lv[l];
        o << "{";
#define I32(x) f(o, #x, (int64_t)L.x)
#define U64(x) u(o, #x, (uint64_t)L.x)
        U64(nsets); U64(nways); U64(block);
        I32(offbits); I32(idxbits); I32(access_time); I32(share);
        I32(ncaches); I32(nchildren); I32(has_bus); I32(bus_q0);
        U64(off_meta); U64(off_ts); U64(off_alive); U64(off_cnt);
#undef I32
#undef U64
        o << "}, ";
    }
    o << "}, .dir = {";
    {
        const DirGeo& D = g.dir;
#define I32(x) f(o, #x, (int64_t)D.x)
#define U64(x) u(o, #x, (uint64_t)D.x)
        U64(nsets); U64(nways); U64(block); U64(csets);
        I32(offbits); I32(idxbits); I32(access_time); I32(nwords);
        I32(pool_entries); I32(cset_shift);
        I32(sh_wide); I32(sh_cap);
        U64(off_line); U64(off_pool); U64(off_pool_free); U64(off_alive); U64(off_cnt);
        U64(off_prog);
#undef I32
#undef U64
    }
    o << "}, .tlb = {";
    {
        const TlbGeo& T = g.tlb;
#define I32(x) f(o, #x, (int64_t)T.x)
#define U64(x) u(o, #x, (uint64_t)T.x)
        U64(nsets); U64(nways); U64(page_size);
        I32(offbits); I32(idxbits); I32(access_time); I32(page_miss_delay);
        U64(off_meta); U64(off_ts); U64(off_ppage); U64(off_cnt);
        U64(off_pages); U64(pages_cap);
#undef I32
#undef U64
    }
    o << "}, ";
#define I32(x) f(o, #x, (int64_t)g.x)
#define U64(x) u(o, #x, (uint64_t)g.x)
    U64(off_qhdr); U64(off_qring); U64(off_stats); U64(off_completion); U64(off_run);
    U64(off_core_shift);
    I32(dram_banks); I32(dram_bank_shift); I32(dram_row_shift); I32(dram_t_rcd);
    I32(dram_t_rp); I32(dram_t_burst);
    U64(off_dram);
    U64(replica_bytes);
#undef I32
#undef U64
    o << "};\n";
    return o.str();
}

}  // namespace pu
