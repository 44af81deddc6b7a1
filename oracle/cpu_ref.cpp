// cpu_ref.cpp — TEST INFRASTRUCTURE ONLY: the CPU restatement ("port") of the
// reference uncore hot path.  It is the checker for the HIP engine and the
// CPU baseline leg of bench.py; the product never links or calls it.
//
// It restates, in our own scalar structure-of-arrays form, the semantics of
//   System::access / mesi_directory / mesi_bus / share / inval /
//   accessDirectoryCache / accessSharedCache / tlb_translate / getHomeId
//                                    reference src/system.cpp:144-946
//   Cache::addrParse/addrCompose/lru/accessLine/replaceLine
//                                    reference src/cache.cpp:145-235
//   Network::transmit/getLoc/getLink reference src/network.cpp:97-307
//   Link::access, Bus::access        reference src/link.cpp:54-60, bus.cpp:55-61
//   QueueModelHistoryTree::computeQueueDelay + QueueModelMG1
//                                    reference src/Graphite/queue_model_history_tree.cpp:42-125,
//                                    queue_model_m_g_1.cpp:16-55
//   Dram::access, PageTable::translate reference src/dram.cpp:43-47, page_table.cpp:56-72
//     (+ the opt-in DRAM bank model of include/primeuncore.h pu_dram_cfg, which
//     has no reference counterpart: its parity is engine vs this restatement)
//   ThreadSched::allocCore            reference src/thread_sched.cpp:55-67
// and the request loop of reference src/prime.cpp:120-137.
//
// The AVL interval tree is restated as a sorted array of free intervals: the
// tree search returns the leftmost interval I (by start) with
//   (I.first <= t && t+p <= I.second) || (t < I.first && I.second-I.first >= p)
// which holds whenever intervals are disjoint with gaps >= 1 — guaranteed for
// processing times >= 1 and min_processing_time >= 1 (checked at create).
// Parity of this restatement is pinned against the reference itself
// (oracle/_ref, tests/golden/*).

#include "cpu_ref.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#ifdef CPUREF_TRACE
void cpuref_trace_link(size_t link, bool tree, size_t intervals);   // defined by the analysis build
static size_t g_trace_k;   // index (from the front) of the interval the last tree search stopped at
static size_t g_trace_n0, g_trace_n1;   // free intervals before the last queue op (after the prune) and after it
#endif

namespace {

enum : uint8_t { I = 0, S = 1, E = 2, M = 3, V = 4, B = 5 };

// ------------------------------------------------------------ queue model
struct Queue {
    std::vector<std::pair<uint64_t, uint64_t>> iv{{0, UINT64_MAX}};
    double sum_sq = 0.0;
    double sum = 0.0;
    uint64_t n = 0;
    uint64_t newest = 0;
};

uint64_t mg1_wait(const Queue& q) {
    if (q.n == 0) return 0;
    volatile double nd = (double)q.n;
    volatile double mean = q.sum / nd;
    volatile double var = (q.sum_sq / nd) - mean * mean;
    volatile double mu = 1.0 / (q.sum / nd);
    volatile double lambda = nd / (double)q.newest;
    if (lambda >= mu) lambda = 0.999 * mu;
    volatile double inv = 1 / (mu * mu);
    volatile double num = 0.5 * mu;
    num = num * lambda;
    num = num * (inv + var);
    volatile double w = num / (mu - lambda);
    return (uint64_t)std::ceil(w);
}

uint64_t queue_delay(Queue& q, uint64_t t, uint64_t p, uint64_t min_proc, uint64_t* mg1_calls) {
    auto& v = q.iv;
    if (v.size() >= 100) v.erase(v.begin());          // prune the minimum
#ifdef CPUREF_TRACE
    g_trace_n0 = v.size();
#endif
    uint64_t d;
    if (v.front().first > t + p) {                     // older than tracked history: M/G/1
        d = mg1_wait(q);
        (*mg1_calls)++;
    } else {
        size_t k = 0;
        for (; k < v.size(); k++) {
            const auto& x = v[k];
            if ((x.first <= t && t + p <= x.second) || (t < x.first && x.second - x.first >= p)) break;
        }
#ifdef CPUREF_TRACE
        g_trace_k = k;
#endif
        auto& x = v[k];
        if (t >= x.first) {
            d = 0;
            if (t - x.first >= min_proc) {
                if (x.second - (t + p) >= min_proc) {
                    std::pair<uint64_t, uint64_t> tail{t + p, x.second};
                    x.second = t;
                    v.insert(v.begin() + (long)k + 1, tail);
                } else {
                    x.second = t;
                }
            } else if (x.second - (t + p) >= min_proc) {
                x.first = t + p;
            } else {
                v.erase(v.begin() + (long)k);
            }
        } else {
            d = x.first - t;
            if (x.second - (x.first + p) >= min_proc) {
                x.first += p;
            } else {
                v.erase(v.begin() + (long)k);
            }
        }
    }
    q.sum_sq += (double)p * (double)p;
    q.sum += (double)p;
    q.n++;
    uint64_t fin = t + d + p;
    if (fin > q.newest) q.newest = fin;
#ifdef CPUREF_TRACE
    g_trace_n1 = v.size();
#endif
    return d;
}

// ------------------------------------------------------------ cache arrays
struct Geo {
    uint64_t nsets = 0, nways = 0, block = 0, offmask = 0;
    int offbits = 0, idxbits = 0, access_time = 0;
    uint64_t index(uint64_t a) const { return (a >> offbits) % nsets; }
    uint64_t tag(uint64_t a) const { return a >> (offbits + idxbits); }
    uint64_t compose(uint64_t index, uint64_t tag) const {
        return (index << offbits) | (tag << (offbits + idxbits));
    }
};

struct CacheArr {
    bool alive = false;
    std::vector<uint8_t> st;
    std::vector<int32_t> id;
    std::vector<uint64_t> tag;
    std::vector<int64_t> ts;
    std::vector<uint64_t> extra;   // TLB: physical page; directory: sharer bitmap
    uint64_t ins = 0, miss = 0, evict = 0, wb = 0;
    bool has_bus = false;
    Queue bus;
    void make(size_t lines, size_t extra_per_line) {
        alive = true;
        st.assign(lines, I);
        id.assign(lines, 0);
        tag.assign(lines, 0);
        ts.assign(lines, 0);
        extra.assign(lines * extra_per_line, 0);
    }
};

long lookup(const CacheArr& c, const Geo& g, uint64_t addr, int prog) {
    uint64_t set = g.index(addr), tg = g.tag(addr);
    for (uint64_t w = 0; w < g.nways; w++) {
        size_t li = (size_t)(set * g.nways + w);
        if (c.id[li] == prog && c.tag[li] == tg && c.st[li] != I) return (long)li;
    }
    return -1;
}

struct Victim {
    uint64_t addr = 0;
    int prog = 0;
};

long replace(CacheArr& c, const Geo& g, uint64_t addr, int prog, Victim* old) {
    uint64_t set = g.index(addr), tg = g.tag(addr);
    size_t base = (size_t)(set * g.nways);
    for (uint64_t w = 0; w < g.nways; w++) {
        if (c.st[base + w] == I) {
            c.id[base + w] = prog;
            c.tag[base + w] = tg;
            return (long)(base + w);
        }
    }
    size_t best = 0;
    for (uint64_t w = 1; w < g.nways; w++)
        if (c.ts[base + w] < c.ts[base + best]) best = (size_t)w;
    size_t li = base + best;
    old->addr = g.compose(set, c.tag[li]);
    old->prog = c.id[li];
    c.id[li] = prog;
    c.tag[li] = tg;
    return (long)li;
}

int ilog2(uint64_t x) { return (int)std::log2((double)x); }

struct Req {
    uint64_t addr;
    int prog;
    int type;
};

// ------------------------------------------------------------ the system
struct Sys {
    pu_sim_cfg cfg;
    int L = 0, cores = 0, N = 0;
    Geo lg[PU_MAX_LEVELS];
    int share[PU_MAX_LEVELS] = {0}, ncaches[PU_MAX_LEVELS] = {0};
    std::vector<CacheArr> caches[PU_MAX_LEVELS];
    Geo dg;
    int nwords = 0;
    std::vector<CacheArr> dirs;
    std::vector<uint8_t> home_stat;
    Geo tg;
    std::vector<CacheArr> tlbs;
    std::map<std::pair<int, uint64_t>, uint64_t> page_map;
    uint64_t next_page = 0;
    int page_bits = 0;
    // network
    int w = 0, net_type = 0, header_flits = 0, data_width = 1;
    uint64_t router = 0, link_delay = 0, inject = 0;
    std::vector<Queue> links;
    // stats
    pu_stats st;
    // per-access scratch (delay[core] / hit_flag[core] of the requesting core)
    int dly = 0;
    bool hit = false;
    // thread map
    std::vector<int> core_stat;
    std::map<std::pair<int, int>, int> core_map;
    std::vector<int64_t> completion;
    int batch_delay = 0;   // running delay of the open message, kept across cpuref_run calls
    bool halted = false;   // prime.cpp:130-134: the handler exits on a negative delay
    int mode = 0;          // CPUREF_CLOSED | CPUREF_NOHALT
    std::vector<int64_t> core_shift;   // closed loop: the core's summed batch delays
    int64_t msg_shift = 0;             // closed loop: the open message's shift
    bool skip_msg = false;             // CPUREF_MSGHALT: the open message went negative
    uint64_t dead_tags = 0;            // CPUREF_MSGHALT: receive threads (tag & 63) that returned
    // opt-in DRAM bank model (pu_dram_cfg): per bank the cycle it is free and
    // its open page + 1 (0 = closed)
    std::vector<int64_t> bank_ready;
    std::vector<uint64_t> bank_open;

    // -------------------------------------------------- geometry
    std::string init(const pu_sim_cfg* c) {
        cfg = *c;
        const pu_sys_cfg& y = cfg.sys;
        L = y.num_levels;
        cores = y.num_cores;
        if (L < 1 || L > PU_MAX_LEVELS) return "num_levels must be 1..4";
        if (cores < 1) return "num_cores must be >= 1";
        for (int l = 0; l < L; l++) {
            const pu_cache_cfg& cc = y.cache[l];
            if (cc.share < 1 || cc.num_ways < 1 || cc.block_size < 1) return "bad cache geometry";
            share[l] = cc.share;
            ncaches[l] = (int)std::ceil((double)cores / cc.share);
            Geo& g = lg[l];
            g.nways = cc.num_ways;
            g.block = cc.block_size;
            g.nsets = cc.size / (cc.block_size * cc.num_ways);
            if (g.nsets < 1) return "cache has no sets";
            g.offbits = ilog2(cc.block_size);
            g.offmask = cc.block_size - 1;
            g.idxbits = ilog2(g.nsets);
            g.access_time = cc.access_time;
            caches[l].resize((size_t)ncaches[l]);
            for (auto& ca : caches[l]) ca.has_bus = cc.share > 1;
        }
        if (share[0] != 1) return "L1 share must be 1 (System::access passes cache[0][core_id], system.cpp:161)";
        for (int l = 1; l < L; l++)
            if (share[l] % share[l - 1] != 0) return "cache shares must nest";
        N = ncaches[L - 1];
        const pu_cache_cfg& dc = y.directory_cache;
        if (dc.size == 0) return "a directory is required (system.cpp:1052, SURVEY Q15)";
        dg.nways = dc.num_ways;
        dg.block = dc.block_size;
        dg.nsets = dc.size / (dc.block_size * dc.num_ways);
        if (dg.nsets < 1) return "directory has no sets";
        dg.offbits = ilog2(dc.block_size);
        dg.offmask = dc.block_size - 1;
        dg.idxbits = ilog2(dg.nsets);
        dg.access_time = dc.access_time;
        nwords = (N + 63) / 64;
        dirs.resize((size_t)N);
        home_stat.assign((size_t)N, 0);
        if (y.tlb_enable) {
            const pu_cache_cfg& tc = y.tlb_cache;
            if (tc.size == 0) return "tlb_enable needs a TLB";
            tg.nways = tc.num_ways;
            tg.block = tc.block_size;
            tg.nsets = tc.size / (tc.block_size * tc.num_ways);
            if (tg.nsets < 1) return "TLB has no sets";
            tg.offbits = ilog2((uint64_t)y.page_size);
            tg.offmask = (uint64_t)y.page_size - 1;
            tg.idxbits = ilog2(tg.nsets);
            tg.access_time = tc.access_time;
            tlbs.resize((size_t)cores);
            for (auto& t : tlbs) t.make((size_t)(tg.nsets * tg.nways), 1);
        }
        page_bits = y.page_size > 0 ? ilog2((uint64_t)y.page_size) : 0;
        if (y.protocol_type == 1 && N != cores) return "limited-pointer broadcast needs one LLC per core (SURVEY Q11)";
        if (y.sys_type == 0 && y.network.link_delay < 1) return "link_delay must be >= 1";
        for (int l = 0; l < L; l++)
            if (share[l] > 1 && y.bus_latency < 1) return "bus_latency must be >= 1 when a level is shared";
        // network
        net_type = y.network.net_type;
        w = net_type == 1 ? (int)std::ceil(std::cbrt((double)N)) : (int)std::ceil(std::sqrt((double)N));
        header_flits = y.network.header_flits;
        data_width = y.network.data_width;
        router = y.network.router_delay;
        link_delay = y.network.link_delay;
        inject = y.network.inject_delay;
        size_t nl = w > 1 ? (size_t)(w - 1) * (size_t)w * (net_type == 1 ? 3 * (size_t)w : 2) : 0;
        links.resize(nl);
        std::memset(&st, 0, sizeof(st));
        st.num_levels = L;
        core_stat.assign((size_t)cores, 0);
        completion.assign((size_t)cores, -1);
        core_shift.assign((size_t)cores, 0);
        const pu_dram_cfg& dm = y.dram;
        if (dm.banks < 0 || (dm.banks & (dm.banks - 1)) != 0) return "dram banks must be 0 or a power of two";
        if (dm.banks > 0 && (dm.row_bytes < 64 || (dm.row_bytes & (dm.row_bytes - 1)) != 0))
            return "dram row_bytes must be a power of two >= 64";
        bank_ready.assign((size_t)dm.banks, 0);
        bank_open.assign((size_t)dm.banks, 0);
        return "";
    }

    // -------------------------------------------------- lazy creation (system.cpp:172-218)
    void ensure_cache(int l, int cid) {
        CacheArr& c = caches[l][(size_t)cid];
        if (!c.alive) c.make((size_t)(lg[l].nsets * lg[l].nways), 0);
        if (l < L - 1) ensure_cache(l + 1, parent(l, cid));
    }
    int parent(int l, int cid) const { return cid * share[l] / share[l + 1]; }
    int nchildren(int l) const { return l == 0 ? 0 : share[l] / share[l - 1]; }
    CacheArr& dir(int home) {
        CacheArr& d = dirs[(size_t)home];
        if (!d.alive) d.make((size_t)(dg.nsets * dg.nways), (size_t)nwords);
        return d;
    }

    // -------------------------------------------------- network
    void loc(int id, int* x, int* y, int* z) const {
        if (net_type == 1) {
            *x = (id % (w * w)) % w;
            *y = (id % (w * w)) / w;
            *z = id / (w * w);
        } else {
            *x = id % w;
            *y = id / w;
            *z = 0;
        }
    }
    // dir: 0 E, 1 W, 2 N, 3 S, 4 U, 5 D  (network.cpp:213-307)
    size_t link_index(int x, int y, int z, int dirn) const {
        int a, b, c;
        if (net_type == 1) {
            switch (dirn) {
                case 0: a = x; b = y; c = z; break;
                case 1: a = x - 1; b = y; c = z; break;
                case 2: a = y - 1; b = z; c = x + w; break;
                case 3: a = y; b = z; c = x + w; break;
                case 4: a = z; b = x; c = y + 2 * w; break;
                default: a = z - 1; b = x; c = y + 2 * w; break;
            }
            return ((size_t)a * (size_t)w + (size_t)b) * (size_t)(3 * w) + (size_t)c;
        }
        switch (dirn) {
            case 0: a = x; b = y; break;
            case 1: a = x - 1; b = y; break;
            case 2: a = y - 1; b = x + w; break;
            default: a = y; b = x + w; break;
        }
        return (size_t)a * (size_t)(2 * w) + (size_t)b;
    }
    uint64_t hop(size_t li, uint64_t t, int plen) {
        st.link_flits += (uint64_t)plen;
#ifdef CPUREF_TRACE   // analysis builds only (tools/reuse/tree_reuse.py): which link, which branch
        const uint64_t m0 = st.mg1_calls;
        const uint64_t d = queue_delay(links[li], t, (uint64_t)plen, link_delay, &st.mg1_calls);
        cpuref_trace_link(li, st.mg1_calls == m0, g_trace_k);
        return d + link_delay;
#else
        return queue_delay(links[li], t, (uint64_t)plen, link_delay, &st.mg1_calls) + link_delay;
#endif
    }
    uint64_t transmit(int src, int dst, int len, uint64_t timer) {
        if (src == dst) return 0;
        int plen = header_flits + (int)std::ceil((double)len / data_width);
        int sx, sy, sz, rx, ry, rz;
        loc(src, &sx, &sy, &sz);
        loc(dst, &rx, &ry, &rz);
        uint64_t t = timer + inject;
        uint64_t dist = 0;
        dist += (uint64_t)std::abs(rx - sx);
        while (sx != rx) {
            t += router;
            int d = rx > sx ? 0 : 1;
            t += hop(link_index(sx, sy, sz, d), t, plen);
            sx += d == 0 ? 1 : -1;
        }
        dist += (uint64_t)std::abs(ry - sy);
        while (sy != ry) {
            t += router;
            int d = ry > sy ? 3 : 2;
            t += hop(link_index(sx, sy, sz, d), t, plen);
            sy += d == 3 ? 1 : -1;
        }
        dist += (uint64_t)std::abs(rz - sz);
        while (sz != rz) {
            t += router;
            int d = rz > sz ? 4 : 5;
            t += hop(link_index(sx, sy, sz, d), t, plen);
            sz += d == 4 ? 1 : -1;
        }
        t += router;
        t += (uint64_t)(plen - 1);
        st.net_accesses++;
        st.net_total_delay += t - timer;
        st.net_router_delay += (dist + 1) * router;
        st.net_link_delay += t - timer - (dist + 1) * router - (uint64_t)(plen - 1) - inject;
        st.net_inject_delay += inject;
        st.net_distance += dist;
        return t - timer;
    }

    // -------------------------------------------------- homes (system.cpp:921-946)
    int home_of(uint64_t addr) const {
        int off = ilog2(dg.block);
        int hm = (int)std::ceil(std::log2((double)N));
        int hb = (int)((addr >> off) % (uint64_t)(1 << hm));
        if (hb < N) return hb;
        return hb % (1 << (hm - 1));
    }

    // Dram::access at cycle t for address addr: fixed latency, or one
    // open-page bank access under pu_dram_cfg (banks > 0; formula in
    // include/primeuncore.h).  Sites whose delay System discards still occupy
    // the bank.
    int dram(uint64_t addr, int64_t t) {
        st.dram_accesses++;
        const pu_dram_cfg& dm = cfg.sys.dram;
        if (dm.banks == 0) return cfg.sys.dram_access_time;
        const uint64_t row = addr / dm.row_bytes;
        const size_t bank = (size_t)(row % (uint64_t)dm.banks);
        const uint64_t page = row / (uint64_t)dm.banks + 1;
        const int64_t start = std::max(t, bank_ready[bank]);
        int64_t act;
        if (bank_open[bank] == page) {
            act = 0;
            st.dram_row_hits++;
        } else if (bank_open[bank] == 0) {
            act = dm.t_rcd;
            st.dram_row_empty++;
        } else {
            act = (int64_t)dm.t_rp + dm.t_rcd;
            st.dram_row_conflicts++;
        }
        bank_ready[bank] = start + act + dm.t_burst;
        bank_open[bank] = page;
        st.dram_bank_wait += (uint64_t)(start - t);
        return (int)(start - t + act) + cfg.sys.dram_access_time;
    }

    // -------------------------------------------------- downward propagation (system.cpp:488-572)
    int share_down(int l, int cid, const Req& r) {
        CacheArr& c = caches[l][(size_t)cid];
        if (!c.alive) return 0;
        st.lockdown_calls++;
        long li = lookup(c, lg[l], r.addr, r.prog);
        int d = lg[l].access_time;
        if (li >= 0 && (c.st[(size_t)li] == M || c.st[(size_t)li] == E)) {
            c.st[(size_t)li] = S;
            d += share_children(l, cid, r);
        }
        return d;
    }
    int share_children(int l, int cid, const Req& r) {
        int mx = 0;
        for (int k = 0; k < nchildren(l); k++) mx = std::max(mx, share_down(l - 1, cid * nchildren(l) + k, r));
        return mx;
    }
    int inval_down(int l, int cid, const Req& r) {
        CacheArr& c = caches[l][(size_t)cid];
        if (!c.alive) return 0;
        st.lockdown_calls++;
        long li = lookup(c, lg[l], r.addr, r.prog);
        int d = lg[l].access_time;
        if (li >= 0) {
            c.st[(size_t)li] = I;
            d += inval_children(l, cid, r);
        }
        return d;
    }
    int inval_children(int l, int cid, const Req& r) {
        int mx = 0;
        for (int k = 0; k < nchildren(l); k++) mx = std::max(mx, inval_down(l - 1, cid * nchildren(l) + k, r));
        return mx;
    }

    // -------------------------------------------------- sharer bitmaps
    uint64_t* sharers(CacheArr& d, long li) { return &d.extra[(size_t)li * (size_t)nwords]; }
    int first_sharer(CacheArr& d, long li) {
        uint64_t* s = sharers(d, li);
        for (int k = 0; k < nwords; k++)
            if (s[k]) return k * 64 + __builtin_ctzll(s[k]);
        st.error_flags |= PU_ERRF_EMPTY_SHARER;
        return 0;
    }
    int count_sharers(CacheArr& d, long li) {
        uint64_t* s = sharers(d, li);
        int n = 0;
        for (int k = 0; k < nwords; k++) n += __builtin_popcountll(s[k]);
        return n;
    }
    void clear_sharers(CacheArr& d, long li) { std::fill_n(sharers(d, li), nwords, 0ull); }
    void add_sharer(CacheArr& d, long li, int cid) { sharers(d, li)[cid / 64] |= 1ull << (cid % 64); }

    // Loops of system.cpp:605-633 / 766-795: home -> sharer -> inval -> home,
    // each leg offset by delay_pipe (+header_flits per sharer), result = max.
    int inval_sharers(CacheArr& d, long li, int home, const Req& r, int64_t base) {
        int last = L - 1, pipe = 0, mx = 0;
        std::vector<uint64_t> snap(sharers(d, li), sharers(d, li) + nwords);
        for (int k = 0; k < nwords; k++) {
            uint64_t word = snap[(size_t)k];
            while (word) {
                int p = k * 64 + __builtin_ctzll(word);
                word &= word - 1;
                int t = pipe;
                t += (int)transmit(home, p, 0, (uint64_t)(base + t));
                t += inval_down(last, p, r);
                t += (int)transmit(p, home, 0, (uint64_t)(base + t));
                mx = std::max(mx, t);
                pipe += header_flits;
            }
        }
        return mx;
    }
    int broadcast(int home, const Req& r, int64_t base) {
        int last = L - 1, pipe = 0, mx = 0;
        st.total_num_broadcast++;
        for (int i = 0; i < cores; i++) {
            int t = pipe;
            t += (int)transmit(home, i, 0, (uint64_t)(base + t));
            t += inval_down(last, i, r);
            t += (int)transmit(i, home, 0, (uint64_t)(base + t));
            mx = std::max(mx, t);
            pipe += header_flits;
        }
        return mx;
    }

    // -------------------------------------------------- home slices
    // accessSharedCache (system.cpp:734-893) when shared, else
    // accessDirectoryCache (system.cpp:577-731).
    int access_home(int cid, int home, const Req& r, int64_t timer, uint8_t* out_state) {
        const bool shared = cfg.sys.shared_llc != 0;
        const int last = L - 1;
        const int blk = (int)lg[last].block;
        CacheArr& d = dir(home);
        home_stat[(size_t)home] = 1;
        long li = lookup(d, dg, r.addr, r.prog);
        d.ins++;
        int delay = dg.access_time;
        if (li < 0 && r.type != PU_WB) {
            Victim old;
            li = replace(d, dg, r.addr, r.prog, &old);
            uint8_t s = d.st[(size_t)li];
            if (s != I) {
                d.evict++;
                Req o{old.addr, old.prog, PU_RD};
                if (s == M || s == E) {
                    int own = first_sharer(d, li);
                    delay += (int)transmit(home, own, 0, (uint64_t)(timer + delay));
                    delay += inval_down(last, own, o);
                    int reply = (!shared || s == M) ? blk : 0;
                    delay += (int)transmit(own, home, reply, (uint64_t)(timer + delay));
                    dram(old.addr, timer + delay);
                } else if (s == S) {
                    delay += inval_sharers(d, li, home, o, timer + delay);
                } else if (s == B) {
                    delay += broadcast(home, o, timer + delay);
                }
            }
            d.st[(size_t)li] = r.type == PU_WR ? M : E;
            d.miss++;
            clear_sharers(d, li);
            add_sharer(d, li, cid);
            delay += dram(r.addr, timer + delay);
        } else if (li < 0) {
            // WB that misses at home: the reference dereferences NULL
            st.error_flags |= PU_ERRF_WB_MISS;
            *out_state = I;
            return delay;
        } else {
            uint8_t s = d.st[(size_t)li];
            if (r.type == PU_WR) {
                if (s == M || s == E) {
                    int own = first_sharer(d, li);
                    delay += (int)transmit(home, own, 0, (uint64_t)(timer + delay));
                    delay += inval_down(last, own, r);
                    delay += (int)transmit(own, home, blk, (uint64_t)(timer + delay));
                } else if (s == S) {
                    delay += inval_sharers(d, li, home, r, timer + delay);
                    if (!shared) delay += dram(r.addr, timer + delay);
                } else if (s == B) {
                    delay += broadcast(home, r, timer + delay);
                    if (!shared) delay += dram(r.addr, timer + delay);
                }
                d.st[(size_t)li] = M;
                clear_sharers(d, li);
                add_sharer(d, li, cid);
            } else if (r.type == PU_RD) {
                if (s == M || s == E) {
                    int own = first_sharer(d, li);
                    delay += (int)transmit(home, own, 0, (uint64_t)(timer + delay));
                    delay += share_down(last, own, r);
                    delay += (int)transmit(own, home, blk, (uint64_t)(timer + delay));
                    d.st[(size_t)li] = S;
                } else if (s == S) {
                    if (!shared) delay += dram(r.addr, timer + delay);
                    bool lim = cfg.sys.protocol_type == 1 && count_sharers(d, li) >= cfg.sys.max_num_sharers;
                    d.st[(size_t)li] = lim ? B : S;
                } else if (s == B) {
                    if (!shared) delay += dram(r.addr, timer + delay);
                } else if (s == V) {
                    d.st[(size_t)li] = E;
                }
                add_sharer(d, li, cid);
            } else {
                d.st[(size_t)li] = shared ? V : I;
                clear_sharers(d, li);
                dram(r.addr, timer + delay);
            }
        }
        uint8_t fs = d.st[(size_t)li];
        *out_state = fs == B ? S : fs;
        d.ts[(size_t)li] = timer;
        return delay;
    }

    // -------------------------------------------------- directory MESI walk (system.cpp:372-482)
    uint8_t mesi_dir(int l, int cid, const Req& r, int64_t timer) {
        ensure_cache(l, cid);
        CacheArr& c = caches[l][(size_t)cid];
        const int last = L - 1;
        if (c.has_bus) {
            st.bus_accesses++;
            int db = (int)queue_delay(c.bus, (uint64_t)(timer + dly), (uint64_t)cfg.sys.bus_latency,
                                      (uint64_t)cfg.sys.bus_latency, &st.mg1_calls);
            st.total_bus_contention += (uint64_t)(int64_t)db;
            dly += db;
        }
        if (!hit) c.ins++;
        dly += lg[l].access_time;
        long li = lookup(c, lg[l], r.addr, r.prog);
        if (li >= 0) {
            c.ts[(size_t)li] = timer + dly;
            hit = true;
            if (r.type == PU_WR) {
                if (l != last) {
                    if (c.st[(size_t)li] != M) {
                        c.st[(size_t)li] = I;
                        uint8_t ns = mesi_dir(l + 1, parent(l, cid), r, timer + dly);
                        c.st[(size_t)li] = ns;
                    }
                } else {
                    if (c.st[(size_t)li] == S) {
                        int home = home_of(r.addr);
                        uint8_t tmp;
                        dly += (int)transmit(cid, home, 0, (uint64_t)(timer + dly));
                        dly += access_home(cid, home, r, timer + dly, &tmp);
                        dly += (int)transmit(home, cid, 0, (uint64_t)(timer + dly));
                    }
                    c.st[(size_t)li] = M;
                }
                return M;
            }
            if (c.st[(size_t)li] != S) dly += share_children(l, cid, r);
            return S;
        }
        Victim old;
        li = replace(c, lg[l], r.addr, r.prog, &old);
        if (c.st[(size_t)li] != I) {
            c.evict++;
            Req o{old.addr, old.prog, PU_RD};
            dly += inval_children(l, cid, o);
            uint8_t s = c.st[(size_t)li];
            if (s == M || s == E) {
                c.wb++;
                if (l == last) {
                    int home = home_of(old.addr);
                    o.type = PU_WB;
                    uint8_t tmp;
                    transmit(cid, home, (int)lg[last].block, (uint64_t)(timer + dly));   // delay discarded (Q3)
                    access_home(cid, home, o, timer + dly, &tmp);                        // delay discarded (Q3)
                }
            }
        }
        c.ts[(size_t)li] = timer + dly;
        if (l != last) {
            uint8_t ns = mesi_dir(l + 1, parent(l, cid), r, timer);   // `timer`, not timer+delay (Q2)
            c.st[(size_t)li] = ns;
        } else {
            int home = home_of(r.addr);
            uint8_t tmp;
            dly += (int)transmit(cid, home, 0, (uint64_t)(timer + dly));
            dly += access_home(cid, home, r, timer + dly, &tmp);
            c.st[(size_t)li] = tmp;
            dly += (int)transmit(home, cid, (int)lg[last].block, (uint64_t)(timer + dly));
        }
        c.miss++;
        return c.st[(size_t)li];
    }

    // -------------------------------------------------- snoopy bus MESI walk (system.cpp:224-368)
    uint8_t mesi_bus(int l, int cid, const Req& r, int64_t timer) {
        ensure_cache(l, cid);
        CacheArr& c = caches[l][(size_t)cid];
        const int last = L - 1;
        if (c.has_bus) {
            st.bus_accesses++;
            int db = (int)queue_delay(c.bus, (uint64_t)(timer + dly), (uint64_t)cfg.sys.bus_latency,
                                      (uint64_t)cfg.sys.bus_latency, &st.mg1_calls);
            st.total_bus_contention += (uint64_t)(int64_t)db;
            dly += db;
        }
        dly += lg[l].access_time;
        if (!hit) c.ins++;
        long li = lookup(c, lg[l], r.addr, r.prog);
        if (li >= 0) {
            c.ts[(size_t)li] = timer + dly;
            hit = true;
            if (r.type == PU_WR) {
                if (l != last) {
                    if (c.st[(size_t)li] != M) {
                        c.st[(size_t)li] = I;
                        uint8_t ns = mesi_bus(l + 1, parent(l, cid), r, timer + dly);
                        c.st[(size_t)li] = ns;
                    }
                } else {
                    if (c.st[(size_t)li] == S) {
                        for (int i = 0; i < ncaches[last]; i++) {
                            if (i == cid) continue;
                            ensure_cache(last, i);
                            CacheArr& o = caches[last][(size_t)i];
                            long lt = lookup(o, lg[last], r.addr, r.prog);
                            if (lt >= 0) {
                                o.st[(size_t)lt] = I;
                                inval_children(last, i, r);
                            }
                        }
                    }
                    c.st[(size_t)li] = M;
                }
                inval_children(l, cid, r);
                return M;
            }
            if (c.st[(size_t)li] != S) share_children(l, cid, r);
            return S;
        }
        Victim old;
        li = replace(c, lg[l], r.addr, r.prog, &old);
        if (c.st[(size_t)li] != I) {
            Req o{old.addr, old.prog, PU_RD};
            inval_children(l, cid, o);
        }
        c.ts[(size_t)li] = timer + dly;
        if (l != last) {
            uint8_t ns = mesi_bus(l + 1, parent(l, cid), r, timer + dly);
            c.st[(size_t)li] = ns;
        } else {
            if (r.type == PU_WR) {
                for (int i = 0; i < ncaches[last]; i++) {
                    if (i == cid) continue;
                    ensure_cache(last, i);
                    CacheArr& o = caches[last][(size_t)i];
                    long lt = lookup(o, lg[last], r.addr, r.prog);
                    if (lt >= 0) {
                        inval_children(last, i, r);
                        uint8_t s = o.st[(size_t)lt];
                        o.st[(size_t)lt] = I;
                        if (s == M || s == E) break;
                    }
                }
                c.st[(size_t)li] = M;
            } else {
                bool shared_line = false;
                for (int i = 0; i < ncaches[last]; i++) {
                    if (i == cid) continue;
                    ensure_cache(last, i);
                    CacheArr& o = caches[last][(size_t)i];
                    long lt = lookup(o, lg[last], r.addr, r.prog);
                    if (lt >= 0) {
                        shared_line = true;
                        share_children(last, i, r);
                        uint8_t s = o.st[(size_t)lt];
                        o.st[(size_t)lt] = S;
                        if (s == M || s == E) break;
                    }
                }
                c.st[(size_t)li] = shared_line ? S : E;
            }
            dly += dram(r.addr, timer + dly);
        }
        c.miss++;
        return c.st[(size_t)li];
    }

    // -------------------------------------------------- TLB (system.cpp:897-918)
    int tlb_translate(Req& r, int core, int64_t timer) {
        CacheArr& t = tlbs[(size_t)core];
        long li = lookup(t, tg, r.addr, r.prog);
        t.ins++;
        int d = tg.access_time;
        if (li < 0) {
            Victim old;
            li = replace(t, tg, r.addr, r.prog, &old);
            if (t.st[(size_t)li] != I) t.evict++;
            t.miss++;
            t.st[(size_t)li] = V;
            auto key = std::make_pair(r.prog, r.addr >> page_bits);
            auto it = page_map.find(key);
            uint64_t pp;
            if (it == page_map.end()) {
                pp = next_page++;
                page_map[key] = pp;
            } else {
                pp = it->second;
            }
            t.extra[(size_t)li] = pp;
            d += cfg.sys.page_miss_delay;
        }
        t.ts[(size_t)li] = timer;
        r.addr = (t.extra[(size_t)li] << page_bits) | (r.addr % (uint64_t)cfg.sys.page_size);
        return d;
    }

    // -------------------------------------------------- System::access (system.cpp:144-168)
    int access(int core, Req r, int64_t timer) {
        if (core >= cores || core < 0) {
            st.error_flags |= PU_ERRF_CORE_RANGE;
            return -1;
        }
        st.requests++;
        hit = false;
        dly = 0;
        int cid = core / share[0];
        if (cfg.sys.tlb_enable) dly = tlb_translate(r, core, timer);
        if (cfg.sys.sys_type == 0)
            mesi_dir(0, cid, r, timer + dly);
        else
            mesi_bus(0, cid, r, timer + dly);
        return dly;
    }

    void fill_stats(pu_stats* o) {
        pu_stats s = st;
        for (int l = 0; l < L; l++) {
            pu_level_stats a{0, 0, 0, 0};
            for (auto& c : caches[l]) {
                if (!c.alive) continue;
                a.ins += c.ins; a.miss += c.miss; a.evict += c.evict; a.wb += c.wb;
            }
            s.level[l] = a;
        }
        pu_level_stats dsum{0, 0, 0, 0};
        for (auto& d : dirs) {
            dsum.ins += d.ins; dsum.miss += d.miss; dsum.evict += d.evict; dsum.wb += d.wb;
        }
        s.directory = dsum;
        pu_level_stats tsum{0, 0, 0, 0};
        for (auto& t : tlbs) {
            tsum.ins += t.ins; tsum.miss += t.miss; tsum.evict += t.evict; tsum.wb += t.wb;
        }
        s.tlb = tsum;
        *o = s;
    }
};

}  // namespace

extern "C" {

void* cpuref_create(const pu_sim_cfg* cfg, char* err, size_t errcap) {
    Sys* s = new Sys();
    std::string e = s->init(cfg);
    if (!e.empty()) {
        if (err && errcap) std::snprintf(err, errcap, "%s", e.c_str());
        delete s;
        return nullptr;
    }
    return s;
}

void cpuref_destroy(void* h) { delete (Sys*)h; }

int cpuref_alloc_core(void* h, int prog, int thread) {
    Sys* s = (Sys*)h;
    for (int i = 0; i < s->cores; i++) {
        if (s->core_stat[(size_t)i] == 0) {
            s->core_stat[(size_t)i] = prog;
            s->core_map[{prog, thread}] = i;
            return i;
        }
    }
    return -1;
}

long cpuref_run(void* h, const pu_req* reqs, size_t n, int32_t* delays) {
    Sys* s = (Sys*)h;
    const bool closed = (s->mode & CPUREF_CLOSED) != 0, keep_halt = (s->mode & CPUREF_NOHALT) == 0;
    if (s->halted && keep_halt) {
        if (delays) std::fill_n(delays, n, 0);
        return n ? -1 : 0;
    }
    // 4: one receive thread of several (the server): a negative running delay
    // skips the rest of its message and that thread (tag) never receives again;
    // 8: a caller of uncore_access that only abandons the message
    const bool msghalt = (s->mode & 12) != 0, thread_dies = (s->mode & 4) != 0;
    int delay = s->batch_delay;
    for (size_t i = 0; i < n; i++) {
        const pu_req& q = reqs[i];
        const bool core_ok = q.core >= 0 && q.core < s->cores;
        if (q.batch_start) {
            delay = 0;
            // MSGHALT: a receive thread that returned never receives again
            // (prime.cpp:133 returns from msgHandler; its tag = pu_req.tag)
            s->skip_msg = msghalt && ((s->dead_tags >> (q.tag & 63)) & 1);
            if (closed && core_ok) s->msg_shift = s->core_shift[(size_t)q.core];
        }
        if (s->skip_msg) {          // MSGHALT: this message's handler thread has returned
            if (delays) delays[i] = 0;
            continue;
        }
        int64_t t = q.timer + (closed ? s->msg_shift : 0) + delay;
        int d = s->access(q.core, Req{q.addr, q.prog_id, (int)q.mem_type}, t);
        if (delays) delays[i] = d;
        delay += d - 1;
        if (core_ok) {
            s->completion[(size_t)q.core] = t + d;
            if (closed) s->core_shift[(size_t)q.core] = s->msg_shift + delay;
        }
        if (delay < 0 && msghalt) {
            if (thread_dies) s->dead_tags |= 1ull << (q.tag & 63);
            s->st.error_flags |= PU_ERRF_NEG_DELAY;
            s->skip_msg = true;
            continue;
        }
        if (delay < 0 && keep_halt) {
            s->st.error_flags |= PU_ERRF_NEG_DELAY;
            s->batch_delay = delay;
            s->halted = true;
            if (delays) std::fill(delays + i + 1, delays + n, 0);
            return (long)i + 1;
        }
    }
    s->batch_delay = delay;
    return 0;
}

int cpuref_set_mode(void* h, int mode) {
    ((Sys*)h)->mode = mode;
    return 0;
}

int cpuref_stats(void* h, pu_stats* out) {
    ((Sys*)h)->fill_stats(out);
    return 0;
}

int cpuref_completion(void* h, int64_t* out, size_t n) {
    Sys* s = (Sys*)h;
    for (size_t i = 0; i < n && i < s->completion.size(); i++) out[i] = s->completion[i];
    return 0;
}

int cpuref_cache_counters(void* h, int level, uint64_t* out, size_t n) {
    Sys* s = (Sys*)h;
    const std::vector<CacheArr>* v = nullptr;
    if (level >= 0 && level < s->L) v = &s->caches[level];
    else if (level == s->L) v = &s->dirs;
    else return -1;
    size_t k = 0;
    for (const auto& c : *v) {
        if (k + 4 > n) break;
        out[k++] = c.ins; out[k++] = c.miss; out[k++] = c.evict; out[k++] = c.wb;
    }
    return (int)(k / 4);
}

int cpuref_network_run(int num_nodes, int net_type, int data_width, int header_flits, uint64_t router_delay,
                       uint64_t link_delay, uint64_t inject_delay, const int32_t* src, const int32_t* dst,
                       const int32_t* len, const uint64_t* timer, size_t n, uint64_t* delay_out, pu_stats* st) {
    Sys s;
    std::memset(&s.st, 0, sizeof(s.st));
    s.N = num_nodes;
    s.net_type = net_type;
    s.w = net_type == 1 ? (int)std::ceil(std::cbrt((double)num_nodes)) : (int)std::ceil(std::sqrt((double)num_nodes));
    s.header_flits = header_flits;
    s.data_width = data_width;
    s.router = router_delay;
    s.link_delay = link_delay;
    s.inject = inject_delay;
    size_t nl = s.w > 1 ? (size_t)(s.w - 1) * (size_t)s.w * (net_type == 1 ? 3 * (size_t)s.w : 2) : 0;
    s.links.resize(nl);
    for (size_t i = 0; i < n; i++) delay_out[i] = s.transmit(src[i], dst[i], len[i], timer[i]);
    if (st) *st = s.st;
    return 0;
}

// mg1_wait on given states (tests/test_gpu_mg1.py, test_units_oracle.py)
int cpuref_mg1_batch(const uint64_t* n, const double* sum, const double* sum_sq, const uint64_t* newest, size_t cnt,
                     uint64_t* out) {
    Queue q;
    for (size_t i = 0; i < cnt; i++) {
        q.n = n[i];
        q.sum = sum[i];
        q.sum_sq = sum_sq[i];
        q.newest = newest[i];
        out[i] = mg1_wait(q);
    }
    return 0;
}

int cpuref_queue_run(uint64_t min_proc, const uint64_t* t, const uint64_t* p, size_t n,
                     uint64_t* delay_out, uint64_t* mg1_calls) {
    Queue q;
    uint64_t calls = 0;
    for (size_t i = 0; i < n; i++) delay_out[i] = queue_delay(q, t[i], p[i], min_proc, &calls);
    if (mg1_calls) *mg1_calls = calls;
    return 0;
}

}  // extern "C"
