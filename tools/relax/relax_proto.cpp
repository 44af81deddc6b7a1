// relax_proto.cpp — RESEARCH PROTOTYPE (not product, not oracle): windowed
// speculative relaxation of one uncore simulation, CPU-sequential but with the
// information flow of the planned GPU sweep.  Measures how many sweeps a window
// needs before its fixed point (== the sequential result) is reached.
//
// Shape: directory MESI, one private L1 level, shared-LLC home slices, full
// map, no TLB (C1/C2/C4/C5 presets).  Semantics follow oracle/cpu_ref.cpp
// (reference system.cpp:372-482, 734-893; network.cpp:97-160;
// queue_model_history_tree.cpp:42-125).
//
// Sweep k over a window of requests [a, b):
//   F  functional fold in canonical order (L1 sets, home sets, sharers, victims)
//      using the stamps (T_r + 1 for L1 lines, home arrival for home lines)
//      of sweep k-1            -> per-request program (which transmits, legs)
//   T  per message, sequential: T_r = timer + D, walk the program; each link
//      visit's queue delay is GUESSED from sweep k-1's result for that visit
//      (departure-preserving: a visit that waited keeps its departure time)
//   L  per link: fold its visits in canonical order from the window-start link
//      state -> exact queue delays for the arrival times T produced
// Fixed point: every visit's L delay == the guess T used, and every stamp T
// produced == the stamp F used.  Then the window equals the sequential run.
//
// usage: relax_proto PREFIX N_CORES WINDOW [max_sweeps] [guess mode 0|1] [bands]
// (bands > 0: print the home-tile band statistics of the first sweep and exit)
// Environment (the GPU sweep measurement, tools/relax/sweep_bench.hip):
//   RELAX_SKIP=K        run the first K requests exactly (sequentially, checked
//                       against PREFIX.delay) before the first window
//   RELAX_DUMP=DIR      relax ONE window after the skip and, at sweep
//   RELAX_DUMP_SWEEP=S  S (default 2), write phase L's input (every link's
//                       window-start state and its visits in canonical order,
//                       with the exact delays this sweep's fold produced) and
//                       phase F's input (the window's home-slice events in
//                       canonical order, the window-start lines of every home
//                       set they touch, and the outcome of each) to DIR
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

struct Req {
    uint64_t addr;
    int64_t timer;
    int32_t core, prog;
    uint8_t type, bstart;
    uint16_t p0;
    int32_t p1;
};
static_assert(sizeof(Req) == 32, "pu_req");

enum : uint8_t { I = 0, S = 1, E = 2, M = 3, V = 4, B = 5 };

// ------------------------------------------------------------------ queue
struct Queue {
    std::vector<std::pair<uint64_t, uint64_t>> iv{{0, UINT64_MAX}};
    double sum_sq = 0.0, sum = 0.0;
    uint64_t n = 0, newest = 0;
};

static uint64_t mg1_wait(const Queue& q) {
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

static uint64_t queue_delay(Queue& q, uint64_t t, uint64_t p, uint64_t min_proc, bool* mg1) {
    auto& v = q.iv;
    if (v.size() >= 100) v.erase(v.begin());
    uint64_t d;
    *mg1 = false;
    if (v.front().first > t + p) {
        d = mg1_wait(q);
        *mg1 = true;
    } else {
        size_t k = 0;
        for (; k < v.size(); k++) {
            const auto& x = v[k];
            if ((x.first <= t && t + p <= x.second) || (t < x.first && x.second - x.first >= p)) break;
        }
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
            if (x.second - (x.first + p) >= min_proc) x.first += p;
            else v.erase(v.begin() + (long)k);
        }
    }
    q.sum_sq += (double)p * (double)p;
    q.sum += (double)p;
    q.n++;
    uint64_t fin = t + d + p;
    if (fin > q.newest) q.newest = fin;
    return d;
}

// ------------------------------------------------------------------ config
struct Cfg {
    int cores = 1024, N = 1024, w = 32;
    int hdr = 3, width = 10;
    int64_t router = 0, link = 1, inject = 1;
    int l1_sets = 64, l1_ways = 8, l1_at = 1, off = 6, l1_idx = 6;
    int d_sets = 512, d_ways = 8, d_at = 10, d_idx = 9;
    int dram = 120, blk = 64;
    int nwords = 16;
};
static Cfg C;

struct Cache {
    // sets are materialised on first touch (a C4 home slice only ever sees 1 of its 512 sets)
    bool alive = false;
    int ways = 0, words = 0;
    std::vector<int32_t> slot;   // set -> first line index in the arrays below, -1 = never touched
    std::vector<uint8_t> st;
    std::vector<int32_t> id;
    std::vector<uint64_t> tag;
    std::vector<int64_t> ts;
    std::vector<uint64_t> shr;   // home: sharer bitmap per line
    void make(int sets, int ways_, int words_) {
        alive = true;
        ways = ways_; words = words_;
        slot.assign((size_t)sets, -1);
    }
    size_t base(uint64_t set) {
        if (slot[set] < 0) {
            slot[set] = (int32_t)st.size();
            st.resize(st.size() + ways, I); id.resize(id.size() + ways, 0); tag.resize(tag.size() + ways, 0);
            ts.resize(ts.size() + ways, 0); shr.resize(shr.size() + (size_t)ways * words, 0);
        }
        return (size_t)slot[set];
    }
};

struct FState {
    std::vector<Cache> l1, home;
};

static int home_of(uint64_t addr) {
    int hm = (int)std::ceil(std::log2((double)C.N));
    int hb = (int)((addr >> C.off) % (uint64_t)(1 << hm));
    return hb < C.N ? hb : hb % (1 << (hm - 1));
}

// ------------------------------------------------------------------ programs
struct Leg { int node; int at; };
struct Prog {
    uint8_t kind = 0;      // 0 hit (no network), 1 miss, 2 upgrade (WR hit on S)
    int wb_home = -1;      // victim write-back transmit target
    int home = -1;
    uint8_t hp = 0;        // 0 none, 1 owner sequence, 2 sharer legs (also broadcast)
    int owner = -1, owner_len = 0, owner_at = 0;
    std::vector<Leg> legs;
    int dram_add = 0;
    int reply_len = 0;
    bool operator==(const Prog& o) const {
        if (kind != o.kind || wb_home != o.wb_home || home != o.home || hp != o.hp || owner != o.owner ||
            owner_len != o.owner_len || owner_at != o.owner_at || dram_add != o.dram_add ||
            reply_len != o.reply_len || legs.size() != o.legs.size())
            return false;
        for (size_t i = 0; i < legs.size(); i++)
            if (legs[i].node != o.legs[i].node || legs[i].at != o.legs[i].at) return false;
        return true;
    }
};

// ---- F: functional fold with given stamps (stampL[r] = L1 stamp, stampH[r] = home stamp)
// One home-slice access of phase F (home_access), as the GPU sweep replays it.
struct HomeEv {
    uint32_t slot;       // (home, set) slot of the dump
    uint32_t type;       // 0 RD, 1 WR, 2 WB
    int32_t prog, cid;
    uint64_t tag;
    int64_t stamp;
    int32_t way;         // outcome: the way the access used
    uint32_t fstate;     // outcome: the line's state after it
};

struct Functional {
    FState s;
    // exact mode: the line the request's home access stamped (patched with the
    // home arrival once the request transmit is timed)
    Cache* last_home = nullptr;
    long last_li = -1;
    std::vector<HomeEv>* rec = nullptr;         // phase F events, when recording
    std::vector<std::pair<int, uint64_t>>* rec_set = nullptr;   // per event (home, set)
    long lookup(Cache& c, int sets, int ways, int idxb, uint64_t addr, int prog) {
        uint64_t set = (addr >> C.off) % (uint64_t)sets, tg = addr >> (C.off + idxb);
        size_t b0 = c.base(set);
        for (int w = 0; w < ways; w++) {
            size_t li = b0 + w;
            if (c.id[li] == prog && c.tag[li] == tg && c.st[li] != I) return (long)li;
        }
        return -1;
    }
    long replace(Cache& c, int sets, int ways, int idxb, uint64_t addr, int prog, uint64_t* oaddr, int* oprog) {
        uint64_t set = (addr >> C.off) % (uint64_t)sets, tg = addr >> (C.off + idxb);
        size_t base = c.base(set);
        for (int w = 0; w < ways; w++)
            if (c.st[base + w] == I) { c.id[base + w] = prog; c.tag[base + w] = tg; return (long)(base + w); }
        size_t best = 0;
        for (int w = 1; w < ways; w++) if (c.ts[base + w] < c.ts[base + best]) best = w;
        size_t li = base + best;
        *oaddr = (set << C.off) | (c.tag[li] << (C.off + idxb));
        *oprog = c.id[li];
        c.id[li] = prog; c.tag[li] = tg;
        return (long)li;
    }
    Cache& l1(int c) { Cache& x = s.l1[c]; if (!x.alive) x.make(C.l1_sets, C.l1_ways, 0); return x; }
    Cache& hm(int h) { Cache& x = s.home[h]; if (!x.alive) x.make(C.d_sets, C.d_ways, C.nwords); return x; }
    int down(int p, uint64_t addr, int prog, bool share) {   // inval_down / share_down on L1 p
        Cache& c = s.l1[p];
        if (!c.alive) return 0;
        long li = lookup(c, C.l1_sets, C.l1_ways, C.l1_idx, addr, prog);
        if (li >= 0) {
            if (!share) c.st[li] = I;
            else if (c.st[li] == M || c.st[li] == E) c.st[li] = S;
        }
        return C.l1_at;
    }
    uint64_t* shr(Cache& h, long li) { return &h.shr[(size_t)li * C.nwords]; }
    int first_sharer(Cache& h, long li) {
        uint64_t* b = shr(h, li);
        for (int k = 0; k < C.nwords; k++) if (b[k]) return k * 64 + __builtin_ctzll(b[k]);
        return 0;
    }
    void legs_of(Cache& h, long li, uint64_t addr, int prog, Prog& P) {
        std::vector<uint64_t> snap(shr(h, li), shr(h, li) + C.nwords);
        P.hp = 2;
        for (int k = 0; k < C.nwords; k++) {
            uint64_t wd = snap[k];
            while (wd) {
                int p = k * 64 + __builtin_ctzll(wd);
                wd &= wd - 1;
                int at = down(p, addr, prog, false);
                P.legs.push_back({p, at});
            }
        }
    }
    // accessSharedCache, functional part; records the probe structure into P
    void home_access(int cid, int h, uint64_t addr, int prog, int type, int64_t stamp, Prog* P, uint8_t* out) {
        Cache& d = hm(h);
        long li = lookup(d, C.d_sets, C.d_ways, C.d_idx, addr, prog);
        if (li < 0 && type != 2) {
            uint64_t oa = 0; int op = 0;
            li = replace(d, C.d_sets, C.d_ways, C.d_idx, addr, prog, &oa, &op);
            uint8_t s0 = d.st[li];
            if (s0 != I) {
                if (s0 == M || s0 == E) {
                    int own = first_sharer(d, li);
                    P->hp = 1; P->owner = own; P->owner_at = down(own, oa, op, false);
                    P->owner_len = s0 == M ? C.blk : 0;
                } else if (s0 == S) {
                    legs_of(d, li, oa, op, *P);
                } else if (s0 == B) {
                    std::fprintf(stderr, "broadcast not in prototype\n"); std::exit(2);
                }
            }
            d.st[li] = type == 1 ? M : E;
            std::fill_n(shr(d, li), C.nwords, 0ull);
            shr(d, li)[cid / 64] |= 1ull << (cid % 64);
            P->dram_add = C.dram;
        } else if (li < 0) {
            std::fprintf(stderr, "WB miss at home\n"); std::exit(2);
        } else {
            uint8_t s0 = d.st[li];
            if (type == 1) {
                if (s0 == M || s0 == E) {
                    int own = first_sharer(d, li);
                    P->hp = 1; P->owner = own; P->owner_at = down(own, addr, prog, false); P->owner_len = C.blk;
                } else if (s0 == S) {
                    legs_of(d, li, addr, prog, *P);
                }
                d.st[li] = M;
                std::fill_n(shr(d, li), C.nwords, 0ull);
                shr(d, li)[cid / 64] |= 1ull << (cid % 64);
            } else if (type == 0) {
                if (s0 == M || s0 == E) {
                    int own = first_sharer(d, li);
                    P->hp = 1; P->owner = own; P->owner_at = down(own, addr, prog, true); P->owner_len = C.blk;
                    d.st[li] = S;
                } else if (s0 == V) {
                    d.st[li] = E;
                }
                shr(d, li)[cid / 64] |= 1ull << (cid % 64);
            } else {
                d.st[li] = V;
                std::fill_n(shr(d, li), C.nwords, 0ull);
            }
        }
        uint8_t fs = d.st[li];
        *out = fs == B ? S : fs;
        d.ts[li] = stamp;
        last_home = &d;
        last_li = li;
        if (rec) {
            const uint64_t set = (addr >> C.off) % (uint64_t)C.d_sets;
            rec->push_back({0, (uint32_t)type, prog, cid, addr >> (C.off + C.d_idx), stamp,
                            (int32_t)(li - (long)d.base(set)), fs});
            rec_set->push_back({h, set});
        }
    }
    // mesi_directory at L1 (the last level)
    void access(const Req& q, int64_t stampL, int64_t stampH, Prog& P) {
        int c = q.core;
        Cache& x = l1(c);
        P = Prog();
        long li = lookup(x, C.l1_sets, C.l1_ways, C.l1_idx, q.addr, q.prog);
        if (li >= 0) {
            x.ts[li] = stampL;
            if (q.type == 1) {
                if (x.st[li] == S) {
                    P.kind = 2; P.home = home_of(q.addr); P.reply_len = 0;
                    uint8_t tmp;
                    home_access(c, P.home, q.addr, q.prog, 1, stampH, &P, &tmp);
                }
                x.st[li] = M;
            }
            return;
        }
        uint64_t oa = 0; int op = 0;
        li = replace(x, C.l1_sets, C.l1_ways, C.l1_idx, q.addr, q.prog, &oa, &op);
        uint8_t s0 = x.st[li];
        if (s0 != I && (s0 == M || s0 == E)) {
            P.wb_home = home_of(oa);
            uint8_t tmp;
            Prog dummy;
            home_access(c, P.wb_home, oa, op, 2, stampL, &dummy, &tmp);
        }
        x.ts[li] = stampL;
        P.kind = 1; P.home = home_of(q.addr); P.reply_len = C.blk;
        uint8_t st;
        home_access(c, P.home, q.addr, q.prog, q.type, stampH, &P, &st);
        x.st[li] = st;
    }
};

// ------------------------------------------------------------------ network geometry
static size_t link_index(int x, int y, int dirn) {
    int a, b;
    switch (dirn) {
        case 0: a = x; b = y; break;
        case 1: a = x - 1; b = y; break;
        case 2: a = y - 1; b = x + C.w; break;
        default: a = y; b = x + C.w; break;
    }
    return (size_t)a * (size_t)(2 * C.w) + (size_t)b;
}

struct VisitRec { uint64_t t; uint64_t qd; uint8_t mg1; uint8_t valid; };

struct Walker {
    // guesses from the previous sweep (per request, per visit index)
    const std::vector<std::vector<VisitRec>>* prev;
    std::vector<std::vector<VisitRec>>* cur;     // t and guess used this sweep
    std::vector<std::vector<std::pair<int, int>>>* link_visits;   // per link: (request, visit idx)
    std::vector<std::vector<int>>* visit_link;   // per request: link of each visit
    std::vector<std::vector<uint8_t>>* visit_p;  // per request: packet length of each visit
    int mode = 1;   // 0: reuse prev qd; 1: departure-preserving
    uint64_t guess(int r, int j, uint64_t t) {
        const auto& pv = (*prev)[r];
        if (j >= (int)pv.size() || !pv[j].valid) return 0;
        const VisitRec& v = pv[j];
        if (mode == 0 || v.mg1) return v.qd;
        if (v.qd == 0) return 0;
        uint64_t dep = v.t + v.qd;
        return dep > t ? dep - t : 0;
    }
    uint64_t walk(int r, int& j, int src, int dst, int len, uint64_t start) {
        if (src == dst) return 0;
        int plen = C.hdr + (int)std::ceil((double)len / C.width);
        int sx = src % C.w, sy = src / C.w, rx = dst % C.w, ry = dst / C.w;
        uint64_t t = start + C.inject;
        auto hop = [&](int d) {
            t += C.router;
            size_t li = link_index(sx, sy, d);
            uint64_t g = guess(r, j, t);
            (*cur)[r].push_back({t, g, 0, 1});
            (*visit_link)[r].push_back((int)li);
            (*visit_p)[r].push_back((uint8_t)plen);
            (*link_visits)[li].push_back({r, j});
            t += g + C.link;
            j++;
        };
        while (sx != rx) { int d = rx > sx ? 0 : 1; hop(d); sx += d == 0 ? 1 : -1; }
        while (sy != ry) { int d = ry > sy ? 3 : 2; hop(d); sy += d == 3 ? 1 : -1; }
        t += C.router;
        t += (uint64_t)(plen - 1);
        return t - start;
    }
};

// Exact sequential execution (the reference's order, live link queues): the
// fast-forward to the measured window.
struct Exact {
    std::vector<Queue>* links;
    uint64_t walk(int src, int dst, int len, uint64_t start) {
        if (src == dst) return 0;
        int plen = C.hdr + (int)std::ceil((double)len / C.width);
        int sx = src % C.w, sy = src / C.w, rx = dst % C.w, ry = dst / C.w;
        uint64_t t = start + C.inject;
        auto hop = [&](int d) {
            t += C.router;
            bool mg;
            t += queue_delay((*links)[link_index(sx, sy, d)], t, (uint64_t)plen, (uint64_t)C.link, &mg) + C.link;
        };
        while (sx != rx) { int d = rx > sx ? 0 : 1; hop(d); sx += d == 0 ? 1 : -1; }
        while (sy != ry) { int d = ry > sy ? 3 : 2; hop(d); sy += d == 3 ? 1 : -1; }
        t += C.router;
        t += (uint64_t)(plen - 1);
        return t - start;
    }
    // one request at running delay D (updated); returns its delay
    int run(Functional& F, const Req& q, int32_t& D) {
        if (q.bstart) D = 0;
        const int64_t T = q.timer + D;
        Prog P;
        F.last_home = nullptr;
        F.access(q, T + C.l1_at, 0, P);   // the home stamp is patched below
        Cache* hc = F.last_home;
        const long hli = F.last_li;
        int d = C.l1_at;
        if (P.wb_home >= 0) walk(q.core, P.wb_home, C.blk, (uint64_t)(T + d));   // delay discarded (Q3)
        if (P.kind != 0) {
            d += (int)walk(q.core, P.home, 0, (uint64_t)(T + d));
            const int64_t th = T + d;
            hc->ts[(size_t)hli] = th;
            int hd = C.d_at;
            if (P.hp == 1) {
                hd += (int)walk(P.home, P.owner, 0, (uint64_t)(th + hd));
                hd += P.owner_at;
                hd += (int)walk(P.owner, P.home, P.owner_len, (uint64_t)(th + hd));
            } else if (P.hp == 2) {
                int pipe = 0, mx = 0;
                for (const Leg& L : P.legs) {
                    int tt = pipe;
                    tt += (int)walk(P.home, L.node, 0, (uint64_t)(th + hd + tt));
                    tt += L.at;
                    tt += (int)walk(L.node, P.home, 0, (uint64_t)(th + hd + tt));
                    mx = std::max(mx, tt);
                    pipe += C.hdr;
                }
                hd += mx;
            }
            hd += P.dram_add;
            d += hd;
            d += (int)walk(P.home, q.core, P.reply_len, (uint64_t)(T + d));
        }
        D += d - 1;
        return d;
    }
};

static void wfile(const std::string& path, const void* p, size_t bytes) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(p, 1, bytes, f) != bytes) { std::fprintf(stderr, "cannot write %s\n", path.c_str()); std::exit(1); }
    std::fclose(f);
}

// Phase L's per-link record for the GPU sweep: the window-start state and the
// range of its visits (l_vis.bin, canonical order).
struct LinkRec {
    uint64_t n, newest;
    double sum, sum_sq;
    uint32_t nint, vis_begin, vis_end, link;
};
struct VisRec { uint64_t t; uint32_t p, pad; };

int main(int argc, char** argv) {
    if (argc < 4) { std::fprintf(stderr, "usage: relax_proto PREFIX N_CORES WINDOW [max_sweeps] [mode]\n"); return 1; }
    std::string pre = argv[1];
    C.cores = C.N = std::atoi(argv[2]);
    C.w = (int)std::ceil(std::sqrt((double)C.N));
    C.nwords = (C.N + 63) / 64;
    size_t W = (size_t)std::atol(argv[3]);
    int max_sweeps = argc > 4 ? std::atoi(argv[4]) : 10000;
    int mode = argc > 5 ? std::atoi(argv[5]) : 1;
    const int bands = argc > 6 ? std::atoi(argv[6]) : 0;   // > 0: home-tile band statistics of sweep 1
    std::vector<Req> reqs;
    std::vector<int32_t> want;
    {
        FILE* f = std::fopen((pre + ".req").c_str(), "rb");
        std::fseek(f, 0, SEEK_END); long n = std::ftell(f) / 32; std::fseek(f, 0, SEEK_SET);
        reqs.resize(n); if (std::fread(reqs.data(), 32, n, f) != (size_t)n) return 1; std::fclose(f);
        f = std::fopen((pre + ".delay").c_str(), "rb");
        want.resize(n); if (std::fread(want.data(), 4, n, f) != (size_t)n) return 1; std::fclose(f);
    }
    size_t n = reqs.size();
    size_t nl = (size_t)(C.w - 1) * C.w * 2;
    std::vector<Queue> links(nl);
    Functional F;
    F.s.l1.resize(C.cores);
    F.s.home.resize(C.N);
    int32_t carryD = 0;   // running delay of a message that spans windows
    size_t mism = 0;
    long total_sweeps = 0, windows = 0, max_s = 0;
    const size_t skip = std::min(n, (size_t)std::atol(getenv("RELAX_SKIP") ? getenv("RELAX_SKIP") : "0"));
    const char* dump_dir = getenv("RELAX_DUMP");
    const int dump_sweep = getenv("RELAX_DUMP_SWEEP") ? std::atoi(getenv("RELAX_DUMP_SWEEP")) : 2;
    if (skip) {
        Exact X{&links};
        size_t bad = 0;
        for (size_t i = 0; i < skip; i++) bad += X.run(F, reqs[i], carryD) != want[i];
        std::printf("exact fast-forward: %zu requests, %zu mismatches\n", skip, bad);
        if (bad) return 1;
        mism += bad;
    }
    for (size_t a = skip; a < n; a += W) {
        size_t b = std::min(n, a + W), wn = b - a;
        std::vector<int64_t> stampL(wn), stampH(wn);
        // sweep-0 stamp guesses: no delay within messages, zero-load home arrival
        for (size_t i = 0; i < wn; i++) { stampL[i] = reqs[a + i].timer + 1; stampH[i] = stampL[i] + 1; }
        std::vector<std::vector<VisitRec>> prev(wn), cur(wn);
        std::vector<Prog> progs(wn);
        std::vector<int32_t> dly(wn);
        FState base = F.s;
        std::vector<Queue> lbase = links;
        int sweep = 0;
        std::vector<std::vector<std::pair<int, int>>> lv(nl);
        std::vector<std::vector<int>> vlink(wn);
        std::vector<std::vector<uint8_t>> vp(wn);
        std::vector<Queue> lwork;
        bool done = false;
        while (!done) {
            sweep++;
            // F
            F.s = base;
            std::vector<HomeEv> fev;
            std::vector<std::pair<int, uint64_t>> fset;
            const bool dumping = dump_dir && sweep == dump_sweep;
            if (dumping) { F.rec = &fev; F.rec_set = &fset; }
            for (size_t i = 0; i < wn; i++) F.access(reqs[a + i], stampL[i], stampH[i], progs[i]);
            F.rec = nullptr;
            F.rec_set = nullptr;
            // T
            for (auto& v : lv) v.clear();
            for (size_t i = 0; i < wn; i++) { cur[i].clear(); vlink[i].clear(); vp[i].clear(); }
            Walker Wk{&prev, &cur, &lv, &vlink, &vp, mode};
            int32_t D = carryD;
            bool stamps_same = true;
            for (size_t i = 0; i < wn; i++) {
                const Req& q = reqs[a + i];
                const Prog& P = progs[i];
                if (q.bstart) D = 0;
                int64_t T = q.timer + D;
                int r = (int)i, j = 0;
                int d = C.l1_at;
                int64_t sL = T + d, sH = sL;
                if (P.wb_home >= 0) Wk.walk(r, j, q.core, P.wb_home, C.blk, (uint64_t)(T + d));
                if (P.kind != 0) {
                    d += (int)Wk.walk(r, j, q.core, P.home, 0, (uint64_t)(T + d));
                    int64_t th = T + d;
                    sH = th;
                    int hd = C.d_at;
                    if (P.hp == 1) {
                        hd += (int)Wk.walk(r, j, P.home, P.owner, 0, (uint64_t)(th + hd));
                        hd += P.owner_at;
                        hd += (int)Wk.walk(r, j, P.owner, P.home, P.owner_len, (uint64_t)(th + hd));
                    } else if (P.hp == 2) {
                        int pipe = 0, mx = 0;
                        for (const Leg& L : P.legs) {
                            int tt = pipe;
                            tt += (int)Wk.walk(r, j, P.home, L.node, 0, (uint64_t)(th + hd + tt));
                            tt += L.at;
                            tt += (int)Wk.walk(r, j, L.node, P.home, 0, (uint64_t)(th + hd + tt));
                            mx = std::max(mx, tt);
                            pipe += C.hdr;
                        }
                        hd += mx;
                    }
                    hd += P.dram_add;
                    d += hd;
                    d += (int)Wk.walk(r, j, P.home, q.core, P.reply_len, (uint64_t)(T + d));
                }
                if (sL != stampL[i] || (P.kind != 0 && sH != stampH[i])) stamps_same = false;
                stampL[i] = sL;
                stampH[i] = sH;
                dly[i] = d;
                D += d - 1;
            }
            if (bands > 0 && sweep == 1) {
                // SURVEY §8e's partition: the mesh's rows in `bands` bands (one per GPU);
                // a link belongs to the band of its lower-row endpoint.  Every change of
                // band along a request's visit sequence is a dependent hand-off between
                // GPUs; so is the end of a request whose last visit is not in the band
                // of the next request's first visit.
                auto band_of = [&](int li) {
                    // link index a*2w + b (network.cpp:213-307): X links have b = y,
                    // Y links have a = the lower endpoint's y
                    const int a = li / (2 * C.w), b = li % (2 * C.w);
                    const int y = b < C.w ? b : a;
                    return y * bands / C.w;
                };
                long cross = 0, single = 0, visits_all = 0;
                for (size_t i2 = 0; i2 < wn; i2++) {
                    const auto& vl = vlink[i2];
                    visits_all += (long)vl.size();
                    int changes = 0;
                    for (size_t k = 1; k < vl.size(); k++) changes += band_of(vl[k]) != band_of(vl[k - 1]);
                    cross += changes;
                    single += changes == 0;
                }
                std::printf("bands %d: %.2f band changes per request (%.1f link visits), %.1f%% of requests in one band\n",
                            bands, (double)cross / wn, (double)visits_all / wn, 100.0 * single / wn);
                return 0;
            }
            // L
            lwork = lbase;
            size_t changed = 0, visits = 0;
            for (size_t li = 0; li < nl; li++) {
                Queue& Q = lwork[li];
                for (auto [r, j] : lv[li]) {
                    VisitRec& v = cur[r][j];
                    bool mg;
                    uint64_t qd = queue_delay(Q, v.t, vlink[r].size() ? vp[r][j] : 0, (uint64_t)C.link, &mg);
                    visits++;
                    if (qd != v.qd) changed++;
                    v.qd = qd;
                    v.mg1 = mg;
                }
            }
            if (changed == 0 && stamps_same) done = true;
            if (dumping) {
                // ---- phase L: every visited link's window-start state, its visits
                std::vector<LinkRec> lr;
                std::vector<uint64_t> liv;      // 128 (first, second) slots per link record
                std::vector<VisRec> vis;
                std::vector<uint64_t> qd;
                for (size_t li = 0; li < nl; li++) {
                    if (lv[li].empty()) continue;
                    const Queue& Q = lbase[li];
                    LinkRec R{Q.n, Q.newest, Q.sum, Q.sum_sq, (uint32_t)Q.iv.size(), (uint32_t)vis.size(), 0,
                              (uint32_t)li};
                    for (size_t k = 0; k < 128; k++) {
                        liv.push_back(k < Q.iv.size() ? Q.iv[k].first : 0);
                        liv.push_back(k < Q.iv.size() ? Q.iv[k].second : 0);
                    }
                    for (auto [r, j] : lv[li]) {
                        vis.push_back({cur[r][j].t, (uint32_t)vp[r][j], 0});
                        qd.push_back(cur[r][j].qd);
                    }
                    R.vis_end = (uint32_t)vis.size();
                    lr.push_back(R);
                }
                const std::string d = dump_dir;
                wfile(d + "/l_links.bin", lr.data(), lr.size() * sizeof(LinkRec));
                wfile(d + "/l_iv.bin", liv.data(), liv.size() * 8);
                wfile(d + "/l_vis.bin", vis.data(), vis.size() * sizeof(VisRec));
                wfile(d + "/l_qd.bin", qd.data(), qd.size() * 8);
                // ---- phase F: home events with their set slots, and the
                // window-start lines of those sets: {state, prog, tag, ts} x ways
                // + the sharer bitmaps (nwords u64 per line)
                std::vector<std::pair<int, uint64_t>> slots;
                std::vector<uint32_t> fslot;
                for (auto& hs : fset) {
                    auto it = std::find(slots.begin(), slots.end(), hs);
                    if (it == slots.end()) { slots.push_back(hs); it = slots.end() - 1; }
                    fslot.push_back((uint32_t)(it - slots.begin()));
                }
                for (size_t e = 0; e < fev.size(); e++) fev[e].slot = fslot[e];
                std::vector<uint64_t> lines;    // per slot, per way: st | prog << 8, tag, ts
                std::vector<uint64_t> shr;
                for (auto [h, set] : slots) {
                    Cache& c = base.home[(size_t)h];
                    const bool have = c.alive && c.slot[set] >= 0;
                    for (int w = 0; w < C.d_ways; w++) {
                        const size_t li = have ? (size_t)c.slot[set] + (size_t)w : 0;
                        lines.push_back(have ? (uint64_t)c.st[li] | ((uint64_t)(uint32_t)c.id[li] << 8) : 0);
                        lines.push_back(have ? c.tag[li] : 0);
                        lines.push_back(have ? (uint64_t)c.ts[li] : 0);
                        for (int k = 0; k < C.nwords; k++) shr.push_back(have ? c.shr[li * C.nwords + k] : 0);
                    }
                }
                wfile(d + "/f_ev.bin", fev.data(), fev.size() * sizeof(HomeEv));
                wfile(d + "/f_lines.bin", lines.data(), lines.size() * 8);
                wfile(d + "/f_shr.bin", shr.data(), shr.size() * 8);
                const uint32_t meta[8] = {(uint32_t)wn, (uint32_t)lr.size(), (uint32_t)vis.size(), (uint32_t)fev.size(),
                                          (uint32_t)slots.size(), (uint32_t)C.d_ways, (uint32_t)C.nwords,
                                          (uint32_t)C.link};
                wfile(d + "/meta.bin", meta, sizeof meta);
                size_t maxv = 0;
                for (auto& R : lr) maxv = std::max<size_t>(maxv, R.vis_end - R.vis_begin);
                std::printf("dump: window [%zu, %zu) sweep %d: %zu links with visits (max %zu visits), %zu visits, "
                            "%zu home events over %zu sets\n", a, b, sweep, lr.size(), maxv, vis.size(), fev.size(),
                            slots.size());
                return 0;
            }
            if (getenv("RELAX_VERBOSE"))
                std::printf("  window %zu sweep %d: visits %zu changed %zu stamps_same %d\n", a / W, sweep, visits,
                            changed, (int)stamps_same);
            prev.swap(cur);
            if (sweep >= max_sweeps && !done) { std::printf("window %zu: no convergence after %d\n", a / W, sweep); break; }
        }
        links = lwork;
        {   // running delay carried into the next window if the message continues
            int32_t D = carryD;
            for (size_t i = 0; i < wn; i++) { if (reqs[a + i].bstart) D = 0; D += dly[i] - 1; }
            carryD = D;
        }
        for (size_t i = 0; i < wn; i++) if (dly[i] != want[a + i]) mism++;
        total_sweeps += sweep; windows++; max_s = std::max<long>(max_s, sweep);
    }
    std::printf("W=%zu windows=%ld sweeps mean %.2f max %ld  mismatches %zu/%zu\n", W, windows,
                (double)total_sweeps / windows, max_s, mism, n);
    return 0;
}
