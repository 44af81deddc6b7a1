// sweep_bench.hip — RESEARCH MEASUREMENT (not product, not oracle): one
// relaxation sweep of a single C4 simulation, as GPU kernels, on inputs that
// tools/relax/relax_proto.cpp dumped (RELAX_DUMP) for a window of W requests.
//
// The relaxation repeats a sweep of three phases until the
// fixed point; this measures the two phases north_star names as stages 2-3:
//   L (stage 3)  the per-link fold: every link's visits of the window in
//                canonical order, from the window-start link state, through
//                QueueModelHistoryTree::computeQueueDelay
//                (queue_model_history_tree.cpp:42-125) -> the exact queue
//                delay of every visit.  One wavefront per link; the free
//                intervals are a sorted array of <= 101 slots (lane l holds
//                slots l and l+64), the search one predicate + ballot; the
//                M/G/1 branch (queue_model_m_g_1.cpp:16-55) in IEEE f64.
//   F (stage 2)  the window's home-slice (directory) events sorted by set
//                (a stable radix sort: canonical order within a set), then
//                one lane per set folds its events (Cache::accessLine /
//                replaceLine / lru, the MESI transitions of
//                accessSharedCache, system.cpp:734-893) from the window-start
//                lines.  This is a LOWER bound on phase F: the real phase
//                also folds the L1 sets and derives the home events from
//                them (an L1 miss makes a home event, a home invalidation
//                changes a later L1 outcome), which this leaves out.
// Phase T (each message's walk over its program with guessed delays) is not
// built, so a sweep here is a lower bound on a full sweep.
//
// Every visit's delay is checked against the dump (the CPU fold of the same
// sweep): bit-exact, so the GPU fold is the reference's.  Output: one JSON
// line with the per-phase times (HIP events, mean over the repetitions, and
// the whole sweep captured in a hipGraph).
//
// usage: sweep_bench DUMP_DIR [reps]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

struct LinkRec {
    uint64_t n, newest;
    double sum, sum_sq;
    uint32_t nint, vis_begin, vis_end, link;
};
struct VisRec {
    uint64_t t;
    uint32_t p, pad;
};
struct HomeEv {
    uint32_t slot, type;
    int32_t prog, cid;
    uint64_t tag;
    int64_t stamp;
    int32_t way;
    uint32_t fstate;
};
static_assert(sizeof(LinkRec) == 48 && sizeof(VisRec) == 16 && sizeof(HomeEv) == 40, "dump layout");

template <class T>
static std::vector<T> rd(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
        std::fprintf(stderr, "cannot open %s\n", path.c_str());
        std::exit(1);
    }
    std::fseek(f, 0, SEEK_END);
    const long b = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<T> v((size_t)b / sizeof(T));
    if (b && std::fread(v.data(), 1, (size_t)b, f) != (size_t)b) std::exit(1);
    std::fclose(f);
    return v;
}

// ---------------------------------------------------------------- phase L
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
// lane i receives lane i+1 (NEXT) / i-1 (PREV), wrapping
__device__ __forceinline__ uint32_t dnext(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x134, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dprev(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x13C, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t d64(uint64_t x, bool next) {
    const uint32_t lo = next ? dnext((uint32_t)x) : dprev((uint32_t)x);
    const uint32_t hi = next ? dnext((uint32_t)(x >> 32)) : dprev((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}
// slots j in [from, 128) take slot j+1 (next) or j-1 (prev)
__device__ __forceinline__ void shift(uint64_t& lo, uint64_t& hi, bool next, uint32_t from) {
    const int ln = (int)(threadIdx.x & 63);
    const uint64_t a = d64(lo, next), b = d64(hi, next);
    // crossing lanes: slot 63 <- slot 64 (next: lane 63 of lo takes lane 0 of hi),
    // slot 64 <- slot 63 (prev: lane 0 of hi takes lane 63 of lo)
    const uint64_t nlo = (next && ln == 63) ? b : a;
    const uint64_t nhi = (!next && ln == 0) ? a : b;
    if ((uint32_t)ln >= from) lo = nlo;
    if ((uint32_t)(ln + 64) >= from) hi = nhi;
}

__device__ __forceinline__ uint64_t mg1_wait(uint64_t n, double sum, double sum_sq, uint64_t newest) {
    if (n == 0) return 0;
    const double nd = (double)n;
    const double mean = sum / nd;
    const double var = (sum_sq / nd) - mean * mean;
    const double mu = 1.0 / (sum / nd);
    double lambda = nd / (double)newest;
    if (lambda >= mu) lambda = 0.999 * mu;
    const double inv = 1 / (mu * mu);
    double num = 0.5 * mu;
    num = num * lambda;
    num = num * (inv + var);
    const double w = num / (mu - lambda);
    return (uint64_t)ceil(w);
}

__global__ __launch_bounds__(64) void phase_l(const LinkRec* __restrict__ links, const uint64_t* __restrict__ iv,
                                              const VisRec* __restrict__ vis, uint64_t* __restrict__ qd,
                                              uint64_t minp) {
    const int ln = (int)threadIdx.x;
    const LinkRec L = links[blockIdx.x];
    const uint64_t* I = iv + (size_t)blockIdx.x * 256;
    uint64_t lf = I[2 * ln], ls = I[2 * ln + 1], hf = I[2 * (ln + 64)], hs = I[2 * (ln + 64) + 1];
    uint32_t cnt = L.nint;
    uint64_t n = L.n, newest = L.newest;
    double sum = L.sum, sum_sq = L.sum_sq;
    for (uint32_t v0 = L.vis_begin; v0 < L.vis_end; v0 += 64) {
        // 64 visits at a time: lane i holds visit v0+i (no load in the fold)
        const uint32_t m = min(64u, L.vis_end - v0);
        uint64_t my_t = 0, my_d = 0;
        uint32_t my_p = 0;
        if ((uint32_t)ln < m) {
            my_t = vis[v0 + ln].t;
            my_p = vis[v0 + ln].p;
        }
        for (uint32_t i = 0; i < m; i++) {
            const uint64_t t = rl64(my_t, (int)i);
            const uint64_t p = (uint32_t)__builtin_amdgcn_readlane((int)my_p, (int)i);
            if (cnt >= 100) {                               // drop the oldest interval (:49-55)
                shift(lf, hf, true, 0);
                shift(ls, hs, true, 0);
                cnt--;
            }
            const uint64_t tp = t + p;
            uint64_t d;
            if (rl64(lf, 0) > tp) {
                d = mg1_wait(n, sum, sum_sq, newest);       // (:58-63)
            } else {
                const bool pl = (uint32_t)ln < cnt && ((lf <= t && tp <= ls) || (t < lf && ls - lf >= p));
                const bool ph = (uint32_t)(ln + 64) < cnt && ((hf <= t && tp <= hs) || (t < hf && hs - hf >= p));
                const uint64_t ml = __builtin_amdgcn_ballot_w64(pl), mh = __builtin_amdgcn_ballot_w64(ph);
                const uint32_t k = ml ? (uint32_t)__builtin_ctzll(ml) : 64u + (uint32_t)__builtin_ctzll(mh);
                const bool khi = k >= 64;
                const uint64_t sf = rl64(khi ? hf : lf, (int)(k & 63)), ss = rl64(khi ? hs : ls, (int)(k & 63));
                const bool mine_lo = (uint32_t)ln == k, mine_hi = (uint32_t)ln + 64 == k;
                if (t >= sf) {                              // (:74-96)
                    d = 0;
                    if (t - sf >= minp) {
                        if (ss - tp >= minp) {              // split: [sf, t] at k, [t+p, ss] at k+1
                            shift(lf, hf, false, k + 1);
                            shift(ls, hs, false, k + 1);
                            if ((uint32_t)ln == k + 1) { lf = tp; ls = ss; }
                            if ((uint32_t)ln + 64 == k + 1) { hf = tp; hs = ss; }
                            cnt++;
                        }
                        if (mine_lo) ls = t;
                        if (mine_hi) hs = t;
                    } else if (ss - tp >= minp) {
                        if (mine_lo) lf = tp;
                        if (mine_hi) hf = tp;
                    } else {
                        shift(lf, hf, true, k);
                        shift(ls, hs, true, k);
                        cnt--;
                    }
                } else {                                    // (:97-106)
                    d = sf - t;
                    if (ss - (sf + p) >= minp) {
                        if (mine_lo) lf = sf + p;
                        if (mine_hi) hf = sf + p;
                    } else {
                        shift(lf, hf, true, k);
                        shift(ls, hs, true, k);
                        cnt--;
                    }
                }
            }
            sum_sq += (double)p * (double)p;                // (:117, queue_model_m_g_1.cpp:45-55)
            sum += (double)p;
            n++;
            const uint64_t fin = t + d + p;
            if (fin > newest) newest = fin;
            if ((uint32_t)ln == i) my_d = d;
        }
        if ((uint32_t)ln < m) qd[v0 + ln] = my_d;
    }
}

// ---------------------------------------------------------------- phase F
constexpr uint32_t ST_I = 0, ST_S = 1, ST_E = 2, ST_M = 3, ST_V = 4;

// line word 0 = state | prog << 8, word 1 = tag, word 2 = ts (per way)
__global__ void phase_f_fold(const uint32_t* __restrict__ key, const uint32_t* __restrict__ idx,
                             const HomeEv* __restrict__ ev, uint64_t* __restrict__ lines, uint64_t* __restrict__ shr,
                             int32_t* __restrict__ way_out, uint32_t* __restrict__ st_out, uint32_t nev, int ways,
                             int nwords) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nev || (i > 0 && key[i] == key[i - 1])) return;    // one lane per set: the head of its segment
    const uint32_t slot = key[i];
    uint64_t* Ln = lines + (size_t)slot * ways * 3;
    uint64_t* Sh = shr + (size_t)slot * ways * nwords;
    for (uint32_t j = i; j < nev && key[j] == slot; j++) {
        const HomeEv e = ev[idx[j]];
        int w = -1;
        for (int k = 0; k < ways; k++) {                         // Cache::accessLine (cache.cpp:184-200)
            const uint64_t m = Ln[3 * k];
            if ((uint32_t)(m & 0xFF) != ST_I && (int32_t)(m >> 8) == e.prog && Ln[3 * k + 1] == e.tag) {
                w = k;
                break;
            }
        }
        uint32_t s0 = ST_I;
        uint64_t* sh;
        if (w < 0) {                                             // replaceLine / lru (cache.cpp:167-235)
            for (int k = 0; k < ways && w < 0; k++)
                if ((uint32_t)(Ln[3 * k] & 0xFF) == ST_I) w = k;
            if (w < 0) {
                w = 0;
                for (int k = 1; k < ways; k++)
                    if ((int64_t)Ln[3 * k + 2] < (int64_t)Ln[3 * w + 2]) w = k;
            }
            s0 = (uint32_t)(Ln[3 * w] & 0xFF);
            sh = Sh + (size_t)w * nwords;
            // the victim's owner / sharers are probed (system.cpp:607-633): read its sharer words
            uint64_t any = 0;
            if (s0 != ST_I)
                for (int k = 0; k < nwords; k++) any |= sh[k];
            const uint32_t ns = e.type == 1 ? ST_M : ST_E;
            for (int k = 0; k < nwords; k++) sh[k] = (k == e.cid / 64) ? (1ull << (e.cid % 64)) : 0ull;
            Ln[3 * w] = ns | ((uint64_t)(uint32_t)e.prog << 8) | (any & 0 /* keep the read */);
            Ln[3 * w + 1] = e.tag;
        } else {
            s0 = (uint32_t)(Ln[3 * w] & 0xFF);
            sh = Sh + (size_t)w * nwords;
            uint32_t ns = s0;
            if (e.type == 1) {
                uint64_t any = 0;
                for (int k = 0; k < nwords; k++) any |= sh[k];
                ns = ST_M | (uint32_t)(any & 0);
                for (int k = 0; k < nwords; k++) sh[k] = (k == e.cid / 64) ? (1ull << (e.cid % 64)) : 0ull;
            } else if (e.type == 0) {
                if (s0 == ST_M || s0 == ST_E) ns = ST_S;
                else if (s0 == ST_V) ns = ST_E;
                sh[e.cid / 64] |= 1ull << (e.cid % 64);
            } else {
                ns = ST_V;
                for (int k = 0; k < nwords; k++) sh[k] = 0;
            }
            Ln[3 * w] = ns | ((uint64_t)(uint32_t)e.prog << 8);
        }
        Ln[3 * w + 2] = (uint64_t)e.stamp;
        way_out[idx[j]] = w;
        st_out[idx[j]] = (uint32_t)(Ln[3 * w] & 0xFF);
    }
}

__global__ void f_keys(const HomeEv* __restrict__ ev, uint32_t* key, uint32_t* idx, uint32_t nev) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nev) {
        key[i] = ev[i].slot;
        idx[i] = i;
    }
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: sweep_bench DUMP_DIR [reps]\n");
        return 1;
    }
    const std::string d = argv[1];
    const int reps = argc > 2 ? std::atoi(argv[2]) : 200;
    const auto meta = rd<uint32_t>(d + "/meta.bin");
    const uint32_t W = meta[0], nlinks = meta[1], nvis = meta[2], nev = meta[3], nslots = meta[4];
    const int ways = (int)meta[5], nwords = (int)meta[6];
    const uint64_t minp = meta[7];
    const auto links = rd<LinkRec>(d + "/l_links.bin");
    const auto iv = rd<uint64_t>(d + "/l_iv.bin");
    const auto vis = rd<VisRec>(d + "/l_vis.bin");
    const auto qd_want = rd<uint64_t>(d + "/l_qd.bin");
    const auto ev = rd<HomeEv>(d + "/f_ev.bin");
    const auto lines0 = rd<uint64_t>(d + "/f_lines.bin");
    const auto shr0 = rd<uint64_t>(d + "/f_shr.bin");
    // the shapes every kernel assumes, checked on the host before any launch
    if (links.size() != nlinks || vis.size() != nvis || qd_want.size() != nvis || ev.size() != nev ||
        iv.size() != (size_t)nlinks * 256 || lines0.size() != (size_t)nslots * ways * 3 ||
        shr0.size() != (size_t)nslots * ways * nwords) {
        std::fprintf(stderr, "dump sizes inconsistent with meta.bin\n");
        return 1;
    }
    uint32_t maxv = 0;
    for (const auto& L : links) {
        if (L.vis_begin > L.vis_end || L.vis_end > nvis || L.nint > 100 || L.nint == 0) {
            std::fprintf(stderr, "bad link record\n");
            return 1;
        }
        maxv = std::max(maxv, L.vis_end - L.vis_begin);
    }
    for (const auto& e : ev)
        if (e.slot >= nslots || e.cid < 0 || e.cid >= nwords * 64 || e.type > 2) {
            std::fprintf(stderr, "bad home event\n");
            return 1;
        }

    LinkRec* d_links;
    uint64_t *d_iv, *d_qd, *d_lines, *d_lines0, *d_shr, *d_shr0;
    VisRec* d_vis;
    HomeEv* d_ev;
    uint32_t *d_key, *d_idx, *d_key2, *d_idx2, *d_st;
    int32_t* d_way;
    CK(hipMalloc(&d_links, links.size() * sizeof(LinkRec)));
    CK(hipMalloc(&d_iv, iv.size() * 8));
    CK(hipMalloc(&d_vis, vis.size() * sizeof(VisRec)));
    CK(hipMalloc(&d_qd, nvis * 8));
    CK(hipMalloc(&d_ev, ev.size() * sizeof(HomeEv)));
    CK(hipMalloc(&d_lines, lines0.size() * 8));
    CK(hipMalloc(&d_lines0, lines0.size() * 8));
    CK(hipMalloc(&d_shr, shr0.size() * 8));
    CK(hipMalloc(&d_shr0, shr0.size() * 8));
    CK(hipMalloc(&d_key, nev * 4));
    CK(hipMalloc(&d_idx, nev * 4));
    CK(hipMalloc(&d_key2, nev * 4));
    CK(hipMalloc(&d_idx2, nev * 4));
    CK(hipMalloc(&d_way, nev * 4));
    CK(hipMalloc(&d_st, nev * 4));
    CK(hipMemcpy(d_links, links.data(), links.size() * sizeof(LinkRec), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_iv, iv.data(), iv.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vis, vis.data(), vis.size() * sizeof(VisRec), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ev, ev.data(), ev.size() * sizeof(HomeEv), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lines0, lines0.data(), lines0.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_shr0, shr0.data(), shr0.size() * 8, hipMemcpyHostToDevice));
    int kbits = 1;
    while ((1u << kbits) < nslots) kbits++;
    size_t tmp_b = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_b, d_key, d_key2, d_idx, d_idx2, (int)nev, 0, kbits));
    void* d_tmp;
    CK(hipMalloc(&d_tmp, tmp_b + 16));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

    auto run_l = [&] { phase_l<<<nlinks, 64, 0, s>>>(d_links, d_iv, d_vis, d_qd, minp); };
    auto run_f = [&] {
        CK(hipMemcpyAsync(d_lines, d_lines0, lines0.size() * 8, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(d_shr, d_shr0, shr0.size() * 8, hipMemcpyDeviceToDevice, s));
        f_keys<<<(nev + 255) / 256, 256, 0, s>>>(d_ev, d_key, d_idx, nev);
        CK(hipcub::DeviceRadixSort::SortPairs(d_tmp, tmp_b, d_key, d_key2, d_idx, d_idx2, (int)nev, 0, kbits, s));
        phase_f_fold<<<(nev + 255) / 256, 256, 0, s>>>(d_key2, d_idx2, d_ev, d_lines, d_shr, d_way, d_st, nev, ways,
                                                        nwords);
    };
    // ---- correctness first (bit-exact against the CPU fold of the same sweep)
    run_l();
    run_f();
    CK(hipStreamSynchronize(s));
    CK(hipGetLastError());
    std::vector<uint64_t> qd(nvis);
    std::vector<int32_t> way(nev);
    std::vector<uint32_t> st(nev);
    CK(hipMemcpy(qd.data(), d_qd, nvis * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(way.data(), d_way, nev * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(st.data(), d_st, nev * 4, hipMemcpyDeviceToHost));
    size_t bad_l = 0, bad_f = 0;
    for (uint32_t i = 0; i < nvis; i++) bad_l += qd[i] != qd_want[i];
    for (uint32_t i = 0; i < nev; i++) bad_f += way[i] != ev[i].way || st[i] != ev[i].fstate;

    // ---- timing: HIP events around `reps` launches of each phase, then of the
    // whole (L + F) sweep captured once in a graph and replayed
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](auto&& body) {
        for (int i = 0; i < 3; i++) body();
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; i++) body();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return 1e3 * ms / reps;   // µs
    };
    const double us_l = timed(run_l);
    const double us_f = timed(run_f);
    const double us_lf = timed([&] {
        run_l();
        run_f();
    });
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    run_l();
    run_f();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const double us_graph = timed([&] { CK(hipGraphLaunch(ge, s)); });
    CK(hipStreamSynchronize(s));
    std::printf("{\"window_requests\": %u, \"links\": %u, \"visits\": %u, \"max_visits_per_link\": %u, "
                "\"home_events\": %u, \"home_sets\": %u, \"l_mismatches\": %zu, \"f_mismatches\": %zu, "
                "\"reps\": %d, \"us_phase_l\": %.2f, \"us_phase_f\": %.2f, \"us_sweep_streamed\": %.2f, "
                "\"us_sweep_graph\": %.2f}\n",
                W, nlinks, nvis, maxv, nev, nslots, bad_l, bad_f, reps, us_l, us_f, us_lf, us_graph);
    return bad_l || bad_f ? 3 : 0;
}
