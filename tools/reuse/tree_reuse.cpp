// tree_reuse.cpp — ANALYSIS BUILD (not product, not oracle): the CPU
// restatement (oracle/cpu_ref.cpp, compiled in with its CPUREF_TRACE hook)
// plus a recorder of every link visit: which link, whether it took the tree
// branch of computeQueueDelay (queue_model_history_tree.cpp:64-112, the
// branch whose free-interval ring the lone wave stages and writes back), and
// the index (from the front of the sorted free-interval list) of the
// interval the tree search stopped at.  The recorder keeps the move-to-front stack of the
// links that took the tree branch, so each tree visit's LRU stack distance
// (distinct tree-visited links since its link's last tree visit) is known:
// the hit rate an on-chip cache of the last K rings would have.
// Driven by tools/reuse/tree_reuse.py through the cpuref_* C API.
#define CPUREF_TRACE 1
#include "../../oracle/cpu_ref.cpp"

#include <cstdint>
#include <vector>

namespace {
constexpr int kMaxDist = 512;
struct Rec {
    bool on = false;
    std::vector<uint32_t> mtf;                      // tree-visited links, most recent first
    uint64_t hist[kMaxDist + 1] = {};               // [d]: stack distance d; [kMaxDist]: beyond (or first)
    uint64_t visits = 0, tree = 0, tree_ks = 0;     // link visits, tree visits, summed found indices
    uint64_t khist[128] = {};                       // tree visits by found index
    uint64_t all_hist[kMaxDist + 1] = {};           // the same over every link visit
    std::vector<uint32_t> all_mtf;
} g;

void mtf_push(std::vector<uint32_t>& s, uint64_t* hist, uint32_t link) {
    size_t d = 0;
    for (; d < s.size() && s[d] != link; d++) {}
    if (d < s.size()) {
        hist[d < (size_t)kMaxDist ? d : kMaxDist]++;
        s.erase(s.begin() + (long)d);
    } else {
        hist[kMaxDist]++;
        if (s.size() >= (size_t)kMaxDist) s.pop_back();
    }
    s.insert(s.begin(), link);
}
}  // namespace

void cpuref_trace_link(size_t link, bool tree, size_t k) {
    if (!g.on) return;
    g.visits++;
    mtf_push(g.all_mtf, g.all_hist, (uint32_t)link);
    if (!tree) return;
    g.tree++;
    g.tree_ks += k;
    g.khist[k < 128 ? k : 127]++;
    mtf_push(g.mtf, g.hist, (uint32_t)link);
}

extern "C" {
// start (on = 1, counts cleared; the stacks keep their history) or stop recording
void trace_enable(int on) {
    g.on = on != 0;
    if (on) {
        for (auto& h : g.hist) h = 0;
        for (auto& h : g.all_hist) h = 0;
        g.visits = g.tree = g.tree_ks = 0;
        for (auto& h : g.khist) h = 0;
    }
}
// out: [0] link visits, [1] tree visits, [2] summed found indices at tree visits,
// then kMaxDist + 1 tree-visit stack-distance bins, then kMaxDist + 1 bins over
// all visits, then 128 bins of tree visits by found index
int trace_read(uint64_t* out, int n) {
    const int need = 3 + 2 * (kMaxDist + 1) + 128;
    if (n < need) return -need;
    out[0] = g.visits;
    out[1] = g.tree;
    out[2] = g.tree_ks;
    for (int i = 0; i <= kMaxDist; i++) out[3 + i] = g.hist[i];
    for (int i = 0; i <= kMaxDist; i++) out[3 + kMaxDist + 1 + i] = g.all_hist[i];
    for (int i = 0; i < 128; i++) out[3 + 2 * (kMaxDist + 1) + i] = g.khist[i];
    return need;
}
}
