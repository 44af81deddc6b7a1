// write_audit.cpp — ANALYSIS BUILD (not product, not oracle): the CPU
// restatement (oracle/cpu_ref.cpp with its CPUREF_TRACE hook) plus a count of
// the free-interval ring slots the engine's tree operation writes back
// (engine.hip tree_op: one slot for a shrink, the shorter side of the ring
// plus the overridden slots for a removal or a split), so the bytes the engine
// writes per access can be attributed.  Driven by
// tools/reuse/write_audit.py through the cpuref_* C API.
#define CPUREF_TRACE 1
#include "../../oracle/cpu_ref.cpp"

#include <cstdint>

namespace {
struct Audit {
    bool on = false;
    uint64_t visits = 0, tree = 0, slots = 0, removes = 0, splits = 0, shrinks = 0;
} g;
}  // namespace

void cpuref_trace_link(size_t, bool tree, size_t k) {
    if (!g.on) return;
    g.visits++;
    if (!tree) return;
    g.tree++;
    const size_t c0 = g_trace_n0, c1 = g_trace_n1;
    if (c1 == c0 + 1) {            // split (queue_model_history_tree.cpp:78-84): engine op 4
        g.splits++;
        g.slots += 2 * k + 1 < c0 ? k + 2 : c0 - k + 1;
    } else if (c1 + 1 == c0) {     // removal: engine op 3 (k == 0: the cursor moves, nothing written)
        g.removes++;
        g.slots += k == 0 ? 0 : (k < c0 - 1 - k ? k : c0 - 1 - k);
    } else {                       // one end of the interval moves: engine ops 1, 2
        g.shrinks++;
        g.slots += 1;
    }
}

extern "C" {
void audit_enable(int on) {
    g.on = on != 0;
    if (on) g = Audit{true};
}
// out: link visits, tree visits, ring slots written, splits, removals, shrinks
int audit_read(uint64_t* out, int n) {
    if (n < 6) return -6;
    out[0] = g.visits; out[1] = g.tree; out[2] = g.slots;
    out[3] = g.splits; out[4] = g.removes; out[5] = g.shrinks;
    return 6;
}
}
