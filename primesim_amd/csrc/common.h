// common.h — host-side helpers shared by the C-ABI translation units.
#pragma once

#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/primeuncore.h"

namespace pu {

// Records a message for pu_last_error() and returns `code`.
int set_error(int code, const std::string& msg);

// pu_run_device with extra kernel flags (PU_KF_*, geometry.h): the server's
// per-receive-thread stop.  use_replay_mode = false launches open-loop whatever
// pu_set_replay_mode left on the handle (live clients' timers are real).
int run_device_flags(pu_handle* h, const pu_req* d_reqs, const uint64_t* d_off, int32_t* d_delay,
                     uint32_t extra_flags, bool use_replay_mode = true);
// RunState.limit_at of replicas [0, n) after the last launch: the index into
// that launch's request array of the first request that raised a
// PU_ERRF_LIMITS bit (UINT64_MAX: none).
int limit_positions(pu_handle* h, uint64_t* out, size_t n);

// ThreadSched (reference src/thread_sched.cpp:55-91) with its quirks: the
// first free core is taken, a busy core is marked with its prog id, a core is
// freed only while core_stat == 1, and getCoreId inserts 0 for an unknown
// (prog, thread) through std::map::operator[].  The map's (prog, thread) order
// is the order ThreadSched::report prints.
struct Sched {
    std::vector<int> stat;
    std::map<std::pair<int, int>, int> map;
    int alloc(int prog, int th) {
        for (size_t i = 0; i < stat.size(); i++)
            if (stat[i] == 0) {
                stat[i] = prog;
                map[{prog, th}] = (int)i;
                return (int)i;
            }
        return -1;
    }
    int dealloc(int prog, int th) {
        int c = map[{prog, th}];
        if (c >= 0 && c < (int)stat.size() && stat[(size_t)c] == 1) {
            stat[(size_t)c] = 0;
            return 1;
        }
        return 0;
    }
    int get(int prog, int th) { return map[{prog, th}]; }
};

}  // namespace pu
