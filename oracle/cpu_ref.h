/* cpu_ref.h — TEST INFRASTRUCTURE ONLY.  C API of the CPU restatement of the
 * reference uncore (oracle/cpu_ref.cpp).  Imported only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker /
 * baseline — never by the product path. */
#ifndef PU_CPU_REF_H
#define PU_CPU_REF_H

#include <stddef.h>
#include <stdint.h>

#include "../include/primeuncore.h"

#ifdef __cplusplus
extern "C" {
#endif

void* cpuref_create(const pu_sim_cfg* cfg, char* err, size_t errcap);
void cpuref_destroy(void* h);
int cpuref_alloc_core(void* h, int prog, int thread);
/* prime.cpp:120-137 loop over reqs; delays may be NULL.  Returns 0 or the
 * index+1 of the first request whose running batch delay went negative. */
long cpuref_run(void* h, const pu_req* reqs, size_t n, int32_t* delays);
/* Replay mode bits: closed loop (timer_i += the core's earlier batch delays,
 * core_manager.cpp:265), no halt (System::access semantics), and the per-
 * message stop of one receive thread among several (the server). */
#define CPUREF_CLOSED 1
#define CPUREF_NOHALT 2
#define CPUREF_MSGHALT 4   /* a negative running delay skips the rest of that message, and its receive
                              thread (pu_req.tag & 63) never receives again (the server) */
#define CPUREF_MSGSKIP 8   /* ... skips the rest of that message only (uncore_access callers) */
int cpuref_set_mode(void* h, int mode);
int cpuref_stats(void* h, pu_stats* out);
int cpuref_completion(void* h, int64_t* out, size_t n);
/* Per-cache counters: level l (0..num_levels-1) or l == num_levels for the
 * directory slices; out holds ncaches*4 entries (ins, miss, evict, wb). */
int cpuref_cache_counters(void* h, int level, uint64_t* out, size_t n);

/* Network::transmit sequence on a fresh mesh (network.cpp:97-160); st gets
 * the network counters. */
int cpuref_network_run(int num_nodes, int net_type, int data_width, int header_flits, uint64_t router_delay,
                       uint64_t link_delay, uint64_t inject_delay, const int32_t* src, const int32_t* dst,
                       const int32_t* len, const uint64_t* timer, size_t n, uint64_t* delay_out, pu_stats* st);

/* Graphite history-tree queue model alone: min_proc, (t_i, p_i) -> delay_i. */
int cpuref_queue_run(uint64_t min_proc, const uint64_t* t, const uint64_t* p, size_t n,
                     uint64_t* delay_out, uint64_t* mg1_calls);

#ifdef __cplusplus
}
#endif
#endif
