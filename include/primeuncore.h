/*
 * primeuncore.h — C ABI of the MI355X-native PriME uncore timing engine.
 *
 * This is the drop-in boundary for the reference's hot path
 *   UncoreManager::uncore_access  (reference src/uncore_manager.cpp:82-85)
 *     -> System::access           (reference src/system.cpp:144-168)
 * i.e. set-associative tag/LRU lookups (Cache), directory / shared-LLC MESI
 * transitions, XY mesh Network/Link timing with the Graphite history-tree +
 * M/G/1 queue model, and fixed-latency Dram (or, opt-in, a DRAM bank model
 * with no reference counterpart: pu_dram_cfg).
 *
 * Plain C: pointers, sizes and PODs only; no exceptions cross this boundary.
 * Every entry point returns 0 (or a non-negative value) on success and a
 * negative PU_E* code on failure; pu_last_error() gives the message.
 *
 * The engine keeps R independent "replicas" of the uncore on one GPU (one
 * wavefront each).  Replica r is a complete System instance; requests for
 * replica r are processed strictly in the order given (the canonical order),
 * exactly as the reference's single-threaded msgHandler loop would
 * (reference src/prime.cpp:120-137).
 */
#ifndef PRIMEUNCORE_H
#define PRIMEUNCORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PU_MAX_LEVELS 4

/* error codes */
#define PU_OK          0
#define PU_EINVAL    (-22)
#define PU_ENOMEM    (-12)
#define PU_ENODEV    (-19)
#define PU_ERANGE    (-34)
#define PU_EIO        (-5)
#define PU_ENOTSUP   (-95)
#define PU_ESTATE    (-71)   /* engine hit a state the reference treats as UB */

/* memory request types — reference src/common.h:61-66 (MemType) */
#define PU_RD 0
#define PU_WR 1
#define PU_WB 2

/* ------------------------------------------------------------------------
 * Configuration: plain-C mirror of the reference's XmlSim/XmlSys/XmlCache/
 * XmlNetwork structs (reference src/xml_parser.h:43-100), same field
 * meaning.  `cache[]` is inline (at most PU_MAX_LEVELS levels).
 * ---------------------------------------------------------------------- */
typedef struct pu_cache_cfg {          /* XmlCache, xml_parser.h:47-55 */
    int32_t  level;
    int32_t  share;
    int32_t  access_time;
    int32_t  _pad;
    uint64_t size;
    uint64_t block_size;
    uint64_t num_ways;
} pu_cache_cfg;

typedef struct pu_net_cfg {            /* XmlNetwork, xml_parser.h:57-65 */
    int32_t  data_width;
    int32_t  header_flits;
    int32_t  net_type;                 /* 0 = 2D mesh, 1 = 3D mesh */
    int32_t  _pad;
    uint64_t router_delay;
    uint64_t link_delay;
    uint64_t inject_delay;
} pu_net_cfg;

/* DRAM bank timing (north_star stage 4).  Opt-in, no reference counterpart:
 * the reference's Dram is a fixed latency plus a counter (dram.cpp:43-47), and
 * banks = 0 (the default; a config without a <dram> element) is exactly that.
 * With banks > 0 every Dram::access call site of System (system.cpp) becomes
 * an access to one bank of an open-page DRAM at that call's cycle t:
 *   row r = addr >> log2(row_bytes);  bank = r & (banks-1);  page = r >> log2(banks)
 *   start = max(t, bank.ready)
 *   act   = 0 (page open: row hit) | t_rcd (bank closed) | t_rp + t_rcd (other page open)
 *   delay = (start - t) + act + dram_access_time
 *   bank.ready = start + act + t_burst;  bank.open = page
 * Call sites whose Dram::access delay the reference discards (write-backs)
 * still occupy the bank.  banks and row_bytes are powers of two. */
typedef struct pu_dram_cfg {
    int32_t  banks;          /* 0 = fixed latency (the reference) */
    int32_t  t_rcd;          /* activate to column command, cycles */
    int32_t  t_rp;           /* precharge, cycles */
    int32_t  t_burst;        /* cycles a bank stays busy after the column command */
    uint64_t row_bytes;      /* bytes of one row (page) of one bank, >= 64 */
} pu_dram_cfg;

typedef struct pu_sys_cfg {            /* XmlSys, xml_parser.h:69-89 */
    int32_t  sys_type;                 /* 0 directory, 1 bus */
    int32_t  protocol_type;            /* 0 full map, 1 limited pointer */
    int32_t  max_num_sharers;
    int32_t  page_size;
    int32_t  tlb_enable;
    int32_t  shared_llc;
    int32_t  verbose_report;
    int32_t  dram_access_time;
    double   cpi_nonmem;
    int32_t  num_levels;
    int32_t  num_cores;
    double   freq;
    int32_t  bus_latency;
    int32_t  page_miss_delay;
    pu_net_cfg   network;
    pu_cache_cfg directory_cache;
    pu_cache_cfg tlb_cache;
    pu_cache_cfg cache[PU_MAX_LEVELS];
    pu_dram_cfg  dram;                 /* optional <dram> element; no XmlSys counterpart */
} pu_sys_cfg;

typedef struct pu_sim_cfg {            /* XmlSim, xml_parser.h:92-100 */
    int32_t  max_msg_size;
    int32_t  num_recv_threads;
    int32_t  thread_sync_interval;
    int32_t  proc_sync_interval;
    int32_t  syscall_cost;
    int32_t  _pad;
    pu_sys_cfg sys;
} pu_sim_cfg;

/* Parse a config_prime XML file (schema of reference tools/config_prime:62-198;
 * replaces XmlParser::parse, reference src/xml_parser.cpp:684-718, including its
 * required-field counts 5/13/4/6/6/6*L and the optional max_num_sharers,
 * net_type and inject_delay).  An optional <dram> element inside <system>
 * (banks, row_bytes, t_rcd, t_rp, t_burst) fills pu_sys_cfg.dram; the
 * reference's parser ignores it.  Returns 0 or PU_EINVAL. */
int pu_config_load_xml(const char* path, pu_sim_cfg* out);
int pu_config_parse_xml(const char* text, size_t len, pu_sim_cfg* out);
/* Write the config back out in config_prime's XML layout. */
int pu_config_write_xml(const pu_sim_cfg* cfg, char* buf, size_t cap, size_t* written);

/* ------------------------------------------------------------------------
 * Requests.  One pu_req per MsgMem record (reference src/common.h:49-59),
 * already resolved to a core id (ThreadSched, reference src/thread_sched.cpp:55)
 * and tagged with the Pin process rank (prime.cpp:125 prog_id = MPI source).
 * batch_start = 1 marks the first request of a MEM_REQUESTS message: the
 * running-delay rule of prime.cpp:129 restarts there:
 *     D = 0 at batch start;  d_i = access(core, req_i, timer_i + D);  D += d_i - 1
 * ---------------------------------------------------------------------- */
typedef struct pu_req {
    uint64_t addr;         /* MsgMem.addr_dmem */
    int64_t  timer;        /* MsgMem.timer (core cycle when issued) */
    int32_t  core;         /* core id */
    int32_t  prog_id;      /* program (Pin process rank, >= 1) */
    uint8_t  mem_type;     /* PU_RD / PU_WR */
    uint8_t  batch_start;  /* 1 = first request of a message */
    uint16_t tag;          /* MPI tag of its message = receive-thread id (prime.cpp:53);
                              only the server's per-thread stop reads it, 0 elsewhere */
    int32_t  _pad1;
} pu_req;                  /* 32 bytes */

/* Compact 16-byte device request record for throughput runs whose requests
 * fit (no reference counterpart: a layout of the same MsgMem fields).
 *   a = addr_dmem
 *   b = timer (bits 0-39) | core (40-55) | prog_id (56-61) | mem_type (62)
 *       | batch_start (63);  tag is 0.
 * pu_pack_req16 packs n records and returns 0, or PU_ERANGE (out untouched
 * past the record it names in the error text) at the first that does not
 * fit: timer outside [0, 2^40), core outside [0, 2^16), prog_id outside
 * [0, 64), mem_type or batch_start above 1, or tag != 0.
 * pu_set_device_req_format(h, PU_REQ_FMT_16) makes pu_run_device,
 * pu_run_device_sliced and pu_run_device_pool read d_reqs as pu_req16
 * records (indices in d_off / d_pos count records either way); those runs
 * use the throughput kernels (a latency launch's helper reads pu_req).
 * Results are identical to the same requests as pu_req.  PU_REQ_FMT_32
 * (the default) restores pu_req.  The host batch paths always take pu_req. */
typedef struct pu_req16 {
    uint64_t a, b;
} pu_req16;
#define PU_REQ_FMT_32 0
#define PU_REQ_FMT_16 1

/* ------------------------------------------------------------------------
 * Statistics — every number System::report prints (reference
 * src/system.cpp:956-1111, network.cpp:310-323, dram.cpp:50-55) plus the
 * extra counters the parity harness obtains from the reference with
 * -Wl,--wrap.
 * ---------------------------------------------------------------------- */
typedef struct pu_level_stats {
    uint64_t ins;
    uint64_t miss;
    uint64_t evict;
    uint64_t wb;
} pu_level_stats;

typedef struct pu_stats {
    uint64_t net_accesses;          /* Network::num_access */
    uint64_t net_distance;          /* Network::total_distance (= link visits) */
    uint64_t net_total_delay;
    uint64_t net_router_delay;
    uint64_t net_link_delay;
    uint64_t net_inject_delay;
    uint64_t dram_accesses;
    uint64_t total_bus_contention;
    int64_t  total_num_broadcast;
    int32_t  num_levels;
    int32_t  _pad;
    pu_level_stats level[PU_MAX_LEVELS];   /* data caches, aggregated per level */
    pu_level_stats directory;              /* directory / shared-LLC slices */
    pu_level_stats tlb;
    /* extra counters */
    uint64_t link_flits;            /* sum of packet_len over Link::access */
    uint64_t mg1_calls;             /* QueueModelMG1::computeQueueDelay calls */
    uint64_t lockdown_calls;        /* Cache::lockDown calls (share/inval visits) */
    uint64_t bus_accesses;          /* Bus::access calls */
    uint64_t requests;              /* uncore_access calls */
    uint64_t error_flags;           /* PU_ERRF_* bits; 0 for a valid run */
    /* DRAM bank model (pu_dram_cfg.banks > 0; all 0 otherwise) */
    uint64_t dram_row_hits;         /* accesses to the open page of their bank */
    uint64_t dram_row_empty;        /* accesses to a closed bank */
    uint64_t dram_row_conflicts;    /* accesses that closed another page */
    uint64_t dram_bank_wait;        /* cycles spent waiting for a busy bank */
} pu_stats;

#define PU_ERRF_CORE_RANGE   (1ull << 0)  /* core_id >= num_cores (system.cpp:147) */
#define PU_ERRF_WB_MISS      (1ull << 1)  /* WB missed at home: NULL deref in ref (Q13) */
#define PU_ERRF_EMPTY_SHARER (1ull << 2)  /* *sharer_set.begin() on empty set */
#define PU_ERRF_QUEUE        (1ull << 3)  /* queue-model precondition violated */
#define PU_ERRF_NEG_DELAY    (1ull << 4)  /* batch delay went negative (prime.cpp:130) */
#define PU_ERRF_POOL         (1ull << 5)  /* sharer-bitmap pool exhausted (engine limit: the
                                             pool holds one entry per directory line up to
                                             2 GiB of bitmaps; PRIMEUNCORE_POOL_ENTRIES) */
#define PU_ERRF_PAGES        (1ull << 6)  /* page table 3/4 full (engine limit: 2^22 slots,
                                             raise PRIMEUNCORE_PAGE_ENTRIES) */
#define PU_ERRF_PROG         (1ull << 7)  /* no longer raised: since 0.2 directory lines
                                             carry any int prog_id (ids outside [0, 1023)
                                             escape to a side array) */
/* The bits that mean the replica stopped where the reference would have
 * continued (an engine limit) or reached a state the reference leaves undefined.
 * Not CORE_RANGE (System::access returns -1 and goes on) nor NEG_DELAY
 * (prime.cpp's own stop).  The host batch paths and the server return /
 * report PU_ESTATE for these. */
#define PU_ERRF_LIMITS (PU_ERRF_WB_MISS | PU_ERRF_EMPTY_SHARER | PU_ERRF_QUEUE | \
                        PU_ERRF_POOL | PU_ERRF_PAGES | PU_ERRF_PROG)

/* ------------------------------------------------------------------------
 * Engine lifetime and the hot path.
 * ---------------------------------------------------------------------- */
typedef struct pu_handle pu_handle;

/* Replaces UncoreManager::init (reference src/uncore_manager.cpp:46-50 ->
 * System::init system.cpp:47-141, ThreadSched::init thread_sched.cpp:44).
 * Allocates `num_replicas` independent uncores on HIP device `device`.
 * Returns NULL on failure (see pu_last_error). */
pu_handle* pu_create(const pu_sim_cfg* cfg, int num_replicas, int device);
void       pu_destroy(pu_handle* h);
/* The replica geometry the engine derives from cfg (layout offsets, set and
 * mesh parameters) as C++ source: a constexpr `Geo kJitGeo = {...};` the engine
 * can be specialised against (compile-time configuration).  Returns the full
 * length like snprintf; no reference counterpart. */
long pu_config_geo_source(const pu_sim_cfg* cfg, char* buf, size_t cap);
/* Compile-time configuration.  pu_create compiles the engine kernel for the
 * configuration's geometry with hipRTC (every cache/mesh/latency value a
 * constant) and launches that code object; compiled code objects are cached on
 * disk (PRIMEUNCORE_JIT_CACHE, else jit_cache/ beside the library).
 * PRIMEUNCORE_JIT=0, or a failed compile, runs the library's ahead-of-time
 * kernels (the same engine source for a runtime geometry).  No reference
 * counterpart (the reference's System reads its XmlSys at run time).
 * pu_config_jit_warm compiles into the cache without a GPU (1: was cached,
 * 0: compiled, PU_E* on failure); pu_compiled_config tells what handle h
 * runs: 2 the compiled configuration for every launch (the default); 1 the
 * compiled configuration for latency launches (at most one replica per CU,
 * headers in LDS) and the ahead-of-time kernels for throughput launches
 * (PRIMEUNCORE_JIT_THROUGHPUT=0; sets wider than 64 ways always take 2);
 * 0 the ahead-of-time kernels only.  pu_compiled_compiler tells which
 * compiler built the two code objects (throughput and latency kernels) handle
 * h runs: 2 hipcc for both (written by pu_config_jit_warm in a process that
 * set PRIMEUNCORE_JIT_OFFLINE=1 and has not used the GPU: the build-time
 * warm-up, tools/jit_warm.py), 1 hipRTC for both (cache misses at run time),
 * 3 one of each, 0 none. */
int pu_config_jit_warm(const pu_sim_cfg* cfg);
int pu_compiled_config(const pu_handle* h);
int pu_compiled_compiler(const pu_handle* h);
/* The 8-hex-digit tag of the engine sources this library compiles: the prefix
 * of every code object it writes to the cache (cache maintenance keeps the
 * code objects whose prefix some library still carries). */
const char* pu_jit_source_tag(void);

/* Diagnostics, no reference counterpart (tools/prof_regions.py --jit): the
 * region cycle counters of the loaded compiled-configuration kernels built
 * with PRIMEUNCORE_JIT_EXTRA=-DPU_PROF, summed over modules into out[0..n);
 * reset != 0 clears them.  Returns n, 0 when no loaded kernel counts regions,
 * < 0 on error. */
int pu_jit_prof_read(unsigned long long* out, int n, int reset);

/* Return all replicas to the just-initialised state (no reallocation). */
int        pu_reset(pu_handle* h);
int        pu_num_replicas(const pu_handle* h);
/* Device bytes held by one replica's state. */
uint64_t   pu_replica_bytes(const pu_handle* h);
/* The share of it held by the sharer-bitmap pool (full-map sets of more than
 * four LLCs).  pu_create sizes the pool exactly (one bitmap per directory line,
 * up to 2 GiB) and shrinks it, with a message on stderr, only when the
 * requested replicas would not fit the device otherwise. */
uint64_t   pu_replica_pool_bytes(const pu_handle* h);
/* Replicas this configuration's throughput kernels (time-sliced and replica
 * pool) keep resident on the device at once (one wave each; registers and LDS
 * bound it, LDS counted in the device's 1,280-B allocation units, which
 * hipOccupancy understates).  A launch over more replicas runs in several
 * rounds.  No reference counterpart (engine sizing). */
int        pu_resident_replicas(const pu_handle* h);

/* Thread -> core map (reference src/thread_sched.cpp:55-91; identical quirks:
 * first free core, a core is marked busy with prog_id, dealloc frees only
 * when core_stat == 1).  Shared by all replicas. */
int pu_alloc_core(pu_handle* h, int prog_id, int thread_id);
int pu_dealloc_core(pu_handle* h, int prog_id, int thread_id);
int pu_get_core_id(pu_handle* h, int prog_id, int thread_id);
/* The same three calls on one replica's own ThreadSched (copied from the
 * shared one on first use; the shared calls above keep updating it).  The
 * server (pu_server_*) gives every session (= replica) its own core map, as a
 * separate prime.cpp process would have.  The replica's report prints its own
 * core allocation. */
int pu_alloc_core_replica(pu_handle* h, int replica, int prog_id, int thread_id);
int pu_dealloc_core_replica(pu_handle* h, int replica, int prog_id, int thread_id);
int pu_get_core_id_replica(pu_handle* h, int replica, int prog_id, int thread_id);

/* Replay of the recorded timers (no reference counterpart; the rule is the
 * core side's, core_manager.cpp:265 `cycle += delay` after every reply):
 *   PU_REPLAY_OPEN   (default) timer_i is used as recorded;
 *   PU_REPLAY_CLOSED timer_i += the sum of the batch delays of that core's
 *                    earlier messages, as if the recording core had waited for
 *                    each reply.  The uncore (System) is untouched. */
#define PU_REPLAY_OPEN   0
#define PU_REPLAY_CLOSED 1
int pu_set_replay_mode(pu_handle* h, int mode);

/* PU_ERRF_* bits of replicas [0, n) (EngineStats.error_flags). */
int pu_error_flags(pu_handle* h, uint64_t* out, size_t n);
/* For replicas [0, n): the index, into the last launch's request array, of
 * the first request that raised a PU_ERRF_LIMITS bit (UINT64_MAX: none).
 * Every request before it was simulated exactly (the server still answers
 * the messages that ended before it). */
int pu_limit_positions(pu_handle* h, uint64_t* out, size_t n);

/* Single-request compatibility path: UncoreManager::uncore_access
 * (uncore_manager.cpp:82-85).  Operates on replica 0; `*addr` is updated in
 * place like InsMem::addr_dmem (system.cpp:916).  Returns the delay (an int,
 * negative when the reference's int wraps) or -1 for core_id >= num_cores,
 * like System::access (system.cpp:147-150).  No prime.cpp halt rule and no
 * closed-loop shift apply here: those belong to the caller's message loop. */
int pu_access(pu_handle* h, int core_id, int prog_id, int mem_type,
              uint64_t* addr, int64_t timer);
/* The same with the status out of band: returns 0 or PU_E*, and the delay
 * (any int, including a wrapped negative one, or -1 for core_id >= num_cores)
 * goes to *delay_out.  pu_access reports errors in-band, so a wrapped delay
 * that happens to equal a PU_E* code is ambiguous there; the C++ and Python
 * mirrors use this entry point. */
int pu_access_status(pu_handle* h, int core_id, int prog_id, int mem_type,
                     uint64_t* addr, int64_t timer, int32_t* delay_out);

/* Batch path from host memory: the per-message loop of prime.cpp:120-137 for
 * replica `replica`.  delay_out[i] receives uncore_access's return value for
 * reqs[i] (may be NULL).  Synchronous.  Returns 0 or PU_E*; PU_ESTATE when
 * the replica carries a PU_ERRF_LIMITS bit (an engine limit stopped it where
 * the reference would continue: later delays are 0, not the reference's). */
int pu_access_batch(pu_handle* h, int replica, const pu_req* reqs, size_t n,
                    int32_t* delay_out);

/* Resident mode (no reference counterpart; the transport under prime.cpp:129's
 * per-request uncore_access and the per-message batch): pu_access,
 * pu_access_status and pu_access_batch of at most 16,384 requests do not
 * launch a kernel per call.  The first such call starts one persistent
 * latency-mode workgroup for that replica, which keeps the replica's queue
 * headers in its CU's LDS and takes every later call through a mailbox in
 * host-coherent pinned memory (requests in, delays and error flags out), each
 * call computing exactly what one launch would.  It leaves by itself after
 * PRIMEUNCORE_RESIDENT_IDLE_MS (default 50) without a call, when another
 * replica or a launch of any kind needs the engine, on pu_reset, pu_synchronize,
 * a read of statistics, completion cycles or the report, and on pu_destroy or
 * process exit.  It needs the compiled configuration and a replica whose queue
 * headers fit one CU's LDS; otherwise (or with PRIMEUNCORE_RESIDENT=0) every
 * call launches as before.  pu_set_resident: mode 1 on, 0 off (joins a running
 * kernel), -1 query; returns the previous mode.  pu_resident_info writes up
 * to n of {kernel running, commands served, kernels launched, eligible, then
 * summed over the commands: the kernel's request-copy, message-loop, close
 * (run state and counters) and mailbox phases in 10-ns ticks (commands with a
 * full answer), the host's post-to-answer time in ns, and how many commands
 * came back as the fast answer (one request, no new error bit, no TLB: the
 * delay and the command number in one 8-B store)} and returns how many it
 * wrote. */
int pu_set_resident(pu_handle* h, int mode);
int pu_resident_info(pu_handle* h, uint64_t* out, size_t n);

/* Batch path from device memory, all replicas at once, asynchronous on
 * `hip_stream` (a hipStream_t; NULL = the engine's own stream, see
 * pu_synchronize).  Replica r
 * processes d_reqs[d_off[r] .. d_off[r+1]) and writes d_delay over the same
 * range.  d_off holds num_replicas+1 entries and lives in device memory.
 * Nothing is copied to or from the host. */
int pu_run_device(pu_handle* h, const pu_req* d_reqs, const uint64_t* d_off,
                  int32_t* d_delay, void* hip_stream);
/* Time-sliced variant for throughput runs of many replicas: replica r
 * processes d_reqs[d_pos[r] .. d_off[r+1]) in order but stops before the first
 * request that would start more than budget_us microseconds (wall clock) after
 * its wavefront started, and writes its next position back to d_pos[r]
 * (device memory, num_replicas entries).  A replica stops only between
 * requests, so calling again continues its stream exactly; results are the
 * same as one unsliced run over the same requests.  budget_us = 0: no limit. */
int pu_run_device_sliced(pu_handle* h, const pu_req* d_reqs, const uint64_t* d_off,
                         int32_t* d_delay, uint64_t* d_pos, uint64_t budget_us, void* hip_stream);
/* Replica pool: pu_run_device_sliced for more replicas than run at once (no
 * reference counterpart; throughput runs).  A launch runs `slots` wavefronts,
 * 1 <= slots <= pu_pool_slots(h) = min(num_replicas, pu_resident_replicas).
 * Each slot continues the replica it held when the previous pool launch
 * ended; a slot whose replica is done (d_pos[r] reached d_off[r+1], or the
 * replica stopped by the prime.cpp:130-134 rule: the rest of its range reads
 * 0) takes the next replica nobody has started, in index order, and goes on
 * within the same slice, so no wavefront idles while unstarted replicas
 * remain.  Per replica the results are those of pu_run_device_sliced (each
 * replica is processed in order, by one wavefront at a time).  d_sched:
 * pu_pool_words(slots) = B + 2*slots uint32 words of device memory,
 * B = (3 + slots) & ~1, all 0 before the first launch of a pool run, the same
 * slots for every launch of it (word 0 = replicas taken so far; word 1
 * unused; then per slot its replica + 1; from word B, per slot one uint64:
 * the 100-MHz ticks its wavefronts have been resident, summed over launches:
 * the busy time of the pool).
 * budget_us > 0. */
int  pu_pool_slots(pu_handle* h);
long pu_pool_words(int slots);
int  pu_run_device_pool(pu_handle* h, const pu_req* d_reqs, const uint64_t* d_off, int32_t* d_delay,
                        uint64_t* d_pos, uint32_t* d_sched, int slots, uint64_t budget_us, void* hip_stream);
int pu_set_device_req_format(pu_handle* h, int fmt);
int pu_pack_req16(const pu_req* in, size_t n, pu_req16* out);
int pu_synchronize(pu_handle* h);

/* Per-core completion cycle of the last request each core issued
 * (last timer_i + D + d_i); out has num_cores entries (-1 = no request). */
int pu_core_completion(pu_handle* h, int replica, int64_t* out, size_t n);

/* Statistics and the report text of UncoreManager::report
 * (uncore_manager.cpp:87-98 -> ThreadSched::report, System::report) for one
 * replica.  With include_time == 0 the wall-clock line is omitted so the
 * text can be compared byte-for-byte.  Returns the full length (like
 * snprintf); writes at most cap bytes including the terminating NUL. */
int pu_stats_get(pu_handle* h, int replica, pu_stats* out);
long pu_report(pu_handle* h, int replica, int include_time, char* buf, size_t cap);

/* Device-time of the last pu_run_device / pu_access_batch launch, in ms,
 * measured with HIP events on the engine's stream (a call served by the
 * resident kernel: its wall time from posting to the answer). */
double pu_last_kernel_ms(pu_handle* h);

/* UncoreManager::getSimStartTime / getSimFinishTime (uncore_manager.cpp:52-60):
 * wall-clock stamps (CLOCK_REALTIME); pu_report(include_time=1) prints their
 * difference as "Total computation time" like UncoreManager::report (:92-93). */
void pu_sim_start_time(pu_handle* h);
void pu_sim_finish_time(pu_handle* h);

const char* pu_last_error(void);
const char* pu_version(void);

/* ------------------------------------------------------------------------
 * Synthetic request streams.  Deterministic: one splitmix64
 * per core seeded seed*2^32 + core; per core timer += 1 + U{0..3}; a core
 * stops at each quantum barrier (q+1)*quantum (core_manager.cpp:104-198);
 * messages of <= max_msg requests never span a barrier; canonical order is
 * quantum-major, then core id, batch-atomic.
 * ---------------------------------------------------------------------- */
#define PU_STREAM_PRIVATE_STREAMING 1  /* C1: blackscholes-like */
#define PU_STREAM_SHARED_UNIFORM    2  /* C2: canneal-like */
#define PU_STREAM_MULTIPROGRAM      3  /* C3: SPEC-like mix, 4 programs */
#define PU_STREAM_UNIFORM_HOTSPOT   4  /* C4: uniform 2^20 lines + 64-line hotspot */
#define PU_STREAM_PRODUCER_CONSUMER 5  /* C5: core pairs sharing buffers */
#define PU_STREAM_UNIFORM           6  /* C4(i): pure uniform */

typedef struct pu_stream_params {
    int32_t  kind;             /* PU_STREAM_* */
    int32_t  num_cores;
    uint64_t seed;
    int32_t  quantum;          /* thread_sync_interval, e.g. 1000 */
    int32_t  num_quanta;       /* quanta to generate */
    int32_t  max_msg;          /* max_msg_size, e.g. 100 */
    int32_t  num_progs;        /* programs; core c belongs to prog 1 + c*num_progs/num_cores */
    int64_t  max_requests;     /* stop after this many requests (<=0: no cap) */
    int32_t  write_pct;        /* percent writes; <0 = kind default */
    int32_t  _pad;
} pu_stream_params;

/* Number of requests the stream holds (call first to size the buffer). */
int64_t pu_stream_count(const pu_stream_params* p);
/* Fill out[0..cap) in canonical order; returns the number written or PU_E*. */
int64_t pu_stream_generate(const pu_stream_params* p, pu_req* out, size_t cap);
/* The (prog_id, thread_id) of core c in a generated stream. */
int pu_stream_thread_of(const pu_stream_params* p, int core, int* prog_id, int* thread_id);

/* Resumable streams: the same requests as pu_stream_generate, produced in
 * consecutive chunks (concatenating the chunks gives exactly the one-shot
 * stream).  pu_stream_next returns the number written (< n at the end).
 * pu_stream_next_many advances `count` streams by up to n_each requests each
 * on `threads` host threads (<= 0: all cores), stream i writing
 * out[i*stride ...]; returns the smallest count written. */
typedef struct pu_stream pu_stream;
pu_stream* pu_stream_open(const pu_stream_params* p);
void       pu_stream_close(pu_stream* s);
int64_t    pu_stream_next(pu_stream* s, pu_req* out, size_t n);
int64_t    pu_stream_position(const pu_stream* s);
int64_t    pu_stream_next_many(pu_stream* const* s, int count, pu_req* out, size_t n_each,
                               size_t stride, int threads);

/* Trace files ("PUTRACE1": header, thread table, pu_req records). */
int pu_trace_write(const char* path, const pu_req* reqs, size_t n,
                   const int32_t* thread_prog, const int32_t* thread_id, int num_threads);

/* ------------------------------------------------------------------------
 * MsgMem message logs: the receive stream of the
 * reference's uncore server, message by message as prime.cpp:53 gets it
 * (MPI source rank + the MsgMem records of reference src/common.h:49-59, 24 B
 * each).  File: "PRIMEMSG" | u32 1 | u32 24, then per message
 * i32 source | i32 n_records | records.  Replay applies prime.cpp:55-137:
 * NEW_THREAD -> allocCore, THREAD_FINISHING -> deallocCore, MEM_REQUESTS ->
 * getCoreId + requests 1..addr_dmem-1 with prog_id = source; other control
 * messages have no uncore effect, PROGRAM_EXITING ends the log.
 * ---------------------------------------------------------------------- */
typedef struct pu_msglog pu_msglog;
/* Open for replay; num_cores sizes the log's own ThreadSched (used when
 * pu_msglog_next gets h == NULL). */
pu_msglog* pu_msglog_open(const char* path, int num_cores);
/* Next requests (<= cap) in receive order, core ids resolved through h's
 * ThreadSched (h may be NULL: the log's own).  batch_start marks each
 * message's first request.  Returns the count, 0 at the end, or PU_E*. */
int64_t    pu_msglog_next(pu_msglog* L, pu_handle* h, pu_req* out, size_t cap);
int64_t    pu_msglog_messages(const pu_msglog* L);
/* Capture: create a log and append messages as received (the three fwrite
 * calls a prime.cpp build would add after MPI_Recv). */
pu_msglog* pu_msglog_create(const char* path);
int        pu_msglog_append(pu_msglog* L, int32_t source, const void* records, int32_t n_records);
int        pu_msglog_close(pu_msglog* L);
/* A canonical-order request stream written as the log its cores would have
 * sent (NEW_THREAD per thread, one MEM_REQUESTS message per batch). */
int pu_msglog_from_requests(const char* path, const pu_req* reqs, size_t n, const int32_t* thread_prog,
                            const int32_t* thread_id, int num_threads, const int32_t* core_thread,
                            int num_cores);

/* ------------------------------------------------------------------------
 * Server front-end: prime.cpp's message loop
 * (reference src/prime.cpp:35-137, main :142-233) behind a Unix-domain socket
 * instead of MPI, feeding the engine a round at a time.
 *
 * A session is one simulation (one prime.cpp process in the reference) and
 * runs on one replica; its clients are the Pin processes of that simulation,
 * identified by their rank (the MPI source, = prog_id).  Clients exchange
 * exactly what core_manager.cpp sends and receives over MPI: MsgMem buffers
 * (24-B records, common.h:49-59) sent with a tag, and int replies received
 * on a tag (pu_client_*; INTEGRATION.md shows the core_manager.cpp edit).
 * Every message is handled with prime.cpp's rules: PROCESS_STARTING /
 * PROCESS_FINISHING / INTER_PROCESS_BARRIERS maintain the program list and
 * release barriers (replies on tag 0), NEW_THREAD allocates a core (reply
 * core % num_recv_threads on tag thread), THREAD_FINISHING frees it,
 * MEM_REQUESTS runs requests 1..msg[0].addr_dmem-1 with the running delay of
 * prime.cpp:129 (reply: the batch delay on tag thread), PROGRAM_EXITING ends
 * one handler thread; a session ends after num_recv_threads of them and
 * writes its report (UncoreManager::report) to <report_prefix>_<session>.
 * A negative batch delay stops that message's receive thread like
 * prime.cpp:130-134 (its handler returns): the message gets no reply, later
 * messages on its tag are never received, and once every receive thread has
 * returned the report is written and the session's connections are closed.
 * An engine limit (PU_ERRF_LIMITS) ends the session with an error instead of
 * replying with delays that are no longer the reference's.
 *
 * Rounds: each round reads everything the clients have sent, takes from every
 * session its pending messages up to the first control message that follows
 * a MEM_REQUESTS message (so control messages never overtake a batch whose
 * outcome could stop the session), and runs all sessions' MEM_REQUESTS
 * batches in ONE engine launch (pu_run_device: one wavefront per session),
 * then sends the replies.  Per session the result is the sequential one of
 * prime.cpp with one receive thread, in the order the server received the
 * messages.
 * ---------------------------------------------------------------------- */
typedef struct pu_server pu_server;

typedef struct pu_server_opts {
    const char* socket_path;   /* Unix-domain socket path to listen on */
    const char* report_prefix; /* session s writes <prefix>_<s> when it ends; NULL = no file */
    int num_sessions;          /* sessions 0..n-1 (<= replicas); run() returns when all have ended */
    int num_recv_threads;      /* XmlSim::num_recv_threads (prime.cpp:182); 0 = 1 */
    int max_msg_size;          /* XmlSim::max_msg_size: records per message beyond the header; 0 = 100 */
    int verbose;               /* print prime.cpp's "[PriME] ..." progress lines */
} pu_server_opts;

typedef struct pu_server_stats {
    uint64_t rounds;           /* service rounds that handled at least one message */
    uint64_t launches;         /* engine launches (rounds with MEM_REQUESTS) */
    uint64_t messages;         /* MsgMem messages handled */
    uint64_t requests;         /* memory requests sent to the engine */
    int32_t  sessions_ended;
    int32_t  sessions_halted;  /* a receive thread stopped by a negative batch delay */
    int32_t  sessions_failed;  /* ended by an engine limit (PU_ERRF_LIMITS): no exact reply possible */
    int32_t  _pad;
} pu_server_stats;

/* Host executor: runs one session's requests in order and writes each
 * request's uncore_access delay (the engine's per-request output).  Lets the
 * protocol be exercised without a GPU (tests); the product path is
 * pu_server_create on an engine handle.  Returns 0, a negative PU_E* (the
 * round fails), or positive PU_ERRF_* bits the session's replica now carries. */
typedef int (*pu_exec_fn)(void* ctx, int session, const pu_req* reqs, size_t n, int32_t* delays);

/* Serve engine handle h (not owned; sessions <= pu_num_replicas(h)). */
pu_server* pu_server_create(pu_handle* h, const pu_server_opts* o);
pu_server* pu_server_create_exec(pu_exec_fn fn, void* ctx, int num_cores, const pu_server_opts* o);
/* Serve until every session has ended or pu_server_stop (which ends this run;
 * calling pu_server_run again resumes serving); 0 or PU_E*. */
int  pu_server_run(pu_server* s);
/* One round, waiting up to timeout_ms for the first message; returns the
 * number of messages handled (>= 0) or PU_E*. */
int  pu_server_round(pu_server* s, int timeout_ms);
void pu_server_stop(pu_server* s);     /* thread-safe */
int  pu_server_get_stats(pu_server* s, pu_server_stats* out);
void pu_server_destroy(pu_server* s);

/* Client: the MPI calls of core_manager.cpp.  One client per Pin thread (or a
 * mutex around a shared one).  send = MPI_Send(records, n*24, MPI_CHAR, 0,
 * tag); recv = MPI_Recv(value, 1, MPI_INT, 0, tag) with MPI's matching (a
 * reply sent before the receive is posted waits at the server). */
typedef struct pu_client pu_client;
pu_client* pu_client_connect(const char* socket_path, int session, int rank);
int  pu_client_send(pu_client* c, int tag, const void* records, int n_records);
int  pu_client_recv(pu_client* c, int tag, int32_t* value);
void pu_client_close(pu_client* c);

/* ------------------------------------------------------------------------
 * Unit hooks: run one engine component alone on the GPU (one wavefront), for
 * the component-level parity tests.
 * ---------------------------------------------------------------------- */
/* QueueModelHistoryTree::computeQueueDelay sequence on a fresh queue
 * (queue_model_history_tree.cpp:42-125 + queue_model_m_g_1.cpp). */
int pu_unit_queue_run(uint64_t min_proc, const uint64_t* t, const uint64_t* p, size_t n,
                      uint64_t* delay_out, uint64_t* mg1_calls, int device);
/* QueueModelMG1::computeQueueDelay (queue_model_m_g_1.cpp:16-42) evaluated by
 * the engine's M/G/1 arithmetic on n given queue states: state i is
 * _num_arrivals = num_arrivals[i] (< 2^53), _sigma_service_time = sum[i],
 * _sigma_service_time_square = sum_sq[i], _newest_arrival_time = newest[i];
 * wait_out[i] = the queue delay.  The arithmetic fuzz of the M/G/1 branch. */
int pu_unit_mg1_run(const uint64_t* num_arrivals, const double* sum, const double* sum_sq,
                    const uint64_t* newest, size_t n, uint64_t* wait_out, int device);
/* Network::transmit sequence on a fresh mesh (network.cpp:97-160); st gets
 * the network counters. */
int pu_unit_network_run(int num_nodes, int net_type, int data_width, int header_flits,
                        uint64_t router_delay, uint64_t link_delay, uint64_t inject_delay,
                        const int32_t* src, const int32_t* dst, const int32_t* len,
                        const uint64_t* timer, size_t n, uint64_t* delay_out, pu_stats* st,
                        int device);

#ifdef __cplusplus
}
#endif
#endif /* PRIMEUNCORE_H */
