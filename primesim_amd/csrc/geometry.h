// geometry.h — replica memory layout and derived geometry, shared by the
// host (uncore.cpp) and the HIP engine (engine.hip).
//
// One replica = one complete uncore (reference System, system.h:80-130) laid
// out structure-of-arrays in a single HBM arena:
//
//   per data-cache level l (reference Cache, cache.h:102-164):
//     meta[l]  : ncaches*nsets*nways x LineMeta (16 B: tag, prog id, state)
//     ts[l]    : ncaches*nsets*nways x int64 LRU timestamps
//     alive[l] : ncaches x u32 (reference creates caches lazily, system.cpp:172)
//     cnt[l]   : ncaches x 4 x u64 (ins, miss, evict, wb)
//   directory / shared-LLC slices (one per network node):
//     dline    : N*csets*nways x DirLine (24 B: tag, ts, packed prog/state/sharers);
//                csets <= nsets: only the sets an address can reach at that
//                home (DirGeo)
//                sharers (std::set<int> in the reference, iterated ascending)
//                are held inline as up to 4 sorted 12-bit ids; a larger set
//                moves to a full-map bitmap taken from a per-replica pool
//     pool     : pool_entries x nwords x u64 bitmaps + a free stack
//     dalive, dcnt : per slice
//   queues (Graphite history tree restated as a ring of sorted free intervals):
//     qhdr : nqueues x 32-B packed header (visit counts of the two packet
//            lengths -> the M/G/1 moments, ring cursor, newest finish, the
//            first interval start, so the M/G/1-vs-tree decision of a hop
//            needs the header only; engine.hip)  — links first, then buses
//     qring: nqueues x 128 x {first,second} (2 KB)
//   dram : banks x DramBank (opt-in bank model, pu_dram_cfg; absent when off)
//   stats (EngineStats), per-core completion cycles, run state.
//
// Lane ownership inside the wavefront that runs a replica: way w of any set
// is always read and written by lane w; sharer word k by lane k; queue ring
// slot s by lane s % 64; every scalar record by lane 0.  Values move between
// lanes only through registers (readlane / shuffles), so every memory
// read-after-write is a same-thread program-order dependency.
#pragma once

#include <stddef.h>
#include <stdint.h>

#define PU_QRING 128          // ring capacity (history tree holds <= 100 intervals)
#define PU_QMAX 100           // QueueModelHistoryTree::_max_free_interval_size
#define PU_MAX_WAYS 64        // ways per set of the ahead-of-time kernels (one lane per way)
#define PU_MAX_WAYS_WIDE 4096  // compiled configurations walk wider sets in 64-way chunks
#define PU_MAX_NWORDS 1024    // sharer bitmap words -> up to 65536 LLC nodes (16-bit inline ids)

// Network geometry helpers shared by host and engine.
static inline void pu_set_net_magic(int w, int header_flits, int data_width, int blk_len, uint64_t* w_magic,
                                    uint64_t* w2_magic, int32_t* w2, int32_t* blk, int32_t* plen_blk) {
    const uint64_t ww = (uint64_t)w * (uint64_t)w;
    *w_magic = ((1ull << 32) + (uint64_t)w - 1) / (uint64_t)w;
    *w2_magic = ((1ull << 32) + ww - 1) / ww;
    *w2 = (int32_t)ww;
    *blk = blk_len;
    // network.cpp:104: header_flits + (int)ceil((double)data_len / data_width), integer form
    *plen_blk = blk_len >= 0 ? header_flits + (blk_len + data_width - 1) / data_width : 0;
}

struct LineMeta {
    uint64_t tag;
    int32_t id;
    uint32_t state;
};

// Directory / shared-LLC line (reference Line, cache.h:77-87, with sharer_set),
// 24 B (measured: 32-B lines made the C4 bench 3.5% slower):
//   w bits  0-47  sharers: up to 4 LLC ids ascending, 12 bits each (<= 4096
//                 nodes; above: 3 ids of 16 bits, DirGeo.sh_wide), or the
//                 pool index of a full-map bitmap
//         bits 48-50  sharer count 0..4, 7 = pool
//         bits 51-53  state
//         bits 54-63  program id if 0 <= id < 1023; 1023 = escaped: the full int
//                     id (InsMem::prog_id) is in the side array DirGeo.off_prog
// The engine works on the unpacked form (16-bit inline ids, nsh PU_SH_POOL).
struct DirLine {
    uint64_t tag;
    int64_t ts;
    uint64_t w;
};
#define PU_SH_INLINE 4
#define PU_SH_POOL 0xFF
#define PU_DIR_PROG_ESC 1023u

// The prune of a full history (size >= 100 at the start of
// computeQueueDelay, queue_model_history_tree.cpp:49-55) is applied eagerly at
// the end of the tree op that fills it — nothing observes the tree in
// between, and an M/G/1 visit never grows it — so the header needs the tree's
// minimum (the M/G/1 test) but not the one after it.
// The engine's packed header is 32 B: a = {n | head, n1 | count}
// (visit counts as exact doubles, the ring cursor in their low bits), b =
// {newest, f0}; every visit rewrites it (one aligned 32-B read-modify-write),
// and the consecutive queues of a route segment share a 128-B line four at a
// time (engine.hip explains the exact moments).  The unit hooks' wide header
// (any packet length) is 48 B as two arrays: {a, b} of every queue (a = {n,
// Σs}, b = {Σs², newest}, 32 B), then c of every queue ({head, count, f0}, 16 B).
constexpr uint32_t PU_HDR_BYTES = 32;                      // per queue, the engine
constexpr uint32_t PU_HDR_AB = 32, PU_HDR_C = 16;          // wide header pieces (unit hooks)
constexpr uint32_t PU_HDR_WIDE_BYTES = PU_HDR_AB + PU_HDR_C;

struct QueueSlot {
    uint64_t first;
    uint64_t second;
};

// Accumulated by the kernel (atomic adds at the end of each launch).
struct EngineStats {
    uint64_t net_accesses, net_distance, net_total_delay, net_router_delay, net_link_delay,
        net_inject_delay, dram_accesses, total_bus_contention;
    int64_t total_num_broadcast;
    uint64_t link_flits, mg1_calls, lockdown_calls, bus_accesses, requests, error_flags;
    uint64_t dram_row_hits, dram_row_empty, dram_row_conflicts, dram_bank_wait;
    // per-level {ins, miss, evict, wb} sums kept by the compiled configuration
    // when Geo.cnt_sum (levels 0-3, [PU_CNT_DIR] the directory slices,
    // [PU_CNT_TLB] the TLBs); the host adds them to the per-cache counters
    uint64_t lvl_cnt[6][4];
};
#define PU_CNT_DIR 4
#define PU_CNT_TLB 5

// One DRAM bank of the opt-in bank model (pu_dram_cfg): the cycle it is free
// again and its open page + 1 (0 = closed).  Zeroed at reset: every bank
// closed and free from cycle 0.
struct DramBank {
    int64_t ready;
    uint64_t open;
};

struct LevelGeo {
    uint64_t nsets, nways, block;
    int32_t offbits, idxbits, access_time, share;
    int32_t ncaches, nchildren, has_bus, bus_q0;   // bus queue index of cache 0
    uint64_t off_meta, off_ts, off_alive, off_cnt;
};

// Only the sets some address can reach at a home are stored: the home id and
// the set index are both taken from the bits above the block offset
// (system.cpp:921-936, cache.cpp:145-152), so every set a home sees is
// congruent to it modulo G' = 2^cset_shift.  A home's set s is stored at
// compact index s >> cset_shift, csets = nsets >> cset_shift per home.
struct DirGeo {
    uint64_t nsets, nways, block, csets;
    int32_t offbits, idxbits, access_time, nwords;
    int32_t pool_entries, cset_shift;
    int32_t sh_wide, sh_cap;   // > 4096 LLC nodes: inline sharer ids are 16-bit, 3 fit (else 12-bit, 4)
    uint64_t off_line, off_pool, off_pool_free, off_alive, off_cnt;
    uint64_t off_prog;     // int32 per line: the full program id of escaped lines
};

// Per-core TLBs and the first-touch page table (reference system.cpp:897-918,
// page_table.cpp:56-72): TLB sets like a data cache (LineMeta + ts) plus the
// physical page per way; the page map is an open-addressing table of
// PageEnt (linear probing, never deleted), numbered in processing order.
struct TlbGeo {
    uint64_t nsets, nways, page_size;
    int32_t offbits, idxbits, access_time, page_miss_delay;
    uint64_t off_meta, off_ts, off_ppage, off_cnt;
    uint64_t off_pages, pages_cap;    // pages_cap: power of two
};
struct PageEnt {
    uint64_t vpage;
    int32_t prog;
    uint32_t used;
    uint64_t ppage;
    uint64_t _pad;
};

struct Geo {
    int32_t num_cores, num_levels, sys_type, protocol_type;
    int32_t max_num_sharers, shared_llc, tlb_enable, dram_access_time;
    int32_t bus_latency, N, net_type, net_width;
    int32_t header_flits, data_width, nlinks, nqueues;
    int32_t home_offbits, home_mask_bits;
    int32_t blk_len, plen_blk;      // last-level block size and its packet length (header + ceil(blk/dw))
    uint64_t w_magic, w2_magic;     // ceil(2^32 / w), ceil(2^32 / w^2): node id -> mesh coordinates
    int32_t w2;                     // (exact division by multiply-high for ids < 2^16)
    int32_t cnt_sum;                // 1 (no verbose_report): the compiled configuration keeps per-level
                                    // {ins, miss, evict, wb} sums (EngineStats.lvl_cnt) instead of per-cache
                                    // counters, and no directory alive bits (only the verbose report lists them)
    uint64_t router_delay, link_delay, inject_delay;
    LevelGeo lv[4];
    DirGeo dir;
    TlbGeo tlb;
    uint64_t off_qhdr, off_qring, off_stats, off_completion, off_run;
    uint64_t off_core_shift;        // closed-loop replay: int64 per core (sum of its batch delays)
    // DRAM bank model (dram_banks = 0: the reference's fixed latency)
    int32_t dram_banks, dram_bank_shift, dram_row_shift, dram_t_rcd;
    int32_t dram_t_rp, dram_t_burst;
    uint64_t off_dram;              // dram_banks x DramBank
    uint64_t replica_bytes;
};

// Kernel flags (per launch).
// Replica pool (pu_run_device_pool): the scheduling words shared by the host
// and the kernel.  sched[0] = next unstarted replica (the queue head);
// sched[PU_POOL_SLOT0 + w] = replica + 1 held by slot w (0 = none), then
// (from the even word PU_POOL_BUSY0) one uint64 per slot: the s_memrealtime
// ticks (100 MHz) its wavefronts have been resident, summed over launches
// (64 bits: 32 would wrap after 43 s per slot).  All zero = nothing started.
#define PU_POOL_SLOT0 2u
#define PU_POOL_BUSY0(slots) ((PU_POOL_SLOT0 + (uint32_t)(slots) + 1u) & ~1u)
#define PU_POOL_WORDS(slots) (PU_POOL_BUSY0(slots) + 2u * (uint32_t)(slots))
#define PU_KF_NOHALT   1u   // System::access semantics: no prime.cpp:130-134 stop (pu_access)
#define PU_KF_MSGHALT  2u   // a negative running delay stops only that message's receive
                            // thread (pu_req.tag): the rest of the message and every later
                            // message with that tag are skipped (the server, prime.cpp:130-134
                            // with num_recv_threads > 1)
#define PU_KF_CLOSED   4u   // closed-loop replay: timer_i += the core's earlier batch delays
                            // (core_manager.cpp:265 `cycle += delay` after each reply)
#define PU_KF_REQ16    8u   // d_reqs holds 16-B pu_req16 records (pu_set_device_req_format;
                            // throughput launches only)

// Resident mode (pu_access / short host batches without a launch per call):
// one latency-mode workgroup stays on the GPU with the replica's queue
// headers in its CU's LDS and serves commands through a mailbox in
// host-coherent pinned memory.  The host writes the requests, then the
// command, then `seq`; the kernel (lane 0 polling `seq` with system-scope
// acquire loads) copies the requests into device memory, runs them exactly as
// one launch would (replica_loop + replica_close), writes every delay into the
// host buffer, then error flags and last_addr, and publishes `ack = seq` after
// a system-scope release.  It leaves (headers back to HBM, `exited = 1`) on a
// STOP command or after `idle` ticks without one.
#define PU_RES_RUN 0u
#define PU_RES_STOP 1u
struct PuResHost {          // written by the host (its own 64-B line), seq last
    uint64_t seq;           // command number: the kernel waits for a change
    uint32_t n;             // requests of the command (n > 1: in PuMailbox's request area)
    uint32_t flags_cmd;     // PU_KF_* of the command | (PU_RES_RUN / PU_RES_STOP) << 16
    uint64_t req0[4];       // n == 1: the request itself (a pu_req, 32 B at offset 16)
    uint64_t _pad[2];
};
struct PuResDev {           // written by the kernel (its own 64-B line)
    uint64_t ack;           // seq of the last command completed
    uint64_t err;           // the replica's EngineStats.error_flags after it
    uint64_t last_addr;     // RunState.last_addr after it (TLB translation)
    uint32_t exited, _pad0; // 1 once the kernel has left (stop or idle)
    uint32_t phase[4];      // the command's phases in s_memrealtime ticks (10 ns): request copy,
                            // replica_loop, replica_close, mailbox writes up to the ack
    uint64_t fast;          // the fast answer of a one-request command: seq (low 32 bits) | delay << 32
    uint64_t _pad;
};
static_assert(sizeof(PuResHost) == 64 && sizeof(PuResDev) == 64, "one 64-B line each");
static_assert(__builtin_offsetof(PuResHost, req0) == 16, "the inline request is lanes 1-2 of the line's 16-B pieces");
// Mailbox: {host line, device line}, then pu_req reqs[cap], then int32 delays[cap].
struct PuMailbox {
    PuResHost h;
    PuResDev d;
};

// Per-replica run state carried across launches.
struct RunState {
    int32_t batch_delay;   // prime.cpp:113 running `delay` of the open message
    int32_t halted;        // 1 once a message's delay went negative: prime.cpp:130-134
                           // prints an error and exits the handler thread, so no
                           // further request reaches the uncore
    uint64_t processed;    // requests processed so far
    int32_t pool_top;      // free entries on the sharer-bitmap pool stack
    int32_t skip_msg;      // PU_KF_MSGHALT: the open message went negative, its rest is skipped
    uint64_t page_next;    // PageTable::empty_page_num (pages allocated so far)
    uint64_t last_addr;    // address of the last request after translation (InsMem::addr_dmem)
    int64_t msg_shift;     // PU_KF_CLOSED: the open message's core shift at its first request
    uint64_t dead_tags;    // PU_KF_MSGHALT: receive threads (pu_req.tag < 64) that have exited
    uint64_t limit_at;     // last launch: index (into its request array) of the first request that
                           // raised a PU_ERRF_LIMITS bit; UINT64_MAX if none did
};
