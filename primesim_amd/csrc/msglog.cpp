// msglog.cpp — MsgMem message logs: the uncore's receive stream, recorded and
// replayed.
//
// The reference records no traces.  What its uncore sees is
// a sequence of MPI messages, each a buffer of MsgMem records (reference
// src/common.h:49-59) received in prime.cpp:53 with its MPI source rank; the
// first record's message_type (union with timer) selects the handler branch
// (prime.cpp:55-137).  A log stores exactly that: per message, the source rank
// and the records as received, in the reference's own 24-byte layout, so a
// maintainer can capture one with three fwrite calls after MPI_Recv
// (INTEGRATION.md).  Replaying a log applies the same handler semantics:
//   NEW_THREAD        -> ThreadSched::allocCore(source, msg[0].mem_size)  (prime.cpp:90-108)
//   THREAD_FINISHING  -> ThreadSched::deallocCore(source, msg[0].mem_size) (prime.cpp:110-114)
//   MEM_REQUESTS      -> core = getCoreId(source, thread = msg[0].mem_size); requests
//                        msg[1 .. msg[0].addr_dmem - 1], prog_id = source   (prime.cpp:120-137)
//   process start/finish, barriers, PROGRAM_EXITING: no uncore effect.
// Requests come out as pu_req in receive order with batch_start on the first
// request of each message (the running-delay restart of prime.cpp:123).
//
// File layout: "PRIMEMSG" | u32 version (1) | u32 sizeof(MsgMem) (24), then per
// message: i32 source | i32 n_records | n_records x MsgMem.

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <utility>
#include <vector>

#include "../../include/primeuncore.h"
#include "common.h"

namespace {

// reference MsgMem (common.h:49-59) as laid out by the x86-64 ABI
struct MsgMemRec {
    uint8_t mem_type;     // bool: 1 write, 0 read
    uint8_t _pad[3];
    int32_t mem_size;     // thread id in a message header
    uint64_t addr_dmem;   // record count in a message header
    int64_t timer;        // message_type in a message header
};
static_assert(sizeof(MsgMemRec) == 24, "MsgMem is 24 bytes");

constexpr char kMagic[8] = {'P', 'R', 'I', 'M', 'E', 'M', 'S', 'G'};
// MessageTypes (common.h:38-47)
constexpr int64_t kProcessStarting = -3, kProcessFinishing = -1, kBarrier = -2, kNewThread = -4,
                  kThreadFinishing = -8, kProgramExiting = -5;

}  // namespace

// ThreadSched for a log replayed without an engine handle (conversion only):
// the same rules as the handle's (pu::Sched, thread_sched.cpp:55-91).
using LocalSched = pu::Sched;

struct pu_msglog {
    FILE* f = nullptr;
    LocalSched sched;              // used when no handle is given
    bool write = false;
    bool ended = false;            // PROGRAM_EXITING seen or end of file
    std::vector<MsgMemRec> msg;    // the message being converted
    size_t next = 1;               // next request record of `msg` (MEM_REQUESTS)
    size_t len = 0;                // records of `msg` that are requests + 1
    int32_t source = 0;
    int32_t core = 0;
    int64_t messages = 0;
};

extern "C" {

pu_msglog* pu_msglog_open(const char* path, int num_cores) {
    FILE* f = path ? std::fopen(path, "rb") : nullptr;
    if (!f) {
        pu::set_error(PU_EIO, "cannot open message log");
        return nullptr;
    }
    char magic[8];
    uint32_t ver = 0, rec = 0;
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, kMagic, 8) != 0 || std::fread(&ver, 4, 1, f) != 1 ||
        std::fread(&rec, 4, 1, f) != 1 || ver != 1 || rec != sizeof(MsgMemRec)) {
        std::fclose(f);
        pu::set_error(PU_EINVAL, "not a PRIMEMSG v1 log of 24-byte MsgMem records");
        return nullptr;
    }
    pu_msglog* L = new (std::nothrow) pu_msglog;
    if (!L) {
        std::fclose(f);
        pu::set_error(PU_ENOMEM, "out of host memory");
        return nullptr;
    }
    L->f = f;
    L->sched.stat.assign(num_cores > 0 ? (size_t)num_cores : 0, 0);
    return L;
}

pu_msglog* pu_msglog_create(const char* path) {
    FILE* f = path ? std::fopen(path, "wb") : nullptr;
    if (!f) {
        pu::set_error(PU_EIO, "cannot create message log");
        return nullptr;
    }
    const uint32_t ver = 1, rec = sizeof(MsgMemRec);
    if (std::fwrite(kMagic, 1, 8, f) != 8 || std::fwrite(&ver, 4, 1, f) != 1 || std::fwrite(&rec, 4, 1, f) != 1) {
        std::fclose(f);
        pu::set_error(PU_EIO, "short write on message log");
        return nullptr;
    }
    pu_msglog* L = new (std::nothrow) pu_msglog;
    if (!L) {
        std::fclose(f);
        pu::set_error(PU_ENOMEM, "out of host memory");
        return nullptr;
    }
    L->f = f;
    L->write = true;
    return L;
}

int pu_msglog_append(pu_msglog* L, int32_t source, const void* records, int32_t n_records) {
    if (!L || !L->write || n_records < 1 || !records) return pu::set_error(PU_EINVAL, "bad arguments");
    if (std::fwrite(&source, 4, 1, L->f) != 1 || std::fwrite(&n_records, 4, 1, L->f) != 1 ||
        std::fwrite(records, sizeof(MsgMemRec), (size_t)n_records, L->f) != (size_t)n_records)
        return pu::set_error(PU_EIO, "short write on message log");
    L->messages++;
    return 0;
}

int pu_msglog_close(pu_msglog* L) {
    if (!L) return 0;
    int rc = 0;
    if (L->f && std::fclose(L->f) != 0) rc = pu::set_error(PU_EIO, "close failed");
    delete L;
    return rc;
}

int64_t pu_msglog_messages(const pu_msglog* L) { return L ? L->messages : PU_EINVAL; }

// Replays messages through h's ThreadSched (or, with h == NULL, the log's own
// over num_cores cores) and fills out[0..cap) with the
// requests they carry.  A message's requests may span calls (batch_start
// marks only its first).  Returns the number written; 0 at the end of the
// log (or after PROGRAM_EXITING); a negative PU_E* on a malformed log or when
// allocCore finds no free core (prime.cpp:94-101 aborts there).
int64_t pu_msglog_next(pu_msglog* L, pu_handle* h, pu_req* out, size_t cap) {
    if (!L || L->write || (!out && cap)) return pu::set_error(PU_EINVAL, "bad arguments");
    size_t k = 0;
    while (k < cap) {
        if (L->next < L->len) {                       // requests left in the current message
            const MsgMemRec& m = L->msg[L->next];
            pu_req& r = out[k++];
            std::memset(&r, 0, sizeof(r));
            r.addr = m.addr_dmem;
            r.timer = m.timer;
            r.core = L->core;
            r.prog_id = L->source;
            r.mem_type = m.mem_type ? PU_WR : PU_RD;
            r.batch_start = L->next == 1 ? 1 : 0;
            L->next++;
            continue;
        }
        if (L->ended) break;
        int32_t src = 0, n = 0;
        if (std::fread(&src, 4, 1, L->f) != 1) {     // clean end of log
            L->ended = true;
            break;
        }
        if (std::fread(&n, 4, 1, L->f) != 1 || n < 1 || n > (1 << 24))
            return pu::set_error(PU_EINVAL, "malformed message header in log");
        L->msg.resize((size_t)n);
        if (std::fread(L->msg.data(), sizeof(MsgMemRec), (size_t)n, L->f) != (size_t)n)
            return pu::set_error(PU_EINVAL, "truncated message in log");
        L->messages++;
        const MsgMemRec& hd = L->msg[0];
        const int64_t type = hd.timer;
        L->next = L->len = 0;
        if (type == kProcessStarting || type == kProcessFinishing || type == kBarrier) continue;
        if (type == kProgramExiting) {
            L->ended = true;
            break;
        }
        if (type == kNewThread) {
            if ((h ? pu_alloc_core(h, src, hd.mem_size) : L->sched.alloc(src, hd.mem_size)) < 0)
                return pu::set_error(PU_ERANGE, "Not enough cores (prime.cpp:94-101)");
            continue;
        }
        if (type == kThreadFinishing) {
            if (h) pu_dealloc_core(h, src, hd.mem_size);
            else L->sched.dealloc(src, hd.mem_size);
            continue;
        }
        // MEM_REQUESTS (prime.cpp:120-137): records 1 .. addr_dmem - 1
        const uint64_t msg_len = hd.addr_dmem;
        if (msg_len > (uint64_t)n) return pu::set_error(PU_EINVAL, "message length exceeds its records");
        L->source = src;
        L->core = h ? pu_get_core_id(h, src, hd.mem_size) : L->sched.get(src, hd.mem_size);
        L->next = 1;
        L->len = (size_t)msg_len;
    }
    return (int64_t)k;
}

}  // extern "C"

extern "C" {

// A synthetic request stream as the message log its cores would have sent:
// one NEW_THREAD per thread (thread_prog/thread_id, allocation order), then
// one MEM_REQUESTS message per batch (header: mem_size = thread id,
// addr_dmem = records incl. header, message_type 0; core_manager.cpp:244-255).
// core_thread[c] gives core c's thread index into the thread table.
int pu_msglog_from_requests(const char* path, const pu_req* reqs, size_t n, const int32_t* thread_prog,
                            const int32_t* thread_id, int num_threads, const int32_t* core_thread, int num_cores) {
    if (!path || (!reqs && n) || num_threads < 0 || num_cores < 0) return pu::set_error(PU_EINVAL, "bad arguments");
    pu_msglog* L = pu_msglog_create(path);
    if (!L) return PU_EIO;
    int rc = 0;
    for (int t = 0; t < num_threads && !rc; t++) {
        MsgMemRec m{};
        m.mem_size = thread_id[t];
        m.timer = kNewThread;
        rc = pu_msglog_append(L, thread_prog[t], &m, 1);
    }
    std::vector<MsgMemRec> msg;
    size_t i = 0;
    while (i < n && !rc) {
        size_t j = i + 1;
        while (j < n && !reqs[j].batch_start) j++;
        const int c = reqs[i].core;
        if (c < 0 || c >= num_cores) {
            rc = pu::set_error(PU_ERANGE, "request core outside the thread table");
            break;
        }
        const int t = core_thread[c];
        msg.assign(j - i + 1, MsgMemRec{});
        msg[0].mem_size = thread_id[t];
        msg[0].addr_dmem = (uint64_t)(j - i + 1);
        msg[0].timer = 0;                               // MEM_REQUESTS
        for (size_t k = i; k < j; k++) {
            MsgMemRec& m = msg[k - i + 1];
            m.mem_type = reqs[k].mem_type == PU_WR ? 1 : 0;
            m.mem_size = 8;
            m.addr_dmem = reqs[k].addr;
            m.timer = reqs[k].timer;
        }
        rc = pu_msglog_append(L, reqs[i].prog_id, msg.data(), (int32_t)msg.size());
        i = j;
    }
    int rc2 = pu_msglog_close(L);
    return rc ? rc : rc2;
}

}  // extern "C"
