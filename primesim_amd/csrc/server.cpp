// server.cpp — prime.cpp's server front-end over a Unix-domain socket
// (SURVEY.md §8f row 4), feeding the engine one launch per round.
//
// The reference's uncore process (src/prime.cpp) receives MsgMem buffers
// from the Pin processes over MPI (MPI_Recv from MPI_ANY_SOURCE, prime.cpp:53)
// and answers with one int per message (MPI_Send).  Here the transport is a
// stream socket with a 16-byte frame header, and the uncore is the HIP engine:
//
//   client -> server   HELLO {session, rank}     (once per connection)
//                      SEND  {tag, n_bytes} + n_bytes of MsgMem records
//                      RECV  {tag}              (post MPI_Recv(.., tag))
//   server -> client   REPLY {tag, value}       (answers the oldest RECV)
//
// Handler rules follow prime.cpp:55-137 message by message (see the header
// comment in include/primeuncore.h).  What is MI355X-specific is the round
// structure: the memory-request batches of every session that are pending in
// a round are laid out replica-major and run by one pu_run_device launch (one
// wavefront per session), instead of one blocking uncore_access loop per
// message on a CPU thread.

#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <set>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/primeuncore.h"
#include "common.h"
#include "geometry.h"

namespace {

// reference MsgMem (common.h:49-59), x86-64 layout
struct MsgRec {
    uint8_t mem_type;
    uint8_t _pad[3];
    int32_t mem_size;
    uint64_t addr_dmem;
    int64_t timer;   // message_type in a header record
};
static_assert(sizeof(MsgRec) == 24, "MsgMem is 24 bytes");

// MessageTypes (common.h:38-47)
constexpr int64_t kProcessStarting = -3, kProcessFinishing = -1, kBarrier = -2, kNewThread = -4,
                  kThreadFinishing = -8, kProgramExiting = -5;

enum : int32_t { kHello = 1, kSend = 2, kRecv = 3, kReply = 4 };
struct Frame {
    int32_t kind, tag, a, b;
};
static_assert(sizeof(Frame) == 16, "frame header");
constexpr int32_t kMaxPayload = 1 << 26;

bool write_all(int fd, const void* p, size_t n) {
    const char* c = (const char*)p;
    while (n) {
        ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
        if (w < 0 && errno == EINTR) continue;
        if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
            pollfd pf{fd, POLLOUT, 0};
            ::poll(&pf, 1, 1000);
            continue;
        }
        if (w <= 0) return false;
        c += w;
        n -= (size_t)w;
    }
    return true;
}

bool read_all(int fd, void* p, size_t n) {
    char* c = (char*)p;
    while (n) {
        ssize_t r = ::recv(fd, c, n, 0);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        c += r;
        n -= (size_t)r;
    }
    return true;
}

struct Conn {
    int fd = -1;
    int session = -1, rank = -1;
    std::vector<char> in;   // bytes received, not yet parsed
    bool dead = false;
};

// One received message of a session, waiting to be handled.
struct Msg {
    Conn* conn;
    int rank;
    int tag;                  // MPI tag = the receive thread that takes it (prime.cpp:53)
    std::vector<MsgRec> rec;
};

// A MEM_REQUESTS message taken into this round's launch.
struct Batch {
    int session, rank, tag;   // tag: the reply tag (the sender's thread id)
    int recv;                 // the receive thread (the message's MPI tag)
    size_t first, n;          // its requests in the session's slice of the round
};

// Executor: runs a round's requests, all sessions at once.
struct Exec {
    virtual ~Exec() = default;
    // reqs: session-major; off[s]..off[s+1] = session s.  delays: same index.
    virtual int run(const std::vector<pu_req>& reqs, const std::vector<uint64_t>& off, int32_t* delays) = 0;
    virtual int alloc(int s, int prog, int th) = 0;
    virtual int dealloc(int s, int prog, int th) = 0;
    virtual int get(int s, int prog, int th) = 0;
    virtual std::string report(int s) = 0;
    // PU_ERRF_LIMITS bits of session s after the last run (0: exact so far)
    virtual uint64_t limit_flags(int) { return 0; }
    // index (into the last run's reqs) of the first request of session s that
    // raised one of them: every request before it is exact.  0 = unknown;
    // UINT64_MAX = none in the last run (the bits then predate it).
    virtual uint64_t limit_at(int) { return 0; }
};

// The product executor: the HIP engine, one wavefront per session.
struct EngineExec : Exec {
    pu_handle* h;
    int R;
    pu_req* d_reqs = nullptr;
    int32_t* d_delays = nullptr;
    uint64_t* d_off = nullptr;
    size_t cap = 0;
    explicit EngineExec(pu_handle* hh) : h(hh), R(pu_num_replicas(hh)) { pu_sim_start_time(hh); }   // prime.cpp:207
    ~EngineExec() override {
        if (d_reqs) (void)hipFree(d_reqs);
        if (d_delays) (void)hipFree(d_delays);
        if (d_off) (void)hipFree(d_off);
    }
    int run(const std::vector<pu_req>& reqs, const std::vector<uint64_t>& off, int32_t* delays) override {
        const size_t n = reqs.size();
        if (n > cap) {
            size_t c = std::max<size_t>(n, 2 * cap);
            if (d_reqs) (void)hipFree(d_reqs);
            if (d_delays) (void)hipFree(d_delays);
            d_reqs = nullptr;
            d_delays = nullptr;
            if (hipMalloc(&d_reqs, c * sizeof(pu_req)) != hipSuccess ||
                hipMalloc(&d_delays, c * sizeof(int32_t)) != hipSuccess)
                return pu::set_error(PU_ENOMEM, "server: request staging");
            cap = c;
        }
        if (!d_off && hipMalloc(&d_off, ((size_t)R + 1) * sizeof(uint64_t)) != hipSuccess)
            return pu::set_error(PU_ENOMEM, "server: offsets");
        // replicas past the served sessions get empty ranges
        std::vector<uint64_t> full((size_t)R + 1, (uint64_t)n);
        std::copy(off.begin(), off.end(), full.begin());
        if (hipMemcpy(d_reqs, reqs.data(), n * sizeof(pu_req), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(d_off, full.data(), full.size() * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess)
            return pu::set_error(PU_EIO, "server: upload");
        // a negative running delay stops only that message's receive thread
        // live client timers already include the earlier replies' delays
        // (core_manager.cpp:265): the server never applies the handle's
        // closed-loop replay shift, whatever mode the handle was left in
        int rc = pu::run_device_flags(h, d_reqs, d_off, d_delays, PU_KF_MSGHALT, /*use_replay_mode=*/false);
        if (!rc) rc = pu_synchronize(h);
        if (rc) return rc;
        if (hipMemcpy(delays, d_delays, n * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
            return pu::set_error(PU_EIO, "server: download");
        flags.assign(off.size() - 1, 0);
        int frc = pu_error_flags(h, flags.data(), flags.size());
        if (frc) return frc;
        at.assign(off.size() - 1, 0);
        return pu::limit_positions(h, at.data(), at.size());
    }
    std::vector<uint64_t> flags, at;
    uint64_t limit_flags(int s) override {
        return (size_t)s < flags.size() ? flags[(size_t)s] & PU_ERRF_LIMITS : 0;
    }
    uint64_t limit_at(int s) override { return (size_t)s < at.size() ? at[(size_t)s] : 0; }
    int alloc(int s, int p, int t) override { return pu_alloc_core_replica(h, s, p, t); }
    int dealloc(int s, int p, int t) override { return pu_dealloc_core_replica(h, s, p, t); }
    int get(int s, int p, int t) override { return pu_get_core_id_replica(h, s, p, t); }
    std::string report(int s) override {
        pu_sim_finish_time(h);                      // prime.cpp:232-233
        long len = pu_report(h, s, 1, nullptr, 0);
        if (len < 0) return std::string();
        std::string out((size_t)len + 1, '\0');
        pu_report(h, s, 1, &out[0], out.size());
        out.resize((size_t)len);
        return out;
    }
};

// Host executor (tests of the protocol without a GPU).
struct FnExec : Exec {
    pu_exec_fn fn;
    void* ctx;
    std::vector<pu::Sched> sched;
    std::vector<uint64_t> flags;
    FnExec(pu_exec_fn f, void* c, int sessions, int cores) : fn(f), ctx(c), sched((size_t)sessions) {
        for (auto& s : sched) s.stat.assign((size_t)cores, 0);
        flags.assign((size_t)sessions, 0);
    }
    int run(const std::vector<pu_req>& reqs, const std::vector<uint64_t>& off, int32_t* delays) override {
        for (size_t s = 0; s + 1 < off.size(); s++) {
            size_t a = off[s], b = off[s + 1];
            if (b > a) {
                int rc = fn(ctx, (int)s, reqs.data() + a, b - a, delays + a);
                if (rc < 0) return rc;
                flags[s] |= (uint64_t)rc;      // > 0: PU_ERRF_* bits of that session's replica
            }
        }
        return 0;
    }
    uint64_t limit_flags(int s) override { return flags[(size_t)s] & PU_ERRF_LIMITS; }
    int alloc(int s, int p, int t) override { return sched[(size_t)s].alloc(p, t); }
    int dealloc(int s, int p, int t) override { return sched[(size_t)s].dealloc(p, t); }
    int get(int s, int p, int t) override { return sched[(size_t)s].get(p, t); }
    std::string report(int) override { return std::string(); }
};

struct Session {
    bool started = false, ended = false, halted = false;
    std::set<int> done_tags;    // receive threads that returned (PROGRAM_EXITING, negative delay)
    std::list<int> prog_list;   // prime.h: list<int> prog_list
    size_t prog_count = 0;
    std::deque<Msg> backlog;
    // MPI matching at the server: values sent to (rank, tag) before a receive
    // is posted, and receives posted before a value arrived
    std::map<std::pair<int, int>, std::deque<int32_t>> mailbox;
    std::map<std::pair<int, int>, std::deque<Conn*>> waiters;
};

}  // namespace

struct pu_server {
    std::unique_ptr<Exec> exec;
    std::string path, prefix;
    int nsessions = 1, nthreads = 1, max_msg = 100, verbose = 0;
    int lfd = -1;
    std::vector<std::unique_ptr<Conn>> conns;
    std::vector<Session> sess;
    std::atomic<bool> stop{false};
    pu_server_stats st{};
};

namespace {

void reply(Conn* c, int tag, int32_t value) {
    if (!c || c->dead) return;
    Frame f{kReply, tag, value, 0};
    if (!write_all(c->fd, &f, sizeof f)) c->dead = true;
}

void deliver(Session& S, int rank, int tag, int32_t value) {
    auto& w = S.waiters[{rank, tag}];
    if (!w.empty()) {
        Conn* c = w.front();
        w.pop_front();
        reply(c, tag, value);
    } else {
        S.mailbox[{rank, tag}].push_back(value);
    }
}

void post_recv(Session& S, Conn* c, int tag) {
    auto& m = S.mailbox[{c->rank, tag}];
    if (!m.empty()) {
        int32_t v = m.front();
        m.pop_front();
        reply(c, tag, v);
    } else {
        S.waiters[{c->rank, tag}].push_back(c);
    }
}

void end_session(pu_server* s, int si) {
    Session& S = s->sess[(size_t)si];
    if (S.ended) return;
    S.ended = true;
    S.backlog.clear();
    s->st.sessions_ended++;
    if (!s->prefix.empty()) {
        std::string text = s->exec->report(si);
        std::string fn = s->prefix + "_" + std::to_string(si);
        if (FILE* f = std::fopen(fn.c_str(), "w")) {
            std::fwrite(text.data(), 1, text.size(), f);
            std::fclose(f);
        }
    }
    // connections of an ended session get EOF (a halted or aborted handler
    // leaves its clients without replies; EOF makes that an error, not a hang)
    // once they have collected the replies already sent to them (MPI_Send
    // buffers them: a client receives them after the handler has returned)
    for (auto& c : s->conns)
        if (c->session == si && !c->dead) {
            bool mail = false;
            for (const auto& kv : S.mailbox) mail |= kv.first.first == c->rank && !kv.second.empty();
            if (!mail) {
                ::shutdown(c->fd, SHUT_RDWR);
                c->dead = true;
            }
        }
}

// prime.cpp:55-118 for one control message; false = MEM_REQUESTS.
bool handle_control(pu_server* s, int si, Msg& m) {
    Session& S = s->sess[(size_t)si];
    const MsgRec& h = m.rec[0];
    const int src = m.rank;
    switch (h.timer) {
    case kProcessStarting:                                      // prime.cpp:55-61
        if (s->verbose) std::printf("[PriME] Process %d begins\n", src);
        S.prog_list.push_back(src);
        S.prog_list.unique();
        return true;
    case kProcessFinishing: {                                   // prime.cpp:63-76
        if (s->verbose) std::printf("[PriME] Process %d finishes\n", src);
        S.prog_list.remove(src);
        int32_t d = (int32_t)S.prog_list.size();
        deliver(S, src, 0, d);
        if (S.prog_count >= S.prog_list.size()) {
            for (int p : S.prog_list) deliver(S, p, 0, d);
            S.prog_count = 0;
        }
        return true;
    }
    case kBarrier:                                              // prime.cpp:78-88
        S.prog_count++;
        if (S.prog_count >= S.prog_list.size()) {
            int32_t d = (int32_t)S.prog_list.size();
            for (int p : S.prog_list) deliver(S, p, 0, d);
            S.prog_count = 0;
        }
        return true;
    case kNewThread: {                                          // prime.cpp:90-108
        int core = s->exec->alloc(si, src, h.mem_size);
        if (core == -1) {
            std::fprintf(stderr, "Not enough cores for process %d thread %d\n", src, h.mem_size);
            end_session(s, si);                                 // report, then MPI_Abort
            return true;
        }
        deliver(S, src, h.mem_size, core % s->nthreads);
        return true;
    }
    case kThreadFinishing:                                      // prime.cpp:110-114
        s->exec->dealloc(si, src, h.mem_size);
        return true;
    case kProgramExiting:                                       // prime.cpp:116-118: thread `tag` returns
        S.done_tags.insert(m.tag);
        if ((int)S.done_tags.size() >= s->nthreads) end_session(s, si);
        return true;
    default:
        return false;
    }
}

int parse_conn(pu_server* s, Conn* c) {
    size_t pos = 0;
    while (c->in.size() - pos >= sizeof(Frame)) {
        Frame f;
        std::memcpy(&f, c->in.data() + pos, sizeof f);
        size_t need = sizeof f + (f.kind == kSend ? (size_t)f.a : 0);
        if (f.kind == kSend && (f.a < 0 || f.a > kMaxPayload || f.a % (int)sizeof(MsgRec))) {
            c->dead = true;
            return 0;
        }
        if (c->in.size() - pos < need) break;
        if (f.kind == kHello) {
            if (f.a < 0 || f.a >= s->nsessions) {
                c->dead = true;
                return 0;
            }
            c->session = f.a;
            c->rank = f.b;
        } else if (c->session < 0) {
            c->dead = true;                     // protocol error: no HELLO
            return 0;
        } else if (f.kind == kRecv) {
            Session& S = s->sess[(size_t)c->session];
            if (!S.ended) {
                post_recv(S, c, f.tag);
            } else {                            // ended: hand out what was sent, then EOF
                auto& m = S.mailbox[{c->rank, f.tag}];
                if (!m.empty()) {
                    reply(c, f.tag, m.front());
                    m.pop_front();
                } else {
                    ::shutdown(c->fd, SHUT_RDWR);
                    c->dead = true;
                    return 0;
                }
            }
        } else if (f.kind == kSend && (f.tag < 0 || f.tag >= s->nthreads)) {
            // prime.cpp:53: handler thread k receives tag k only, k < num_recv_threads;
            // a message with any other tag is never received (and must not count as
            // some thread's PROGRAM_EXITING: the engine's dead-thread mask is tag & 63)
            std::fprintf(stderr, "[primeuncore] session %d: dropped a message with tag %d (receive threads 0..%d)\n",
                         c->session, f.tag, s->nthreads - 1);
        } else if (f.kind == kSend) {
            Session& S = s->sess[(size_t)c->session];
            int nrec = f.a / (int)sizeof(MsgRec);
            if (!S.ended && nrec > 0) {
                Msg m{c, c->rank, f.tag, std::vector<MsgRec>((size_t)nrec)};
                std::memcpy(m.rec.data(), c->in.data() + pos + sizeof f, (size_t)f.a);
                S.started = true;
                S.backlog.push_back(std::move(m));
            }
        } else {
            c->dead = true;
            return 0;
        }
        pos += need;
    }
    c->in.erase(c->in.begin(), c->in.begin() + (ptrdiff_t)pos);
    return 0;
}

void accept_all(pu_server* s) {
    for (;;) {
        int fd = ::accept(s->lfd, nullptr, nullptr);
        if (fd < 0) return;
        int fl = ::fcntl(fd, F_GETFL, 0);
        ::fcntl(fd, F_SETFL, fl | O_NONBLOCK);
        auto c = std::make_unique<Conn>();
        c->fd = fd;
        s->conns.push_back(std::move(c));
    }
}

// Read what the clients sent (waiting up to timeout_ms for anything).
void pump(pu_server* s, int timeout_ms) {
    std::vector<pollfd> pf;
    pf.push_back({s->lfd, POLLIN, 0});
    for (auto& c : s->conns) pf.push_back({c->fd, POLLIN, 0});
    int r = ::poll(pf.data(), pf.size(), timeout_ms);
    if (r <= 0) return;
    if (pf[0].revents & POLLIN) accept_all(s);
    char buf[1 << 16];
    for (size_t i = 1; i < pf.size(); i++) {
        Conn* c = s->conns[i - 1].get();
        if (!(pf[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        for (;;) {
            ssize_t n = ::recv(c->fd, buf, sizeof buf, 0);
            if (n > 0) {
                c->in.insert(c->in.end(), buf, buf + n);
                continue;
            }
            if (n == 0 || (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)) c->dead = true;
            break;
        }
        parse_conn(s, c);
    }
}

void reap(pu_server* s) {
    for (auto& S : s->sess)
        for (auto& kv : S.waiters) {
            auto& d = kv.second;
            d.erase(std::remove_if(d.begin(), d.end(), [](Conn* c) { return c->dead; }), d.end());
        }
    for (auto& S : s->sess)
        for (auto& m : S.backlog)
            if (m.conn && m.conn->dead) m.conn = nullptr;
    s->conns.erase(std::remove_if(s->conns.begin(), s->conns.end(),
                                  [](const std::unique_ptr<Conn>& c) {
                                      if (c->dead) ::close(c->fd);
                                      return c->dead;
                                  }),
                   s->conns.end());
}

int serve_round(pu_server* s, int timeout_ms) {
    bool backlog = false;
    for (auto& S : s->sess) backlog |= !S.backlog.empty();
    pump(s, backlog ? 0 : timeout_ms);
    std::vector<pu_req> reqs;
    std::vector<uint64_t> off((size_t)s->nsessions + 1, 0);
    std::vector<Batch> batches;
    std::vector<int> pending_exit;
    int handled = 0;
    for (int si = 0; si < s->nsessions; si++) {
        Session& S = s->sess[(size_t)si];
        off[(size_t)si] = reqs.size();
        bool mem = false;
        while (!S.backlog.empty() && !S.ended) {
            Msg& m = S.backlog.front();
            bool is_ctl = m.rec[0].timer == kProcessStarting || m.rec[0].timer == kProcessFinishing ||
                          m.rec[0].timer == kBarrier || m.rec[0].timer == kNewThread ||
                          m.rec[0].timer == kThreadFinishing || m.rec[0].timer == kProgramExiting;
            if (is_ctl && mem) break;           // wait for this round's batches to finish first
            handled++;
            if (S.done_tags.count(m.tag)) {     // its receive thread has returned: never received
                S.backlog.pop_front();
                continue;
            }
            if (is_ctl) {
                handle_control(s, si, m);
                if (!S.ended) S.backlog.pop_front();
                continue;
            }
            // MEM_REQUESTS (prime.cpp:120-137)
            const MsgRec& h = m.rec[0];
            const int thread_id = h.mem_size;
            int64_t msg_len = (int64_t)h.addr_dmem;
            msg_len = std::min<int64_t>(msg_len, (int64_t)m.rec.size());
            msg_len = std::min<int64_t>(msg_len, (int64_t)s->max_msg + 1);
            const int core = s->exec->get(si, m.rank, thread_id);
            Batch b{si, m.rank, thread_id, m.tag, reqs.size() - off[(size_t)si], 0};
            for (int64_t i = 1; i < msg_len; i++) {
                pu_req q;
                std::memset(&q, 0, sizeof q);
                q.addr = m.rec[(size_t)i].addr_dmem;
                q.timer = m.rec[(size_t)i].timer;
                q.core = core;
                q.prog_id = m.rank;
                q.mem_type = m.rec[(size_t)i].mem_type ? 1 : 0;
                q.batch_start = i == 1;
                q.tag = (uint16_t)m.tag;
                reqs.push_back(q);
                b.n++;
            }
            batches.push_back(b);
            mem = true;
            S.backlog.pop_front();
        }
    }
    off[(size_t)s->nsessions] = reqs.size();
    if (!reqs.empty()) {
        std::vector<int32_t> delays(reqs.size());
        int rc = s->exec->run(reqs, off, delays.data());
        if (rc) return rc;
        s->st.launches++;
        s->st.requests += reqs.size();
        for (const Batch& b : batches) {
            Session& S = s->sess[(size_t)b.session];
            if (S.ended) continue;
            const uint64_t lim = s->exec->limit_flags(b.session);
            const uint64_t at = s->exec->limit_at(b.session);
            // the limit bits are sticky across launches, the position is this
            // launch's: a bit with no position here was raised before this
            // launch (a handle stopped before serving, or served again after
            // pu_server_stop), so every request of this launch is suspect
            if (lim && (at == UINT64_MAX || off[(size_t)b.session] + b.first + b.n > at)) {
                // an engine limit stopped the replica where the reference continues:
                // batches that ended before the request that hit it were answered
                // exactly above; no reply is exact from here on: end the session
                std::fprintf(stderr, "[primeuncore] session %d stopped by an engine limit (error flags 0x%llx)\n",
                             b.session, (unsigned long long)lim);
                s->st.sessions_failed++;
                end_session(s, b.session);
                continue;
            }
            if (S.done_tags.count(b.recv)) continue;         // an earlier batch stopped this thread
            const int32_t* d = delays.data() + off[(size_t)b.session] + b.first;
            const pu_req* q = reqs.data() + off[(size_t)b.session] + b.first;
            int32_t D = 0;
            bool neg = false;
            for (size_t i = 0; i < b.n; i++) {
                D += d[i] - 1;                                  // prime.cpp:129
                if (D < 0) {                                    // prime.cpp:130-134
                    std::fprintf(stderr, "Error: negative delay: %d %d %d %d %llu\n", q[i].core, b.rank, b.tag,
                                 (int)q[i].mem_type, (unsigned long long)q[i].addr);
                    neg = true;
                    break;
                }
            }
            if (neg) {                                          // that handler thread returns, unanswered
                S.done_tags.insert(b.recv);
                if (!S.halted) s->st.sessions_halted++;
                S.halted = true;
                if ((int)S.done_tags.size() >= s->nthreads) end_session(s, b.session);
                continue;
            }
            deliver(S, b.rank, b.tag, D);                       // prime.cpp:136
        }
    } else {
        for (const Batch& b : batches) deliver(s->sess[(size_t)b.session], b.rank, b.tag, 0);
    }
    if (handled) s->st.rounds++;
    s->st.messages += (uint64_t)handled;
    reap(s);
    return handled;
}

pu_server* make_server(Exec* ex, const pu_server_opts* o) {
    std::unique_ptr<Exec> own(ex);
    if (!o || !o->socket_path || !*o->socket_path) {
        pu::set_error(PU_EINVAL, "server: socket path required");
        return nullptr;
    }
    auto s = std::make_unique<pu_server>();
    s->exec = std::move(own);
    s->path = o->socket_path;
    s->prefix = o->report_prefix ? o->report_prefix : "";
    s->nsessions = o->num_sessions > 0 ? o->num_sessions : 1;
    s->nthreads = o->num_recv_threads > 0 ? o->num_recv_threads : 1;
    if (s->nthreads > 64) {
        pu::set_error(PU_ENOTSUP, "server: at most 64 receive threads (the engine's per-thread stop mask)");
        return nullptr;
    }
    s->max_msg = o->max_msg_size > 0 ? o->max_msg_size : 100;
    s->verbose = o->verbose;
    s->sess.resize((size_t)s->nsessions);
    sockaddr_un addr;
    std::memset(&addr, 0, sizeof addr);
    addr.sun_family = AF_UNIX;
    if (s->path.size() >= sizeof(addr.sun_path)) {
        pu::set_error(PU_EINVAL, "server: socket path too long");
        return nullptr;
    }
    std::strcpy(addr.sun_path, s->path.c_str());
    s->lfd = ::socket(AF_UNIX, SOCK_STREAM, 0);
    if (s->lfd < 0) {
        pu::set_error(PU_EIO, "server: socket()");
        return nullptr;
    }
    ::unlink(s->path.c_str());
    if (::bind(s->lfd, (sockaddr*)&addr, sizeof addr) != 0 || ::listen(s->lfd, 256) != 0) {
        pu::set_error(PU_EIO, std::string("server: bind/listen ") + s->path + ": " + std::strerror(errno));
        ::close(s->lfd);
        return nullptr;
    }
    int fl = ::fcntl(s->lfd, F_GETFL, 0);
    ::fcntl(s->lfd, F_SETFL, fl | O_NONBLOCK);
    return s.release();
}

}  // namespace

extern "C" {

pu_server* pu_server_create(pu_handle* h, const pu_server_opts* o) {
    if (!h) {
        pu::set_error(PU_EINVAL, "server: null handle");
        return nullptr;
    }
    if (o && o->num_sessions > pu_num_replicas(h)) {
        pu::set_error(PU_ERANGE, "server: more sessions than replicas");
        return nullptr;
    }
    return make_server(new EngineExec(h), o);
}

pu_server* pu_server_create_exec(pu_exec_fn fn, void* ctx, int num_cores, const pu_server_opts* o) {
    if (!fn || num_cores < 1) {
        pu::set_error(PU_EINVAL, "server: executor and core count required");
        return nullptr;
    }
    int ns = o && o->num_sessions > 0 ? o->num_sessions : 1;
    return make_server(new FnExec(fn, ctx, ns, num_cores), o);
}

int pu_server_round(pu_server* s, int timeout_ms) {
    if (!s) return pu::set_error(PU_EINVAL, "null server");
    return serve_round(s, timeout_ms);
}

namespace {
// A live connection of an ended session still holds replies it has not collected.
bool undelivered(pu_server* s) {
    for (auto& c : s->conns) {
        if (c->dead || c->session < 0) continue;
        const Session& S = s->sess[(size_t)c->session];
        if (!S.ended) continue;
        for (const auto& kv : S.mailbox)
            if (kv.first.first == c->rank && !kv.second.empty()) return true;
    }
    return false;
}
}  // namespace

int pu_server_run(pu_server* s) {
    if (!s) return pu::set_error(PU_EINVAL, "null server");
    s->stop.store(false);        // pu_server_stop ends a run; a later run serves again
    std::chrono::steady_clock::time_point all_ended{};
    while (!s->stop.load()) {
        if (s->st.sessions_ended >= s->nsessions) {
            // every session has ended: keep serving receives while clients still
            // collect replies sent before the end (for at most 10 s)
            const auto now = std::chrono::steady_clock::now();
            if (all_ended == std::chrono::steady_clock::time_point{}) all_ended = now;
            if (!undelivered(s) || now - all_ended > std::chrono::seconds(10)) {
                for (auto& c : s->conns)             // EOF for whatever a client still waits on
                    if (!c->dead) {
                        ::shutdown(c->fd, SHUT_RDWR);
                        c->dead = true;
                    }
                return 0;
            }
        }
        int rc = serve_round(s, 50);
        if (rc < 0) return rc;
    }
    return 0;
}

void pu_server_stop(pu_server* s) {
    if (s) s->stop.store(true);
}

int pu_server_get_stats(pu_server* s, pu_server_stats* out) {
    if (!s || !out) return pu::set_error(PU_EINVAL, "bad arguments");
    *out = s->st;
    return 0;
}

void pu_server_destroy(pu_server* s) {
    if (!s) return;
    for (auto& c : s->conns) ::close(c->fd);
    if (s->lfd >= 0) ::close(s->lfd);
    ::unlink(s->path.c_str());
    delete s;
}

// ------------------------------------------------------------------ client
struct pu_client {
    int fd = -1;
    // replies that arrived for another tag than the one being waited for
    std::deque<std::pair<int, int32_t>> early;
};

pu_client* pu_client_connect(const char* socket_path, int session, int rank) {
    if (!socket_path) {
        pu::set_error(PU_EINVAL, "client: socket path required");
        return nullptr;
    }
    sockaddr_un addr;
    std::memset(&addr, 0, sizeof addr);
    addr.sun_family = AF_UNIX;
    if (std::strlen(socket_path) >= sizeof(addr.sun_path)) {
        pu::set_error(PU_EINVAL, "client: socket path too long");
        return nullptr;
    }
    std::strcpy(addr.sun_path, socket_path);
    int fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
    if (fd < 0 || ::connect(fd, (sockaddr*)&addr, sizeof addr) != 0) {
        pu::set_error(PU_EIO, std::string("client: connect ") + socket_path + ": " + std::strerror(errno));
        if (fd >= 0) ::close(fd);
        return nullptr;
    }
    Frame f{kHello, 0, session, rank};
    if (!write_all(fd, &f, sizeof f)) {
        ::close(fd);
        pu::set_error(PU_EIO, "client: hello");
        return nullptr;
    }
    auto* c = new pu_client;
    c->fd = fd;
    return c;
}

int pu_client_send(pu_client* c, int tag, const void* records, int n_records) {
    if (!c || (!records && n_records) || n_records < 0 ||
        (int64_t)n_records * (int64_t)sizeof(MsgRec) > kMaxPayload)
        return pu::set_error(PU_EINVAL, "client: bad send");
    Frame f{kSend, tag, n_records * (int32_t)sizeof(MsgRec), 0};
    std::vector<char> buf(sizeof f + (size_t)f.a);
    std::memcpy(buf.data(), &f, sizeof f);
    if (n_records) std::memcpy(buf.data() + sizeof f, records, (size_t)f.a);
    if (!write_all(c->fd, buf.data(), buf.size())) return pu::set_error(PU_EIO, "client: send");
    return 0;
}

int pu_client_recv(pu_client* c, int tag, int32_t* value) {
    if (!c || !value) return pu::set_error(PU_EINVAL, "client: bad recv");
    for (auto it = c->early.begin(); it != c->early.end(); ++it)
        if (it->first == tag) {
            *value = it->second;
            c->early.erase(it);
            return 0;
        }
    Frame f{kRecv, tag, 0, 0};
    if (!write_all(c->fd, &f, sizeof f)) return pu::set_error(PU_EIO, "client: recv request");
    for (;;) {
        Frame r;
        if (!read_all(c->fd, &r, sizeof r)) return pu::set_error(PU_EIO, "client: server closed the session");
        if (r.kind != kReply) return pu::set_error(PU_EIO, "client: bad reply");
        if (r.tag == tag) {
            *value = r.a;
            return 0;
        }
        c->early.emplace_back(r.tag, r.a);
    }
}

void pu_client_close(pu_client* c) {
    if (!c) return;
    if (c->fd >= 0) ::close(c->fd);
    delete c;
}

}  // extern "C"
