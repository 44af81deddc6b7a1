// stream.cpp — deterministic synthetic request streams and trace files.
//
// The reference records no traces and ships no streams, so
// the parity harness and the benchmark drive the uncore with seeded synthetic
// streams that follow the request-stream semantics of the reference's core
// model (core_manager.cpp:240-269):
//   * one splitmix64 per core, seeded seed*2^32 + core;
//   * a core issues a memory request at its current cycle, then advances
//     by 1 + U{0..3} cycles (cpi_nonmem = 1 gaps);
//   * every `quantum` cycles the core reaches a barrier (core_manager.cpp:104-198):
//     it flushes its partial message, so a message never spans a barrier;
//   * messages hold at most `max_msg` requests (core_manager.cpp:251);
//   * canonical order: quantum-major, then core id,
//     message-atomic.  Timers are recorded values (open-loop replay).
//
// Address patterns (PARSEC/Pin are unavailable, so C1/C2 are
// labelled stand-ins):
//   C1 private streaming   90% reads; 95% sequential 8-B words over a 2 MB
//                          private region, 5% random reads of a 64 KB table
//   C2 shared uniform      70% uniform over 64 MB, 30% re-use of one of the
//                          core's last 16 addresses; 30% writes
//   C3 multiprogram        4 programs, footprints 4/16/32/64 MB, same virtual
//                          range per program; 50% per-core streaming, 50%
//                          uniform over the program footprint; 20% writes
//   C4 uniform + hotspot   80% uniform over 2^20 lines (64 MB), 20% over a
//                          64-line hotspot; 25% writes
//   C5 producer/consumer   core p and p + C/2 share a 1024-line buffer; 50% writes
//   uniform                100% uniform over 2^20 lines; 25% writes

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "../../include/primeuncore.h"
#include "common.h"

namespace {

struct SplitMix64 {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
};

constexpr uint64_t kLine = 64;
constexpr uint64_t kMB = 1ull << 20;

struct CoreGen {
    SplitMix64 rng;
    int64_t cycle = 0;
    uint64_t stream_pos = 0;      // streaming word index
    uint64_t recent[16] = {0};    // C2 re-use ring
    int n_recent = 0;
    int recent_head = 0;
};

int default_write_pct(int kind) {
    switch (kind) {
        case PU_STREAM_PRIVATE_STREAMING: return 10;
        case PU_STREAM_SHARED_UNIFORM: return 30;
        case PU_STREAM_MULTIPROGRAM: return 20;
        case PU_STREAM_UNIFORM_HOTSPOT: return 25;
        case PU_STREAM_PRODUCER_CONSUMER: return 50;
        case PU_STREAM_UNIFORM: return 25;
        default: return -1;
    }
}

int prog_of(const pu_stream_params* p, int core) {
    int np = p->num_progs > 0 ? p->num_progs : 1;
    return 1 + (int)((int64_t)core * np / p->num_cores);
}

// One request's address and type for core `c`.
void make_request(const pu_stream_params* p, int c, CoreGen& g, int wpct,
                  uint64_t* addr, uint8_t* type) {
    uint64_t r0 = g.rng.next();
    uint64_t r1 = g.rng.next();
    uint64_t word = (r1 >> 20) & 7;  // 8-byte word within the line
    bool wr = (int)(r1 % 100) < wpct;
    uint64_t a = 0;
    switch (p->kind) {
        case PU_STREAM_PRIVATE_STREAMING: {
            if (r0 % 100 < 5) {  // shared read-mostly table
                a = 0x10000000ull + (r0 >> 8) % (64 * 1024 / 8) * 8;
                wr = false;
            } else {
                uint64_t base = 0x100000000ull + (uint64_t)c * 16 * kMB;
                a = base + (g.stream_pos * 8) % (2 * kMB);
                g.stream_pos++;
            }
            break;
        }
        case PU_STREAM_SHARED_UNIFORM: {
            if (r0 % 100 < 30 && g.n_recent > 0) {
                a = g.recent[(r0 >> 8) % (uint64_t)g.n_recent];
            } else {
                a = 0x40000000ull + (r0 >> 8) % (64 * kMB / 8) * 8;
                g.recent[g.recent_head] = a;
                g.recent_head = (g.recent_head + 1) & 15;
                if (g.n_recent < 16) g.n_recent++;
            }
            break;
        }
        case PU_STREAM_MULTIPROGRAM: {
            static const uint64_t fp_mb[4] = {4, 16, 32, 64};
            int prog = prog_of(p, c);
            uint64_t fp = fp_mb[(prog - 1) & 3] * kMB;
            uint64_t base = 0x80000000ull;
            if (r0 % 100 < 50) {
                int np = p->num_progs > 0 ? p->num_progs : 1;
                int per = p->num_cores / np > 0 ? p->num_cores / np : 1;
                uint64_t slice = fp / (uint64_t)per;
                if (slice < kLine) slice = kLine;
                uint64_t first = (uint64_t)(c % per) * slice;
                a = base + (first + (g.stream_pos * 8) % slice) % fp;
                g.stream_pos++;
            } else {
                a = base + (r0 >> 8) % (fp / 8) * 8;
            }
            break;
        }
        case PU_STREAM_UNIFORM_HOTSPOT: {
            if (r0 % 100 < 20) {
                a = 0x20000000ull + ((r0 >> 8) % 64) * kLine + word * 8;
            } else {
                a = 0x40000000ull + ((r0 >> 8) % (1ull << 20)) * kLine + word * 8;
            }
            break;
        }
        case PU_STREAM_PRODUCER_CONSUMER: {
            int half = p->num_cores / 2 > 0 ? p->num_cores / 2 : 1;
            int pair = c % half;
            a = 0x100000000ull + (uint64_t)pair * 1024 * kLine + ((r0 >> 8) % 1024) * kLine + word * 8;
            break;
        }
        case PU_STREAM_UNIFORM:
        default: {
            a = 0x40000000ull + ((r0 >> 8) % (1ull << 20)) * kLine + word * 8;
            break;
        }
    }
    *addr = a;
    *type = wr ? PU_WR : PU_RD;
}

bool params_ok(const pu_stream_params* p) {
    if (!p) return false;
    if (p->kind < PU_STREAM_PRIVATE_STREAMING || p->kind > PU_STREAM_UNIFORM) return false;
    if (p->num_cores <= 0 || p->quantum <= 0 || p->num_quanta < 0 || p->max_msg <= 0) return false;
    return true;
}

// The generator's whole state, so a stream can be produced in consecutive
// chunks (pu_stream_next) that concatenate to exactly pu_stream_generate's
// output: per-core RNG/cycle state plus the (quantum, core, message) cursor.
struct StreamGen {
    pu_stream_params p{};
    int wpct = 0;
    std::vector<CoreGen> gens;
    int q = 0;            // current quantum
    int c = 0;            // current core within the quantum
    int in_msg = 0;       // requests already in the core's open message
    int64_t n = 0;        // requests produced so far
    int64_t limit = INT64_MAX;

    void init(const pu_stream_params* pp) {
        p = *pp;
        wpct = p.write_pct >= 0 ? p.write_pct : default_write_pct(p.kind);
        gens.assign((size_t)p.num_cores, CoreGen{});
        for (int k = 0; k < p.num_cores; k++) gens[(size_t)k].rng.s = p.seed * 0x100000000ull + (uint64_t)k;
        limit = p.max_requests > 0 ? p.max_requests : INT64_MAX;
    }

    // Up to `cap` more requests in canonical order (quantum-major, then core
    // id, message-atomic); out == nullptr only counts.
    int64_t next(pu_req* out, int64_t cap) {
        int64_t k = 0;
        while (q < p.num_quanta && n < limit && k < cap) {
            const int64_t barrier = (int64_t)(q + 1) * p.quantum;
            CoreGen& g = gens[(size_t)c];
            if (g.cycle >= barrier) {          // core c reached the barrier: next core / quantum
                in_msg = 0;
                if (++c == p.num_cores) {
                    c = 0;
                    q++;
                }
                continue;
            }
            uint64_t a;
            uint8_t t;
            make_request(&p, c, g, wpct, &a, &t);
            if (out) {
                pu_req& r = out[k];
                std::memset(&r, 0, sizeof(r));
                r.addr = a;
                r.timer = g.cycle;
                r.core = c;
                r.prog_id = prog_of(&p, c);
                r.mem_type = t;
                r.batch_start = in_msg == 0 ? 1 : 0;
            }
            k++;
            n++;
            in_msg = (in_msg + 1) % p.max_msg;
            g.cycle += 1 + (int64_t)(g.rng.next() & 3);
        }
        return k;
    }
};

// Generates the whole stream; when out == nullptr only counts.
int64_t run(const pu_stream_params* p, pu_req* out, size_t cap) {
    if (!params_ok(p)) return PU_EINVAL;
    StreamGen g;
    g.init(p);
    if (!out) return g.next(nullptr, INT64_MAX);
    int64_t got = g.next(out, (int64_t)cap);
    if (got == (int64_t)cap && g.next(nullptr, 1) != 0) return PU_ERANGE;   // more than cap requests
    return got;
}

}  // namespace

extern "C" {

int64_t pu_stream_count(const pu_stream_params* p) { return run(p, nullptr, 0); }

int64_t pu_stream_generate(const pu_stream_params* p, pu_req* out, size_t cap) {
    if (!out) return PU_EINVAL;
    return run(p, out, cap);
}

int pu_stream_thread_of(const pu_stream_params* p, int core, int* prog_id, int* thread_id) {
    if (!params_ok(p) || core < 0 || core >= p->num_cores) return PU_EINVAL;
    int prog = prog_of(p, core);
    int first = core;
    while (first > 0 && prog_of(p, first - 1) == prog) first--;
    if (prog_id) *prog_id = prog;
    if (thread_id) *thread_id = core - first;
    return 0;
}

struct pu_stream {
    StreamGen g;
};

pu_stream* pu_stream_open(const pu_stream_params* p) {
    if (!params_ok(p)) {
        pu::set_error(PU_EINVAL, "invalid stream parameters");
        return nullptr;
    }
    pu_stream* s = new (std::nothrow) pu_stream;
    if (!s) {
        pu::set_error(PU_ENOMEM, "out of host memory");
        return nullptr;
    }
    s->g.init(p);
    return s;
}

void pu_stream_close(pu_stream* s) { delete s; }

int64_t pu_stream_next(pu_stream* s, pu_req* out, size_t n) {
    if (!s || (!out && n)) return PU_EINVAL;
    return s->g.next(out, (int64_t)n);
}

int64_t pu_stream_position(const pu_stream* s) { return s ? s->g.n : PU_EINVAL; }

int64_t pu_stream_next_many(pu_stream* const* s, int count, pu_req* out, size_t n_each, size_t stride,
                            int threads) {
    if (!s || count < 0 || (!out && n_each && count) || stride < n_each) return PU_EINVAL;
    for (int i = 0; i < count; i++)
        if (!s[i]) return PU_EINVAL;
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (threads > count) threads = count;
    if (threads < 1) threads = 1;
    std::vector<int64_t> got((size_t)count, 0);
    auto work = [&](int t0) {
        for (int i = t0; i < count; i += threads) got[(size_t)i] = s[i]->g.next(out + (size_t)i * stride, (int64_t)n_each);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    int64_t mn = count ? got[0] : 0;
    for (int64_t v : got) mn = v < mn ? v : mn;
    return mn;
}

int pu_trace_write(const char* path, const pu_req* reqs, size_t n, const int32_t* thread_prog,
                   const int32_t* thread_id, int num_threads) {
    if (!path || (!reqs && n) || num_threads < 0) return PU_EINVAL;
    FILE* f = std::fopen(path, "wb");
    if (!f) return pu::set_error(PU_EIO, "cannot open trace file");
    const char magic[8] = {'P', 'U', 'T', 'R', 'A', 'C', 'E', '1'};
    uint64_t nn = n;
    int32_t nt = num_threads;
    bool ok = std::fwrite(magic, 1, 8, f) == 8 && std::fwrite(&nt, 4, 1, f) == 1;
    for (int i = 0; ok && i < num_threads; i++) {
        ok = std::fwrite(&thread_prog[i], 4, 1, f) == 1 && std::fwrite(&thread_id[i], 4, 1, f) == 1;
    }
    ok = ok && std::fwrite(&nn, 8, 1, f) == 1;
    ok = ok && (n == 0 || std::fwrite(reqs, sizeof(pu_req), n, f) == n);
    std::fclose(f);
    return ok ? 0 : pu::set_error(PU_EIO, "short write on trace file");
}

}  // extern "C"
